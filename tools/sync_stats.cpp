// sync_stats — self-synchronisation distances of the JPEG entropy decode.
//
// For a baseline JPEG (no restart markers): decode the destuffed scan
// sequentially and record the (block-in-MCU, coefficient index) state at
// every symbol boundary; then for each subsequence start k*S decode from the
// guess (symbol boundary, r = 0, z = 0) until the decode lands on a true
// boundary with the true state, and report the distance in bits.  This is
// what bounds the sync iterations of k_huff_sync.
//   g++ -O2 -std=c++17 -I datago_amd/csrc tools/sync_stats.cpp datago_amd/csrc/host/jpeg_header.cpp -o /tmp/sync_stats
//   /tmp/sync_stats S file.jpg...   -> one line per file: n p50 p90 p99 p999 max (bits)
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "dg_entropy.h"
#include "host/jpeg_header.h"

using namespace dg;

static std::vector<uint8_t> read_file(const char *p) {
  std::vector<uint8_t> v;
  FILE *f = fopen(p, "rb");
  if (!f) return v;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  v.resize((size_t)n);
  if (fread(v.data(), 1, (size_t)n, f) != (size_t)n) v.clear();
  fclose(f);
  return v;
}

struct Dec {
  std::vector<uint8_t> ds;
  std::vector<HuffTable> tabs;
  uint32_t slotmap = 0, comp_bits = 0, bpm = 0;
  uint32_t bits(uint32_t pos) const {  // 32 bits at pos, big-endian
    uint32_t i = pos >> 3;
    uint64_t v = 0;
    for (int k = 0; k < 5; k++) v = (v << 8) | (i + k < ds.size() ? ds[i + k] : 0);
    return (uint32_t)((v << (pos & 7)) >> 8);
  }
  // one symbol from (pos, r, z); returns false past the end
  void step(uint32_t &pos, uint32_t &r, uint32_t &z) const {
    const uint32_t comp = (comp_bits >> (2 * r)) & 3u;
    const bool isdc = z == 0;
    const uint32_t slot = (slotmap >> (((comp << 1) | (isdc ? 0u : 1u)) << 2)) & 15u;
    const uint32_t b = bits(pos);
    const uint32_t e = huff_lookup(tabs[slot], b);
    const uint32_t len = e >> 8, sym = e & 0xFF, size = sym & 15, run = isdc ? 0 : sym >> 4;
    pos += len + size;
    if (isdc) {
      z = 1;
    } else {
      const bool eob = size == 0 && run != 15;
      z = eob ? 64 : z + run + 1;
    }
    if (z >= 64) {
      z = 0;
      r = r + 1 == bpm ? 0 : r + 1;
    }
  }
};

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  const uint32_t S = (uint32_t)atoi(argv[1]);
  std::vector<uint32_t> all;
  for (int a = 2; a < argc; a++) {
    std::vector<uint8_t> f = read_file(argv[a]);
    JpegHeader h;
    parse_jpeg_header(f.data(), f.size(), h);
    if (h.status != JH_OK || h.restart) continue;
    Dec d;
    for (size_t i = h.scan_off; i < h.scan_end; i++) {
      d.ds.push_back(f[i]);
      if (f[i] == 0xFF && i + 1 < h.scan_end && f[i + 1] == 0x00) i++;
    }
    uint32_t bpm = 0;
    for (int c = 0; c < h.ncomp; c++) {
      const int nb = h.ncomp == 1 ? 1 : h.comp[c].h * h.comp[c].v;
      for (int j = 0; j < nb; j++) d.comp_bits |= (uint32_t)c << (2 * (bpm + j));
      bpm += nb;
      HuffTable t;
      build_huff_table(h.dc[h.comp[c].td], t);
      d.slotmap |= (uint32_t)d.tabs.size() << ((2 * c) * 4);
      d.tabs.push_back(t);
      build_huff_table(h.ac[h.comp[c].ta], t);
      d.slotmap |= (uint32_t)d.tabs.size() << ((2 * c + 1) * 4);
      d.tabs.push_back(t);
    }
    d.bpm = bpm;
    const uint32_t total = (uint32_t)d.ds.size() * 8;
    std::vector<uint16_t> truth(total + 64, 0);  // (r << 7 | z) + 1 at true boundaries
    uint64_t nsym = 0;
    uint32_t worst = 0;  // most symbols in any S-bit window starting at a multiple of S
    {
      uint32_t pos = 0, r = 0, z = 0, wstart = 0, wcount = 0;
      while (pos < total) {
        truth[pos] = (uint16_t)(((r << 7) | z) + 1);
        d.step(pos, r, z);
        nsym++;
        wcount++;
        if (pos - wstart >= S) {
          worst = std::max(worst, wcount);
          wstart += S;
          wcount = 0;
        }
      }
    }
    printf("  symbols=%llu bits=%u bits/sym=%.2f worst_syms_per_S=%u mean_syms_per_S=%.0f\n", (unsigned long long)nsym,
           total, (double)total / (double)nsym, worst, (double)nsym * S / total);
    std::vector<uint32_t> dist;
    for (uint32_t a0 = S; a0 + 64 < total; a0 += S) {
      uint32_t pos = a0, r = 0, z = 0, n = 0;
      for (;;) {
        if (pos < total && truth[pos] == (uint16_t)(((r << 7) | z) + 1)) break;
        if (pos >= total || ++n > 200000) {
          pos = a0 + 1000000;
          break;
        }
        d.step(pos, r, z);
      }
      dist.push_back(pos - a0);
    }
    if (dist.empty()) continue;
    all.insert(all.end(), dist.begin(), dist.end());
    std::sort(dist.begin(), dist.end());
    auto pct = [&](double p) { return dist[std::min(dist.size() - 1, (size_t)(p * dist.size()))]; };
    printf("%s %ux%u comps=%d bpm=%u n=%zu p50=%u p90=%u p99=%u max=%u\n", argv[a], h.width, h.height, h.ncomp, bpm,
           dist.size(), pct(0.5), pct(0.9), pct(0.99), dist.back());
  }
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
  if (!all.empty())
    printf("ALL n=%zu p50=%u p90=%u p99=%u p999=%u max=%u\n", all.size(), pct(0.5), pct(0.9), pct(0.99), pct(0.999),
           all.back());
  return 0;
}
