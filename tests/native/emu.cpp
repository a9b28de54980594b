// CPU emulation of the GPU entropy-decoding pipeline (test infrastructure).
// Runs the product's own dg_entropy.h decode_range() with the exact phase
// structure of k_huff_sync / k_huff_fix / k_huff_scan / k_huff_write
// (sequential over the threads of a workgroup, same read-then-write
// iteration semantics), so the parallel algorithm's logic can be checked
// against the oracle without a GPU.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "dg_entropy.h"
#include "host/jpeg_header.h"

using namespace dg;

static uint32_t g_lead = 0;
extern "C" void emu_set_lead(uint32_t lead) { g_lead = lead; }
// lead-ins whose multi-symbol result (k_huff_sync's) differs from the single-step one
static int64_t g_multi_mismatch = 0, g_multi_checked = 0;
extern "C" int64_t emu_multi_mismatch() { return g_multi_mismatch; }
extern "C" int64_t emu_multi_checked() { return g_multi_checked; }
// k_huff_sync2's two-chain SyncChain decode vs lead_in + decode_range per slot
// (entry state, accumulators, exit state and every checkpoint record)
static int64_t g_two_mismatch = 0, g_two_checked = 0;
extern "C" int64_t emu_two_mismatch() { return g_two_mismatch; }
extern "C" int64_t emu_two_checked() { return g_two_checked; }

extern "C" int emu_decode_coefs(const uint8_t *data, size_t len, uint32_t sub_bits, int16_t *out,
                                size_t cap_blocks, size_t *nblocks, int64_t *stats) {
  JpegHeader h;
  parse_jpeg_header(data, len, h);
  if (h.status != JH_OK) return h.status;
  ImageDesc d;
  memset(&d, 0, sizeof(d));
  const uint32_t W = h.width, H = h.height;
  d.ncomp = (uint8_t)h.ncomp;
  d.hmax = h.hmax;
  d.vmax = h.vmax;
  d.mcux = (W + 8 * d.hmax - 1) / (8 * d.hmax);
  d.mcuy = (H + 8 * d.vmax - 1) / (8 * d.vmax);
  uint32_t bpm = 0, cbw0 = 0, cbh0 = 0;
  for (int c = 0; c < h.ncomp; c++) {
    if (h.ncomp == 1) {
      uint32_t dsw = (W * h.comp[c].h + d.hmax - 1) / d.hmax, dsh = (H * h.comp[c].v + d.vmax - 1) / d.vmax;
      cbw0 = (dsw + 7) / 8;
      cbh0 = (dsh + 7) / 8;
      d.blk_comp[0] = 0;
      bpm = 1;
    } else {
      for (int j = 0; j < h.comp[c].h * h.comp[c].v; j++) d.blk_comp[bpm + j] = (uint8_t)c;
      bpm += h.comp[c].h * h.comp[c].v;
    }
  }
  d.bpm = bpm;
  for (uint32_t k = 0; k < bpm; k++) d.comp_bits |= (uint32_t)d.blk_comp[k] << (2 * k);
  d.total_blocks = h.ncomp == 1 ? cbw0 * cbh0 : d.mcux * d.mcuy * bpm;
  d.restart = h.restart;
  d.blocks_per_seg = d.restart * bpm;
  std::vector<HuffTable> tabs;
  d.slotmap = 0;
  for (int c = 0; c < h.ncomp; c++) {
    HuffTable t;
    build_huff_table(h.dc[h.comp[c].td], t);
    d.slotmap |= (uint32_t)tabs.size() << ((2 * c) * 4);
    tabs.push_back(t);
    build_huff_table(h.ac[h.comp[c].ta], t);
    d.slotmap |= (uint32_t)tabs.size() << ((2 * c + 1) * 4);
    tabs.push_back(t);
  }
  // k_huff_sync's multi-symbol lookups: one per component's AC table here (slots 2c + 1)
  std::vector<uint16_t> mt;
  uint32_t acm = 0xFFu;
  for (int c = 0; c < h.ncomp && c < (int)kMultiLuts; c++) {
    for (uint32_t p = 0; p < (1u << kMultiBits); p++) mt.push_back((uint16_t)multi_entry(tabs[2 * c + 1], p));
    acm = (acm & ~(3u << (2 * c))) | ((uint32_t)c << (2 * c));
  }
  d.scan_len = (uint32_t)(h.scan_end - h.scan_off);
  const uint8_t *raw = data + h.scan_off;
  // destuff exactly as k_destuff_* do (per byte, same classification function)
  std::vector<uint8_t> ds;
  std::vector<uint32_t> mk;
  for (uint32_t i = 0; i < d.scan_len; i++) {
    uint32_t prev = i ? raw[i - 1] : 0, next = i + 1 < d.scan_len ? raw[i + 1] : 0xD9, m;
    uint32_t keep = destuff_keep(prev, raw[i], next, i == 0, &m);
    if (m) mk.push_back((uint32_t)ds.size() * 8);
    if (keep) ds.push_back(raw[i]);
  }
  d.ds_bits = (uint32_t)ds.size() * 8;
  d.nmk = (uint32_t)mk.size();
  ds.resize(((ds.size() + 3) & ~(size_t)3) + 64, 0);
  d.sub_bits = sub_bits;
  d.lead_bits = g_lead;
  d.nsub = d.scan_len ? (uint32_t)(((uint64_t)d.scan_len * 8 + sub_bits - 1) / sub_bits) : 1;
  // the kernels' word-interleaved layout (ds_word_index)
  d.ds_lsw = 0;
  while ((32u << d.ds_lsw) < sub_bits) d.ds_lsw++;
  std::vector<uint32_t> phys((size_t)ds_words_alloc(d.nsub, d.ds_lsw), 0u);
  for (size_t wi = 0; wi * 4 < ds.size(); wi++) {
    uint32_t v;
    memcpy(&v, &ds[wi * 4], 4);
    const uint32_t pi = ds_word_index((uint32_t)wi, d.ds_lsw);
    if (pi < phys.size()) phys[pi] = v;
  }
  const uint8_t *scan = (const uint8_t *)phys.data();
  const uint32_t *mkp = mk.data();
  std::vector<SubState> subs(d.nsub);
  const uint32_t NCK = num_ckpt(d.sub_bits);
  std::vector<Ckpt> ck((size_t)d.nsub * (NCK ? NCK : 1));
  const uint32_t U = kSubPerWg - 1;  // useful subsequences per workgroup (thread 0 = lead-in)
  const uint32_t NW = (d.nsub + U - 1) / U;
  int64_t redo_total = 0, iters_max = 0, fix_wgs = 0, rounds = 0;
  auto ckp = [&](uint32_t s) { return NCK ? &ck[(size_t)s * NCK] : (Ckpt *)nullptr; };
  // ---- k_huff_sync2's chains: slots t and t + 128 of a workgroup on one lane
  {
    std::vector<Ckpt> ck1((size_t)d.nsub * (NCK ? NCK : 1)), ck2((size_t)d.nsub * (NCK ? NCK : 1));
    for (uint32_t wg = 0; wg < NW; wg++) {
      const uint32_t s0 = wg * U;
      for (uint32_t t = 0; t < 128; t++) {
        SyncChain<HuffTable> ch[2];
        uint32_t sv[2];
        bool act[2];
        for (int hh = 0; hh < 2; hh++) {
          const uint32_t q = t + 128 * hh;
          const int64_t si = (int64_t)s0 + q - 1;
          act[hh] = si >= 0 && si < (int64_t)d.nsub;
          sv[hh] = act[hh] ? (uint32_t)si : 0u;
          schain_begin(ch[hh], d, tabs.data(), scan, mkp, sv[hh], d.lead_bits, act[hh],
                       (q > 0 && act[hh] && NCK) ? &ck2[(size_t)sv[hh] * NCK] : (Ckpt *)nullptr, mt.data(), acm);
        }
        schain_run2(ch[0], ch[1], d, tabs.data(), scan, mkp, mt.data(), acm);
        for (int hh = 0; hh < 2; hh++) {
          if (!act[hh]) continue;
          const uint32_t q = t + 128 * hh;
          const uint32_t in = lead_in(d, tabs.data(), scan, mkp, sv[hh], d.lead_bits, mt.data(), acm, false);
          RangeAcc a;
          Ckpt *c1 = (q > 0 && NCK) ? &ck1[(size_t)sv[hh] * NCK] : (Ckpt *)nullptr;
          decode_range<false>(d, tabs.data(), scan, mkp, sv[hh], in, a, nullptr, c1, false, 0, nullptr, mt.data(), acm,
                              0u);
          const RangeAcc &b = ch[hh].acc;
          bool bad = in != ch[hh].in || a.out != b.out || a.m != b.m || a.n != b.n || a.dc[0] != b.dc[0] ||
                     a.dc[1] != b.dc[1] || a.dc[2] != b.dc[2];
          if (c1)
            for (uint32_t j = 0; j < NCK; j++) {
              const Ckpt &x = c1[j], &y = ck2[(size_t)sv[hh] * NCK + j];
              bad = bad || x.st != y.st || x.m != y.m || x.n != y.n || x.dc[0] != y.dc[0] || x.dc[1] != y.dc[1] ||
                    x.dc[2] != y.dc[2];
            }
          g_two_checked++;
          g_two_mismatch += bad ? 1 : 0;
        }
      }
    }
  }
  // ---- k_huff_sync (mirrors the kernel: threads in lockstep phases)
  for (uint32_t wg = 0; wg < NW; wg++) {
    const uint32_t s0 = wg * U;
    std::vector<uint32_t> ex(kSubPerWg, 0), ins(kSubPerWg, 0);
    std::vector<RangeAcc> acc(kSubPerWg);
    std::vector<char> active(kSubPerWg, 0), head(kSubPerWg, 0);
    for (uint32_t t = 0; t < (uint32_t)kSubPerWg; t++) {
      int64_t si = (int64_t)s0 + t - 1;
      active[t] = si >= 0 && si < (int64_t)d.nsub;
      head[t] = (t == 0) || (s0 == 0 && t == 1);
      if (!active[t]) continue;
      ins[t] = lead_in(d, tabs.data(), scan, mkp, (uint32_t)si, d.lead_bits, mt.data(), acm, true);
      if (d.lead_bits) {
        g_multi_checked++;
        g_multi_mismatch += ins[t] != lead_in(d, tabs.data(), scan, mkp, (uint32_t)si, d.lead_bits);
      }
      decode_range<false>(d, tabs.data(), scan, mkp, (uint32_t)si, ins[t], acc[t], nullptr, t ? ckp((uint32_t)si) : nullptr,
                          false, 0, nullptr, mt.data(), acm, true);
      ex[t] = acc[t].out;
    }
    int64_t it = 0;
    for (;;) {
      std::vector<uint32_t> pin(kSubPerWg, 0);
      std::vector<char> redo(kSubPerWg, 0);
      bool any = false;
      for (uint32_t t = 1; t < (uint32_t)kSubPerWg; t++)
        if (active[t] && !head[t] && ins[t] != ex[t - 1]) { redo[t] = 1; pin[t] = ex[t - 1]; any = true; }
      for (uint32_t t = 1; t < (uint32_t)kSubPerWg; t++)
        if (redo[t]) {
          uint32_t si = s0 + t - 1;
          decode_range<false>(d, tabs.data(), scan, mkp, si, pin[t], acc[t], nullptr, ckp(si), true, ex[t], nullptr,
                              mt.data(), acm, true);
          ex[t] = acc[t].out;
          ins[t] = pin[t];
          redo_total++;
        }
      it++;
      if (!any) break;
    }
    if (it > iters_max) iters_max = it;
    for (uint32_t t = 1; t < (uint32_t)kSubPerWg; t++) {
      if (!active[t]) continue;
      SubState &o = subs[s0 + t - 1];
      o.in = ins[t]; o.out = ex[t]; o.m = acc[t].m; o.n = acc[t].n;
      o.dc[0] = acc[t].dc[0]; o.dc[1] = acc[t].dc[1]; o.dc[2] = acc[t].dc[2];
    }
  }
  // ---- k_huff_fix until no workgroup's last exit changes
  for (;;) {
    rounds++;
    bool chain = false;
    std::vector<SubState> snap = subs;  // all workgroups read the launch-start values
    for (uint32_t wg = 1; wg < NW; wg++) {
      const uint32_t s0 = wg * U;
      const uint32_t n = d.nsub - s0 < U ? d.nsub - s0 : U;
      uint32_t first_in = snap[s0 - 1].out;
      if (subs[s0].in == first_in) continue;
      fix_wgs++;
      std::vector<uint32_t> ex(n), ins(n);
      std::vector<RangeAcc> acc(n);
      std::vector<char> mine(n, 0);
      for (uint32_t t = 0; t < n; t++) {
        ex[t] = subs[s0 + t].out; ins[t] = subs[s0 + t].in;
        acc[t].m = subs[s0 + t].m; acc[t].n = subs[s0 + t].n;
        for (int c = 0; c < 3; c++) acc[t].dc[c] = subs[s0 + t].dc[c];
      }
      uint32_t orig_last = ex[n - 1];
      for (;;) {
        std::vector<uint32_t> pin(n, 0);
        std::vector<char> redo(n, 0);
        bool any = false;
        for (uint32_t t = 0; t < n; t++) {
          uint32_t want = t == 0 ? first_in : ex[t - 1];
          if (ins[t] != want) { redo[t] = 1; pin[t] = want; any = true; }
        }
        for (uint32_t t = 0; t < n; t++)
          if (redo[t]) {
            decode_range<false>(d, tabs.data(), scan, mkp, s0 + t, pin[t], acc[t], nullptr, ckp(s0 + t), true, ex[t]);
            ex[t] = acc[t].out; ins[t] = pin[t]; mine[t] = 1; redo_total++;
          }
        if (!any) break;
      }
      for (uint32_t t = 0; t < n; t++)
        if (mine[t]) {
          SubState &o = subs[s0 + t];
          o.in = ins[t]; o.out = ex[t]; o.m = acc[t].m; o.n = acc[t].n;
          o.dc[0] = acc[t].dc[0]; o.dc[1] = acc[t].dc[1]; o.dc[2] = acc[t].dc[2];
        }
      if (n == U && s0 + n < d.nsub && ex[n - 1] != orig_last) chain = true;
    }
    if (!chain || rounds > 64) break;
  }
  // ---- k_huff_scan (segmented exclusive scan)
  uint32_t cm = 0, cn = 0;
  int32_t cd[3] = {0, 0, 0};
  for (uint32_t i = 0; i < d.nsub; i++) {
    subs[i].seg = cm; subs[i].nin = cn;
    subs[i].dcin[0] = cd[0]; subs[i].dcin[1] = cd[1]; subs[i].dcin[2] = cd[2];
    if (subs[i].m) { cm += subs[i].m; cn = subs[i].n; for (int c = 0; c < 3; c++) cd[c] = subs[i].dc[c]; }
    else { cn += subs[i].n; for (int c = 0; c < 3; c++) cd[c] += subs[i].dc[c]; }
  }
  uint64_t decoded = d.blocks_per_seg ? (uint64_t)cm * d.blocks_per_seg + cn : cn;
  // ---- k_huff_write
  std::vector<int16_t> coef((size_t)d.total_blocks * 64, (int16_t)0x7777);  // poison: every slot must be written
  int64_t mismatch = 0;
  int16_t blk[64];
  for (uint32_t s = 0; s < d.nsub; s++) {
    WriteCtx w;
    w.blk = blk; w.coef = coef.data(); w.seg = subs[s].seg; w.nin = subs[s].nin;
    for (int c = 0; c < 3; c++) w.pred[c] = subs[s].dcin[c];
    w.blocks_per_seg = d.blocks_per_seg; w.total_blocks = d.total_blocks; w.cur = -1; w.zs = 0;
    RangeAcc acc;
    decode_range<true>(d, tabs.data(), scan, mkp, s, subs[s].in, acc, &w, nullptr, false, 0, nullptr, nullptr, 0xFFu,
                       3u);  // k_huff_write's multi-symbol steps (up to 3 more symbols per peek)
    if (acc.out != subs[s].out) mismatch++;
  }
  // zigzag -> natural
  static const int nat[64] = {0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
                              41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
                              30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
  *nblocks = d.total_blocks;
  for (size_t b = 0; b < d.total_blocks && b < cap_blocks; b++)
    for (int k = 0; k < 64; k++) out[b * 64 + nat[k]] = coef[b * 64 + k];
  if (stats) {
    stats[0] = d.nsub; stats[1] = redo_total; stats[2] = iters_max; stats[3] = fix_wgs;
    stats[4] = rounds; stats[5] = mismatch; stats[6] = (int64_t)decoded; stats[7] = d.total_blocks;
  }
  return 0;
}
