// jpeg_header.cpp — see jpeg_header.h.
#include "jpeg_header.h"

#include <string.h>

namespace dg {

static const int kNat[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

static inline int rd16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

bool is_jpeg(const uint8_t *d, size_t n) { return n >= 3 && d[0] == 0xFF && d[1] == 0xD8 && d[2] == 0xFF; }
bool jpeg_sniff_progressive(const uint8_t *d, size_t n) {
  if (!is_jpeg(d, n)) return false;
  size_t p = 2;
  while (p + 4 <= n) {
    if (d[p] != 0xFF) return false;
    const uint8_t m = d[p + 1];
    if (m == 0xFF) {  // fill byte
      p++;
      continue;
    }
    if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) return m == 0xC2;
    if (m == 0xD9 || m == 0xDA) return false;
    p += 2 + (((size_t)d[p + 2] << 8) | d[p + 3]);
  }
  return false;
}

bool is_png(const uint8_t *d, size_t n) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  return n >= 8 && memcmp(d, sig, 8) == 0;
}

static void fail(JpegHeader &h, int st, const char *why) {
  h.status = st;
  h.why = why;
}

void parse_jpeg_header(const uint8_t *d, size_t n, JpegHeader &h) {
  h = JpegHeader();
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return fail(h, JH_CORRUPT, "not a JPEG (no SOI)");
  bool saw_sof = false;
  size_t p = 2;
  for (;;) {
    while (p < n && d[p] != 0xFF) p++;
    while (p < n && d[p] == 0xFF) p++;
    if (p >= n) return fail(h, JH_CORRUPT, "truncated before SOS");
    int m = d[p++];
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) return fail(h, JH_CORRUPT, "EOI before SOS");
    if (p + 2 > n) return fail(h, JH_CORRUPT, "truncated marker");
    int L = rd16(d + p);
    if (L < 2 || p + (size_t)L > n) return fail(h, JH_CORRUPT, "bad marker length");
    const uint8_t *s = d + p + 2;
    int len = L - 2;
    if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      // SOFn
      if (len < 6) return fail(h, JH_CORRUPT, "short SOF");
      h.sof = m;
      h.progressive = (m == 0xC2 || m == 0xC6 || m == 0xCA || m == 0xCE);
      h.arithmetic = (m >= 0xC9);
      h.lossless = (m == 0xC3 || m == 0xC7 || m == 0xCB || m == 0xCF);
      h.precision = s[0];
      h.height = (uint32_t)rd16(s + 1);
      h.width = (uint32_t)rd16(s + 3);
      h.ncomp = s[5];
      if (h.ncomp < 1 || h.ncomp > 4 || len < 6 + 3 * h.ncomp) return fail(h, JH_CORRUPT, "bad SOF components");
      for (int c = 0; c < h.ncomp; c++) {
        h.comp[c].id = s[6 + 3 * c];
        h.comp[c].h = s[7 + 3 * c] >> 4;
        h.comp[c].v = s[7 + 3 * c] & 15;
        h.comp[c].tq = s[8 + 3 * c];
        if (h.comp[c].h < 1 || h.comp[c].h > 4 || h.comp[c].v < 1 || h.comp[c].v > 4 || h.comp[c].tq > 3)
          return fail(h, JH_CORRUPT, "bad sampling factors");
      }
      if (h.width == 0 || h.height == 0) return fail(h, JH_CORRUPT, "zero dimension");
      saw_sof = true;
    } else if (m == 0xC4) {
      int o = 0;
      while (o < len) {
        if (o + 17 > len) return fail(h, JH_CORRUPT, "short DHT");
        int tc = s[o] >> 4, th = s[o] & 15;
        if (tc > 1 || th > 3) return fail(h, JH_CORRUPT, "bad DHT class/id");
        HuffSpec &t = tc ? h.ac[th] : h.dc[th];
        int total = 0;
        t.bits[0] = 0;
        for (int i = 1; i <= 16; i++) {
          t.bits[i] = s[o + i];
          total += s[o + i];
        }
        if (total > 256 || o + 17 + total > len) return fail(h, JH_CORRUPT, "bad DHT counts");
        memset(t.vals, 0, sizeof(t.vals));
        memcpy(t.vals, s + o + 17, (size_t)total);
        t.nvals = total;
        t.present = true;
        o += 17 + total;
      }
    } else if (m == 0xDB) {
      int o = 0;
      while (o < len) {
        int pq = s[o] >> 4, tq = s[o] & 15;
        if (tq > 3 || pq > 1 || o + 1 + 64 * (pq + 1) > len) return fail(h, JH_CORRUPT, "bad DQT");
        for (int k = 0; k < 64; k++)
          h.q[tq][kNat[k]] = pq ? (uint16_t)rd16(s + o + 1 + 2 * k) : (uint16_t)s[o + 1 + k];
        h.qpresent[tq] = true;
        o += 1 + 64 * (pq + 1);
      }
    } else if (m == 0xDD) {
      if (len < 2) return fail(h, JH_CORRUPT, "short DRI");
      h.restart = rd16(s);
    } else if (m == 0xE0) {
      if (len >= 5 && memcmp(s, "JFIF\0", 5) == 0) h.jfif = true;
    } else if (m == 0xEE) {
      if (len >= 12 && memcmp(s, "Adobe", 5) == 0) {
        h.adobe = true;
        h.adobe_transform = s[11];
      }
    } else if (m == 0xDA) {
      if (!saw_sof) return fail(h, JH_CORRUPT, "SOS before SOF");
      int ns = s[0];
      if (ns < 1 || ns > 4 || len < 1 + 2 * ns + 3) return fail(h, JH_CORRUPT, "bad SOS");
      h.scan_ncomp = ns;
      for (int i = 0; i < ns; i++) {
        int cid = s[1 + 2 * i], c;
        for (c = 0; c < h.ncomp; c++)
          if (h.comp[c].id == cid) break;
        if (c == h.ncomp) return fail(h, JH_CORRUPT, "SOS names unknown component");
        h.scan_comp[i] = c;
        h.comp[c].td = s[2 + 2 * i] >> 4;
        h.comp[c].ta = s[2 + 2 * i] & 15;
        if (h.comp[c].td > 3 || h.comp[c].ta > 3) return fail(h, JH_CORRUPT, "bad table selector");
      }
      h.scan_off = p + (size_t)L;
      if (h.progressive) {
        // T.81 G.1.2 scan parameters (libjpeg jdphuff.c start_pass_phuff_decoder checks)
        JpegScan sc;
        sc.ns = ns;
        sc.ss = s[1 + 2 * ns];
        sc.se = s[2 + 2 * ns];
        sc.ah = s[3 + 2 * ns] >> 4;
        sc.al = s[3 + 2 * ns] & 15;
        sc.restart = h.restart;
        if (sc.ss == 0 ? sc.se != 0 : (sc.se < sc.ss || sc.se > 63 || ns != 1))
          return fail(h, JH_CORRUPT, "bad progressive scan band");
        if ((sc.ah != 0 && sc.al != sc.ah - 1) || sc.al > 13) return fail(h, JH_CORRUPT, "bad successive approximation");
        for (int i = 0; i < ns; i++) {
          const JpegComponent &k = h.comp[h.scan_comp[i]];
          sc.comp[i] = h.scan_comp[i];
          if (sc.ss == 0 && sc.ah == 0) {
            if (!h.dc[k.td].present) return fail(h, JH_CORRUPT, "missing Huffman table");
            sc.dc_tab[i] = (int)h.tables.size();
            h.tables.push_back(h.dc[k.td]);
          }
        }
        if (sc.ss > 0) {
          const JpegComponent &k = h.comp[h.scan_comp[0]];
          if (!h.ac[k.ta].present) return fail(h, JH_CORRUPT, "missing Huffman table");
          sc.ac_tab = (int)h.tables.size();
          h.tables.push_back(h.ac[k.ta]);
        }
        // the scan's data ends at the first marker that is not RSTn
        size_t q = h.scan_off;
        for (;;) {
          const uint8_t *f = (const uint8_t *)memchr(d + q, 0xFF, n - q);
          if (!f || (size_t)(f - d) + 1 >= n) return fail(h, JH_CORRUPT, "truncated progressive scan");
          q = (size_t)(f - d);
          const uint8_t c = d[q + 1];
          if (c != 0x00 && c != 0xFF && !(c >= 0xD0 && c <= 0xD7)) break;
          q++;
        }
        sc.off = h.scan_off;
        sc.end = q;
        h.scans.push_back(sc);
        if (h.scans.size() > kProgMaxScans) return fail(h, JH_UNSUPPORTED, "more than 256 progressive scans");
        p = q;
        if (d[q + 1] == 0xD9) break;  // EOI
        continue;
      }
      h.scan_end = n;
      if (n >= 2 && d[n - 2] == 0xFF && d[n - 1] == 0xD9) {
        h.scan_end = n - 2;
      } else {  // trailing data / truncated file: entropy data ends at the first non-RST marker
        for (size_t q = h.scan_off; q + 1 < n; q++) {
          if (d[q] == 0xFF && d[q + 1] != 0x00 && d[q + 1] != 0xFF && !(d[q + 1] >= 0xD0 && d[q + 1] <= 0xD7)) {
            h.scan_end = q;
            break;
          }
        }
      }
      if (h.scan_end < h.scan_off) return fail(h, JH_CORRUPT, "empty scan");
      break;
    }
    p += (size_t)L;
  }
  // ---- what the GPU path decodes
  if (h.arithmetic) return fail(h, JH_UNSUPPORTED, "arithmetic-coded JPEG");
  if (h.lossless || (h.sof != 0xC0 && h.sof != 0xC1 && h.sof != 0xC2)) return fail(h, JH_UNSUPPORTED, "unsupported SOF type");
  if (h.precision != 8) return fail(h, JH_UNSUPPORTED, "12/16-bit JPEG");
  if (h.ncomp != 1 && h.ncomp != 3) return fail(h, JH_UNSUPPORTED, "CMYK/2-component JPEG");
  if (!h.progressive && h.scan_ncomp != h.ncomp) return fail(h, JH_UNSUPPORTED, "non-interleaved multi-scan JPEG");
  if (h.progressive) {
    // coefficient precision after the last scan (libjpeg coef_bits): the DC and
    // AC 1..9 must end exact, or libjpeg would smooth blocks (jdcoefct.c smoothing_ok)
    int bits[4][64];
    for (int c = 0; c < 4; c++)
      for (int k = 0; k < 64; k++) bits[c][k] = -1;
    for (const JpegScan &sc : h.scans)
      for (int i = 0; i < sc.ns; i++)
        for (int k = sc.ss; k <= sc.se; k++) bits[sc.comp[i]][k] = sc.al;
    // recorded, not refused here: libjpeg-turbo semantics refuse such files
    // (plan_image / dg_probe), zune-jpeg applies no smoothing and decodes the
    // coefficients as they stand
    for (int c = 0; c < h.ncomp; c++)
      for (int k = 0; k < 10; k++)
        if (bits[c][k] != 0) h.incomplete_refinement = true;
    h.scan_end = h.scans.empty() ? h.scan_off : h.scans.back().end;
  }
  h.hmax = h.vmax = 1;
  for (int c = 0; c < h.ncomp; c++) {
    if (h.comp[c].h > h.hmax) h.hmax = h.comp[c].h;
    if (h.comp[c].v > h.vmax) h.vmax = h.comp[c].v;
  }
  if (h.ncomp == 3) {
    int blocks = 0;
    for (int c = 0; c < 3; c++) {
      const JpegComponent &k = h.comp[c];
      if (h.hmax % k.h || h.vmax % k.v) return fail(h, JH_UNSUPPORTED, "fractional sampling ratio");
      int hr = h.hmax / k.h, vr = h.vmax / k.v;
      if (!((hr == 1 && vr == 1) || (hr == 2 && vr == 1) || (hr == 2 && vr == 2)))
        return fail(h, JH_UNSUPPORTED, "chroma sampling other than 4:4:4/4:2:2/4:2:0");
      blocks += k.h * k.v;
    }
    if (blocks > 10) return fail(h, JH_CORRUPT, "too many blocks per MCU");
  }
  for (int c = 0; c < h.ncomp; c++) {
    if (!h.qpresent[h.comp[c].tq]) return fail(h, JH_CORRUPT, "missing quantisation table");
    if (!h.progressive && (!h.dc[h.comp[c].td].present || !h.ac[h.comp[c].ta].present))
      return fail(h, JH_CORRUPT, "missing Huffman table");
  }
  // colour space guess (libjpeg jdapimin.c default_decompress_parms)
  if (h.ncomp == 1) {
    h.colorspace = CS_GRAY;
  } else if (h.jfif) {
    h.colorspace = CS_YCC;
  } else if (h.adobe) {
    h.colorspace = h.adobe_transform == 0 ? CS_RGB : CS_YCC;
  } else if (h.comp[0].id == 82 && h.comp[1].id == 71 && h.comp[2].id == 66) {
    h.colorspace = CS_RGB;
  } else {
    h.colorspace = CS_YCC;
  }
  // image's default limits: 512 MiB allocation (B4); reject absurd sizes
  if ((uint64_t)h.width * h.height * h.ncomp > (512ull << 20)) return fail(h, JH_UNSUPPORTED, "image exceeds decode limits");
  h.status = JH_OK;
  h.why = "";
}

bool build_huff_table(const HuffSpec &spec, HuffTable &out) {
  memset(&out, 0, sizeof(out));
  int32_t mincode[17], maxcode[17], valptr[17];
  int code = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    valptr[l] = k;
    mincode[l] = code;
    code += spec.bits[l];
    k += spec.bits[l];
    maxcode[l] = spec.bits[l] ? code - 1 : -1;
    if (code > (1 << l)) return false;
    code <<= 1;
  }
  if (k > 256) return false;
  for (int l = 1; l <= 16; l++) {
    out.lim[l] = spec.bits[l] ? (uint32_t)(maxcode[l] + 1) << (16 - l) : 0u;
    out.valoff[l] = valptr[l] - mincode[l];
  }
  memcpy(out.vals, spec.vals, 256);
  // first level: codes of length <= kLutBits
  for (uint32_t pfx = 0; pfx < (1u << kLutBits); pfx++) {
    for (int l = 1; l <= kLutBits; l++) {
      int32_t c = (int32_t)(pfx >> (kLutBits - l));
      if (spec.bits[l] && c <= maxcode[l]) {
        if (c >= mincode[l]) out.lut[pfx] = (uint16_t)((l << 8) | spec.vals[(valptr[l] + c - mincode[l]) & 255]);
        break;
      }
    }
  }
  // second level: every 16-bit peek whose first kLutBits bits are not a
  // complete code; subtables are allocated per such prefix (up to kMaxSubTables)
  int nsub = 0;
  bool overflow = false;
  for (uint32_t pfx = 0; pfx < (1u << kLutBits); pfx++) {
    if (out.lut[pfx]) continue;
    uint16_t tmp[1 << kSubBits];
    bool any = false;
    for (uint32_t lo = 0; lo < (1u << kSubBits); lo++) {
      uint32_t pk = (pfx << kSubBits) | lo;  // 16-bit peek
      tmp[lo] = 0;
      for (int l = kLutBits + 1; l <= 16; l++) {
        int32_t c = (int32_t)(pk >> (16 - l));
        if (spec.bits[l] && c <= maxcode[l]) {
          if (c >= mincode[l]) tmp[lo] = (uint16_t)((l << 8) | spec.vals[(valptr[l] + c - mincode[l]) & 255]);
          break;
        }
      }
      any |= tmp[lo] != 0;
    }
    if (!any) continue;  // invalid prefix: stays 0 (fallback returns "invalid" too)
    if (nsub == kMaxSubTables) {
      overflow = true;
      continue;
    }
    memcpy(out.sub[nsub], tmp, sizeof(tmp));
    out.lut[pfx] = (uint16_t)(0x8000u | (uint32_t)nsub);
    nsub++;
  }
  (void)overflow;  // prefixes beyond kMaxSubTables keep lut = 0 and use the lim[] fallback
  return true;
}

}  // namespace dg
