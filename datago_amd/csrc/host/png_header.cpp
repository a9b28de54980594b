// png_header.cpp — PNG chunk walk (see png_header.h).
//
// Behaviour follows png 0.18.0 as image 0.25.9 drives it (EXPAND): colour
// types 0/2/3/4/6, depths per the spec table; 16-bit samples and Adam7
// interlacing are valid but outside the GPU path (PH_UNSUPPORTED: the Rust
// glue keeps its CPU decode for them).  Chunk CRCs are not verified here
// (decoding never depends on them) and, like png's default
// (ignore_adler32), neither is the zlib Adler-32 trailer.
#include "png_header.h"

#include "../dg_types.h"

#include <string.h>

namespace dg {

static uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static void fail(PngHeader &h, int st, const char *why) {
  h.status = st;
  h.why = why;
}

void parse_png_header(const uint8_t *d, size_t n, PngHeader &h) {
  h = PngHeader();
  memset(h.pal, 0, sizeof(h.pal));
  for (int i = 0; i < 256; i++) h.pal[i][3] = 255;
  if (!is_png(d, n)) return fail(h, PH_CORRUPT, "not a PNG");
  size_t pos = 8;
  bool ihdr = false, iend = false;
  while (pos + 8 <= n) {
    const uint32_t len = be32(d + pos);
    const uint8_t *t = d + pos + 4;
    if (len > 0x7FFFFFFFu || pos + 12 + (size_t)len > n) return fail(h, PH_CORRUPT, "truncated PNG chunk");
    const uint8_t *c = d + pos + 8;
    if (!ihdr && memcmp(t, "IHDR", 4)) return fail(h, PH_CORRUPT, "PNG: first chunk is not IHDR");
    if (!memcmp(t, "IHDR", 4)) {
      if (ihdr || len != 13) return fail(h, PH_CORRUPT, "PNG: bad IHDR");
      h.width = be32(c);
      h.height = be32(c + 4);
      h.depth = c[8];
      h.ctype = c[9];
      h.interlace = c[12];
      if (c[10] != 0 || c[11] != 0 || h.interlace > 1) return fail(h, PH_CORRUPT, "PNG: bad IHDR method");
      if (h.width == 0 || h.height == 0 || h.width > 0x7FFFFFFFu || h.height > 0x7FFFFFFFu)
        return fail(h, PH_CORRUPT, "PNG: bad dimensions");
      ihdr = true;
    } else if (!memcmp(t, "PLTE", 4)) {
      h.npal = (int)(len / 3) > 256 ? 256 : (int)(len / 3);
      for (int i = 0; i < h.npal; i++) {
        h.pal[i][0] = c[3 * i];
        h.pal[i][1] = c[3 * i + 1];
        h.pal[i][2] = c[3 * i + 2];
      }
    } else if (!memcmp(t, "tRNS", 4)) {
      h.has_trns = 1;
      if (h.ctype == 3) {
        for (uint32_t i = 0; i < len && i < 256; i++) h.pal[i][3] = c[i];
      } else if (h.ctype == 0 && len >= 2) {
        h.trns[0] = (uint16_t)((c[0] << 8) | c[1]);
      } else if (h.ctype == 2 && len >= 6) {
        for (int k = 0; k < 3; k++) h.trns[k] = (uint16_t)((c[2 * k] << 8) | c[2 * k + 1]);
      } else {
        h.has_trns = 0;  // tRNS on a colour type with alpha: ignored
      }
    } else if (!memcmp(t, "IDAT", 4)) {
      if (len) {
        h.idat_off.push_back((uint32_t)(pos + 8));
        h.idat_len.push_back(len);
        h.zlen += len;
      }
    } else if (!memcmp(t, "IEND", 4)) {
      iend = true;
      break;
    }
    pos += 12 + (size_t)len;
  }
  (void)iend;
  if (!ihdr) return fail(h, PH_CORRUPT, "PNG: no IHDR");
  if (h.idat_off.empty()) return fail(h, PH_CORRUPT, "PNG: no image data");
  const int ct = h.ctype, dp = h.depth;
  const bool ok = (ct == 0 && (dp == 1 || dp == 2 || dp == 4 || dp == 8 || dp == 16)) ||
                  (ct == 3 && (dp == 1 || dp == 2 || dp == 4 || dp == 8)) ||
                  ((ct == 2 || ct == 4 || ct == 6) && (dp == 8 || dp == 16));
  if (!ok) return fail(h, PH_CORRUPT, "PNG: invalid colour type / bit depth");
  if (ct == 3 && h.npal == 0) return fail(h, PH_CORRUPT, "PNG: palette image without PLTE");
  h.spp = ct == 2 ? 3 : ct == 4 ? 2 : ct == 6 ? 4 : 1;
  switch (ct) {
    case 0: h.out_c = h.has_trns ? 2 : 1; break;
    case 2: h.out_c = h.has_trns ? 4 : 3; break;
    case 3: h.out_c = h.has_trns ? 4 : 3; break;
    case 4: h.out_c = 2; break;
    default: h.out_c = 4; break;
  }
  const uint64_t bits = (uint64_t)h.spp * (uint64_t)dp * h.width;
  if ((bits + 7) / 8 > 0x7FFFFFF0ull) return fail(h, PH_UNSUPPORTED, "PNG: scanline too long");
  h.rowbytes = (uint32_t)((bits + 7) / 8);
  h.bpp = (int)(((uint64_t)h.spp * dp + 7) / 8);
  if (dp == 16) return fail(h, PH_UNSUPPORTED, "PNG: 16-bit samples (CPU path)");
  // Adam7 (PNG spec 8.2): seven sub-images back to back, empty ones absent
  h.rawlen = h.unflen = 0;
  for (uint32_t p = 0; p < (h.interlace ? 7u : 1u); p++) {
    uint32_t pw = h.width, ph = h.height;
    if (h.interlace) png_adam7_pass(h.width, h.height, p, pw, ph);
    if (!pw || !ph) continue;
    const uint64_t rb = ((uint64_t)h.spp * dp * pw + 7) / 8;
    h.rawlen += (uint64_t)ph * (rb + 1);
    h.unflen += (uint64_t)ph * ((rb + 15) / 16 * 16);
  }
  h.status = PH_OK;
}

static uint32_t crc32_bytes(const uint8_t *p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int k = 0; k < 8; k++) c = (c & 1u) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
  }
  return ~c;
}

std::vector<uint8_t> png_enc_header(uint32_t w, uint32_t h, uint32_t C) {
  static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
  std::vector<uint8_t> o(sig, sig + 8);
  auto be32 = [&](uint32_t v) {
    for (int s = 24; s >= 0; s -= 8) o.push_back((uint8_t)(v >> s));
  };
  be32(13);
  const size_t t0 = o.size();
  for (char c : {'I', 'H', 'D', 'R'}) o.push_back((uint8_t)c);
  be32(w);
  be32(h);
  o.push_back(8);                                                // bit depth
  o.push_back((uint8_t)(C == 1 ? 0 : C == 2 ? 4 : C == 3 ? 2 : 6));  // colour type
  o.push_back(0);                                                // deflate
  o.push_back(0);                                                // adaptive filtering
  o.push_back(0);                                                // no interlace
  be32(crc32_bytes(o.data() + t0, o.size() - t0));
  return o;
}

uint64_t png_enc_bound(uint32_t w, uint32_t h, uint32_t C) {
  const uint64_t n = (uint64_t)h * ((uint64_t)w * C + 1);  // filtered stream
  return 33 + 8 + 2 + (3 + 9 * n + 7 + 7) / 8 + 4 + 4 + 12 + 16;
}

}  // namespace dg
