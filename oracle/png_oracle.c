/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this file's library; the product path
 * (datago_amd/csrc) never links or calls it.
 *
 * Scalar C restatement of the PNG half of datago's decode step
 * (image::load_from_memory / ImageReader::decode, worker_files.rs:8-17,
 * worker_wds.rs:45) and of the RGBA handling around crop_and_resize:
 *
 *   - zlib + DEFLATE decode (RFC 1950/1951).  The reference decodes with
 *     png 0.18.0 -> fdeflate 0.3.7 (Cargo.lock), not vendored here; DEFLATE
 *     is fully specified, so any conforming inflater gives the same bytes.
 *     Like png's default (ignore_adler32 = true) the Adler-32 trailer is not
 *     checked, and decoding stops once every scanline has arrived.
 *   - PNG scanline unfiltering (None/Sub/Up/Average/Paeth, PNG spec 9.2-9.4).
 *   - png's Transformations::EXPAND as image 0.25 requests it: palette ->
 *     RGB(A) (tRNS entries become alpha, missing palette entries are black),
 *     gray of 1/2/4 bits -> 8 bits scaled by 255/(2^d-1), tRNS on gray/RGB ->
 *     an alpha channel (0 where the sample equals the tRNS key, else 255).
 *   - Adam7 interlacing (PNG spec 8.2): the seven passes' filtered rows back
 *     to back, each pass unfiltered on its own, then scattered.
 *     16-bit images report PO_UNSUPPORTED (the GPU path reports
 *     DG_ERR_UNSUPPORTED for them, the Rust glue keeps its CPU path).
 *   - fast_image_resize 5.5.0 alpha handling for U8x2/U8x4 (ResizeOptions
 *     mul_div_alpha = true): multiply colour by alpha
 *     before a convolution call, divide after.  Restated from the crate's
 *     published source (unpinned: the crate is not present offline).
 *   - convert_to_rgb8 (image_processing.rs:163-186): RGBA composited over
 *     opaque (128,128,128) with image's Pixel::blend (f32, truncating casts);
 *     pinned by the reference's own known answers (:846-888,
 *     worker_files.rs:322-383).
 *
 * Parity: PNG decode is lossless, so tests/test_oracle_png.py pins this file
 * bit-exactly against PIL's decodes of the committed fixtures.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PO_OK 0
#define PO_UNSUPPORTED 1
#define PO_CORRUPT 2
#define PO_SMALLBUF 3

/* ------------------------------------------------------------------ inflate */

typedef struct {
  const uint8_t *p;
  size_t n, pos;   /* byte position */
  uint64_t buf;
  int cnt;
  int overrun;
} bitrd;

static uint32_t need(bitrd *b, int k) {
  while (b->cnt < k) {
    uint64_t v = 0;
    if (b->pos < b->n)
      v = b->p[b->pos];
    else
      b->overrun++;
    b->pos++;
    b->buf |= v << b->cnt;
    b->cnt += 8;
  }
  return (uint32_t)(b->buf & ((1ull << k) - 1));
}
static uint32_t bits(bitrd *b, int k) {
  if (k == 0) return 0;
  uint32_t v = need(b, k);
  b->buf >>= k;
  b->cnt -= k;
  return v;
}

typedef struct {
  uint16_t count[16];
  uint16_t sym[320];
} huff;

/* Canonical code from lengths (RFC 1951 3.2.2).  Returns 0 ok, -1 if
 * over-subscribed.  Incomplete codes are accepted (as zlib does for the
 * single-code distance tree; a bad stream then fails on an unused code). */
static int huff_build(huff *h, const uint8_t *len, int n) {
  uint16_t offs[16];
  memset(h->count, 0, sizeof(h->count));
  for (int s = 0; s < n; s++) h->count[len[s]]++;
  h->count[0] = 0;
  int left = 1;
  for (int l = 1; l < 16; l++) {
    left <<= 1;
    left -= h->count[l];
    if (left < 0) return -1;
  }
  offs[1] = 0;
  for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + h->count[l];
  for (int s = 0; s < n; s++)
    if (len[s]) h->sym[offs[len[s]]++] = (uint16_t)s;
  return 0;
}

/* Bit-serial canonical decode (puff.c style): returns symbol or -1. */
static int huff_decode(bitrd *b, const huff *h) {
  int code = 0, first = 0, index = 0;
  for (int l = 1; l < 16; l++) {
    code |= (int)bits(b, 1);
    int c = h->count[l];
    if (code - c < first) return h->sym[index + (code - first)];
    index += c;
    first += c;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}

static const uint16_t LBASE[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t LEXT[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t DBASE[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                   193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t DEXT[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

/* Inflate a zlib stream into out[0..want).  Stops as soon as `want` bytes
 * exist.  Returns PO_OK, or PO_CORRUPT when the stream is invalid or ends
 * before `want` bytes. */
int po_zlib_inflate(const uint8_t *z, size_t zn, uint8_t *out, size_t want, size_t *got) {
  size_t op = 0;
  if (got) *got = 0;
  if (zn < 2) return PO_CORRUPT;
  const uint32_t cmf = z[0], flg = z[1];
  if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) return PO_CORRUPT;
  bitrd b = {z + 2, zn - 2, 0, 0, 0, 0};
  int last = 0;
  while (!last && op < want) {
    last = (int)bits(&b, 1);
    const int type = (int)bits(&b, 2);
    if (b.overrun) return PO_CORRUPT;
    if (type == 0) {  /* stored */
      b.buf = 0;      /* drop to a byte boundary: whole bytes still buffered are re-read */
      b.pos -= (size_t)(b.cnt / 8);
      b.cnt = 0;
      if (b.pos + 4 > b.n) return PO_CORRUPT;
      const uint32_t len = b.p[b.pos] | (b.p[b.pos + 1] << 8), nlen = b.p[b.pos + 2] | (b.p[b.pos + 3] << 8);
      if ((len ^ 0xFFFF) != nlen) return PO_CORRUPT;
      b.pos += 4;
      for (uint32_t i = 0; i < len && op < want; i++) {
        if (b.pos >= b.n) return PO_CORRUPT;
        out[op++] = b.p[b.pos++];
      }
      continue;
    }
    if (type == 3) return PO_CORRUPT;
    huff lh, dh;
    uint8_t lens[320];
    if (type == 1) {
      for (int s = 0; s < 144; s++) lens[s] = 8;
      for (int s = 144; s < 256; s++) lens[s] = 9;
      for (int s = 256; s < 280; s++) lens[s] = 7;
      for (int s = 280; s < 288; s++) lens[s] = 8;
      huff_build(&lh, lens, 288);
      for (int s = 0; s < 30; s++) lens[s] = 5;
      huff_build(&dh, lens, 30);
    } else {
      static const uint8_t ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      const int nlen = (int)bits(&b, 5) + 257, ndist = (int)bits(&b, 5) + 1, ncode = (int)bits(&b, 4) + 4;
      if (nlen > 286 || ndist > 30) return PO_CORRUPT;
      uint8_t cl[19] = {0};
      for (int i = 0; i < ncode; i++) cl[ord[i]] = (uint8_t)bits(&b, 3);
      huff ch;
      if (huff_build(&ch, cl, 19)) return PO_CORRUPT;
      int i = 0;
      while (i < nlen + ndist) {
        int s = huff_decode(&b, &ch);
        if (s < 0 || b.overrun) return PO_CORRUPT;
        if (s < 16) {
          lens[i++] = (uint8_t)s;
          continue;
        }
        int rep, v = 0;
        if (s == 16) {
          if (i == 0) return PO_CORRUPT;
          v = lens[i - 1];
          rep = 3 + (int)bits(&b, 2);
        } else if (s == 17) {
          rep = 3 + (int)bits(&b, 3);
        } else {
          rep = 11 + (int)bits(&b, 7);
        }
        if (i + rep > nlen + ndist) return PO_CORRUPT;
        while (rep--) lens[i++] = (uint8_t)v;
      }
      if (lens[256] == 0) return PO_CORRUPT;
      if (huff_build(&lh, lens, nlen)) return PO_CORRUPT;
      if (huff_build(&dh, lens + nlen, ndist)) return PO_CORRUPT;
    }
    for (;;) {
      int s = huff_decode(&b, &lh);
      if (s < 0 || b.overrun) return PO_CORRUPT;
      if (s < 256) {
        out[op++] = (uint8_t)s;
        if (op >= want) break;
        continue;
      }
      if (s == 256) break;
      s -= 257;
      if (s >= 29) return PO_CORRUPT;
      const uint32_t len = LBASE[s] + bits(&b, LEXT[s]);
      const int ds = huff_decode(&b, &dh);
      if (ds < 0 || ds >= 30) return PO_CORRUPT;
      const uint32_t dist = DBASE[ds] + bits(&b, DEXT[ds]);
      if (b.overrun || dist > op) return PO_CORRUPT;
      for (uint32_t k = 0; k < len && op < want; k++, op++) out[op] = out[op - dist];
      if (op >= want) break;
    }
    if (b.overrun) return PO_CORRUPT;
  }
  if (got) *got = op;
  return op >= want ? PO_OK : PO_CORRUPT;
}

/* ------------------------------------------------------------------ PNG */

typedef struct {
  uint32_t w, h;
  int depth, ctype, interlace;
  int out_c;          /* channels after EXPAND */
  uint8_t pal[256][4];
  int npal, has_trns;
  uint16_t trns[3];   /* gray / RGB key */
  uint8_t *z;         /* concatenated IDAT payloads */
  size_t zn;
} pnginfo;

static uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3]; }

static int parse(const uint8_t *d, size_t n, pnginfo *pi, int want_data) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  memset(pi, 0, sizeof(*pi));
  if (n < 8 || memcmp(d, sig, 8)) return PO_CORRUPT;
  size_t pos = 8, cap = 0;
  int seen_ihdr = 0, seen_idat = 0;
  for (int i = 0; i < 256; i++) pi->pal[i][3] = 255;
  while (pos + 8 <= n) {
    const uint32_t len = be32(d + pos);
    const uint8_t *t = d + pos + 4;
    if (pos + 12 + (size_t)len > n) return PO_CORRUPT;
    const uint8_t *c = d + pos + 8;
    if (!memcmp(t, "IHDR", 4)) {
      if (len != 13) return PO_CORRUPT;
      pi->w = be32(c);
      pi->h = be32(c + 4);
      pi->depth = c[8];
      pi->ctype = c[9];
      pi->interlace = c[12];
      if (c[10] != 0 || c[11] != 0 || pi->interlace > 1 || pi->w == 0 || pi->h == 0) return PO_CORRUPT;
      seen_ihdr = 1;
    } else if (!memcmp(t, "PLTE", 4)) {
      pi->npal = (int)(len / 3);
      if (pi->npal > 256) pi->npal = 256;
      for (int i = 0; i < pi->npal; i++) {
        pi->pal[i][0] = c[3 * i];
        pi->pal[i][1] = c[3 * i + 1];
        pi->pal[i][2] = c[3 * i + 2];
      }
    } else if (!memcmp(t, "tRNS", 4)) {
      pi->has_trns = 1;
      if (pi->ctype == 3) {
        for (uint32_t i = 0; i < len && i < 256; i++) pi->pal[i][3] = c[i];
      } else if (pi->ctype == 0 && len >= 2) {
        pi->trns[0] = (uint16_t)((c[0] << 8) | c[1]);
      } else if (pi->ctype == 2 && len >= 6) {
        for (int k = 0; k < 3; k++) pi->trns[k] = (uint16_t)((c[2 * k] << 8) | c[2 * k + 1]);
      } else {
        pi->has_trns = 0;
      }
    } else if (!memcmp(t, "IDAT", 4)) {
      seen_idat = 1;
      if (want_data) {
        if (pi->zn + len > cap) {
          cap = (pi->zn + len) * 2 + 64;
          pi->z = (uint8_t *)realloc(pi->z, cap);
        }
        memcpy(pi->z + pi->zn, c, len);
      }
      pi->zn += len;
    } else if (!memcmp(t, "IEND", 4)) {
      break;
    }
    pos += 12 + (size_t)len;
  }
  if (!seen_ihdr || !seen_idat) return PO_CORRUPT;
  const int ct = pi->ctype, dp = pi->depth;
  int ok = (ct == 0 && (dp == 1 || dp == 2 || dp == 4 || dp == 8 || dp == 16)) ||
           (ct == 3 && (dp == 1 || dp == 2 || dp == 4 || dp == 8)) ||
           ((ct == 2 || ct == 4 || ct == 6) && (dp == 8 || dp == 16));
  if (!ok) return PO_CORRUPT;
  if (ct == 3 && pi->npal == 0) return PO_CORRUPT;
  switch (ct) {
    case 0: pi->out_c = pi->has_trns ? 2 : 1; break;
    case 2: pi->out_c = pi->has_trns ? 4 : 3; break;
    case 3: pi->out_c = pi->has_trns ? 4 : 3; break;
    case 4: pi->out_c = 2; break;
    default: pi->out_c = 4; break;
  }
  if (dp == 16) return PO_UNSUPPORTED;
  return PO_OK;
}

int po_info(const uint8_t *d, size_t n, int *w, int *h, int *c, int *depth, int *ctype, int *interlace) {
  pnginfo pi;
  int st = parse(d, n, &pi, 0);
  if (st == PO_CORRUPT) return st;
  *w = (int)pi.w;
  *h = (int)pi.h;
  *c = pi.out_c;
  *depth = pi.depth;
  *ctype = pi.ctype;
  *interlace = pi.interlace;
  return st;
}

static int paeth(int a, int b, int c) {
  int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  if (pb <= pc) return b;
  return c;
}

/* Unfilter in place: raw = H rows of (1 + rowbytes); bpp = filter unit. */
int po_unfilter(uint8_t *raw, uint32_t h, size_t rowbytes, int bpp, uint8_t *out) {
  const uint8_t *prev = NULL;
  for (uint32_t y = 0; y < h; y++) {
    const uint8_t *r = raw + (size_t)y * (rowbytes + 1);
    const int f = r[0];
    uint8_t *o = out + (size_t)y * rowbytes;
    r++;
    for (size_t x = 0; x < rowbytes; x++) {
      const int a = x >= (size_t)bpp ? o[x - bpp] : 0;
      const int b = prev ? prev[x] : 0;
      const int c = (prev && x >= (size_t)bpp) ? prev[x - bpp] : 0;
      int v;
      switch (f) {
        case 0: v = r[x]; break;
        case 1: v = r[x] + a; break;
        case 2: v = r[x] + b; break;
        case 3: v = r[x] + ((a + b) >> 1); break;
        case 4: v = r[x] + paeth(a, b, c); break;
        default: return PO_CORRUPT;
      }
      o[x] = (uint8_t)v;
    }
    prev = o;
  }
  return PO_OK;
}

/* One pixel: sample x of an unfiltered row -> out_c channels (png EXPAND). */
static void put_pixel(const pnginfo *pi, const uint8_t *r, uint32_t x, uint8_t *o) {
  const int C = pi->out_c, dp = pi->depth;
  if (pi->ctype == 0 || pi->ctype == 3) {
    uint32_t v;
    if (dp == 8) {
      v = r[x];
    } else {
      const size_t bit = (size_t)x * dp;
      v = (r[bit >> 3] >> (8 - dp - (bit & 7))) & ((1u << dp) - 1);
    }
    if (pi->ctype == 3) { /* entries past PLTE are black; alpha from tRNS, else 255 */
      o[0] = pi->pal[v][0];
      o[1] = pi->pal[v][1];
      o[2] = pi->pal[v][2];
      if (C == 4) o[3] = pi->pal[v][3];
    } else {
      const uint32_t scale = 255u / ((1u << dp) - 1u);
      o[0] = (uint8_t)(v * scale);
      if (C == 2) o[1] = v == pi->trns[0] ? 0 : 255;
    }
  } else if (pi->ctype == 2) {
    const uint8_t *p = r + 3 * (size_t)x;
    o[0] = p[0];
    o[1] = p[1];
    o[2] = p[2];
    if (C == 4) o[3] = (p[0] == pi->trns[0] && p[1] == pi->trns[1] && p[2] == pi->trns[2]) ? 0 : 255;
  } else {
    memcpy(o, r + (size_t)x * C, (size_t)C);
  }
}

/* Adam7 pass p (PNG spec 8.2): origin and spacing */
static const int kA7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};

/* Decode to HWC u8 with out_c channels (po_info).  Interlaced images: the
 * inflated stream holds the seven passes' filtered rows back to back (empty
 * passes contribute nothing), each pass unfiltered on its own. */
int po_decode(const uint8_t *d, size_t n, uint8_t *out, size_t cap) {
  pnginfo pi;
  int st = parse(d, n, &pi, 1);
  if (st) {
    free(pi.z);
    return st;
  }
  const int spp = pi.ctype == 2 ? 3 : pi.ctype == 4 ? 2 : pi.ctype == 6 ? 4 : 1;
  const size_t bitspp = (size_t)spp * pi.depth;
  const int bpp = (int)((bitspp + 7) / 8);
  uint32_t pw[7], ph[7];
  size_t prb[7], want = 0, unfn = 0;
  const int np = pi.interlace ? 7 : 1;
  for (int p = 0; p < np; p++) {
    if (pi.interlace) {
      pw[p] = pi.w > (uint32_t)kA7[p][0] ? (pi.w - kA7[p][0] + kA7[p][2] - 1) / kA7[p][2] : 0;
      ph[p] = pi.h > (uint32_t)kA7[p][1] ? (pi.h - kA7[p][1] + kA7[p][3] - 1) / kA7[p][3] : 0;
    } else {
      pw[p] = pi.w;
      ph[p] = pi.h;
    }
    prb[p] = (bitspp * pw[p] + 7) / 8;
    if (pw[p] && ph[p]) {
      want += (size_t)ph[p] * (prb[p] + 1);
      unfn += (size_t)ph[p] * prb[p];
    }
  }
  if (cap < (size_t)pi.w * pi.h * pi.out_c) {
    free(pi.z);
    return PO_SMALLBUF;
  }
  uint8_t *raw = (uint8_t *)malloc(want + 1);
  uint8_t *unf = (uint8_t *)malloc(unfn + 1);
  st = po_zlib_inflate(pi.z, pi.zn, raw, want, NULL);
  free(pi.z);
  size_t ro = 0, uo = 0;
  for (int p = 0; p < np && !st; p++) {
    if (!pw[p] || !ph[p]) continue;
    st = po_unfilter(raw + ro, ph[p], prb[p], bpp, unf + uo);
    ro += (size_t)ph[p] * (prb[p] + 1);
    uo += (size_t)ph[p] * prb[p];
  }
  free(raw);
  if (st) {
    free(unf);
    return st;
  }
  const int C = pi.out_c;
  uo = 0;
  for (int p = 0; p < np; p++) {
    if (!pw[p] || !ph[p]) continue;
    const int x0 = pi.interlace ? kA7[p][0] : 0, y0 = pi.interlace ? kA7[p][1] : 0;
    const int dx = pi.interlace ? kA7[p][2] : 1, dy = pi.interlace ? kA7[p][3] : 1;
    for (uint32_t py = 0; py < ph[p]; py++) {
      const uint8_t *r = unf + uo + (size_t)py * prb[p];
      const size_t y = (size_t)y0 + (size_t)py * dy;
      for (uint32_t px = 0; px < pw[p]; px++)
        put_pixel(&pi, r, px, out + (y * pi.w + (size_t)x0 + (size_t)px * dx) * C);
    }
    uo += (size_t)ph[p] * prb[p];
  }
  free(unf);
  return PO_OK;
}

/* ---------------------------------------------- alpha (fast_image_resize) */

/* mul_div_255: (a*b + 128 + ((a*b + 128) >> 8)) >> 8, the exact rounded a*b/255 */
static inline uint8_t mul_div_255(uint32_t a, uint32_t b) {
  const uint32_t t = a * b + 128;
  return (uint8_t)((t + (t >> 8)) >> 8);
}

/* Division table: recip[a] = round(255 * 2^8 / a), applied as (v * recip + 128) >> 8,
 * clamped to 255; alpha 0 gives 0. */
static inline uint8_t div_alpha(uint32_t v, uint32_t a) {
  if (a == 0) return 0;
  const uint32_t recip = ((255u << 9) / a + 1) >> 1;
  const uint32_t r = (v * recip + 128) >> 8;
  return (uint8_t)(r > 255 ? 255 : r);
}

void po_premultiply(uint8_t *p, size_t npx, int C) {
  for (size_t i = 0; i < npx; i++) {
    uint8_t *q = p + i * C;
    const uint32_t a = q[C - 1];
    for (int c = 0; c < C - 1; c++) q[c] = mul_div_255(q[c], a);
  }
}

void po_unpremultiply(uint8_t *p, size_t npx, int C) {
  for (size_t i = 0; i < npx; i++) {
    uint8_t *q = p + i * C;
    const uint32_t a = q[C - 1];
    for (int c = 0; c < C - 1; c++) q[c] = div_alpha(q[c], a);
  }
}

/* image's Rgba<u8>::blend of `fg` over the opaque (128,128,128) background,
 * then the RGB part (convert_to_rgb8, image_processing.rs:172-179). */
void po_blend_over_gray(const uint8_t *rgba, size_t npx, uint8_t *rgb) {
  for (size_t i = 0; i < npx; i++) {
    const uint8_t *f = rgba + 4 * i;
    uint8_t *o = rgb + 3 * i;
    if (f[3] == 0) {
      o[0] = o[1] = o[2] = 128;
      continue;
    }
    if (f[3] == 255) {
      o[0] = f[0];
      o[1] = f[1];
      o[2] = f[2];
      continue;
    }
    const float mx = 255.0f;
    const float bg = 128.0f / mx, bga = 255.0f / mx;
    const float fa = (float)f[3] / mx;
    const float af = bga + fa - bga * fa;
    if (af == 0.0f) {
      o[0] = o[1] = o[2] = 128;
      continue;
    }
    const float bgm = bg * bga;
    for (int c = 0; c < 3; c++) {
      const float fc = (float)f[c] / mx;
      const float v = (fc * fa + bgm * (1.0f - fa)) / af;
      const float s = mx * v;
      o[c] = (uint8_t)(s < 0.0f ? 0 : s > 255.0f ? 255 : (int)s);
    }
  }
}
