/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this file's library; the product path
 * (datago_amd/csrc) never links or calls it.
 *
 * Scalar C restatement of the re-encode step of image_to_payload
 * (reference /root/reference/src/image_processing.rs:374-395:
 * JpegEncoder::new_with_quality(cursor, quality).encode(bytes, w, h, color)),
 * i.e. image 0.25.9's baseline JPEG encoder (third-party, not vendored here;
 * restated from its published source):
 *   - quality q in [1,100] -> scale = q < 50 ? 5000/q : 200 - 2q; every entry of
 *     the ITU-T T.81 Annex K luma / chroma tables -> clamp((v*scale + 50)/100, 1, 255);
 *   - one component (L8 / La8) or three (Rgb8 / Rgba8), all 1x1 sampled (no
 *     chroma subsampling), standard Annex K Huffman tables, no restart markers;
 *   - 8x8 blocks in raster order, pixels past the right / bottom edge
 *     replicate the last column / row;
 *   - RGB -> YCbCr in f32 (JFIF coefficients scaled to 255, `as u8` casts:
 *     truncation, saturating);
 *   - libjpeg's integer FDCT (jfdctint "islow", CONST_BITS 13, PASS1_BITS 2,
 *     output scaled by 8);
 *   - quantisation ((coef / 8) as f32 / q).round() (integer division first,
 *     then f32, half away from zero);
 *   - headers: SOI, APP0 JFIF 1.02 (aspect 1:1), SOF0, DQT (one segment per
 *     table), DHT (one segment per table), SOS, scan, pad with 1-bits, EOI.
 * The byte stream is NOT pinned to the crate (not present offline);
 * tests/test_oracle_jpeg_enc.py pins the tables against libjpeg (PIL) and the
 * codec round trip through PIL's decoder.  The GPU encoder is checked
 * bit-exactly against this file.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const uint8_t ZZ[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                               12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                               35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                               58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

static const uint8_t STD_LUMA_Q[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                                       14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                                       18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                                       49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const uint8_t STD_CHROMA_Q[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                                         24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                                         99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                                         99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

const uint8_t oe_dc_luma_bits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t oe_dc_chroma_bits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t oe_dc_vals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t oe_ac_luma_bits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t oe_ac_luma_vals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t oe_ac_chroma_bits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t oe_ac_chroma_vals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

/* quality -> natural-order tables (t = 0 luma, 1 chroma) */
void oe_qtables(int quality, uint8_t q[2][64]) {
  int s = quality < 1 ? 1 : quality > 100 ? 100 : quality;
  s = s < 50 ? 5000 / s : 200 - 2 * s;
  for (int i = 0; i < 64; i++) {
    uint32_t a = ((uint32_t)STD_LUMA_Q[i] * (uint32_t)s + 50) / 100, b = ((uint32_t)STD_CHROMA_Q[i] * (uint32_t)s + 50) / 100;
    q[0][i] = (uint8_t)(a < 1 ? 1 : a > 255 ? 255 : a);
    q[1][i] = (uint8_t)(b < 1 ? 1 : b > 255 ? 255 : b);
  }
}

/* canonical codes of a standard table: code/len per symbol */
static void huff_codes(const uint8_t bits[16], const uint8_t *vals, uint16_t code[256], uint8_t len[256]) {
  memset(len, 0, 256);
  uint32_t c = 0, k = 0;
  for (int l = 1; l <= 16; l++) {
    for (int i = 0; i < bits[l - 1]; i++, k++) {
      code[vals[k]] = (uint16_t)c;
      len[vals[k]] = (uint8_t)l;
      c++;
    }
    c <<= 1;
  }
}

/* RGB -> YCbCr as image's rgb_to_ycbcr (f32, truncating saturating casts) */
static uint8_t sat_u8(float v) { return (uint8_t)(v <= 0.0f ? 0 : v >= 255.0f ? 255 : (int)v); }
void oe_rgb_to_ycbcr(uint8_t r8, uint8_t g8, uint8_t b8, uint8_t out[3]) {
  const float mx = 255.0f;
  const float r = (float)r8, g = (float)g8, b = (float)b8;
  const float y = 76.245f / mx * r + 149.685f / mx * g + 29.07f / mx * b;
  const float cb = -43.0185f / mx * r - 84.4815f / mx * g + 127.5f / mx * b + 128.0f;
  const float cr = 127.5f / mx * r - 106.7685f / mx * g - 20.7315f / mx * b + 128.0f;
  out[0] = sat_u8(y);
  out[1] = sat_u8(cb);
  out[2] = sat_u8(cr);
}

#define CONST_BITS 13
#define PASS1_BITS 2
#define FIX_0_298631336 2446
#define FIX_0_390180644 3196
#define FIX_0_541196100 4433
#define FIX_0_765366865 6270
#define FIX_0_899976223 7373
#define FIX_1_175875602 9633
#define FIX_1_501321110 12299
#define FIX_1_847759065 15137
#define FIX_1_961570560 16069
#define FIX_2_053119869 16819
#define FIX_2_562915447 20995
#define FIX_3_072711026 25172

/* libjpeg jfdctint (islow), output scaled by 8 (natural order) */
void oe_fdct(const uint8_t s[64], int32_t c[64]) {
  for (int y = 0; y < 8; y++) {
    const int y0 = y * 8;
    int32_t t0 = (int32_t)s[y0] + s[y0 + 7], t1 = (int32_t)s[y0 + 1] + s[y0 + 6];
    int32_t t2 = (int32_t)s[y0 + 2] + s[y0 + 5], t3 = (int32_t)s[y0 + 3] + s[y0 + 4];
    const int32_t t10 = t0 + t3, t12 = t0 - t3, t11 = t1 + t2, t13 = t1 - t2;
    t0 = (int32_t)s[y0] - s[y0 + 7];
    t1 = (int32_t)s[y0 + 1] - s[y0 + 6];
    t2 = (int32_t)s[y0 + 2] - s[y0 + 5];
    t3 = (int32_t)s[y0 + 3] - s[y0 + 4];
    c[y0] = (t10 + t11 - 8 * 128) << PASS1_BITS;
    c[y0 + 4] = (t10 - t11) << PASS1_BITS;
    int32_t z1 = (t12 + t13) * FIX_0_541196100 + (1 << (CONST_BITS - PASS1_BITS - 1));
    c[y0 + 2] = (z1 + t12 * FIX_0_765366865) >> (CONST_BITS - PASS1_BITS);
    c[y0 + 6] = (z1 - t13 * FIX_1_847759065) >> (CONST_BITS - PASS1_BITS);
    int32_t u12 = t0 + t2, u13 = t1 + t3;
    z1 = (u12 + u13) * FIX_1_175875602 + (1 << (CONST_BITS - PASS1_BITS - 1));
    u12 = u12 * (-FIX_0_390180644) + z1;
    u13 = u13 * (-FIX_1_961570560) + z1;
    z1 = (t0 + t3) * (-FIX_0_899976223);
    int32_t v0 = t0 * FIX_1_501321110 + z1 + u12;
    int32_t v3 = t3 * FIX_0_298631336 + z1 + u13;
    z1 = (t1 + t2) * (-FIX_2_562915447);
    int32_t v1 = t1 * FIX_3_072711026 + z1 + u13;
    int32_t v2 = t2 * FIX_2_053119869 + z1 + u12;
    c[y0 + 1] = v0 >> (CONST_BITS - PASS1_BITS);
    c[y0 + 3] = v1 >> (CONST_BITS - PASS1_BITS);
    c[y0 + 5] = v2 >> (CONST_BITS - PASS1_BITS);
    c[y0 + 7] = v3 >> (CONST_BITS - PASS1_BITS);
  }
  for (int x = 0; x < 8; x++) {
    int32_t t0 = c[x] + c[x + 56], t1 = c[x + 8] + c[x + 48], t2 = c[x + 16] + c[x + 40], t3 = c[x + 24] + c[x + 32];
    const int32_t t10 = t0 + t3 + (1 << (PASS1_BITS - 1)), t12 = t0 - t3, t11 = t1 + t2, t13 = t1 - t2;
    t0 = c[x] - c[x + 56];
    t1 = c[x + 8] - c[x + 48];
    t2 = c[x + 16] - c[x + 40];
    t3 = c[x + 24] - c[x + 32];
    c[x] = (t10 + t11) >> PASS1_BITS;
    c[x + 32] = (t10 - t11) >> PASS1_BITS;
    int32_t z1 = (t12 + t13) * FIX_0_541196100 + (1 << (CONST_BITS + PASS1_BITS - 1));
    c[x + 16] = (z1 + t12 * FIX_0_765366865) >> (CONST_BITS + PASS1_BITS);
    c[x + 48] = (z1 - t13 * FIX_1_847759065) >> (CONST_BITS + PASS1_BITS);
    int32_t u12 = t0 + t2, u13 = t1 + t3;
    z1 = (u12 + u13) * FIX_1_175875602 + (1 << (CONST_BITS + PASS1_BITS - 1));
    u12 = u12 * (-FIX_0_390180644) + z1;
    u13 = u13 * (-FIX_1_961570560) + z1;
    z1 = (t0 + t3) * (-FIX_0_899976223);
    int32_t v0 = t0 * FIX_1_501321110 + z1 + u12;
    int32_t v3 = t3 * FIX_0_298631336 + z1 + u13;
    z1 = (t1 + t2) * (-FIX_2_562915447);
    int32_t v1 = t1 * FIX_3_072711026 + z1 + u13;
    int32_t v2 = t2 * FIX_2_053119869 + z1 + u12;
    c[x + 8] = v0 >> (CONST_BITS + PASS1_BITS);
    c[x + 24] = v1 >> (CONST_BITS + PASS1_BITS);
    c[x + 40] = v2 >> (CONST_BITS + PASS1_BITS);
    c[x + 56] = v3 >> (CONST_BITS + PASS1_BITS);
  }
}

/* ((coef / 8) as f32 / q).round() */
static int32_t quant(int32_t coef, uint8_t q) {
  const float v = (float)(coef / 8) / (float)q;
  return (int32_t)roundf(v);
}

typedef struct {
  uint8_t *p;
  size_t n, cap;
  uint32_t acc;
  int nacc;
  int overflow;
} bw_t;

static void put_byte(bw_t *w, uint8_t b) {
  if (w->n < w->cap)
    w->p[w->n] = b;
  else
    w->overflow = 1;
  w->n++;
}
static void put_bits(bw_t *w, uint32_t v, int n) {
  for (int i = n - 1; i >= 0; i--) {
    w->acc = (w->acc << 1) | ((v >> i) & 1u);
    if (++w->nacc == 8) {
      put_byte(w, (uint8_t)w->acc);
      if ((w->acc & 0xFF) == 0xFF) put_byte(w, 0);
      w->acc = 0;
      w->nacc = 0;
    }
  }
}
static void put_seg(bw_t *w, uint8_t marker, const uint8_t *d, int n) {
  put_byte(w, 0xFF);
  put_byte(w, marker);
  put_byte(w, (uint8_t)((n + 2) >> 8));
  put_byte(w, (uint8_t)(n + 2));
  for (int i = 0; i < n; i++) put_byte(w, d[i]);
}

/* the header bytes up to and including SOS (shared with the GPU path's host
 * header builder in spirit; restated here independently) */
size_t oe_header(int w, int h, int ncomp, int quality, uint8_t *out, size_t cap) {
  bw_t W = {out, 0, cap, 0, 0, 0};
  uint8_t q[2][64], b[256];
  oe_qtables(quality, q);
  put_byte(&W, 0xFF);
  put_byte(&W, 0xD8);
  const uint8_t jfif[14] = {'J', 'F', 'I', 'F', 0, 1, 2, 0, 0, 1, 0, 1, 0, 0};
  put_seg(&W, 0xE0, jfif, 14);
  int n = 0;
  b[n++] = 8;
  b[n++] = (uint8_t)(h >> 8);
  b[n++] = (uint8_t)h;
  b[n++] = (uint8_t)(w >> 8);
  b[n++] = (uint8_t)w;
  b[n++] = (uint8_t)ncomp;
  for (int c = 0; c < ncomp; c++) {
    b[n++] = (uint8_t)(c + 1);
    b[n++] = 0x11;
    b[n++] = (uint8_t)(c ? 1 : 0);
  }
  put_seg(&W, 0xC0, b, n);
  for (int t = 0; t < (ncomp == 1 ? 1 : 2); t++) {
    b[0] = (uint8_t)t;
    for (int i = 0; i < 64; i++) b[1 + i] = q[t][ZZ[i]];
    put_seg(&W, 0xDB, b, 65);
  }
  const uint8_t *bits[4] = {oe_dc_luma_bits, oe_ac_luma_bits, oe_dc_chroma_bits, oe_ac_chroma_bits};
  const uint8_t *vals[4] = {oe_dc_vals, oe_ac_luma_vals, oe_dc_vals, oe_ac_chroma_vals};
  const uint8_t cls[4] = {0x00, 0x10, 0x01, 0x11};
  for (int t = 0; t < (ncomp == 1 ? 2 : 4); t++) {
    n = 0;
    b[n++] = cls[t];
    int nv = 0;
    for (int i = 0; i < 16; i++) {
      b[n++] = bits[t][i];
      nv += bits[t][i];
    }
    for (int i = 0; i < nv; i++) b[n++] = vals[t][i];
    put_seg(&W, 0xC4, b, n);
  }
  n = 0;
  b[n++] = (uint8_t)ncomp;
  for (int c = 0; c < ncomp; c++) {
    b[n++] = (uint8_t)(c + 1);
    b[n++] = c ? 0x11 : 0x00;
  }
  b[n++] = 0;
  b[n++] = 63;
  b[n++] = 0;
  put_seg(&W, 0xDA, b, n);
  return W.overflow ? 0 : W.n;
}

/* Encode HWC u8 (C = 1..4; alpha dropped, La8 -> L, Rgba8 -> RGB) to a JPEG.
 * Returns the byte count, 0 if `cap` is too small. */
size_t oe_encode(const uint8_t *px, int w, int h, int C, int quality, uint8_t *out, size_t cap) {
  const int ncomp = C <= 2 ? 1 : 3;
  size_t hn = oe_header(w, h, ncomp, quality, out, cap);
  if (!hn) return 0;
  bw_t W = {out, hn, cap, 0, 0, 0};
  uint8_t q[2][64];
  oe_qtables(quality, q);
  uint16_t code[4][256];
  uint8_t len[4][256];
  huff_codes(oe_dc_luma_bits, oe_dc_vals, code[0], len[0]);
  huff_codes(oe_ac_luma_bits, oe_ac_luma_vals, code[1], len[1]);
  huff_codes(oe_dc_chroma_bits, oe_dc_vals, code[2], len[2]);
  huff_codes(oe_ac_chroma_bits, oe_ac_chroma_vals, code[3], len[3]);
  int32_t prev[3] = {0, 0, 0};
  for (int by = 0; by < h; by += 8)
    for (int bx = 0; bx < w; bx += 8) {
      uint8_t blk[3][64];
      for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
          const int sx = bx + x < w ? bx + x : w - 1, sy = by + y < h ? by + y : h - 1;
          const uint8_t *p = px + ((size_t)sy * w + sx) * C;
          if (ncomp == 1) {
            blk[0][y * 8 + x] = p[0];
          } else {
            uint8_t ycc[3];
            oe_rgb_to_ycbcr(p[0], p[1], p[2], ycc);
            blk[0][y * 8 + x] = ycc[0];
            blk[1][y * 8 + x] = ycc[1];
            blk[2][y * 8 + x] = ycc[2];
          }
        }
      for (int c = 0; c < ncomp; c++) {
        int32_t co[64];
        oe_fdct(blk[c], co);
        const uint8_t *qt = q[c ? 1 : 0];
        int32_t zq[64];
        for (int i = 0; i < 64; i++) zq[i] = quant(co[ZZ[i]], qt[ZZ[i]]);
        const int t = c ? 2 : 0;
        const int32_t diff = zq[0] - prev[c];
        prev[c] = zq[0];
        {
          const uint32_t a = (uint32_t)(diff < 0 ? -diff : diff);
          int sz = 0;
          while ((a >> sz) != 0) sz++;
          put_bits(&W, code[t][sz], len[t][sz]);
          if (sz) put_bits(&W, diff < 0 ? (uint32_t)(diff - 1) & ((1u << sz) - 1u) : (uint32_t)diff, sz);
        }
        int run = 0;
        for (int k = 1; k < 64; k++) {
          const int32_t v = zq[k];
          if (v == 0) {
            run++;
            continue;
          }
          while (run > 15) {
            put_bits(&W, code[t + 1][0xF0], len[t + 1][0xF0]);
            run -= 16;
          }
          const uint32_t a = (uint32_t)(v < 0 ? -v : v);
          int sz = 0;
          while ((a >> sz) != 0) sz++;
          const int sym = (run << 4) | sz;
          put_bits(&W, code[t + 1][sym], len[t + 1][sym]);
          put_bits(&W, v < 0 ? (uint32_t)(v - 1) & ((1u << sz) - 1u) : (uint32_t)v, sz);
          run = 0;
        }
        if (zq[63] == 0) put_bits(&W, code[t + 1][0x00], len[t + 1][0x00]);
      }
    }
  if (W.nacc) put_bits(&W, 0x7F, 8 - W.nacc);  /* pad with 1-bits */
  put_byte(&W, 0xFF);
  put_byte(&W, 0xD9);
  return W.overflow ? 0 : W.n;
}

/* Upper bound of oe_encode's output (what the caller must allocate). */
size_t oe_bound(int w, int h, int C) {
  const size_t ncomp = C <= 2 ? 1 : 3;
  const size_t blocks = (size_t)((w + 7) / 8) * (size_t)((h + 7) / 8) * ncomp;
  return 1024 + blocks * 420;
}
