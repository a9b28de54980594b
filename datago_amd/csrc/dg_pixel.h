// dg_pixel.h — per-pixel arithmetic shared by the HIP kernels and the CPU
// emulator: ISLOW IDCT, chroma upsampling, YCbCr->RGB, Lanczos3 coefficients.
//
// Semantics follow libjpeg-turbo (the decoder the oracle is pinned against:
// tests/test_oracle_jpeg.py) and fast_image_resize 5.5.0's Convolution
// (reference image_processing.rs:288-323), see oracle/*.c for the restatements
// these kernels are checked against bit for bit.
#pragma once
#include "dg_types.h"

namespace dg {

// ---------------------------------------------------------------- ISLOW IDCT
// T.81 A.3.3 inverse DCT in the fixed-point factorisation of libjpeg's
// jidctint.c (CONST_BITS 13, PASS1_BITS 2).
constexpr int32_t kConstBits = 13, kPass1Bits = 2;

// a * b where both fit a signed 24-bit value (M24): the device's full-rate
// v_mul_i32_i24 (v_mul_lo_u32 is quarter rate) gives the same low 32 bits
template <bool M24>
DG_HD int32_t imul(int32_t a, int32_t b) {
#if defined(DG_DEVICE)
  if (M24) return __mul24(a, b);
#endif
  return a * b;
}

template <bool M24 = false>
DG_HD void idct_1d(const int32_t i0, const int32_t i1, const int32_t i2, const int32_t i3,
                   const int32_t i4, const int32_t i5, const int32_t i6, const int32_t i7,
                   int32_t o[8]) {
  int32_t z1, z2, z3, z4, z5, t0, t1, t2, t3, t10, t11, t12, t13;
  z2 = i2;
  z3 = i6;
  z1 = imul<M24>(z2 + z3, 4433);
  t2 = z1 + imul<M24>(z3, -15137);
  t3 = z1 + imul<M24>(z2, 6270);
  t0 = (int32_t)((uint32_t)(i0 + i4) << kConstBits);
  t1 = (int32_t)((uint32_t)(i0 - i4) << kConstBits);
  t10 = t0 + t3;
  t13 = t0 - t3;
  t11 = t1 + t2;
  t12 = t1 - t2;
  t0 = i7;
  t1 = i5;
  t2 = i3;
  t3 = i1;
  z1 = t0 + t3;
  z2 = t1 + t2;
  z3 = t0 + t2;
  z4 = t1 + t3;
  z5 = imul<M24>(z3 + z4, 9633);
  t0 = imul<M24>(t0, 2446);
  t1 = imul<M24>(t1, 16819);
  t2 = imul<M24>(t2, 25172);
  t3 = imul<M24>(t3, 12299);
  z1 = imul<M24>(z1, -7373);
  z2 = imul<M24>(z2, -20995);
  z3 = imul<M24>(z3, -16069);
  z4 = imul<M24>(z4, -3196);
  z3 += z5;
  z4 += z5;
  t0 += z1 + z3;
  t1 += z2 + z4;
  t2 += z2 + z3;
  t3 += z1 + z4;
  o[0] = t10 + t3;
  o[7] = t10 - t3;
  o[1] = t11 + t2;
  o[6] = t11 - t2;
  o[2] = t12 + t1;
  o[5] = t12 - t1;
  o[3] = t13 + t0;
  o[4] = t13 - t0;
}

DG_HD int32_t descale(int32_t x, int n) { return (x + (1 << (n - 1))) >> n; }

DG_HD uint8_t idct_out(int32_t x) {
  // libjpeg-turbo's SIMD IDCT output stage: saturate to int8, then +128
  x = descale(x, kConstBits + kPass1Bits + 3);
  x = x < -128 ? -128 : (x > 127 ? 127 : x);
  return (uint8_t)(x + 128);
}

// ------------------------------------------- zune-jpeg decode semantics
// Option "decode_semantics" = 1 (ImageDesc::sem): the pixel stages of the
// reference's own decoder, zune-jpeg 0.5.12, as oracle/jpeg_oracle.c
// restates them (OJ_SEM_ZUNE; unpinned -- the crate is not vendored).
// IDCT `idct_int`: stb_image's factorisation with 12-bit constants; o[k] are
// the pre-bias sums, pass 1 takes (o + 512) >> 10, pass 2
// (o + 65536 + (128 << 17)) >> 17 clamped to 0..255.
template <bool M24 = false>
DG_HD void idct_1d_stb(const int32_t s0, const int32_t s1, const int32_t s2, const int32_t s3,
                       const int32_t s4, const int32_t s5, const int32_t s6, const int32_t s7, int32_t o[8]) {
  int32_t p2 = s2, p3 = s6;
  int32_t p1 = imul<M24>(p2 + p3, 2217);
  const int32_t u2 = p1 + imul<M24>(p3, -7567), u3 = p1 + imul<M24>(p2, 3135);
  const int32_t t0e = (int32_t)((uint32_t)(s0 + s4) << 12), t1e = (int32_t)((uint32_t)(s0 - s4) << 12);
  const int32_t x0 = t0e + u3, x3 = t0e - u3, x1 = t1e + u2, x2 = t1e - u2;
  int32_t t0 = s7, t1 = s5, t2 = s3, t3 = s1;
  p3 = t0 + t2;
  int32_t p4 = t1 + t3;
  p1 = t0 + t3;
  p2 = t1 + t2;
  const int32_t p5 = imul<M24>(p3 + p4, 4816);
  t0 = imul<M24>(t0, 1223);
  t1 = imul<M24>(t1, 8410);
  t2 = imul<M24>(t2, 12586);
  t3 = imul<M24>(t3, 6149);
  p1 = p5 + imul<M24>(p1, -3685);
  p2 = p5 + imul<M24>(p2, -10497);
  p3 = imul<M24>(p3, -8034);
  p4 = imul<M24>(p4, -1597);
  t3 += p1 + p4;
  t2 += p2 + p3;
  t1 += p2 + p4;
  t0 += p1 + p3;
  o[0] = x0 + t3;
  o[7] = x0 - t3;
  o[1] = x1 + t2;
  o[6] = x1 - t2;
  o[2] = x2 + t1;
  o[5] = x2 - t1;
  o[3] = x3 + t0;
  o[4] = x3 - t0;
}
DG_HD int32_t idct_stb_pass1(int32_t o) { return (o + 512) >> 10; }
DG_HD uint8_t idct_stb_out(int32_t o) {
  const int32_t v = (o + 65536 + (128 << 17)) >> 17;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// Pass 1 of one column from its 8 dequantised inputs: the workspace values,
// saturated to 16 bits like libjpeg-turbo's SIMD IDCTs (vpackssdw between the
// passes; no valid coefficient block comes near the limits).  Pass 2 of one
// row of workspace values: 8 output samples.  Both decode semantics.
DG_HD int32_t sat16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
// M24: the caller knows every input is below 2^20 in magnitude (sums of up
// to four stay within 24 bits), so the products may use 24-bit multiplies.
template <bool M24 = false>
DG_HD void idct_col(bool zune, const int32_t v[8], int32_t ws[8]) {
  int32_t o[8];
  if (zune) {
    idct_1d_stb<M24>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], o);
#pragma unroll
    for (int r = 0; r < 8; r++) ws[r] = sat16(idct_stb_pass1(o[r]));
  } else {
    idct_1d<M24>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], o);
#pragma unroll
    for (int r = 0; r < 8; r++) ws[r] = sat16(descale(o[r], kConstBits - kPass1Bits));
  }
}
// Pass 2's inputs are the 16-bit-saturated workspace, so every product's
// operands fit 24 bits (sums of up to four of them times constants < 2^15):
// full-rate 24-bit multiplies, bit-exact.
DG_HD void idct_row(bool zune, const int32_t w[8], uint32_t px[8]) {
  int32_t o[8];
  if (zune) {
    idct_1d_stb<true>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
#pragma unroll
    for (int i = 0; i < 8; i++) px[i] = idct_stb_out(o[i]);
  } else {
    idct_1d<true>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
#pragma unroll
    for (int i = 0; i < 8; i++) px[i] = idct_out(o[i]);
  }
}

// Component and block coordinates (in that component's plane) of the
// decode-order block `idx` of a sequential scan: raster order for a single
// component, MCU-interleaved otherwise.
DG_HD void block_pos(const ImageDesc &im, uint32_t idx, uint32_t &c, uint32_t &by, uint32_t &bx) {
  if (im.ncomp == 1) {
    c = 0;
    by = idx / im.cbw[0];
    bx = idx - by * im.cbw[0];
    return;
  }
  const uint32_t mcu = idx / im.bpm, r = idx - mcu * im.bpm;
  c = (im.comp_bits >> (2 * r)) & 3u;
  const uint32_t j = r - im.cfirst[c], vy = j / im.ch[c], hx = j - vy * im.ch[c];
  const uint32_t my = mcu / im.mcux, mx = mcu - my * im.mcux;
  by = my * im.cv[c] + vy;
  bx = mx * im.ch[c] + hx;
}

// zigzag index -> natural index
#if defined(DG_DEVICE)
__constant__
#endif
static const uint8_t kZigzagToNatural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// --------------------------------------------------------- colour conversion
// libjpeg jdcolor.c build_ycc_rgb_table, SCALEBITS 16, computed inline.
DG_HD uint8_t clamp255(int32_t v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

DG_HD void ycc_to_rgb(int32_t y, int32_t cb, int32_t cr, uint8_t &r, uint8_t &g, uint8_t &b) {
  const int32_t F140200 = 91881;  // (int)(1.40200 * 65536 + 0.5)
  const int32_t F177200 = 116130;
  const int32_t F071414 = 46802;
  const int32_t F034414 = 22554;
  int32_t xcr = cr - 128, xcb = cb - 128;
#if defined(DG_DEVICE)
  // |x| <= 128 and the constants are < 2^17: 24-bit multiplies are exact and
  // full rate (hipcc otherwise emits the quarter-rate v_mul_lo_u32 here)
  int32_t crr = (__mul24(F140200, xcr) + 32768) >> 16;
  int32_t cbb = (__mul24(F177200, xcb) + 32768) >> 16;
  int32_t g_ = (__mul24(-F034414, xcb) + 32768 + __mul24(-F071414, xcr)) >> 16;
#else
  int32_t crr = (F140200 * xcr + 32768) >> 16;
  int32_t cbb = (F177200 * xcb + 32768) >> 16;
  int32_t g_ = (-F034414 * xcb + 32768 + -F071414 * xcr) >> 16;
#endif
  r = clamp255(y + crr);
  g = clamp255(y + g_);
  b = clamp255(y + cbb);
}

// zune-jpeg ycbcr_to_rgb (color_convert/scalar.rs): 5- and 6-bit constants
DG_HD void ycc_to_rgb_zune(int32_t y, int32_t cb, int32_t cr, uint8_t &r, uint8_t &g, uint8_t &b) {
  const int32_t xcb = cb - 128, xcr = cr - 128;
  r = clamp255(y + ((45 * xcr) >> 5));
  g = clamp255(y - ((11 * xcb + 23 * xcr) >> 5));
  b = clamp255(y + ((113 * xcb) >> 6));
}

// ----------------------------------------------------------- upsampling
// Value of component `c` at full-resolution pixel (x, y) — libjpeg-turbo
// jdsample.c: h2v1/h2v2 "fancy" triangle filters (box replication when
// downsampled_width <= 2), edges replicated (jdmainct.c context rows).
DG_HD uint32_t upsample_at(const uint8_t *pl, uint32_t stride, uint32_t hr, uint32_t vr,
                           uint32_t dsw, uint32_t dsh, uint32_t x, uint32_t y) {
  if (hr == 1 && vr == 1) return pl[(size_t)y * stride + x];
  uint32_t c = x >> 1;
  bool fancy = dsw > 2;
  if (vr == 1) {  // h2v1
    const uint8_t *in = pl + (size_t)y * stride;
    if (!fancy) return in[c];
    int32_t a = in[c] * 3;
    if (x & 1) {
      uint32_t n = c + 1 < dsw ? c + 1 : dsw - 1;
      return (uint32_t)((a + in[n] + 2) >> 2);
    }
    uint32_t n = c > 0 ? c - 1 : 0;
    return (uint32_t)((a + in[n] + 1) >> 2);
  }
  // h2v2
  uint32_t r = y >> 1;
  if (!fancy) return pl[(size_t)r * stride + c];
  int32_t rn = (y & 1) ? (int32_t)r + 1 : (int32_t)r - 1;
  if (rn < 0) rn = 0;
  if (rn > (int32_t)dsh - 1) rn = (int32_t)dsh - 1;
  const uint8_t *i0 = pl + (size_t)r * stride, *i1 = pl + (size_t)rn * stride;
  int32_t cs = i0[c] * 3 + i1[c];
  if (x & 1) {
    uint32_t n = c + 1 < dsw ? c + 1 : dsw - 1;
    int32_t ns = i0[n] * 3 + i1[n];
    return (uint32_t)((cs * 3 + ns + 7) >> 4);
  }
  uint32_t n = c > 0 ? c - 1 : 0;
  int32_t ps = i0[n] * 3 + i1[n];
  return (uint32_t)((cs * 3 + ps + 8) >> 4);
}

// --------------------------------------------------------------- Lanczos3
// Portable sin (fdlibm algorithm, < 1 ULP): identical on host and device so
// coefficient tables are bit-reproducible; within 1 ULP of glibc's sin.
// Callers compile with -ffp-contract=off.
DG_HD double k_sin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

DG_HD double k_cos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  double ax = x < 0 ? -x : x;
  if (ax < 0.3) return 1.0 - (0.5 * z - (z * r - x * y));
  double qx;
  if (ax > 0.78125) {
    qx = 0.28125;
  } else {
    uint64_t bits;
    __builtin_memcpy(&bits, &ax, 8);
    bits = (bits - 0x0020000000000000ULL) & 0xFFFFFFFF00000000ULL;
    __builtin_memcpy(&qx, &bits, 8);
  }
  double hz = 0.5 * z - qx, a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}

DG_HD double dg_sin(double x) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11;
  double ax = x < 0 ? -x : x;
  if (ax <= 0.785398163397448279) return k_sin(x, 0.0, 0);
  double fn = __builtin_floor(ax * invpio2 + 0.5);
  int n = (int)fn;
  double r = ax - fn * pio2_1, w = fn * pio2_1t;
  double y0 = r - w, y1 = (r - y0) - w;
  double s;
  switch (n & 3) {
    case 0: s = k_sin(y0, y1, 1); break;
    case 1: s = k_cos(y0, y1); break;
    case 2: s = -k_sin(y0, y1, 1); break;
    default: s = -k_cos(y0, y1); break;
  }
  return x < 0 ? -s : s;
}

DG_HD double sinc(double x) {
  if (x == 0.0) return 1.0;
  x *= 3.14159265358979323846;
  return dg_sin(x) / x;
}

DG_HD double lanczos3(double x) { return (x >= -3.0 && x < 3.0) ? sinc(x) * sinc(x / 3.0) : 0.0; }

// fast_image_resize precompute_coefficients for output index o.  Writes the
// normalised f64 weights (n of them) into w[] and returns the bound.
// ksize slots are enough by construction (ceil(support)*2+1).
DG_HD void fir_weights(uint32_t in_size, double in0, double in1, uint32_t out_size, uint32_t o,
                       double *w, int32_t &start, int32_t &n) {
  double scale = (in1 - in0) / (double)out_size;
  double filter_scale = scale > 1.0 ? scale : 1.0;
  double support = 3.0 * filter_scale;
  double recip = 1.0 / filter_scale;
  double center = in0 + ((double)o + 0.5) * scale;
  double fl = __builtin_floor(center - support);
  double cl = __builtin_ceil(center + support);
  int32_t xmin = fl < 0.0 ? 0 : (int32_t)fl;
  int32_t xmax = cl > (double)in_size ? (int32_t)in_size : (int32_t)cl;
  double c = center - 0.5;
  int32_t st = xmin, cnt = 0;
  double ww = 0.0;
  for (int32_t x = xmin; x < xmax; x++) {
    double v = lanczos3(((double)x - c) * recip);
    if (x == st && v == 0.0) {
      st++;
    } else {
      w[cnt++] = v;
      ww += v;
    }
  }
  while (cnt > 0 && w[cnt - 1] == 0.0) cnt--;
  if (ww != 0.0)
    for (int32_t i = 0; i < cnt; i++) w[i] /= ww;
  start = st;
  n = cnt;
}

DG_HD uint32_t fir_ksize(double in0, double in1, uint32_t out_size) {
  double scale = (in1 - in0) / (double)out_size;
  double filter_scale = scale > 1.0 ? scale : 1.0;
  return (uint32_t)__builtin_ceil(3.0 * filter_scale) * 2 + 1;
}

// Pillow-SIMD / fast_image_resize Normalizer16 precision for max weight m.
DG_HD int32_t fir_precision(double maxw) {
  int32_t precision = 0;
  for (int32_t p = 0; p < 22; p++) {
    precision = p;
    double nv = __builtin_round(maxw * (double)(1 << (p + 1)));
    if ((int32_t)nv >= (1 << 15)) break;
  }
  return precision;
}

DG_HD int16_t fir_quant(double v, int32_t precision) {
  double q = __builtin_round(v * (double)(1 << precision));
  if (q > 32767.0) q = 32767.0;
  if (q < -32768.0) q = -32768.0;
  return (int16_t)q;
}

}  // namespace dg
