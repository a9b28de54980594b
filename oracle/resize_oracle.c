/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this file's library; the product path
 * (datago_amd/csrc) never links or calls it.
 *
 * Scalar C restatement of datago's crop_and_resize for 8-bit pixels
 * (reference /root/reference/src/image_processing.rs:254-337):
 *   scale = max(tw/W, th/H); new = round(W*s), round(H*s)      (:278-286)
 *   Resizer::resize(Lanczos3 convolution) -> new_w x new_h      (:288-298)
 *   CropBox::fit_src_into_dst_size(new_w,new_h,tw,th)          (:304-310)
 *   Resizer::resize with crop -> tw x th                        (:312-323)
 *
 * The convolution is fast_image_resize 5.5.0's `Convolution` (third-party,
 * not vendored; Cargo.lock pins it).  Its published algorithm is Pillow-SIMD's
 * separable resampler: f64 Lanczos3 weights normalised per output pixel,
 * quantised to i16 with one dynamic precision per pass (largest precision that
 * keeps 2*max_weight < 2^15), i32 accumulate with a 1<<(prec-1) bias, >>prec,
 * clamp to u8; horizontal pass first over only the rows the vertical pass
 * reads; a pass is skipped when it is the identity.
 *
 * MODE_PILLOW switches the coefficient bounds/quantisation to stock Pillow's
 * (22-bit i32, bounds rounded with (int)(x+0.5)); everything else is shared.
 * tests/test_oracle_resize.py pins MODE_PILLOW bit-exactly against PIL's own
 * Image.resize(..., LANCZOS, box=...), which pins the shared structure, and
 * checks MODE_FIR against PIL within 1 LSB.  fast_image_resize itself cannot
 * run here: its i16 rounding is restated, not pinned.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MODE_FIR 0
#define MODE_PILLOW 1

typedef struct {
  int start, size;
} or_bound;

/* Portable sin for |t| < ~1e5 (fdlibm's algorithm: Cody-Waite pi/2 reduction
 * with a 33+53-bit split, __kernel_sin/__kernel_cos minimax polynomials, < 1
 * ULP).  The product computes the same function on the GPU, so the two agree
 * bit-for-bit; vs glibc sin (what fast_image_resize calls) it differs by at
 * most 1 ULP (tests/test_oracle_resize.py), and the i16 tables, bounds and
 * precisions it yields are identical to glibc's for every pass of the
 * configs[1] and configs[2] size distributions
 * (tests/test_oracle_sin_tables.py). Built with -ffp-contract=off. */
static double k_sin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
static double k_cos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  double ax = fabs(x);
  if (ax < 0.3) return 1.0 - (0.5 * z - (z * r - x * y));
  double qx;
  if (ax > 0.78125) {
    qx = 0.28125;
  } else {
    uint64_t b;
    memcpy(&b, &ax, 8);
    b = (b - 0x0020000000000000ULL) & 0xFFFFFFFF00000000ULL; /* x/4, low word cleared */
    memcpy(&qx, &b, 8);
  }
  double hz = 0.5 * z - qx, a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}
double or_sin(double x) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11;
  double ax = fabs(x);
  if (ax <= 0.785398163397448279) return k_sin(x, 0.0, 0);
  double fn = floor(ax * invpio2 + 0.5);
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

static int use_libm_sin = 0;
void or_use_libm_sin(int on) { use_libm_sin = on; }

static double sinc(double x) {
  if (x == 0.0) return 1.0;
  x *= 3.14159265358979323846;
  return (use_libm_sin ? sin(x) : or_sin(x)) / x;
}

static double lanczos3(double x) {
  if (x >= -3.0 && x < 3.0) return sinc(x) * sinc(x / 3.0);
  return 0.0;
}

/* Returns ksize (window size); fills bounds[out_size] and coeffs[out_size*ksize]
 * as integers plus the precision.  Caller frees *coeffs_out. */
int or_coeffs(int in_size, double in0, double in1, int out_size, int mode, or_bound *bounds,
              int32_t **coeffs_out, int *precision_out) {
  double scale = (in1 - in0) / (double)out_size;
  double filter_scale = scale > 1.0 ? scale : 1.0;
  double support = 3.0 * filter_scale;
  int ksize = (int)ceil(support) * 2 + 1;
  double *kk = (double *)calloc((size_t)out_size * ksize, sizeof(double));
  double maxw = 0.0;
  for (int xx = 0; xx < out_size; xx++) {
    double center = in0 + (xx + 0.5) * scale;
    double ww = 0.0;
    double *k = kk + (size_t)xx * ksize;
    int xmin, xmax, n = 0;
    if (mode == MODE_PILLOW) {
      double ss = 1.0 / filter_scale;
      xmin = (int)(center - support + 0.5);
      if (xmin < 0) xmin = 0;
      xmax = (int)(center + support + 0.5);
      if (xmax > in_size) xmax = in_size;
      n = xmax - xmin;
      for (int x = 0; x < n; x++) {
        double w = lanczos3((x + xmin - center + 0.5) * ss);
        k[x] = w;
        ww += w;
      }
    } else {
      /* fast_image_resize precompute_coefficients: floor/ceil bounds, kernel
       * evaluated at (x - (center - 0.5)) * (1/filter_scale), leading zero
       * weights trimmed from the bound. */
      double recip = 1.0 / filter_scale;
      double fl = floor(center - support);
      double cl = ceil(center + support);
      xmin = fl < 0.0 ? 0 : (int)fl;
      xmax = cl > (double)in_size ? in_size : (int)cl;
      double c = center - 0.5;
      int start = xmin;
      for (int x = xmin; x < xmax; x++) {
        double w = lanczos3(((double)x - c) * recip);
        if (x == start && w == 0.0) {
          start++;
        } else {
          k[n++] = w;
          ww += w;
        }
      }
      while (n > 0 && k[n - 1] == 0.0) n--;
      xmin = start;
    }
    if (ww != 0.0)
      for (int x = 0; x < n; x++) k[x] /= ww;
    for (int x = 0; x < n; x++)
      if (k[x] > maxw) maxw = k[x];
    bounds[xx].start = xmin;
    bounds[xx].size = n;
  }
  int32_t *ci = (int32_t *)calloc((size_t)out_size * ksize, sizeof(int32_t));
  int precision;
  if (mode == MODE_PILLOW) {
    precision = 22;
    for (size_t i = 0; i < (size_t)out_size * ksize; i++)
      ci[i] = kk[i] < 0 ? (int32_t)(-0.5 + kk[i] * (1 << 22)) : (int32_t)(0.5 + kk[i] * (1 << 22));
  } else {
    precision = 0;
    for (int p = 0; p < 22; p++) {
      precision = p;
      double nv = round(maxw * (double)(1 << (p + 1)));
      if ((int32_t)nv >= (1 << 15)) break;
    }
    double sc = (double)(1 << precision);
    for (size_t i = 0; i < (size_t)out_size * ksize; i++) {
      double v = round(kk[i] * sc);
      if (v > 32767.0) v = 32767.0;
      if (v < -32768.0) v = -32768.0;
      ci[i] = (int32_t)(int16_t)v;
    }
  }
  free(kk);
  *coeffs_out = ci;
  *precision_out = precision;
  return ksize;
}

static inline uint8_t clip8(int64_t ss, int prec) {
  int64_t v = ss >> prec;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

/* One resample call: src (sw x sh x C) -> dst (dw x dh x C) over box
 * [x0,x1) x [y0,y1) (Pillow ImagingResampleInner / FIR resample_convolution). */
int or_resample(const uint8_t *src, int sw, int sh, int C, uint8_t *dst, int dw, int dh,
                double x0, double y0, double x1, double y1, int mode) {
  int need_h = dw != sw || x0 != 0.0 || x1 != (double)dw;
  int need_v = dh != sh || y0 != 0.0 || y1 != (double)dh;
  or_bound *bh = (or_bound *)malloc(sizeof(or_bound) * (size_t)dw);
  or_bound *bv = (or_bound *)malloc(sizeof(or_bound) * (size_t)dh);
  int32_t *kh = NULL, *kv = NULL;
  int ph = 0, pv = 0;
  int ksh = or_coeffs(sw, x0, x1, dw, mode, bh, &kh, &ph);
  int ksv = or_coeffs(sh, y0, y1, dh, mode, bv, &kv, &pv);
  int yfirst = bv[0].start;
  int ylast = bv[dh - 1].start + bv[dh - 1].size;
  const uint8_t *cur = src;
  int cw = sw, row0 = 0;
  uint8_t *tmp = NULL;
  if (need_h) {
    int rows = ylast - yfirst;
    if (!need_v) { yfirst = 0; rows = sh; }
    tmp = (uint8_t *)malloc((size_t)dw * rows * C + 1);
    for (int y = 0; y < rows; y++) {
      const uint8_t *in = src + (size_t)(y + yfirst) * sw * C;
      uint8_t *o = tmp + (size_t)y * dw * C;
      for (int x = 0; x < dw; x++) {
        const int32_t *k = kh + (size_t)x * ksh;
        for (int c = 0; c < C; c++) {
          int64_t ss = (int64_t)1 << (ph - 1);
          for (int i = 0; i < bh[x].size; i++) ss += (int64_t)in[(size_t)(bh[x].start + i) * C + c] * k[i];
          o[(size_t)x * C + c] = clip8(ss, ph);
        }
      }
    }
    cur = tmp;
    cw = dw;
    row0 = yfirst;
  }
  if (need_v) {
    for (int y = 0; y < dh; y++) {
      const int32_t *k = kv + (size_t)y * ksv;
      int s = bv[y].start - row0;
      for (int x = 0; x < cw * C; x++) {
        int64_t ss = (int64_t)1 << (pv - 1);
        for (int i = 0; i < bv[y].size; i++) ss += (int64_t)cur[(size_t)(s + i) * cw * C + x] * k[i];
        dst[(size_t)y * dw * C + x] = clip8(ss, pv);
      }
    }
  } else {
    memcpy(dst, cur, (size_t)dw * dh * C);
  }
  free(tmp);
  free(bh);
  free(bv);
  free(kh);
  free(kv);
  return 0;
}

static double rround(double x) { return x >= 0 ? floor(x + 0.5) : -floor(-x + 0.5); }

/* image_processing.rs:278-286 */
void or_scaled_size(int w, int h, int tw, int th, int *nw, int *nh) {
  double sx = (double)tw / (double)w, sy = (double)th / (double)h;
  double s = sx > sy ? sx : sy;
  *nw = (int)rround((double)w * s);
  *nh = (int)rround((double)h * s);
}

/* fast_image_resize CropBox::fit_src_into_dst_size (Pillow ImageOps.fit) */
void or_fit_crop(int sw, int sh, int dw, int dh, double *l, double *t, double *cw, double *ch) {
  double width = sw, height = sh;
  double ir = width / height, rr = (double)dw / (double)dh;
  double w, h;
  if (fabs(ir - rr) < 2.220446049250313e-16) { w = width; h = height; }
  else if (ir >= rr) { w = rr * height; h = height; }
  else { w = width; h = width / rr; }
  *l = (width - w) * 0.5;
  *t = (height - h) * 0.5;
  *cw = w;
  *ch = h;
}

/* fast_image_resize mul_div_alpha: a U8x2/U8x4 convolution call
 * premultiplies a copy of its source, resamples, and divides the result; a
 * call that is a plain copy (same size, integral box) touches no alpha.
 * po_premultiply/po_unpremultiply live in png_oracle.c. */
void po_premultiply(uint8_t *p, size_t npx, int C);
void po_unpremultiply(uint8_t *p, size_t npx, int C);

static int resample_call(const uint8_t *src, int sw, int sh, int C, uint8_t *dst, int dw, int dh, double x0,
                         double y0, double x1, double y1, int mode) {
  /* a crop box of the destination's size at integral offsets is a copy */
  const int is_copy = x1 - x0 == (double)dw && y1 - y0 == (double)dh && x0 == floor(x0) && y0 == floor(y0);
  if (is_copy) {
    for (int y = 0; y < dh; y++)
      memcpy(dst + (size_t)y * dw * C, src + ((size_t)(y + (int)y0) * sw + (size_t)x0) * C, (size_t)dw * C);
    return 0;
  }
  if (!(C == 2 || C == 4)) return or_resample(src, sw, sh, C, dst, dw, dh, x0, y0, x1, y1, mode);
  const size_t n = (size_t)sw * sh;
  uint8_t *pm = (uint8_t *)malloc(n * C + 1);
  memcpy(pm, src, n * C);
  po_premultiply(pm, n, C);
  int r = or_resample(pm, sw, sh, C, dst, dw, dh, x0, y0, x1, y1, mode);
  po_unpremultiply(dst, (size_t)dw * dh, C);
  free(pm);
  return r;
}

/* Whole crop_and_resize for C in {1,2,3,4}: src W x H -> dst tw x th. */
int or_crop_and_resize(const uint8_t *src, int w, int h, int C, int tw, int th, uint8_t *dst, int mode) {
  if (w == tw && h == th) { memcpy(dst, src, (size_t)w * h * C); return 0; }
  int nw, nh;
  or_scaled_size(w, h, tw, th, &nw, &nh);
  uint8_t *mid = (uint8_t *)malloc((size_t)nw * nh * C + 1);
  resample_call(src, w, h, C, mid, nw, nh, 0.0, 0.0, (double)w, (double)h, mode);
  double l, t, cw, ch;
  or_fit_crop(nw, nh, tw, th, &l, &t, &cw, &ch);
  resample_call(mid, nw, nh, C, dst, tw, th, l, t, l + cw, t + ch, mode);
  free(mid);
  return 0;
}
