// dg_band.hip — the JPEG pixel path of one image band in one kernel:
// dequantisation + IDCT, chroma upsampling, colour conversion and the first
// horizontal Lanczos3 pass (fast_image_resize call 1, image_processing.rs:
// 288-298 after the decode of worker_files.rs:14-16), with the pass's
// convolution on the matrix cores.
//
// Why: the split path materialises two intermediates per image -- the
// Y/Cb/Cr planes (k_idct -> HBM -> the band H kernel's fill) -- and its fill
// waits on ~13 small plane loads per octet.  Here a workgroup takes
// kDecCols output columns of the H pass and walks the image's MCU rows in
// strips of kDecRows = 16 source rows; per strip it
//   1. IDCTs the coefficient blocks that cover its source segment into LDS
//      planes (8 lanes per block, libjpeg-turbo ISLOW or zune-jpeg's IDCT),
//      keeping the chroma block rows above and below in a three-row ring so
//      h2v2 fancy upsampling has its context rows without recomputing them;
//   2. upsamples and colour-converts from LDS into planar per-channel rows
//      (signed bytes p - 128: the i8 MFMA operand);
//   3. convolves: out[row][x] = sum_k src[row][k] * w_x[k] is a product of
//      the 16 x K strip with a banded K x 16 weight matrix per 16-column
//      subtile, so each subtile is v_mfma_i32_16x16x64_i8 over its window
//      (one or two K steps).  The i16 weight splits into three i8 operands,
//      w = 2^14 * a + 2^7 * b + c with a in [-2, 1], b and c in [0, 127]
//      (fast_image_resize's precision choice puts the largest weight of a
//      pass in [2^14, 2^15), so two base-128 digits do not fit a signed
//      byte), the pixel offset comes back as 128 * sum(w); every product and
//      sum is an exact i32, so the result equals fast_image_resize's i32
//      accumulation bit for bit;
//   4. stores the 16 rows of the H intermediate with 16-byte writes.
// The planes and the full-size RGB image never reach HBM; per image the
// kernel reads the coefficients once (plus the tile and strip-group edges)
// and writes the H intermediate once.
#include <hip/hip_runtime.h>

#include "dg_pixel.h"
#include "dg_types.h"
#include "kernels.h"

namespace dg {

typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kDecRows = 16;    // strip height: the MFMA M dimension
constexpr uint32_t kDecSub = 16;     // output columns per MFMA subtile (N)
constexpr uint32_t kDecThreads = 512; // 8 waves: one 16-column MFMA subtile each
constexpr uint32_t kDecRound = 64;   // IDCT blocks per round (one per 8-lane group)

__device__ __forceinline__ uint32_t dec_xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t per = n >> 3, rem = n & 7, x = b & 7, l = b >> 3;
  return x * per + (x < rem ? x : rem) + l;
}

__device__ __forceinline__ uint32_t dec_pack4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
  const uint32_t lo = __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm(b3, b2, 0x0c0c0400u);
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// LDS layout of one workgroup (SEG = widest source segment, pixels).
// Planar operand rows are read 16 bytes per lane, 16 rows per lane group: a
// row stride of an odd multiple of 16 bytes (mod 256) puts the 16 rows on
// distinct 4-bank groups.
constexpr uint32_t dec_row_stride(uint32_t need) {
  uint32_t a = (need + 15) / 16 * 16;
  while (((a / 16) & 1u) == 0) a += 16;
  return a;
}
template <uint32_t SEG, int KS>
struct DecSmem {
  static constexpr uint32_t YS = SEG;                   // Y plane row stride
  static constexpr uint32_t CS = SEG;                   // chroma row stride (h2: SEG/2 + 32 used)
  static constexpr uint32_t AS = dec_row_stride(SEG + 64 * KS);  // planar operand rows (reads reach 64 * KS past k0)
  __attribute__((aligned(16))) int16_t qt[3][64];       // quant tables, transposed: qt[c][col * 8 + row]
  uint32_t ext[4];
  __attribute__((aligned(16))) int32_t corr[kDecCols];  // per output column: 128 * sum(w) + rounding bias
  __attribute__((aligned(16))) uint8_t yp[kDecRows * YS];
  __attribute__((aligned(16))) uint8_t cp[2][kDecRows * CS];  // 4:4:4 / 4:2:2 rows, or the 4:2:0 ring (24 rows of SEG/2 + 32)
  union {
    __attribute__((aligned(16))) uint8_t ap[3][kDecRows * AS];  // planar operand rows (i8)
    int32_t blk[kDecRound * 72];                                // IDCT transpose scratch
  };
  // the next strip's coefficient blocks (zigzag int16, 128 B each, job order), landed by LDS-DMA
  // while this strip fills and convolves; jobs past STG load from HBM in their round
  static constexpr uint32_t STG = KS == 1 ? 128 : 64;
  __attribute__((aligned(16))) uint8_t stg[STG * 128];
};

// 8 libjpeg-turbo fancy-upsampled chroma samples at full-resolution columns
// x0..x0+7 (x0 % 8 == 0) of one row: r0 = its chroma row, r1 = the vertical
// neighbour row (h2v2) or null (h2v1); rows are indexed by absolute chroma
// column.  Same arithmetic as upsample8 (kernels.hip) and the oracle.
__device__ __forceinline__ void dec_ups_lj(const uint8_t *r0, const uint8_t *r1, uint32_t dsw, uint32_t x0,
                                           int32_t o[8]) {
  const uint32_t c0 = x0 >> 1;
  const bool fancy = dsw > 2;
  const uint32_t cl = c0 > 0 ? c0 - 1 : 0, cr = c0 + 4 < dsw ? c0 + 4 : dsw - 1;
  int32_t cs[6];
  if (!r1) {
    const uint32_t v = *(const uint32_t *)(r0 + c0);
    cs[0] = r0[cl];
#pragma unroll
    for (int k = 0; k < 4; k++) cs[k + 1] = (v >> (8 * k)) & 0xFF;
    cs[5] = r0[cr];
    if (c0 + 5 > dsw) {  // past the downsampled width: the edge sample (re-read: no dynamic register index)
      const int32_t edge = r0[dsw - 1];
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (c0 + k >= dsw) cs[k + 1] = edge;
    }
    if (!fancy) {
#pragma unroll
      for (int k = 0; k < 8; k++) o[k] = cs[1 + (k >> 1)];
      return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t a = cs[k + 1] * 3;
      const int32_t nl = (c0 + k + 1 < dsw) ? cs[k + 2] : cs[k + 1];
      o[2 * k] = (a + cs[k] + 1) >> 2;
      o[2 * k + 1] = (a + nl + 2) >> 2;
    }
    if (c0 == 0) o[0] = (cs[1] * 3 + cs[1] + 1) >> 2;
    return;
  }
  if (!fancy) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t c = c0 + (k >> 1);
      o[k] = r0[c < dsw ? c : dsw - 1];
    }
    return;
  }
  const uint32_t v0 = *(const uint32_t *)(r0 + c0), v1 = *(const uint32_t *)(r1 + c0);
  cs[0] = r0[cl] * 3 + r1[cl];
#pragma unroll
  for (int k = 0; k < 4; k++) cs[k + 1] = (int32_t)((v0 >> (8 * k)) & 0xFF) * 3 + (int32_t)((v1 >> (8 * k)) & 0xFF);
  cs[5] = r0[cr] * 3 + r1[cr];
  if (c0 + 5 > dsw) {
    const int32_t edge = r0[dsw - 1] * 3 + r1[dsw - 1];
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (c0 + k >= dsw) cs[k + 1] = edge;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int32_t nl = (c0 + k + 1 < dsw) ? cs[k + 2] : cs[k + 1];
    o[2 * k] = (cs[k + 1] * 3 + cs[k] + 8) >> 4;
    o[2 * k + 1] = (cs[k + 1] * 3 + nl + 7) >> 4;
  }
}

// zune-jpeg 0.5.12 upsampling of the same 8 samples (upsample8_zune): over
// the MCU-padded row of n = cbw * 8 samples, h2v2 vertically first.
__device__ __forceinline__ void dec_ups_zune(const uint8_t *r0, const uint8_t *r1, uint32_t n, uint32_t x0,
                                             int32_t o[8]) {
  const uint32_t c0 = x0 >> 1;
  const uint32_t cl = c0 > 0 ? c0 - 1 : 0, cr = c0 + 4 < n ? c0 + 4 : n - 1;
  int32_t cs[6];
  if (!r1) {
    const uint32_t v = *(const uint32_t *)(r0 + c0);
    cs[0] = r0[cl];
#pragma unroll
    for (int k = 0; k < 4; k++) cs[k + 1] = (v >> (8 * k)) & 0xFF;
    cs[5] = r0[cr];
  } else {
    const uint32_t v0 = *(const uint32_t *)(r0 + c0), v1 = *(const uint32_t *)(r1 + c0);
    cs[0] = (3 * (int32_t)r0[cl] + 2 + (int32_t)r1[cl]) >> 2;
#pragma unroll
    for (int k = 0; k < 4; k++)
      cs[k + 1] = (3 * (int32_t)((v0 >> (8 * k)) & 0xFF) + 2 + (int32_t)((v1 >> (8 * k)) & 0xFF)) >> 2;
    cs[5] = (3 * (int32_t)r0[cr] + 2 + (int32_t)r1[cr]) >> 2;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t i = c0 + (uint32_t)k;
    const int32_t a = 3 * cs[k + 1] + 2;
    int32_t ev = (a + cs[k]) >> 2, od = (a + cs[k + 2]) >> 2;
    if (i == 0) ev = cs[1];
    if (i + 1 == n) {
      ev = (3 * cs[k] + cs[k + 1] + 2) >> 2;
      od = cs[k + 1];
    }
    o[2 * k] = ev;
    o[2 * k + 1] = od;
  }
}

// n / d for n, d < 2^16 by one multiply-high with m = ceil(2^32 / d) (the
// error n * (m - 2^32 / d) / 2^32 < 2^-16 < 1 / d never crosses an integer).
// (m = 0 stands for d = 1; one 32-bit division per divisor, no 64-bit one)
__device__ __forceinline__ uint32_t dec_magic(uint32_t d) { return d <= 1 ? 0u : 0xFFFFFFFFu / d + 1u; }
__device__ __forceinline__ uint32_t dec_div(uint32_t n, uint32_t m) { return m ? __umulhi(n, m) : n; }

// Per-component block ranges of the workgroup's segment (uniform).
struct DecComp {
  uint32_t b0, nb;    // block columns [b0, b0 + nb) held in LDS
  uint32_t hr, vr;    // upsampling factors
  uint32_t lim;       // clamp width of the horizontal filter (libjpeg: downsampled width; zune: padded)
};

template <uint32_t SEG, int KS>
__global__ __launch_bounds__(kDecThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_band_dec(const ImageDesc *__restrict__ imgs, const WgItem *__restrict__ list,
                                                  const QuantTable *__restrict__ qpool, uint32_t strips_arg) {
  using SM = DecSmem<SEG, KS>;
  const uint32_t strips_per_wg = strips_arg & 0xFFFFu, dbg = strips_arg >> 16;  // dbg: timing experiments only
  __shared__ SM sm;
  const WgItem it = list[dec_xcd_remap(blockIdx.x, gridDim.x)];
  const ImageDesc &im = imgs[it.image];
  const ResizePass &ps = im.pass[0];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const uint32_t tiles = (ps.width + kDecCols - 1) / kDecCols;
  const uint32_t group = it.item0 / tiles, tile = it.item0 - group * tiles;
  const uint32_t x0 = tile * kDecCols;
  const uint32_t x1 = x0 + kDecCols < ps.width ? x0 + kDecCols : ps.width;
  const DG_GLOBAL int32_t *bounds = gp<const int32_t>(ps.bounds) + 2 * ps.out0;
  const DG_GLOBAL int16_t *coef = gp<const int16_t>(ps.coef) + (size_t)ps.out0 * ps.ksize;
  const uint32_t ncomp = im.ncomp, C = ncomp == 3 ? 3u : 1u;
  const bool zune = im.sem != 0;
  const int32_t prec = ps.precision;

  // ---- segment of the tile: [p0, p1) source columns, p0 16-aligned
  if (t == 0) {
    sm.ext[0] = 0xFFFFFFFFu;
    sm.ext[1] = 0;
  }
  if (t < 192) {
    const uint32_t c = t >> 6, k = t & 63;
    const DG_GLOBAL uint16_t *q = gp<const uint16_t>((uint64_t)(uintptr_t)qpool[im.qpool[c < ncomp ? c : 0]].q);
    sm.qt[c][(k & 7) * 8 + (k >> 3)] = (int16_t)q[k];
  }
  __syncthreads();
  if (t < kDecCols && x0 + t < x1) {
    const uint32_t st = (uint32_t)bounds[2 * (x0 + t)], n = (uint32_t)bounds[2 * (x0 + t) + 1];
    atomicMin(&sm.ext[0], st);
    atomicMax(&sm.ext[1], st + n);
  }
  __syncthreads();
  const uint32_t p0 = sm.ext[0] & ~15u;
  const uint32_t p1 = sm.ext[1];
  const uint32_t pe = (p1 + 7) & ~7u;  // fill end (<= cbw[0] * 8)
  const uint32_t nu = (pe - p0) >> 3;   // 8-pixel fill units per row

  // ---- per-component LDS block columns
  DecComp cc[3];
#pragma unroll
  for (uint32_t c = 0; c < 3; c++) {
    const uint32_t cq = c < ncomp ? c : 0;
    cc[c].hr = im.hmax / im.ch[cq];
    cc[c].vr = im.vmax / im.cv[cq];
    cc[c].lim = zune ? im.cbw[cq] * 8 : im.cdsw[cq];
    if (cc[c].hr == 1) {
      cc[c].b0 = p0 >> 3;
      cc[c].nb = (pe >> 3) - cc[c].b0;
    } else {
      const uint32_t lo = (p0 >> 1) > 0 ? (p0 >> 1) - 1 : 0;
      const uint32_t hi0 = (pe >> 1) + 4, hi = hi0 < cc[c].lim - 1 ? hi0 : cc[c].lim - 1;
      cc[c].b0 = lo >> 3;
      const uint32_t b1 = (hi >> 3) + 1 < im.cbw[cq] ? (hi >> 3) + 1 : im.cbw[cq];
      cc[c].nb = b1 - cc[c].b0;
    }
  }
  const bool ring = ncomp == 3 && cc[1].vr == 2;  // h2v2 chroma: three-block-row ring
  const uint32_t cstr = (ncomp == 3 && cc[1].hr == 2) ? SEG / 2 + 32 : SEG;

  // ---- MFMA weights of this wave's subtile (set up once)
  // lane: column n = lane & 15 of the subtile, k group g = lane >> 4
  const uint32_t n = lane & 15, g = lane >> 4;
  i32x4 wlo[KS], wmid[KS], whi[KS];  // weight digits c, b, a per K step
  uint32_t k0, steps;
  const uint32_t sub = wave;
  {
    const uint32_t xs = x0 + sub * kDecSub + n;
    const bool valid = xs < x1;
    uint32_t st = 0, cnt = 0;
    if (valid) {
      st = (uint32_t)bounds[2 * xs];
      cnt = (uint32_t)bounds[2 * xs + 1];
    }
    uint32_t mn = valid ? st : 0xFFFFFFFFu, mx = valid ? st + cnt : 0u;
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      const uint32_t a = (uint32_t)__shfl_xor((int)mn, m, 64), b = (uint32_t)__shfl_xor((int)mx, m, 64);
      mn = a < mn ? a : mn;
      mx = b > mx ? b : mx;
    }
    k0 = mn == 0xFFFFFFFFu ? p0 : (mn & ~15u);
    steps = mx > k0 ? (mx - k0 + 63) / 64 : 0;
    if (steps > (uint32_t)KS) steps = KS;  // host guarantees windows <= 64 * KS (band_dec_mode)
    const DG_GLOBAL int16_t *kp = coef + (size_t)(valid ? xs : x0) * ps.ksize;
    int32_t sum = 0;  // of column n's weights: this lane's K groups, then over the four groups
#pragma unroll
    for (int s = 0; s < KS; s++) {
      uint32_t lo[4] = {0, 0, 0, 0}, md[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
      const int32_t kb = (int32_t)(k0 + 64 * s + 16 * g) - (int32_t)st;
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int32_t i = kb + e;
        const int32_t w = (valid && i >= 0 && i < (int32_t)cnt) ? (int32_t)kp[i] : 0;
        sum += w;
        lo[e >> 2] |= (uint32_t)(w & 127) << (8 * (e & 3));
        md[e >> 2] |= (uint32_t)((w >> 7) & 127) << (8 * (e & 3));
        hi[e >> 2] |= (uint32_t)((w >> 14) & 0xFF) << (8 * (e & 3));
      }
      wlo[s] = i32x4{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3]};
      wmid[s] = i32x4{(int)md[0], (int)md[1], (int)md[2], (int)md[3]};
      whi[s] = i32x4{(int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    if (g == 0) sm.corr[sub * kDecSub + n] = sum * 128 + (1 << (prec - 1));
  }

  // ---- strips of this workgroup
  const uint32_t s_first = ps.row0 / kDecRows;
  const uint32_t s_end = (ps.row0 + ps.rows + kDecRows - 1) / kDecRows;
  const uint32_t sa = s_first + group * strips_per_wg;
  const uint32_t sb = sa + strips_per_wg < s_end ? sa + strips_per_wg : s_end;
  const DG_GLOBAL int16_t *cf = gp<const int16_t>(im.coef);

  // IDCT jobs of strip s: Y block rows 2s, 2s+1, then the chroma block rows
  // of the strip (4:4:4 / 4:2:2) or the ring's new rows (4:2:0: rows s-1..s+1
  // at the group's first strip, s+1 after), block columns of the segment
  struct Jobs {
    uint32_t ny_r0, nyj, c_r0, ncj, njobs, m_ncj;
  };
  const uint32_t m_nby = dec_magic(cc[0].nb ? cc[0].nb : 1u), m_nbc = dec_magic(cc[1].nb ? cc[1].nb : 1u);
  const uint32_t m_nu = dec_magic(nu ? nu : 1u);
  auto jobs_of = [&](uint32_t s, bool first) -> Jobs {
    Jobs J;
    J.ny_r0 = 2 * s;
    const uint32_t ny_rows = (2 * s + 2 <= im.cbh[0] ? 2u : (2 * s < im.cbh[0] ? 1u : 0u));
    uint32_t c_rows = 0;
    J.c_r0 = 0;
    if (ncomp == 3) {
      if (ring) {
        J.c_r0 = first ? (s > 0 ? s - 1 : 0) : s + 1;
        const uint32_t c_end = s + 2 < im.cbh[1] ? s + 2 : im.cbh[1];
        c_rows = c_end > J.c_r0 ? c_end - J.c_r0 : 0;
      } else {
        J.c_r0 = 2 * s;
        c_rows = (2 * s + 2 <= im.cbh[1] ? 2u : (2 * s < im.cbh[1] ? 1u : 0u));
      }
    }
    J.nyj = ny_rows * cc[0].nb;
    J.ncj = c_rows * cc[1].nb;
    J.m_ncj = dec_magic(J.ncj ? J.ncj : 1u);
    J.njobs = (dbg & 1) ? 0u : J.nyj + 2 * J.ncj;
    return J;
  };
  // job j of J -> (component, block row, block column); false past the end
  // (uniform divisors: multiply-high by precomputed magics, no division loops)
  auto job_at = [&](const Jobs &J, uint32_t j, uint32_t &c, uint32_t &r, uint32_t &b) -> bool {
    c = r = b = 0;
    if (j >= J.njobs) return false;
    if (j < J.nyj) {
      const uint32_t q = dec_div(j, m_nby);
      r = J.ny_r0 + q;
      b = cc[0].b0 + (j - q * cc[0].nb);
      return true;
    }
    j -= J.nyj;
    c = 1 + dec_div(j, J.m_ncj);
    j -= (c - 1) * J.ncj;
    const uint32_t q = dec_div(j, m_nbc);
    r = J.c_r0 + q;
    b = cc[1].b0 + (j - q * cc[1].nb);
    return true;
  };
  // Each 8-lane group of a wave owns one block of a round (wave w: scratch
  // blocks 8w..8w+7), so a round needs only wave-level ordering.  The
  // blocks come from the LDS staging, which LDS-DMA filled during the
  // previous strip's fill and convolution (~16 KiB per workgroup in flight
  // without a register), or, past STG jobs, straight from HBM.
  const uint32_t slot = t >> 3, l8 = t & 7;
  auto block_ptr = [&](uint32_t c, uint32_t r, uint32_t b) -> const DG_GLOBAL int16_t * {
    uint32_t idx;
    if (ncomp == 1) {
      idx = r * im.cbw[0] + b;
    } else {
      const uint32_t my = r / im.cv[c], vy = r - my * im.cv[c];
      const uint32_t mx = b / im.ch[c], hx = b - mx * im.ch[c];
      idx = (my * im.mcux + mx) * im.bpm + im.cfirst[c] + vy * im.ch[c] + hx;
    }
    return cf + (size_t)idx * 64;
  };
  // LDS-DMA of jobs [0, min(njobs, STG)): one wave instruction = 8 blocks (1 KiB), lane l the 16-byte
  // chunk l % 8 of block l / 8; wave w takes instructions w, w + 8, ...
  auto stage = [&](const Jobs &J) {
    const uint32_t nst = J.njobs < SM::STG ? J.njobs : SM::STG;
    for (uint32_t i = wave; i * 8 < nst; i += kDecThreads / 64) {
      const uint32_t j = i * 8 + (lane >> 3);
      uint32_t c, r, b;
      if (j < nst && job_at(J, j, c, r, b))
        __builtin_amdgcn_global_load_lds((const DG_GLOBAL void *)((const DG_GLOBAL uint8_t *)block_ptr(c, r, b) +
                                                                  (lane & 7) * 16),
                                         (__attribute__((address_space(3))) void *)(sm.stg + i * 1024), 16, 0, 0);
    }
  };
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  Jobs cur = jobs_of(sa, true);
  stage(cur);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (uint32_t s = sa; s < sb; s++) {
    // -- 1. IDCT into the LDS planes
    Jobs nxt = cur;
    if (s + 1 < sb) nxt = jobs_of(s + 1, false);
    for (uint32_t r0 = 0; r0 < cur.njobs; r0 += kDecRound) {
      uint32_t comp, brow, bcol;
      const uint32_t jb = r0 + slot;
      const bool act = job_at(cur, jb, comp, brow, bcol);
      u32x4 raw = u32x4{0u, 0u, 0u, 0u};
      if (jb < SM::STG)
        raw = *(const u32x4 *)(sm.stg + jb * 128 + l8 * 16);
      else if (act)
        raw = *(const DG_GLOBAL u32x4 *)(block_ptr(comp, brow, bcol) + l8 * 8);
      constexpr int LD = 72, RS = 9;
      int32_t *bv = sm.blk + slot * LD;
      {
        int16_t a[8];
        __builtin_memcpy(a, &raw, 16);
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const int nn = kZigzagToNatural[l8 * 8 + i];
          bv[(nn >> 3) * RS + (nn & 7)] = a[i];
        }
      }
      wave_sync();
      // pass 1: column l8, dequantised (each lane owns its column: no sync between read and write)
      {
        // column l8 of the component's quant table: one 16-byte read
        const u32x4 qv = *(const u32x4 *)(sm.qt[comp] + l8 * 8);
        int16_t qc[8];
        __builtin_memcpy(qc, &qv, 16);
        int32_t v[8], w[8];
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = bv[r * RS + l8] * (int32_t)qc[r];
        idct_col(zune, v, w);
#pragma unroll
        for (int r = 0; r < 8; r++) bv[r * RS + l8] = w[r];
      }
      wave_sync();
      // pass 2: row l8 -> 8 samples into the component's LDS plane
      if (act) {
        const int32_t *w = bv + l8 * RS;
        int32_t row[8];
        uint32_t px[8];
#pragma unroll
        for (int i = 0; i < 8; i++) row[i] = w[i];
        idct_row(zune, row, px);
        uint8_t *dst;
        if (comp == 0) {
          dst = sm.yp + ((brow - cur.ny_r0) * 8 + l8) * SM::YS + (bcol - cc[0].b0) * 8;
        } else if (ring) {
          dst = sm.cp[comp - 1] + ((brow % 3) * 8 + l8) * cstr + (bcol - cc[1].b0) * 8;
        } else {
          dst = sm.cp[comp - 1] + ((brow - cur.c_r0) * 8 + l8) * cstr + (bcol - cc[1].b0) * 8;
        }
        *(u32x2 *)dst = u32x2{dec_pack4(px[0], px[1], px[2], px[3]), dec_pack4(px[4], px[5], px[6], px[7])};
      }
      wave_sync();
    }
    __syncthreads();  // planes complete, staging consumed
    if (s + 1 < sb) stage(nxt);  // lands during the fill and the convolution

    // -- 2. fill: planar operand rows (p - 128) for the strip's 16 rows, columns [p0, pe)
    for (uint32_t j = t; j < ((dbg & 2) ? 0u : kDecRows * nu); j += kDecThreads) {
      const uint32_t r = dec_div(j, m_nu), u = j - r * nu;
      const uint32_t xo = 8 * u, xa = p0 + xo;  // offset in the segment, absolute column
      const uint32_t y = s * kDecRows + r;       // image row
      const u32x2 yv = *(const u32x2 *)(sm.yp + r * SM::YS + xo);
      if (ncomp == 1) {
        *(u32x2 *)(sm.ap[0] + r * SM::AS + xo) = u32x2{yv.x ^ 0x80808080u, yv.y ^ 0x80808080u};
        continue;
      }
      int32_t Y[8], Cb[8], Cr[8];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        Y[k] = (yv.x >> (8 * k)) & 0xFF;
        Y[k + 4] = (yv.y >> (8 * k)) & 0xFF;
      }
#pragma unroll
      for (uint32_t c = 1; c < 3; c++) {
        int32_t *o = c == 1 ? Cb : Cr;
        const uint8_t *pl = sm.cp[c - 1];
        if (cc[c].hr == 1) {
          const u32x2 v = *(const u32x2 *)(pl + r * cstr + xo);
#pragma unroll
          for (int k = 0; k < 4; k++) {
            o[k] = (v.x >> (8 * k)) & 0xFF;
            o[k + 4] = (v.y >> (8 * k)) & 0xFF;
          }
          continue;
        }
        const uint8_t *r0p, *r1p = nullptr;
        const int32_t cbase = (int32_t)(cc[c].b0 * 8);
        if (cc[c].vr == 1) {
          r0p = pl + r * cstr - cbase;
        } else {
          const uint32_t cr = y >> 1;  // chroma plane row
          uint32_t rn;
          if (zune) {
            const uint32_t ph = im.cbh[c] * 8;
            rn = (y & 1) ? (cr + 1 < ph ? cr + 1 : cr) : (cr > 0 ? cr - 1 : 0);
          } else {
            const int32_t dsh = (int32_t)im.cdsh[c];
            int32_t q = (y & 1) ? (int32_t)cr + 1 : (int32_t)cr - 1;
            q = q < 0 ? 0 : (q > dsh - 1 ? dsh - 1 : q);
            rn = (uint32_t)q;
          }
          r0p = pl + (((cr >> 3) % 3) * 8 + (cr & 7)) * cstr - cbase;
          r1p = pl + (((rn >> 3) % 3) * 8 + (rn & 7)) * cstr - cbase;
        }
        if (zune)
          dec_ups_zune(r0p, r1p, cc[c].lim, xa, o);
        else
          dec_ups_lj(r0p, r1p, cc[c].lim, xa, o);
      }
      uint32_t R[2] = {0, 0}, G[2] = {0, 0}, Bv[2] = {0, 0};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        uint8_t rr, gg, bb;
        if (im.colorspace == CS_RGB) {
          rr = (uint8_t)Y[k];
          gg = (uint8_t)Cb[k];
          bb = (uint8_t)Cr[k];
        } else if (zune) {
          ycc_to_rgb_zune(Y[k], Cb[k], Cr[k], rr, gg, bb);
        } else {
          ycc_to_rgb(Y[k], Cb[k], Cr[k], rr, gg, bb);
        }
        R[k >> 2] |= (uint32_t)rr << (8 * (k & 3));
        G[k >> 2] |= (uint32_t)gg << (8 * (k & 3));
        Bv[k >> 2] |= (uint32_t)bb << (8 * (k & 3));
      }
      *(u32x2 *)(sm.ap[0] + r * SM::AS + xo) = u32x2{R[0] ^ 0x80808080u, R[1] ^ 0x80808080u};
      *(u32x2 *)(sm.ap[1] + r * SM::AS + xo) = u32x2{G[0] ^ 0x80808080u, G[1] ^ 0x80808080u};
      *(u32x2 *)(sm.ap[2] + r * SM::AS + xo) = u32x2{Bv[0] ^ 0x80808080u, Bv[1] ^ 0x80808080u};
    }
    __syncthreads();

    // -- 3. convolution on the matrix cores, D = W . P for this wave's subtile
    // and channel: A = the weight digits (output column n, K group g), B =
    // the strip's pixels (row n, K group g), so lane (n, g) receives output
    // columns 4g .. 4g+3 of strip row n -- 4 adjacent pixels, stored
    // straight to HBM (12 bytes RGB / 4 bytes gray) without an LDS staging.
    const uint32_t y = s * kDecRows + n;  // this lane's image row
    const bool row_ok = y >= ps.row0 && y < ps.row0 + ps.rows;
    if (x0 + sub * kDecSub < x1 && steps != 0 && !(dbg & 4)) {  // wave-uniform
      uint32_t px[3] = {0, 0, 0};  // channel c of columns 4g .. 4g+3, packed
      for (uint32_t c = 0; c < C; c++) {
        const uint8_t *brow = sm.ap[c] + n * SM::AS + (k0 - p0) + 16 * g;  // B: strip row n, K group g
        i32x4 alo = *(const i32x4 *)(sm.corr + sub * kDecSub + 4 * g), amd = {0, 0, 0, 0}, ahi = {0, 0, 0, 0};
        {
          const i32x4 b = *(const i32x4 *)brow;
          alo = __builtin_amdgcn_mfma_i32_16x16x64_i8(wlo[0], b, alo, 0, 0, 0);
          amd = __builtin_amdgcn_mfma_i32_16x16x64_i8(wmid[0], b, amd, 0, 0, 0);
          ahi = __builtin_amdgcn_mfma_i32_16x16x64_i8(whi[0], b, ahi, 0, 0, 0);
        }
        if (KS > 1 && steps > 1) {
          const i32x4 b = *(const i32x4 *)(brow + 64);
          alo = __builtin_amdgcn_mfma_i32_16x16x64_i8(wlo[KS - 1], b, alo, 0, 0, 0);
          amd = __builtin_amdgcn_mfma_i32_16x16x64_i8(wmid[KS - 1], b, amd, 0, 0, 0);
          ahi = __builtin_amdgcn_mfma_i32_16x16x64_i8(whi[KS - 1], b, ahi, 0, 0, 0);
        }
        uint32_t o[4];
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
          const int32_t v = ((ahi[rr] << 14) + (amd[rr] << 7) + alo[rr]) >> prec;
          o[rr] = (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
        const uint32_t w4 = dec_pack4(o[0], o[1], o[2], o[3]);
        px[0] = c == 0 ? w4 : px[0];
        px[1] = c == 1 ? w4 : px[1];
        px[2] = c == 2 ? w4 : px[2];
      }
      const uint32_t xs = x0 + sub * kDecSub + 4 * g;  // first of the lane's 4 columns
      if (row_ok && !(dbg & 8) && xs < x1) {
      DG_GLOBAL uint8_t *d = gp<uint8_t>(ps.dst) + (size_t)(y - ps.row0) * ps.dst_stride + (size_t)xs * C;
      if (C == 1) {
        if (xs + 4 <= x1 && (((uintptr_t)d) & 3) == 0) {
          *(DG_GLOBAL uint32_t *)d = px[0];
        } else {
          for (uint32_t k = 0; k < 4 && xs + k < x1; k++) d[k] = (uint8_t)(px[0] >> (8 * k));
        }
      } else {
      // [R0 G0 B0 R1] [G1 B1 R2 G2] [B2 R3 G3 B3]
      const uint32_t rg = __builtin_amdgcn_perm(px[1], px[0], 0x05010400u);   // R0 G0 R1 G1
      const uint32_t rg2 = __builtin_amdgcn_perm(px[1], px[0], 0x07030602u);  // R2 G2 R3 G3
      const uint32_t d0 = __builtin_amdgcn_perm(px[2], rg, 0x02040100u);      // R0 G0 B0 R1
      const uint32_t gb = __builtin_amdgcn_perm(px[2], rg, 0x0c0c0503u);      // G1 B1 0 0
      const uint32_t d1 = __builtin_amdgcn_perm(rg2, gb, 0x05040100u);        // G1 B1 R2 G2
      const uint32_t d2 = __builtin_amdgcn_perm(rg2, px[2], 0x03070602u);     // B2 R3 G3 B3
      if (xs + 4 <= x1 && (((uintptr_t)d) & 3) == 0) {
        DG_GLOBAL uint32_t *d4 = (DG_GLOBAL uint32_t *)d;
        d4[0] = d0;
        d4[1] = d1;
        d4[2] = d2;
      } else {
        const uint32_t w[3] = {d0, d1, d2};
        for (uint32_t k = 0; k < 12 && xs + k / 3 < x1; k++) d[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
      }
      }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's staging DMA for the next strip landed
    __syncthreads();  // ... every wave's; and the next strip's IDCT scratch aliases the operand rows
    // (the next strip's IDCT writes yp / cp / the scratch aliasing ap, all
    // read before the barriers above; ob is next written after two barriers)
    cur = nxt;
  }
}

void launch_band_dec(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2],
                     const QuantTable *qpool, uint32_t strips_per_wg) {
  if (ncls[0])
    hipLaunchKernelGGL((k_band_dec<kDecSeg0, 1>), dim3(ncls[0]), dim3(kDecThreads), 0, st, imgs, list, qpool, strips_per_wg);
  if (ncls[1])
    hipLaunchKernelGGL((k_band_dec<kDecSeg1, 2>), dim3(ncls[1]), dim3(kDecThreads), 0, st, imgs, list + ncls[0], qpool,
                       strips_per_wg);
}

}  // namespace dg
