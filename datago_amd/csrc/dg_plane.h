// dg_plane.h — how the IDCT writers store a block row of pixels into a
// component plane, and how the upsampling readers load it.
//
// Plain planes: one byte per sample, rows of cbw*8 bytes.
//
// Chroma records (ImageDesc::crec bit c; components sampled at half the
// horizontal rate, h2v1 / h2v2): the fused colour fill of the first H pass
// upsamples 8 output pixels from the 6 chroma samples c0-1 .. c0+4 of a row
// (c0 = x0 / 2, a multiple of 4).  In a plain plane that is one dword plus
// two edge bytes per chroma row, with clamping branches at the row ends.  A
// record plane stores each group of 4 samples of a row as one aligned 8-byte
// record -- bytes 0..3 samples 4g..4g+3, byte 4 sample 4g-1, byte 5 sample
// 4g+4, bytes 6..7 unused -- with every column clamped to [0, lim-1]
// (libjpeg: lim = the downsampled width, whose last sample jdsample.c
// replicates; zune: lim = the padded width it upsamples over), so one
// aligned 8-byte load gives the octet's six columns with the row ends
// already replicated.  Rows are cbw*16 bytes (twice the plain plane).
//
// A writer owns block bx's two records except their outer edge bytes:
// record 2bx's byte 4 (column 8bx-1) is written by block bx-1's writer and
// record 2bx+1's byte 5 (column 8bx+8) by block bx+1's, as byte stores, so
// writers of neighbouring blocks (other lanes, workgroups or kernels) never
// store to the same byte.  The plane's first and last records get their
// outer edge from their own block (clamped).
#pragma once
#include "dg_types.h"

#if defined(DG_DEVICE)
namespace dg {

__device__ __forceinline__ uint32_t plane_pack4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
  // v_perm byte selects (shift/or packing of clamped values miscompiles on
  // hipcc 7.2 for gfx950: see pack4 in kernels.hip)
  const uint32_t lo = __builtin_amdgcn_perm(b1, b0, 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm(b3, b2, 0x0c0c0400u);
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

__device__ __forceinline__ bool plane_is_rec(const ImageDesc &im, uint32_t c) { return (im.crec >> c) & 1u; }

// the column limit of component c's records (see above)
__device__ __forceinline__ uint32_t crec_lim(const ImageDesc &im, uint32_t c) {
  return im.sem ? im.cbw[c] * 8 : im.cdsw[c];
}

// Columns at or past lim take sample lim-1, which lies in this block (the
// last one) whenever any column of it does: lim > 8 * (cbw - 1).  v = px
// with that clamp applied (e = lim - 1 - 8 bx).
__device__ __forceinline__ void crec_clamp(int32_t e, const uint32_t px[8], uint32_t v[8]) {
  if (e < 7) {
    uint32_t pe = px[0];
#pragma unroll
    for (int k = 1; k < 8; k++) pe = k == e ? px[k] : pe;
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = k > e ? pe : px[k];
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = px[k];
  }
}

// Block bx's two records of one row (clamped samples v).  L / R: the outer
// edge samples (column 8bx-1, 8bx+8) when the caller knows them (have_l /
// have_r: a neighbour in the same workgroup, or the plane's end, where they
// clamp to v[0] / v[7]); then both records go out as one 16-byte store.  An
// unknown edge belongs to a neighbour block another writer handles: this
// writer leaves that byte alone and stores its own boundary sample into the
// neighbour's record instead (see above).
__device__ __forceinline__ void store_crec_pair(DG_GLOBAL uint8_t *row, uint32_t bx, uint32_t cbw, const uint32_t v[8],
                                                uint32_t l, uint32_t r, bool have_l, bool have_r) {
  DG_GLOBAL uint8_t *r0 = row + bx * 16, *r1 = r0 + 8;
  const uint32_t a = plane_pack4(v[0], v[1], v[2], v[3]), b = plane_pack4(v[4], v[5], v[6], v[7]);
  if (have_l && have_r) {
    *(DG_GLOBAL u32x4 *)r0 = u32x4{a, (l & 0xFFu) | ((v[4] & 0xFFu) << 8), b, (v[3] & 0xFFu) | ((r & 0xFFu) << 8)};
    return;
  }
  *(DG_GLOBAL uint32_t *)r0 = a;
  *(DG_GLOBAL uint32_t *)r1 = b;
  r0[5] = (uint8_t)v[4];
  r1[4] = (uint8_t)v[3];
  if (have_l)
    r0[4] = (uint8_t)l;
  else
    r0[-3] = (uint8_t)v[0];  // record 2bx-1, byte 5
  if (have_r)
    r1[5] = (uint8_t)r;
  else
    r1[12] = (uint8_t)v[7];  // record 2bx+2, byte 4
}

__device__ __forceinline__ DG_GLOBAL uint8_t *crec_row(const ImageDesc &im, uint32_t c, uint32_t y) {
  return (DG_GLOBAL uint8_t *)(uintptr_t)im.plane[c] + (size_t)y * (im.cbw[c] * 16);
}

// Row `y` (in samples) of block column bx of component c: 8 pixel values px,
// written without knowledge of the neighbour blocks (the scattered writers:
// k_idct_list, the fused IDCT of k_huff_write).
__device__ __forceinline__ void store_plane_row8(const ImageDesc &im, uint32_t c, uint32_t y, uint32_t bx,
                                                 const uint32_t px[8]) {
  const uint32_t cbw = im.cbw[c];
  if (!plane_is_rec(im, c)) {
    DG_GLOBAL uint8_t *dst = (DG_GLOBAL uint8_t *)(uintptr_t)im.plane[c] + (size_t)y * (cbw * 8) + bx * 8;
    *(DG_GLOBAL u32x2 *)dst = u32x2{plane_pack4(px[0], px[1], px[2], px[3]), plane_pack4(px[4], px[5], px[6], px[7])};
    return;
  }
  uint32_t v[8];
  crec_clamp((int32_t)crec_lim(im, c) - 1 - (int32_t)(bx * 8), px, v);
  store_crec_pair(crec_row(im, c, y), bx, cbw, v, v[0], v[7], bx == 0, bx + 1 == cbw);
}

// The six samples c0-1 .. c0+4 (c0 % 4 == 0) of record row `row` of a record
// plane with sample stride `stride` (= cbw * 8): one aligned 8-byte load.
template <class P>
__device__ __forceinline__ void load_crec6(P pl, uint32_t stride, uint32_t row, uint32_t c0, int32_t cs[6]) {
  const u32x2 v = *(const DG_GLOBAL u32x2 *)(pl + (size_t)__umul24(row, 2 * stride) + 2 * c0);
  cs[0] = (int32_t)(v.y & 0xFF);
#pragma unroll
  for (int k = 0; k < 4; k++) cs[k + 1] = (int32_t)((v.x >> (8 * k)) & 0xFF);
  cs[5] = (int32_t)((v.y >> 8) & 0xFF);
}

}  // namespace dg
#endif  // DG_DEVICE
