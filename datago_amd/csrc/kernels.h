// kernels.h — launchers for the HIP kernels in kernels.hip (host-callable).
#pragma once
#include <hip/hip_runtime.h>

#include "dg_types.h"

namespace dg {

// Destuffing: raw scan -> clean bit stream + RST marker positions
void launch_destuff_count(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_destuff_scan(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_destuff_write(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_destuff_one(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg, uint64_t *state);
// Entropy decode (one 256-thread workgroup per 256 subsequences of one image)
// (sync/fix: 255 useful subsequences per workgroup, see kernels.hip)
struct Ckpt;
// stage: decode-once staging (ImageDesc::stage), see k_huff_scatter
// max_slots: the largest ImageDesc::nslots in the batch (dynamic LDS for the tables);
// max_ac: the most distinct AC tables of an image (multi-symbol lead-in lookups, 0 = off)
void launch_huff_sync(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                      const HuffTable *pool, SubState *subs, Ckpt *ck, BatchFlags *flags, bool stage,
                      uint32_t max_slots, uint32_t max_ac, bool pair, bool two = false);
void launch_huff_fix(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                     const HuffTable *pool, SubState *subs, Ckpt *ck, BatchFlags *flags, bool stage,
                     uint32_t max_slots);
// one workgroup per image
void launch_huff_scan(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg, SubState *subs);
void launch_huff_write(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                       const HuffTable *pool, const SubState *subs, BatchFlags *flags, uint32_t max_slots,
                       const QuantTable *qpool, uint32_t pair, const Ckpt *ckpt);
// fused IDCT leftovers (BatchFlags::idct_list), grid-strided over the device-side count
void launch_idct_list(hipStream_t st, const ImageDesc *imgs, const QuantTable *qpool, const BatchFlags *flags,
                      uint32_t nwg);
// decode-once: blocks from the staged coefficients (replaces k_huff_write when ImageDesc::stage is set)
void launch_huff_scatter(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                         const SubState *subs);
// dequant + IDCT: 64 blocks of one block row per workgroup
void launch_idct_t(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, const QuantTable *qpool);
void launch_idct(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg,
                 const QuantTable *qpool);
// upsample + colour convert: 256 x 4-pixel quads per workgroup
void launch_color(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
// Lanczos coefficient tables: one workgroup per (image, stage)
void launch_coeffs(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg);
// resize passes of one stage: 256 output pixels (H) / 4-byte units (V) per workgroup
void launch_resize_h(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int stage);
// band H pass: kHBandCols x kHBandRows outputs per workgroup (see kernels.hip);
// `list` holds ncls[k] items of weight-count class k (<=8, <=16, <=32, more) in order
// ncls[fused][class]: the list holds the fused (colour-fill) items first, then the byte-fill ones,
// each ordered by weight-count class (<= 8, 16, 32 taps, more)
void launch_resize_hb(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2][4],
                      int stage,
                      bool prefetch, bool planar, bool zune);
// band H pass on the matrix cores (k_resize_hm): ncls[fused][ks - 1] items, launched fused KS 1, fused KS 2,
// byte-fill KS 1, byte-fill KS 2 (KS = 64-wide K steps of a 16-column subtile's window)
void launch_resize_hm(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2][2],
                      int stage);
// fused first H + V pass (pass[0].mode & kHVFused): lists of H weight classes <= 8, <= 16 taps
void launch_resize_hv(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2]);
void launch_resize_v(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int stage,
                     uint32_t vunits);
void launch_resize_vt(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int stage,
                      uint32_t rows);
// k_band_dec (dg_band.hip): IDCT + upsampling + colour + the first H pass of images with pass[0].mode &
// kHDecode; list = ncls[0] items of the 320-pixel class, then ncls[1] of the 640-pixel class
void launch_band_dec(hipStream_t st, const ImageDesc *imgs, const WgItem *list, const uint32_t ncls[2],
                     const QuantTable *qpool, uint32_t strips_per_wg);
// final copy / gray->RGB expansion: 256 output pixels per workgroup
void launch_copy(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
// bytes (rounded up to 16) from page-locked host memory to device memory, read by the GPU
void launch_meta_pull(hipStream_t st, const void *src, void *dst, size_t bytes);
// progressive JPEG (dg_prog.hip): zero coefficients (kProgZeroBytes per
// workgroup), then one wave per work item (a scan, or a chain of scans linked
// by ProgScan::next): pipelined launches with pflags (progress words, zeroed,
// 1 + scans; dg_types.h ProgScan) and ticket (a zeroed counter handing out the
// items in list order), or one level per launch with both null.  ntab: Huffman
// tables in LDS (1: AC scans only; 4: any scan).  ptime (debug, may be null):
// {start, end} s_memrealtime per scan.  serial bit 0: serial bit reader for
// every scan; bit 1 (test switch): every scan with unchained dependencies
// times out on its first wait
void launch_prog_zero(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_prog_scan(hipStream_t st, const ImageDesc *imgs, const ProgScan *scans, const WgItem *list, uint32_t n,
                      const HuffTable *pool, uint32_t serial, uint32_t *pflags, uint32_t *ticket, uint64_t *ptime,
                      int ntab);

}  // namespace dg

// PNG (dg_png.hip)
namespace dg {
void launch_png_gather(hipStream_t st, const GatherJob *jobs, const WgItem *list, uint32_t nwg);
// one 64-thread workgroup (one wave) per image
// mode: 0 unchunked streams only, 1 chunked-path fallbacks only, 2 both
void launch_png_inflate(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg, int mode,
                        BatchFlags *flags, uint32_t ncu);
// tasks: (image, pass << 24 | band) in ticket order; flags: ntasks + 1 zeroed words;
// dbg bit 0: band 1 of every plane times out on its first wait (test switch)
void launch_png_unfilter(hipStream_t st, ImageDesc *imgs, const WgItem *tasks, uint32_t ntasks, uint32_t *flags,
                         uint32_t ncu, uint32_t maxbpp, uint32_t dbg,
                         uint32_t units, uint32_t max_per_cu);  // max_per_cu: workers per CU cap (0: LDS-bound)
// 256 pixels per workgroup
void launch_png_expand(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
// alpha program at `point` (0 before call 1, 1 between the calls, 2 after call 2): 256 pixels per workgroup
void launch_alpha(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg, int point);
size_t png_inflate_smem();
// chunk-parallel inflate (see InfChunk): find = one wave per chunk > 0 (list item.image = chunk),
// decode = one lane per chunk, resolve = one 1024-thread workgroup per chunked image
// stage3: Kraft survivors queued before a full header check round (8, 16, 32 or 64)
void launch_inf_find(hipStream_t st, const ImageDesc *imgs, InfChunk *ch, const WgItem *list, uint32_t nwg,
                     uint32_t stage3);
void launch_inf_decode(hipStream_t st, const ImageDesc *imgs, InfChunk *ch, uint32_t nch, uint32_t variant);
void launch_inf_resolve(hipStream_t st, ImageDesc *imgs, const InfChunk *ch, const WgItem *list, uint32_t nwg);
}  // namespace dg

// JPEG re-encode (dg_enc.hip)
namespace dg {
// fdct: 256 MCUs per workgroup; count / write: 256 blocks per workgroup;
// scan / stuff: one 1024-thread workgroup per image
void launch_enc_fdct(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_enc_count(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_enc_scan(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_enc_write(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_enc_stuff(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg);
// PNG re-encode (dg_penc.hip): 4 rows / 256 pieces / 1 image per workgroup
void launch_penc_filter(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_penc_count(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_penc_write(hipStream_t st, const ImageDesc *imgs, const WgItem *list, uint32_t nwg);
void launch_penc_final(hipStream_t st, ImageDesc *imgs, const WgItem *list, uint32_t nwg);
}  // namespace dg
