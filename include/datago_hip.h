/*
 * datago_hip.h — C ABI of the MI355X decode + aspect-ratio-bucket resize stage.
 *
 * Drop-in boundary for datago's CPU hot path.  The Rust workers call these
 * entry points at the places where the reference decodes and transforms a
 * sample (see INTEGRATION.md for the Rust `extern "C"` block):
 *
 *   reference (Rust, /root/reference/src)                   replaced by
 *   -----------------------------------------------------   ---------------------------------
 *   ImageTransformConfig::get_ar_aware_transform             dg_bucket_table_build
 *       image_processing.rs:77-121 (+ build_image_size_list :188-219)
 *   aspect_ratio_to_str            image_processing.rs:130-133   dg_aspect_ratio_to_str / dg_bucket_get
 *   ARAwareTransform::get_closest_aspect_ratio  :222-252      dg_closest_bucket
 *   aspect_ratio_to_size.get(key)  :264, panic :334-336       dg_bucket_find_key (-1 = not found)
 *   ImageReader::with_guessed_format (header sniff)
 *       worker_files.rs:14-16                                dg_probe
 *   image_from_path + image_to_payload
 *       worker_files.rs:8-30, image_processing.rs:341-431    dg_decode_one (sync)
 *   image::load_from_memory + image_to_payload (per member)
 *       worker_wds.rs:45-66, worker_http.rs:64,129-137       dg_submit / dg_wait (batched)
 *   ImagePayload {data, original_*, height, width, channels, bit_depth, is_encoded}
 *       structs.rs:52-71                                     dg_payload_meta (+ caller-owned data buffer)
 *   reference-first AR propagation of a sample
 *       worker_wds.rs:33,68-76, worker_http.rs:126-214       dg_sample_align
 *   ImageError -> sample dropped (worker_files.rs:63-70)     DG_ERR_CORRUPT
 *   panic!/assert! (Cargo.toml:54 panic="abort")             DG_ERR_BAD_BUCKET / DG_ERR_INVALID (never abort)
 *
 * Conventions: every function returns a dg_status (0 = OK) unless stated;
 * plain pointers and sizes only; the caller owns every buffer it passes;
 * dg_last_error() returns a thread-local message for the last failure on the
 * calling thread.  All entry points are reentrant; one dg_ctx may be shared
 * by many host threads (submissions are serialised on its HIP stream).
 */
#ifndef DATAGO_HIP_H
#define DATAGO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DG_ABI_VERSION 3  /* 2: dg_image_config.decode_semantics; 3: dg_wait_ready, progressive on by default */

typedef enum dg_status {
  DG_OK = 0,
  DG_ERR_UNSUPPORTED = 1, /* valid image the GPU path does not decode (arithmetic, 12-bit,
                             CMYK, 16-bit PNG, non-JPEG/PNG...): caller keeps its CPU path */
  DG_ERR_CORRUPT = 2,     /* maps to image::ImageError::Decoding: drop the sample */
  DG_ERR_OOM = 3,         /* device or host allocation failed */
  DG_ERR_BAD_BUCKET = 4,  /* forced aspect-ratio key/index not in the table (the reference panics) */
  DG_ERR_INVALID = 5,     /* invalid argument / config (the reference asserts) */
  DG_ERR_SMALL_BUFFER = 6,/* caller's output buffer is too small; meta holds the size needed */
  DG_ERR_DEVICE = 7,      /* HIP runtime error */
  DG_ERR_NOT_READY = 8    /* dg_poll: batch still running; meta.status of a progressive member
                             dg_wait_ready left running */
} dg_status;

/* Image formats reported by dg_probe. */
enum { DG_FMT_UNKNOWN = 0, DG_FMT_JPEG = 1, DG_FMT_PNG = 2 };

/* Mirrors ImageTransformConfig (image_processing.rs:43-70) + ImageEncoding (:24-30). */
typedef struct dg_image_config {
  int32_t crop_and_resize;      /* required true when an image_config is given */
  uint32_t default_image_size;  /* e.g. 1024 */
  uint32_t downsampling_ratio;  /* e.g. 32 */
  double min_aspect_ratio;      /* e.g. 0.5 */
  double max_aspect_ratio;      /* e.g. 2.0 */
  int32_t pre_encode_images;    /* re-encode on the GPU: JPEG (dg_enc.hip) or PNG (dg_penc.hip) per encode_format */
  int32_t image_to_rgb8;        /* gray -> RGB expansion after resize (:367-372) */
  int32_t encode_format;        /* 0 = PNG, 1 = JPEG (EncodeFormat, :16-22) */
  int32_t jpeg_quality;         /* default 92 (:14) */
  /* JPEG pixel semantics (IDCT, chroma upsampling, YCbCr->RGB, progressive block smoothing):
   * 0 = libjpeg-turbo (pinned bit-exact to PIL; refuses progressive files libjpeg would block-smooth),
   * 1 = zune-jpeg 0.5.12, the reference's own decoder (worker_files.rs:14-16 -> image 0.25.9 ->
   *     zune-jpeg), restated from the crate's published source (unpinned offline).
   * The Rust drop-in sets 1; same as the context option "decode_semantics". */
  int32_t decode_semantics;
} dg_image_config;

/* ------------------------------------------------------------ buckets */

typedef struct dg_bucket_table dg_bucket_table;

/* ImageTransformConfig::get_ar_aware_transform: builds the bucket list, the
 * "%.3f" key -> (w,h) map (last insert wins) and the keys sorted by value. */
dg_status dg_bucket_table_build(uint32_t default_image_size, uint32_t downsampling_ratio,
                                double min_aspect_ratio, double max_aspect_ratio,
                                dg_bucket_table **out);
void dg_bucket_table_free(dg_bucket_table *t);
/* Number of distinct keys (buckets), sorted ascending by aspect ratio. */
int32_t dg_bucket_count(const dg_bucket_table *t);
/* Bucket i: width, height and its "%.3f" key (key buffer >= 16 bytes). */
dg_status dg_bucket_get(const dg_bucket_table *t, int32_t i, uint32_t *w, uint32_t *h, char *key,
                        size_t key_cap);
/* get_closest_aspect_ratio(width, height) -> bucket index (ties go right). */
int32_t dg_closest_bucket(const dg_bucket_table *t, int32_t width, int32_t height);
/* aspect_ratio_to_size lookup by key string; -1 if absent. */
int32_t dg_bucket_find_key(const dg_bucket_table *t, const char *key);
/* aspect_ratio_to_str((w,h)) -> "%.3f" of w/h (buffer >= 32 bytes). */
dg_status dg_aspect_ratio_to_str(uint32_t w, uint32_t h, char *out, size_t cap);

/* ------------------------------------------------------------ probe */

typedef struct dg_probe_info {
  int32_t format;         /* DG_FMT_* */
  uint32_t width, height;
  int32_t components;     /* 1 (L8) or 3 (RGB8) for JPEG */
  int32_t bit_depth;      /* bits per channel (8) */
  int32_t h_samp[4], v_samp[4];
  int32_t progressive, arithmetic, precision, restart_interval;
  int32_t gpu_supported;  /* 1 if dg_submit would decode it on the GPU */
} dg_probe_info;

/* Header-only: lets the caller compute the bucket and size the output before
 * any GPU work.  Returns DG_ERR_CORRUPT for unparseable data. */
dg_status dg_probe(const uint8_t *bytes, size_t len, dg_probe_info *out);

/* ------------------------------------------------------------ context */

typedef struct dg_ctx dg_ctx;

/* device: HIP device ordinal (rank -> device).  cfg may be NULL (no resize:
 * image_config absent -> decode only, like img_tfm = None). */
dg_status dg_ctx_create(int32_t device, const dg_image_config *cfg, dg_ctx **out);
/* Waits for every call on ctx to return, then for its GPU work, and frees it.
 * A process may also exit with contexts alive: an exit hook of the library
 * (registered at the first dg_ctx_create, so it runs before the HIP
 * runtime's own teardown) runs them down when no thread is inside one of
 * their calls; calls made afterwards return DG_ERR_INVALID.
 * DG_NO_EXIT_HOOK=1 disables it. */
void dg_ctx_destroy(dg_ctx *ctx);
const dg_bucket_table *dg_ctx_buckets(const dg_ctx *ctx);

/* Output metadata, mirrors ImagePayload (structs.rs:52-71).  channels and
 * bit_depth are the decoded image's (pre-transform, image_processing.rs:347-351)
 * unless image_to_rgb8 converted it (then 3 / 8). */
typedef struct dg_payload_meta {
  uint32_t original_width, original_height;
  uint32_t width, height;
  int32_t channels;       /* -1 when encoded */
  int32_t bit_depth;
  int32_t is_encoded;
  int32_t status;         /* dg_status of this image */
  int32_t bucket;         /* bucket index used, -1 without transform */
  uint64_t nbytes;        /* bytes written (or needed) in the output buffer */
} dg_payload_meta;

/* Multi-payload alignment of one sample (worker_wds.rs:33,68-76; worker_http.rs:126-152,159-214):
 * the reference payload (the first whose header gives dimensions; the generator
 * sorts it first, generator_wds.rs:154-166) takes the closest bucket (or
 * forced_first >= 0); every later payload is forced to the bucket whose key is
 * aspect_ratio_to_str(reference output size).  Header-only, so all payloads
 * of a sample go to the GPU in one batch.  forced_out[i]: -1 = closest
 * (payloads before the reference, and everything without an image_config),
 * -2 = no such key (the reference panics; dg_submit reports DG_ERR_BAD_BUCKET). */
dg_status dg_sample_align(const dg_bucket_table *t /* dg_ctx_buckets(ctx); NULL = no image_config */,
                          int32_t n, const uint8_t *const *srcs, const size_t *lens, int32_t forced_first,
                          int32_t *forced_out);

/* Bytes needed for image `bytes` (after probe + bucket choice). */
dg_status dg_output_size(dg_ctx *ctx, const uint8_t *bytes, size_t len, int32_t forced_bucket,
                         uint64_t *nbytes);

/* Batched decode + transform from HOST memory to HOST memory (the path the
 * Rust workers take).  forced_bucket[i] = -1 selects the closest bucket
 * (aspect_ratio "" in image_to_payload), otherwise that bucket index is used
 * (the WebDataset / DB alignment of worker_wds.rs:68-76).  forced_bucket may
 * be NULL.  outs[i] must hold out_caps[i] bytes.  Inputs are copied before
 * return; outputs and metas are valid after dg_wait(ticket). */
dg_status dg_submit(dg_ctx *ctx, int32_t n, const uint8_t *const *srcs, const size_t *lens,
                    const int32_t *forced_bucket, uint8_t *const *outs, const uint64_t *out_caps,
                    dg_payload_meta *metas, uint64_t *ticket);
dg_status dg_wait(dg_ctx *ctx, uint64_t ticket);
dg_status dg_poll(dg_ctx *ctx, uint64_t ticket);
/* Progressive JPEGs of a submission (option "prog_split", default on) do not
 * run in its batch: a refinement scan is one serial chain (~0.1-1 s for a
 * large file), so they join a progressive aggregate that runs on slots of its
 * own (launched at "prog_batch" images, after "prog_flush_us", or when a
 * caller blocks on one of them in dg_wait).  dg_wait(ticket) completes every
 * member as before.  dg_wait_ready(ticket) returns once every other member is
 * complete (outputs and metas valid); *pending (may be NULL) = progressive
 * members still running, whose metas read status DG_ERR_NOT_READY (even while
 * their aggregate is already decoding) until they are complete.  *pending == 0
 * means they are: outputs copied, metas published -- by that dg_wait_ready
 * call when the aggregate's kernels are done, or by a later dg_wait(ticket) --
 * so a loader hands its baseline samples on at the baseline pace and the
 * progressive ones when their aggregate is done, polling dg_wait_ready or
 * blocking in dg_wait.  dg_submit's status covers the caller's submission
 * only: an aggregate launch it triggers that fails is reported in the members'
 * metas and by dg_wait on their tickets. */
dg_status dg_wait_ready(dg_ctx *ctx, uint64_t ticket, int32_t *pending);

/* Synchronous single image (image_payload_from_path equivalent).  Calls from
 * concurrent threads are coalesced into shared GPU batches (one 0.3 MP image
 * cannot fill the GPU): a call waits until the batch is full ("coalesce_max"),
 * every concurrent caller is waiting, or "coalesce_us" has passed.  Returns
 * the image's status. */
dg_status dg_decode_one(dg_ctx *ctx, const uint8_t *src, size_t len, int32_t forced_bucket,
                        uint8_t *out, uint64_t out_cap, dg_payload_meta *meta);

/* Device-resident batch: coded bytes already in HBM (d_srcs[i], device
 * pointers); h_srcs[i] is a host copy the header parser reads (only the bytes
 * up to the start of scan are touched).  Outputs are written to device
 * pointers d_outs[i] (capacity out_caps[i]).  Asynchronous on the context's
 * stream; dg_wait(ticket) completes it. */
dg_status dg_submit_device(dg_ctx *ctx, int32_t n, const uint8_t *const *h_srcs,
                           const uint8_t *const *d_srcs, const size_t *lens,
                           const int32_t *forced_bucket, uint8_t *const *d_outs,
                           const uint64_t *out_caps, dg_payload_meta *metas, uint64_t *ticket);

/* Device memory helpers for callers without a GPU runtime of their own. */
dg_status dg_device_alloc(dg_ctx *ctx, size_t bytes, void **dptr);
dg_status dg_device_free(dg_ctx *ctx, void *dptr);
dg_status dg_memcpy_h2d(dg_ctx *ctx, void *dst, const void *src, size_t bytes);
dg_status dg_memcpy_d2h(dg_ctx *ctx, void *dst, const void *src, size_t bytes);
dg_status dg_synchronize(dg_ctx *ctx);

/* Page-lock a caller-owned host range (hipHostRegister) for the host-out path:
 * outputs of dg_submit / dg_decode_one whose buffer lies inside a registered
 * range (or in memory the HIP runtime already pins) are copied by DMA straight
 * from HBM into it -- no pinned staging buffer, no host memcpy, no first-touch
 * page faults.  Meant for a reused output-buffer pool (the Rust glue's payload
 * arena); registering costs about as much as touching the pages once. */
dg_status dg_host_register(dg_ctx *ctx, void *ptr, size_t bytes);
dg_status dg_host_unregister(dg_ctx *ctx, void *ptr);

/* Per-kernel timing of the last completed batch (HIP events on the context's
 * stream).  names[i] points to static strings; returns the number of stages. */
int32_t dg_last_batch_timings(dg_ctx *ctx, const char **names, float *ms, int32_t cap);

/* Tuning knobs:
 *   "sub_bits"    entropy-decoder subsequence size in bits (multiple of 32,
 *                 64..65536; 0 = auto per batch, the default)
 *   "lead_bits"   entropy lead-in before each subsequence (-1 = auto per image)
 *   "small_coded" batches under this many bytes of coded data take "sub_small" (512) bit ranges and
 *                 "lead_small" (1024) bit lead-ins (default 0 = off; measured slower for dg_decode_one)
 *   "v_units"     k_resize_v: 256-unit (4 KiB) strides per workgroup item, 1..8 (default 2)
 *   "lead_big"    the auto lead-in of images with 4- or 6-block MCUs (default 4096; others 2048)
 *   "coalesce_max" dg_decode_one: most images merged into one GPU batch (1 = off; default 64)
 *   "coalesce_us" dg_decode_one: longest wait for other callers (default 500)
 *   "coalesce_inflight" dg_decode_one: coalesced batches in flight (0 = "slots"; default 3)
 *   "wg_timing"   debug: per-workgroup timestamps of the entropy kernels
 *   "timing"      1 = record per-kernel HIP events (dg_last_batch_timings)
 *   "side_stream" 1 = Lanczos tables on a second stream (default 1)
 *   "decode_semantics" 0 / 1: overrides dg_image_config.decode_semantics
 *   "debug_flags" internal switches: bit 0 = direct H-pass kernel only (bisection); bit 16 / 17 =
 *                 force an entropy write-pass mismatch / a resync that never settles; bit 18 / 19 = force
 *                 a PNG unfilter band wait / a progressive scan wait to time out (tests of the per-image
 *                 DG_ERR_UNSUPPORTED those failures return)
 *   "progressive" 1 = decode progressive JPEGs on the GPU (default 1; 0: DG_ERR_UNSUPPORTED, the
 *                 caller's CPU decoder takes them)
 *   "prog_split"  1 = progressive members of a dg_submit run in the progressive aggregate (default 1,
 *                 see dg_wait_ready); 0 = in the submission's own batch
 *   "prog_batch"  progressive aggregate: launched once it holds this many images (default 2048)
 *   "prog_flush_us" ... or once it is this old at a dg_submit / dg_poll / dg_wait_ready (default 20000)
 *   "prog_lanes"  dg_decode_one: progressive files coalesce into batches of their own, this many in
 *                 flight on the progressive slots (0..2, default 1; 0 = mixed into the baseline batches)
 *   "prog_queue"  streams of the progressive slots: 0 plain, 1 high / 2 low priority (default), 3 CU-masked;
 *                 1-3 give them hardware queues of their own (a plain stream may share one with a baseline
 *                 slot, whose kernels then wait behind the refinement chains: 10% mix 4.4 vs 15.8 Gpx/s)
 *   "slot_queue"  streams of the baseline slots: 0 plain, 1 high priority (default), 2 low priority,
 *                 3 CU-masked.  1-3 take hardware queues apart from the process's shared ones, so one slot's
 *                 long kernels (PNG inflate) stop serialising another's: PNG pairs 9.4 -> 11.2 (1) / 12.6 (3)
 *                 Gpx/s, JPEG 95 (0, 1) / 90 (3) Gpx/s
 *   "side_queue"  the baseline slots' side streams (serial PNG mask inflate, progressive DC items): -1 as
 *                 slot_queue, else a slot_queue mode; default 3 (CU-masked over every CU: a queue of its own,
 *                 so a slot's serial mask inflate never holds back another slot's main stream: PNG pairs
 *                 14.5 -> 17.1 Gpx/s, JPEG unchanged).  Main streams are created first, so the slots in use
 *                 start on distinct hardware queues
 *   "prog_chain"  progressive work items: dependency groups costing <= this % of the batch's longest scan
 *                 run back to back in one wave (default 100; 0 = one wave per scan)
 *   "prog_pipe"   1 = all scans of a batch in one pipelined launch (default); 0 = one launch per level
 *   "prog_serial" 1 = serial bit reader for every scan (A/B; scans with restart intervals always use it)
 *   "prog_side"   1 = progressive scans on the slot's side stream (default 0: measured slower)
 *   "multi_lead"  1 = multi-symbol AC steps in k_huff_sync's state-only decodes (default 1)
 *   "write_pair"  k_huff_write: up to this many more AC symbols per step out of one 32-bit peek (0..3,
 *                 default 3)
 *   "sync_pair"   1 = the same in k_huff_sync after a single-symbol step (default 0: measured slower)
 *   "slots"       baseline batches in flight, 1..6 (default 4), each with its own scratch arena, pinned
 *                 staging and streams; progressive batches use two slots of their own
 *   "hb_bands"    band H kernel: 8-row bands per workgroup, 1..64 (default 16)
 *   "entropy_lpt" 1 = dispatch the slowest entropy workgroups first (default 1)
 *   "entropy_prio" 0-3: wave issue priority (s_setprio) of k_huff_sync / k_huff_write over the other
 *                 batches' pixel kernels sharing their SIMDs (default 0)
 *   "entropy_once" 1 = decode-once staging + scatter instead of a second decode (default 0; slower)
 *   "png_chunked" 0 = inflate every PNG with the serial kernel (test switch; default 1)
 *   "inf_chunk"   chunk-parallel inflate: compressed bytes per chunk (power of two, 4096..65536; default 32768)
 *   "inf_stage3"  8, 16, 32 or 64 (default 32): PNG block finder, Kraft survivors queued before each round
 *                 of full header checks
 *   "uf_units"    1 or 2 (default 1): PNG unfilter filter units per lane per diagonal step (1: half the LDS
 *                 per worker, twice the workers per CU: configs[4] 18.5 -> 19.4 Gpx/s, unfilter 17.5 -> 13.7 ms)
 *   "uf_per_cu"   PNG unfilter: persistent workers per CU at most (default 0: as many as the LDS holds)
 *   "inf_decode"  0..28 (not 10): chunk-parallel inflate lookup bits (literal/length, distance) per lane in LDS:
 *                 0 9/7 (80 KiB per wave), 1 8/6, 2 7/6 (24 KiB), 3 7/5 (20 KiB; round 5: configs[4]
 *                 19.1-19.4 -> 20.1-20.3 Gpx/s), 4 6/5, 5 6/4; 6 / 7 = 2 / 1 with
 *                 the next 8 stream words of every lane in registers, refilled wave-wide; 8 / 9 / 11 = 7/6, 6/5,
 *                 8/6 bits with the symbol tables of longer codes in LDS too (64 / 52 / 96 KiB per wave); 12 / 13 =
 *                 8 / 9 with the register buffer; 14 = 0 with it; 15 = 11 with it; 16 = 3 with it;
 *                 17 7/4, 18 8/5, 19 8/4 bits; 20 / 21 / 22 = 17 / 4 / 5 with the register buffer;
 *                 23 / 24 / 25 / 26 / 27 = 16 with a 4 / 12 / 16 / 24 / 32-word buffer; 28 = 20 with 16 words.
 *                 Default 25 (7/5 bits, 16 words: configs[4] 20.5 -> 22.5-22.8 Gpx/s)
 *   "copy_threads" host threads copying a host-out batch's outputs to the caller's buffers (default 8)
 *   "write_split" 1 = k_huff_write decodes each entropy range as two halves split at the sync pass's
 *                 half-way checkpoint (images without restart markers; default); 0 = one lane per range
 *   "meta_pull"   1 = the GPU reads each batch's descriptors and work lists from page-locked staging (default);
 *                 2 = also a host batch's coded inputs; 0 = hipMemcpyAsync for both
 *   "plan_threads" host threads parsing a submission's headers (default 4; 1 = the submitting thread only)
 *   "hv_fused"     1 = fuse the first H and V passes of colour JPEGs where they fit (default 0; slower)
 *   "h_mfma"       1 = band H passes on the matrix cores (k_resize_hm, i8 MFMA; default 0: measured slower); 0 = VALU kernel
 *   "h_planar"     1 = the first H pass of a colour JPEG with up to 16 taps over a planar LDS segment of u16
 *                 pixel pairs (k_resize_hbp; zune fills in packed 16-bit arithmetic; default 1: resize_h1
 *                 1.79 -> 1.60 ms per configs[1] batch); 0 = k_resize_hb for every class.  Same bytes either way
 *   "band_dec"     1 = IDCT + upsampling + colour + the first H pass of a JPEG in one kernel (k_band_dec,
 *                 MFMA convolution; default 0: measured slower); 0 = IDCT to planes + the band H kernel
 *   "dec_strips"   k_band_dec: 16-row strips per workgroup (default 8)
 *   "reset_host_us" clears the host submit phase timers (stats "host_us_*")
 *   "sub_auto"    subsequence size of batches over 64 MiB of coded data when "sub_bits" is 0 (default 8192)
 *   "sparse_coef" 1 = k_huff_write stores, and k_idct_t loads, only the 16-byte zigzag parts of each
 *                 coefficient block up to its last nonzero coefficient (default 1); 0 = whole 128-byte blocks
 *   "max_device_mb" device memory budget of the context in MiB (default 0 = none).  A batch that does
 *                 not fit beside the other slots' buffers takes the highest other slot out of turn (its
 *                 batch finished, its buffers freed): the context settles on fewer batches in flight (stat
 *                 "budget_slots").  A submission whose plan does not fit -- after the retired buffers and
 *                 the other slots' buffers are freed -- is split into sub-batches under the caller's one ticket; an
 *                 image that alone exceeds it comes back DG_ERR_OOM.  Without a budget a failed device
 *                 allocation takes the same path (drain the other slots, then split)
 * Stats: "batches", "coalesced_batches", "coalesced_images", "resync_rounds", "fix_workgroups", "write_mismatch",
 * "unsettled_batches", "sync_iters_max", "sub_bits" (last batch), "hpool", "qpool" (tables pooled now),
 * "pool_flushes" (times the table pools were started over), "png_chunks", "png_serial_fallbacks",
 * "png_small_streams" (PNG streams below two chunks, inflated serially by one wave),
 * "band_dec_images" (images whose first H pass ran in k_band_dec), "prog_items", "prog_chains" (work items / chains
 * of the pipelined progressive launches), "prog_aggregates", "prog_aggregate_images",
 * "meta_bytes" (the last batch's descriptor/list upload), "allocs", "alloc_mb", "alloc_us", "reclaims",
 * "retire_syncs" (device / page-locked buffer growth: count, MiB, wall microseconds; OOM reclaims; device-wide
 * syncs that freed grown-out buffers), "device_mb" / "peak_device_mb" (device memory the context holds now /
 * at most), "budget_slots" (baseline slots in turn under the budget), "budget_splits", "budget_frees",
 * "budget_oom" (sub-batch splits, slot buffers freed, images
 * failed with DG_ERR_OOM under the budget or after a failed allocation), "host_us_<phase>" / "host_cpu_us_<phase>" (wall / thread
 * CPU microseconds in dg_submit* per phase: plan, pools, layout, lists, upload (staging copy), h2d, launch;
 * "host_us_slotwait": waiting for a free slot); -1 if unknown.
 *
 * Entropy-decode self-checks: an image whose write pass disagrees with the sync pass, or every sequential JPEG of
 * a batch whose boundary repair did not settle, is returned DG_ERR_UNSUPPORTED (the caller's CPU decoder takes
 * it), never DG_OK with unverified pixels. */
dg_status dg_ctx_set_option(dg_ctx *ctx, const char *key, int64_t value);
int64_t dg_ctx_get_stat(dg_ctx *ctx, const char *key);

/* ------------------------------------------------------------ WebDataset shards */

/* One tar member: its bytes are tar[data_off, data_off + data_len) (zero-copy);
 * its path is names[name_off, name_off + name_len) (NUL-terminated). */
typedef struct dg_wds_member {
  uint64_t name_off, data_off, data_len;
  uint32_t name_len, pad;
} dg_wds_member;
/* One sample: members[first, first + count), the reference extension first. */
typedef struct dg_wds_sample {
  uint32_t first, count;
} dg_wds_sample;

/* Index a WebDataset shard held in memory (pull_tarballs, generator_wds.rs:56-204):
 * regular-file entries (ustar, GNU long names, pax paths), sample key =
 * Path::file_stem of the path, kept when world_size <= 1 or
 * dg_wds_key_hash(key) % world_size == rank (:133-148), consecutive equal keys
 * grouped, members ending with reference_ext first (:154-166).  Call with
 * NULL/0 capacities to get the counts (DG_ERR_SMALL_BUFFER), then again. */
dg_status dg_wds_index(const uint8_t *tar, size_t len, int32_t rank, int32_t world_size, const char *reference_ext,
                       dg_wds_member *members, int64_t members_cap, int64_t *n_members, char *names,
                       size_t names_cap, size_t *names_len, dg_wds_sample *samples, int64_t samples_cap,
                       int64_t *n_samples);
/* Rust's DefaultHasher (SipHash-1-3, keys 0/0) of a &str: hash_fn (generator_wds.rs:50-54). */
uint64_t dg_wds_key_hash(const char *key, size_t len);

const char *dg_last_error(void);
int32_t dg_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DATAGO_HIP_H */
