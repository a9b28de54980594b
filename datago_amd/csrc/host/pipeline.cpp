// pipeline.cpp — batch planner + runtime for the decode/bucket-resize stage.
//
// Host work per image is header-only (parse + bucket + buffer layout); all
// pixel and coefficient arithmetic runs in kernels.hip.  A batch is laid out
// in one device scratch arena, its descriptors and workgroup lists go up in
// one H2D copy, and every kernel of the batch is launched on the context's
// stream back to back.  The reference equivalent is one tokio task per sample
// (worker_files.rs:32-72 -> image_processing.rs:341-431).
#include "pipeline.h"

#include <string.h>

#include <algorithm>
#include <time.h>
#include <atomic>
#include <chrono>
#include <cmath>
#include <thread>

#include "../dg_entropy.h"
#include "../dg_pixel.h"
#include "../kernels.h"

namespace dg {

thread_local std::string g_last_error;
void set_error(const std::string &s) { g_last_error = s; }

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      set_error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x);          \
      return DG_ERR_DEVICE;                                                                \
    }                                                                                      \
  } while (0)

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static double thread_cpu_us() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (double)ts.tv_sec * 1e6 + (double)ts.tv_nsec * 1e-3;
}

// Boundary-repair rounds (finish()) before a batch is declared unsettled.
static constexpr int kMaxResyncRounds = 64;
// submit(): the batch does not fit the device (budget or allocation); the
// caller splits it (submit_split).  Never returned through the C ABI.
static constexpr dg_status kNeedSplit = (dg_status)15;  // (inside the enum's value range)

// 64-row unfilter bands of pass p of a PNG (the image itself when not
// interlaced); k_png_unfilter numbers its progress flags the same way.
static uint32_t png_pass_bands(const ImageDesc &d, uint32_t p) {
  if (!d.png.interlace) return p == 0 ? (d.height + 63) / 64 : 0u;
  uint32_t pw, ph;
  png_adam7_pass(d.width, d.height, p, pw, ph);
  return pw && ph ? (ph + 63) / 64 : 0u;
}
static uint32_t png_bands(const ImageDesc &d) {
  uint32_t n = 0;
  for (uint32_t p = 0; p < 7; p++) n += png_pass_bands(d, p);
  return n;
}

// Host-side copies of a finished batch's outputs (pinned staging -> the
// caller's buffers, ~3 MB per 1024-bucket image): split into 1 MiB pieces
// and spread over up to `nthreads` threads -- one thread's memcpy (~6-8 GB/s)
// was the limit of the host-in/host-out path, not PCIe.
struct CopyJob {
  void *dst;
  const void *src;
  size_t n;
};
static void parallel_copy(const std::vector<CopyJob> &jobs, int nthreads) {
  constexpr size_t kPiece = 1 << 20;
  std::vector<CopyJob> pieces;
  size_t total = 0;
  for (const CopyJob &j : jobs) {
    for (size_t o = 0; o < j.n; o += kPiece)
      pieces.push_back({(char *)j.dst + o, (const char *)j.src + o, std::min(kPiece, j.n - o)});
    total += j.n;
  }
  const int nt = (int)std::min<size_t>((size_t)std::max(1, nthreads), std::max<size_t>(1, total / (4 * kPiece)));
  if (nt <= 1) {
    for (const CopyJob &p : pieces) memcpy(p.dst, p.src, p.n);
    return;
  }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < pieces.size();) memcpy(pieces[k].dst, pieces[k].src, pieces[k].n);
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < nt; t++) ts.emplace_back(work);
  work();
  for (std::thread &t : ts) t.join();
}

static const char *kStageNames[] = {"upload",     "png_inflate", "png_unfilter", "destuff",   "prog_scans",
                                    "huff_sync",  "huff_fix",    "huff_scan",    "huff_write", "coeffs",
                                    "idct",       "color",       "resize_h1",    "resize_v1", "resize_h2",
                                    "resize_v2",  "copy",        "encode",       "download"};
static const int kNumStages = 19;

Context::Context(int device, const dg_image_config *cfg) : device_(device) {
  if (cfg && cfg->crop_and_resize) {
    has_cfg_ = true;
    cfg_ = *cfg;
  } else if (cfg) {
    cfg_ = *cfg;
  }
  if (cfg) decode_sem_ = cfg->decode_semantics == 1 ? 1 : 0;
}

Context::~Context() {
  plan_pool_.reset();  // join the planning workers before any HIP object goes
  hipSetDevice(device_);
  sync_all();
  for (int g = 0; g < kPoolGens; g++)
    for (DevBuf *b : {&d_hpool_[g], &d_qpool_[g]})
      if (b->p) hipFree(b->p);
  free_retired();
  for (Slot &sl : slots_) {
    for (auto e : sl.ev) hipEventDestroy(e);
    if (sl.done) hipEventDestroy(sl.done);
    for (hipEvent_t e : {sl.ev_meta, sl.ev_coef, sl.ev_zero, sl.ev_prog, sl.ev_png0, sl.ev_png1})
      if (e) hipEventDestroy(e);
    if (sl.coef.p && !sl.views) hipFree(sl.coef.p);
    for (hipStream_t q : {sl.st, sl.side})
      if (q) hipStreamDestroy(q);
    if (sl.wgt.p) hipFree(sl.wgt.p);
    for (DevBuf *b : {&sl.scratch, &sl.meta, &sl.input})
      if (b->p && (b == &sl.meta || !sl.views)) hipFree(b->p);
    if (sl.arena.p) hipFree(sl.arena.p);
    for (PinBuf *b : {&sl.stage, &sl.out})
      if (b->p) hipHostFree(b->p);
  }
  if (side_) hipStreamSynchronize(side_);
  if (ev_meta_) hipEventDestroy(ev_meta_);
  if (ev_coef_) hipEventDestroy(ev_coef_);
  if (side_) hipStreamDestroy(side_);
  if (stream_) hipStreamDestroy(stream_);
}

dg_status Context::init() {
  if (has_cfg_) {
    // ImageTransformConfig::get_ar_aware_transform asserts (image_processing.rs:78-93)
    if (cfg_.default_image_size == 0 || cfg_.downsampling_ratio == 0 || !(cfg_.min_aspect_ratio > 0.0) ||
        !(cfg_.max_aspect_ratio >= cfg_.min_aspect_ratio)) {
      set_error("invalid image_config (default_image_size/downsampling_ratio/aspect ratios)");
      return DG_ERR_INVALID;
    }
    buckets_.reset(new BucketTable(cfg_.default_image_size, cfg_.downsampling_ratio, cfg_.min_aspect_ratio,
                                   cfg_.max_aspect_ratio));
    if (buckets_->buckets().empty()) {
      set_error("empty bucket table");
      return DG_ERR_INVALID;
    }
  }
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device_ < 0 || device_ >= ndev) {
    set_error("device ordinal out of range");
    return DG_ERR_INVALID;
  }
  HIPCHK(hipSetDevice(device_));
  {
    int ncu = 0;
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device_));
    if (ncu > 0) ncu_ = (uint32_t)ncu;
  }
  HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&ev_meta_, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&ev_coef_, hipEventDisableTiming));
  for (Slot &sl : slots_) {
    sl.ev.resize(kNumStages + 1);
    for (auto &e : sl.ev) HIPCHK(hipEventCreate(&e));
    HIPCHK(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));

    HIPCHK(hipEventCreateWithFlags(&sl.ev_meta, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_coef, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_zero, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_prog, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_png0, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&sl.ev_png1, hipEventDisableTiming));
  }
  return make_streams(0, kMaxInflight, slot_queue_, 0, side_queue_);  // the progressive slots' on first use
}

// Streams of the progressive slots (option "prog_queue").  A progressive
// batch holds its stream for ~0.1-1 s; HIP maps streams onto the process's
// few hardware queues (GPU_MAX_HW_QUEUES, 4), and kernels behind it in the
// same queue wait for it -- a baseline slot's stream sharing that queue then
// stalls behind the refinement chains.  0: plain streams; 1 / 2: highest /
// lowest priority; 3: a CU mask over every CU (a masked stream gets a
// hardware queue of its own).
dg_status Context::make_prog_streams() {
  return make_streams(kMaxInflight, kProgSlots, prog_queue_, prog_cus_, -1);
}

// A slot's streams on first use: the baseline slots past "slots" and the
// progressive slots have none until a batch goes to them -- every stream
// with a queue of its own is a hardware queue, and eight processes sharing
// one device run out of them (each rank would hold 16).
dg_status Context::slot_streams(Slot &sl) {
  if (sl.st) return DG_OK;
  const int j = (int)(&sl - slots_);
  return j < kMaxInflight ? make_streams(j, 1, slot_queue_, 0, side_queue_)
                          : make_streams(j, 1, prog_queue_, prog_cus_, -1, kAllSlots);
}

// (Re)create the main and side streams of slots [first, first + count):
// mode 0 plain, 1 / 2 highest / lowest priority, 3 a CU mask over `cus` CUs
// (0 = all).  Modes 1-3 get hardware queues of their own.  HIP hands a new
// stream the least-used queue of its pool, so the main streams are made
// first: the slots in use then start on distinct queues, and a side stream
// (side_mode, -1 = mode) shares a queue with at most one other slot's stream.
// Only slots below `limit` (-1: "slots") get streams now; the others on
// first use (slot_streams).
dg_status Context::make_streams(int first, int count, int mode, int cus, int side_mode, int limit) {
  if (limit < 0) limit = nslots_;
  HIPCHK(hipSetDevice(device_));
  int least = 0, greatest = 0;
  HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  for (int j = first; j < first + count; j++) {
    Slot &sl = slots_[j];
    for (hipStream_t *q : {&sl.st, &sl.side}) {
      if (*q) {
        HIPCHK(hipStreamSynchronize(*q));
        HIPCHK(hipStreamDestroy(*q));
        *q = nullptr;
      }
    }
  }
  for (int pass = 0; pass < 2; pass++) {
    const int m = pass == 1 && side_mode >= 0 ? side_mode : mode;
    for (int j = first; j < first + count && (j < limit || count == 1); j++) {
      hipStream_t *q = pass == 0 ? &slots_[j].st : &slots_[j].side;
      if (m == 1 || m == 2) {
        HIPCHK(hipStreamCreateWithPriority(q, hipStreamNonBlocking, m == 1 ? greatest : least));
      } else if (m == 3) {  // cus of the CUs, spread evenly (every ncu/cus-th)
        std::vector<uint32_t> mask((ncu_ + 31) / 32, 0u);
        const uint32_t want = cus > 0 && (uint32_t)cus < ncu_ ? (uint32_t)cus : ncu_;
        for (uint32_t k = 0; k < want; k++) {
          const uint32_t cu = (uint32_t)(((uint64_t)k * ncu_) / want);
          mask[cu / 32] |= 1u << (cu % 32);
        }
        HIPCHK(hipExtStreamCreateWithCUMask(q, (uint32_t)mask.size(), mask.data()));
      } else {
        HIPCHK(hipStreamCreateWithFlags(q, hipStreamNonBlocking));
      }
    }
  }
  return DG_OK;
}

dg_status Context::host_register(void *ptr, size_t bytes) {
  HIPCHK(hipSetDevice(device_));
  if (hipHostRegister(ptr, bytes, hipHostRegisterDefault) != hipSuccess) {
    set_error("hipHostRegister failed");
    return DG_ERR_DEVICE;
  }
  std::lock_guard<std::mutex> lk(reg_mu_);
  registered_.push_back({(uintptr_t)ptr, bytes});
  return DG_OK;
}

dg_status Context::host_unregister(void *ptr) {
  {
    std::lock_guard<std::mutex> lk(reg_mu_);
    for (size_t i = 0; i < registered_.size(); i++)
      if (registered_[i].first == (uintptr_t)ptr) {
        registered_.erase(registered_.begin() + (long)i);
        break;
      }
  }
  sync_all();  // no copy into the range may still be in flight
  HIPCHK(hipSetDevice(device_));
  return hipHostUnregister(ptr) == hipSuccess ? DG_OK : DG_ERR_INVALID;
}

bool Context::host_pinned(const void *ptr, size_t bytes) {
  const uintptr_t a = (uintptr_t)ptr;
  {
    std::lock_guard<std::mutex> lk(reg_mu_);
    for (const auto &r : registered_)
      if (a >= r.first && a + bytes <= r.first + r.second) return true;
  }
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, ptr) != hipSuccess) {
    (void)hipGetLastError();  // plain pageable memory: not an error
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

dg_status Context::sync_all() {
  bool ok = true;
  for (hipStream_t q : {stream_, side_})
    if (q) ok &= hipStreamSynchronize(q) == hipSuccess;
  for (Slot &sl : slots_)
    for (hipStream_t q : {sl.st, sl.side})
      if (q) ok &= hipStreamSynchronize(q) == hipSuccess;
  if (!ok) {
    set_error("HIP stream synchronisation failed");
    return DG_ERR_DEVICE;
  }
  return DG_OK;
}

// H pass kernel choice.  The band kernel stages the source pixels of
// kHBandCols consecutive outputs in LDS: at most 255 * scale + 2 * support
// (+ window rounding, 8-pixel alignment and ksize slack) pixels, which must
// fit kHSegPx.  Wider segments (extreme downscales) use the direct kernel;
// the first pass of a colour JPEG in the band kernel upsamples and converts
// colour in its fill.
static double h_pass_span(const ResizePass &ps) {
  const double scale = (ps.in1 - ps.in0) / (double)ps.out_size;
  const double fs = scale > 1.0 ? scale : 1.0;
  return std::ceil((kHBandCols - 1) * scale + 6.0 * fs) + 2.0 + 8.0 + (double)ps.ksize + 8.0;
}
static uint32_t h_pass_mode(const ResizePass &ps, bool colour_source) {
  if (h_pass_span(ps) > (double)kHSegPx) return kHDirect;
  return colour_source ? kHFused : 0u;
}
// k_resize_hv takes the first H and V passes of a colour JPEG together when
// its smaller segment and ring fit them and the H taps are in the <= 16 class
static bool hv_fusable(const ResizePass &h, const ResizePass &v) {
  return h.kind == 1 && (h.mode & kHFused) && !(h.mode & kHDirect) && v.kind == 2 && h.C == 3 && h.row0 == 0 &&
         v.row0 == 0 &&
         h.ksize + 1 <= 16 && v.ksize <= kHVTapsMax && h_pass_span(h) <= (double)kHVSegPx;
}

// k_band_dec takes pass[0] of a JPEG when its sampling is one the fused fill
// knows (gray; 4:4:4, 4:2:2, 4:2:0 with luma at the maximum factors) and its
// segments fit: the 128-column tile's source segment (plus the 16-pixel
// alignment) in the class's LDS, every 16-column MFMA subtile's window in the
// class's K steps (320-pixel class: one 64-wide step, downscales up to ~2x;
// 640-pixel class: two).  Returns the mode bits (0: not eligible).
static uint32_t band_dec_mode(const ImageDesc &d, const ResizePass &ps) {
  if (ps.kind != 1 || (ps.mode & (kHDirect | kHVFused)) || d.idct_fused) return 0;
  if (d.ncomp == 3) {
    if (!(ps.mode & kHFused)) return 0;
    if (d.ch[0] != d.hmax || d.cv[0] != d.vmax || d.ch[1] != d.ch[2] || d.cv[1] != d.cv[2]) return 0;
    if (d.hmax % d.ch[1] || d.vmax % d.cv[1]) return 0;
    const uint32_t hr = d.hmax / d.ch[1], vr = d.vmax / d.cv[1];
    if (hr > 2 || vr > 2 || (hr == 1 && vr == 2)) return 0;
  } else if (d.ncomp != 1) {
    return 0;
  }
  const double scale = (ps.in1 - ps.in0) / (double)ps.out_size;
  const double window = 15.0 + std::ceil(15.0 * scale) + (double)ps.ksize + 2.0;  // a subtile's K range
  const double span = h_pass_span(ps) + 16.0;
  if (span <= (double)kDecSeg0 && window <= 64.0) return kHDecode;  // one K step
  if (span <= (double)kDecSeg1 && window <= 128.0) return kHDecode | kHDecWide;
  return 0;
}

// k_resize_hm takes a band H pass when every 16-column subtile's window fits
// one or two 64-wide K steps and the 16-aligned segment fits kHSegPx: returns
// the K steps (0: the VALU band kernel runs it).
static uint32_t h_mfma_steps(const ResizePass &ps) {
  if (ps.kind != 1 || (ps.mode & (kHDirect | kHVFused | kHDecode)) || ps.C < 1 || ps.C > 4) return 0;
  if (h_pass_span(ps) + 8.0 > (double)kHSegPx) return 0;
  const double scale = (ps.in1 - ps.in0) / (double)ps.out_size;
  const double window = 15.0 + std::ceil(15.0 * scale) + (double)ps.ksize + 2.0;
  return window <= 64.0 ? 1u : (window <= 128.0 ? 2u : 0u);
}

// A rejected option names itself, the value and the accepted range in
// dg_last_error (the range as the condition that rejects it).
static dg_status opt_error(const std::string &k, int64_t v, const std::string &why) {
  set_error("dg_ctx_set_option(\"" + k + "\", " + std::to_string(v) + "): " + why);
  return DG_ERR_INVALID;
}

dg_status Context::set_option(const std::string &k, int64_t v) {
  if (k == "sub_bits") {
    if (v != 0 && (v < 64 || v > 65536 || (v & (v - 1)))) return opt_error(k, v, "valid unless v != 0 && (v < 64 || v > 65536 || (v & (v - 1)))");  // power of two
    sub_bits_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "sub_auto") {
    if (v < 1024 || v > 65536 || (v & (v - 1))) return opt_error(k, v, "valid unless v < 1024 || v > 65536 || (v & (v - 1))");
    sub_auto_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "lead_bits") {
    if (v < -1 || v > (1 << 20)) return opt_error(k, v, "valid unless v < -1 || v > (1 << 20)");
    lead_bits_ = v;
    return DG_OK;
  }
  if (k == "coalesce_max") {
    if (v < 1 || v > 4096) return opt_error(k, v, "valid unless v < 1 || v > 4096");
    std::lock_guard<std::mutex> lk(cmu_);
    coalesce_max_ = (int)v;
    return DG_OK;
  }
  if (k == "coalesce_inflight") {  // dg_decode_one: coalesced baseline batches in flight (0 = "slots")
    if (v < 0 || v > kMaxInflight) return opt_error(k, v, "valid unless v < 0 || v > " + std::to_string(kMaxInflight));
    std::lock_guard<std::mutex> lk(cmu_);
    coalesce_inflight_ = (int)v;
    return DG_OK;
  }
  if (k == "coalesce_us") {
    if (v < 0 || v > 1000000) return opt_error(k, v, "valid unless v < 0 || v > 1000000");
    std::lock_guard<std::mutex> lk(cmu_);
    coalesce_us_ = (int)v;
    return DG_OK;
  }
  if (k == "wg_timing") {
    wg_timing_ = v != 0;
    return DG_OK;
  }
  if (k == "timing") {
    timing_ = v != 0;
    return DG_OK;
  }
  if (k == "side_stream") {
    side_stream_ = v != 0;
    return DG_OK;
  }
  if (k == "coef_cache_mb") {  // Lanczos table cache arena (0: off); takes effect at the next reset
    if (v < 0 || v > 65536) return opt_error(k, v, "valid unless v < 0 || v > 65536");
    std::lock_guard<std::mutex> lk(mu_);
    for (const Slot &o : slots_)
      if (o.batch && !o.batch->done && o.batch->uses_ccache) return opt_error(k, v, "not while a batch in flight uses the table cache");  // not while tables are in use
    ccache_cap_ = (size_t)v << 20;
    ccache_index_clear();
    ccache_.clear();
    ccache_off_ = 0;
    ccache_full_ = false;
    if (d_ccache_.p) hipFree(d_ccache_.p);
    d_ccache_.p = nullptr;
    d_ccache_.cap = 0;
    return DG_OK;
  }
  if (k == "entropy_prio") {  // wave issue priority (s_setprio) of the entropy kernels, 0-3
    if (v < 0 || v > 3) return opt_error(k, v, "valid unless v < 0 || v > 3");
    entropy_prio_ = (int)v;
    return DG_OK;
  }
  if (k == "max_device_mb") {  // device memory budget of the context (0: none)
    if (v < 0) return opt_error(k, v, "valid unless v < 0");
    max_dev_bytes_ = (size_t)v << 20;
    budget_slots_ = kMaxInflight;
    budget_planned_ = false;
    // Contexts under a budget are the ones that share a device (several
    // ranks, or a loader beside training): their slot streams share the
    // process's hardware queues instead of taking two of their own each --
    // 8 ranks x 4 slots x 2 own queues oversubscribed the device's queues
    // (profiles/r05/ranks: 6-9 Gpx/s at 4 slots, 104 at 2).  An explicit
    // slot_queue / side_queue wins.
    if (v > 0 && !queue_set_ && (slot_queue_ != 0 || side_queue_ != -1)) {
      std::lock_guard<std::mutex> lk(mu_);
      for (int j = 0; j < kMaxInflight; j++) {
        Slot &sl = slots_[j];
        if (sl.batch && !sl.batch->done) {
          dg_status st = finish(sl);
          if (st) return st;
        }
      }
      slot_queue_ = 0;
      side_queue_ = -1;
      bool any = false;
      for (int j = 0; j < kMaxInflight; j++) any = any || slots_[j].st;
      if (any) return make_streams(0, kMaxInflight, slot_queue_, 0, side_queue_);
    }
    return DG_OK;
  }
  if (k == "budget_plan") {  // 1: the first batch under a budget sizes every slot (no growth later); 0: grow and trade
    budget_plan_ = v != 0;
    budget_planned_ = false;
    return DG_OK;
  }
  if (k == "slots") {
    if (v < 1 || v > (int64_t)kMaxInflight) return opt_error(k, v, "valid unless v < 1 || v > " + std::to_string(kMaxInflight));
    nslots_ = (int)v;
    next_slot_ %= nslots_;
    return DG_OK;
  }
  if (k == "progressive") {
    // Progressive JPEGs on the GPU (dg_prog.hip; default on).  A refinement
    // scan decodes serially in one wave, so a large file takes ~0.1-1 s: the
    // progressive members of a submission run apart from the rest (prog_split)
    // in aggregate batches on slots of their own.  0: DG_ERR_UNSUPPORTED (the
    // caller's CPU decoder takes them).
    progressive_ = v != 0;
    return DG_OK;
  }
  if (k == "prog_lanes") {  // dg_decode_one: progressive batches in flight on the progressive slots; 0: mixed in
    if (v < 0 || v > kProgSlots) return opt_error(k, v, "valid unless v < 0 || v > " + std::to_string(kProgSlots));
    prog_lanes_ = (int)v;
    return DG_OK;
  }
  if (k == "prog_queue") {  // progressive slots' streams: 0 plain, 1 high / 2 low priority, 3 CU-masked
    if (v < 0 || v > 3) return opt_error(k, v, "valid unless v < 0 || v > 3");
    {
      std::lock_guard<std::mutex> lk(pmu_);
      if (!pagg_.empty()) flush_pagg_locked();
    }
    std::lock_guard<std::mutex> lk(mu_);
    for (int j = 0; j < kProgSlots; j++) {
      Slot &sl = slots_[kMaxInflight + j];
      if (sl.batch && !sl.batch->done) {
        dg_status st = finish(sl);
        if (st) return st;
      }
    }
    prog_queue_ = (int)v;
    return make_prog_streams();
  }
  if (k == "slot_queue") {  // baseline slots' streams: 0 plain, 1 high / 2 low priority, 3 CU-masked (own queues)
    if (v < 0 || v > 3) return opt_error(k, v, "valid unless v < 0 || v > 3");
    queue_set_ = true;
    std::lock_guard<std::mutex> lk(mu_);
    for (int j = 0; j < kMaxInflight; j++) {
      Slot &sl = slots_[j];
      if (sl.batch && !sl.batch->done) {
        dg_status st = finish(sl);
        if (st) return st;
      }
    }
    slot_queue_ = (int)v;
    return make_streams(0, kMaxInflight, slot_queue_, 0, side_queue_);
  }
  if (k == "side_queue") {  // the baseline slots' side streams: -1 as slot_queue, else a slot_queue mode
    if (v < -1 || v > 3) return opt_error(k, v, "valid unless v < -1 || v > 3");
    queue_set_ = true;
    std::lock_guard<std::mutex> lk(mu_);
    for (int j = 0; j < kMaxInflight; j++) {
      Slot &sl = slots_[j];
      if (sl.batch && !sl.batch->done) {
        dg_status st = finish(sl);
        if (st) return st;
      }
    }
    side_queue_ = (int)v;
    return make_streams(0, kMaxInflight, slot_queue_, 0, side_queue_);
  }
  if (k == "prog_cus") {  // prog_queue 3: CUs the progressive streams may use (0 = all); set before prog_queue
    if (v < 0 || v > 4096) return opt_error(k, v, "valid unless v < 0 || v > 4096");
    prog_cus_ = (int)v;
    return DG_OK;
  }
  if (k == "prog_split") {  // dg_submit: progressive members into the progressive aggregate (0: decoded in the batch)
    prog_split_ = v != 0;
    return DG_OK;
  }
  if (k == "prog_batch") {  // progressive aggregate: launched once it holds this many images
    if (v < 1 || v > 65536) return opt_error(k, v, "valid unless v < 1 || v > 65536");
    prog_batch_ = (int)v;
    return DG_OK;
  }
  if (k == "prog_flush_us") {  // ... or once it is this old at a submit / poll / wait_ready
    if (v < 0 || v > 100000000) return opt_error(k, v, "valid unless v < 0 || v > 100000000");
    prog_flush_us_ = (int)v;
    return DG_OK;
  }
  if (k == "sync2") {  // k_huff_sync2: two lead-in + range chains per lane (0: one, k_huff_sync)
    sync2_ = v != 0;
    return DG_OK;
  }
  if (k == "sync_pair") {  // k_huff_sync: a second AC symbol per single step from the same peek (A/B)
    sync_pair_ = v != 0;
    return DG_OK;
  }
  if (k == "write_pair") {  // k_huff_write: up to v more AC symbols per step from the same peek (0..3)
    if (v < 0 || v > 3) return opt_error(k, v, "valid unless v < 0 || v > 3");
    write_pair_ = (int)v;
    return DG_OK;
  }
  if (k == "multi_lead") {  // multi-symbol AC steps in k_huff_sync's lead-in (A/B)
    multi_lead_ = v != 0;
    return DG_OK;
  }
  if (k == "prog_side") {  // progressive scans on the side stream, beside the baseline entropy decode
    prog_side_ = v != 0;
    return DG_OK;
  }
  if (k == "prog_chain") {  // chain dependency groups costing <= this % of the batch's longest scan (0: off)
    if (v < 0 || v > 100000) return opt_error(k, v, "valid unless v < 0 || v > 100000");
    prog_chain_ = (int)v;
    return DG_OK;
  }
  if (k == "prog_pipe") {  // 0: one k_prog_scan launch per level (A/B)
    prog_pipe_ = v != 0;
    return DG_OK;
  }
  if (k == "prog_serial") {  // every progressive scan on the serial reader (A/B; restart scans always are)
    prog_serial_ = v != 0;
    return DG_OK;
  }
  if (k == "entropy_once") {  // decode-once: k_huff_sync stages coefficients, k_huff_scatter writes them
    entropy_once_ = v != 0;
    return DG_OK;
  }
  if (k == "entropy_lpt") {
    entropy_lpt_ = v != 0;
    return DG_OK;
  }
  if (k == "hb_bands") {  // band H kernel: 8-row bands per workgroup
    if (v < 1 || v > 64) return opt_error(k, v, "valid unless v < 1 || v > 64");
    hb_bands_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "idct_fused") {  // IDCT inside k_huff_write's block flush (default 0: measured slower)
    idct_fused_ = v != 0;
    return DG_OK;
  }
  if (k == "idct_thread") {
    idct_thread_ = v != 0;
    return DG_OK;
  }
  if (k == "sparse_coef") {
    sparse_coef_ = v != 0;
    return DG_OK;
  }
  if (k == "h_prefetch") {
    h_prefetch_ = v != 0;
    return DG_OK;
  }
  if (k == "h_planar") {
    h_planar_ = v != 0;
    return DG_OK;
  }
  if (k == "destuff_one") {
    destuff_one_ = v != 0;
    return DG_OK;
  }
  if (k == "chroma_rec") {
    chroma_rec_ = v != 0;
    return DG_OK;
  }
  if (k == "reset_host_us") {  // zero the host_us_* / host_cpu_us_* stats
    for (double &x : host_us_) x = 0;
    for (double &x : host_cpu_us_) x = 0;
    return DG_OK;
  }
  if (k == "hv_fused") {  // fused first H + V pass of colour JPEGs where it fits (default 0: slower)
    hv_fused_ = v != 0;
    return DG_OK;
  }
  if (k == "copy_threads") {  // host threads for the output copies of a host-out batch (default 8)
    if (v < 1 || v > 64) return opt_error(k, v, "valid unless v < 1 || v > 64");
    copy_threads_ = (int)v;
    return DG_OK;
  }
  if (k == "ckpt") {  // entropy checkpoints for early merging of re-decodes (default 1)
    ckpt_ = v != 0;
    return DG_OK;
  }
  if (k == "decode_semantics") {  // 0: libjpeg-turbo (pinned), 1: zune-jpeg 0.5.12 restated (unpinned)
    if (v != 0 && v != 1) return opt_error(k, v, "valid unless v != 0 && v != 1");
    decode_sem_ = (int)v;
    return DG_OK;
  }
  if (k == "small_coded") {  // batches under this many coded bytes take sub_small / lead_small (0 = off)
    if (v < 0) return opt_error(k, v, "valid unless v < 0");
    small_coded_ = (uint64_t)v;
    return DG_OK;
  }
  if (k == "sub_small") {
    if (v < 64 || v > 65536 || (v & (v - 1))) return opt_error(k, v, "valid unless v < 64 || v > 65536 || (v & (v - 1))");
    sub_small_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "lead_small") {
    if (v < 0 || v > (1 << 16)) return opt_error(k, v, "valid unless v < 0 || v > (1 << 16)");
    lead_small_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "v_tile") {  // V pass output rows per column tile (k_resize_vt); 0: one thread per 16 output bytes
    if (v != 0 && v != 2 && v != 4 && v != 8) return opt_error(k, v, "valid: 0, 2, 4, 8");
    v_tile_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "v_units") {  // k_resize_v: 256-unit strides per workgroup item
    if (v < 1 || v > 8) return opt_error(k, v, "valid unless v < 1 || v > 8");
    v_units_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "lead_big") {  // auto lead-in of images with >= 4-block MCUs (4:2:0), bits
    if (v < 0 || v > (1 << 16)) return opt_error(k, v, "valid unless v < 0 || v > (1 << 16)");
    lead_big_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "write_split") {  // 1: k_huff_write decodes each range as two halves (see k_huff_write)
    write_split_ = v != 0;
    return DG_OK;
  }
  if (k == "meta_pull") {  // the GPU reads from page-locked staging: 1 the descriptors, 2 also host inputs
    if (v < 0 || v > 2) return opt_error(k, v, "valid unless v < 0 || v > 2");
    meta_pull_ = (int)v;
    return DG_OK;
  }
  if (k == "plan_threads") {  // host threads parsing a submission's headers (1 = the caller only)
    if (v < 1 || v > 64) return opt_error(k, v, "valid unless v < 1 || v > 64");
    plan_threads_ = (int)v;
    return DG_OK;
  }
  if (k == "inf_stage3") {  // k_inf_find: Kraft survivors queued per full header check round
    if (v != 8 && v != 16 && v != 32 && v != 64) return opt_error(k, v, "valid unless v != 8 && v != 16 && v != 32 && v != 64");
    inf_stage3_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "inf_cap") {  // chunk-parallel inflate: entries per chunk, in tenths of the image's expansion of a span
    if (v < 10 || v > 100) return opt_error(k, v, "valid unless v < 10 || v > 100");
    inf_cap_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "png_alias") {  // PNG chunk entries share device memory with the later stages' buffers
    png_alias_ = v != 0;
    return DG_OK;
  }
  if (k == "inf_pad") {  // chunk-parallel inflate: entries per chunk on top of inf_cap's
    if (v < 0 || v > (1 << 20)) return opt_error(k, v, "valid unless v < 0 || v > 2^20");
    inf_pad_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "inf_chunk") {  // compressed bytes per chunk of the chunk-parallel inflate
    if (v < 4096 || v > 65536 || (v & (v - 1))) return opt_error(k, v, "valid unless v < 4096 || v > 65536 || (v & (v - 1))");
    inf_chunk_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "png_chunked") {  // 0: every PNG inflates serially (test switch)
    chunked_off_ = v == 0;
    return DG_OK;
  }
  if (k == "lead_density") {
    lead_density_ = v != 0;
    return DG_OK;
  }
  if (k == "sub_density") {  // bits-per-block threshold for shorter subsequences (0 = off)
    if (v < 0 || v > 4096) return opt_error(k, v, "valid unless v < 0 || v > 4096");
    sub_density_ = (double)v;
    return DG_OK;
  }
  if (k == "uf_per_cu") {  // PNG unfilter: persistent workers per CU at most (0: as many as the LDS holds)
    if (v < 0 || v > 16) return opt_error(k, v, "valid unless v < 0 || v > 16");
    uf_per_cu_ = (int)v;
    return DG_OK;
  }
  if (k == "uf_units") {  // PNG unfilter: filter units per lane per step (1: half the LDS per worker)
    if (v < 1 || v > 2) return opt_error(k, v, "valid unless v < 1 || v > 2");
    uf_units_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "inf_decode") {  // k_inf_decode lookup bits (literal/length, distance): 0 9/7, 1 8/6, 2 7/6, 3 7/5, 4 6/5,
                            // 5 6/4; 6, 7 = 2, 1 with the wave-batched register stream buffer; 8 / 9 / 11 =
                            // 7/6, 6/5, 8/6 with the canonical walk's symbol tables in LDS; 12 / 13 = 8 / 9
                            // with the register buffer; 14 = 0 with it, 15 = 11 with it; 16 = 3 with it;
                            // 17 7/4, 18 8/5, 19 8/4; 20 / 21 / 22 = 17 / 4 / 5 with the register buffer;
                            // 23 / 24 / 25 / 26 / 27 = 16 with a 4 / 12 / 16 / 24 / 32-word buffer;
                            // 28 = 20 with a 16-word buffer
    if (v < 0 || v > 28 || v == 10) return opt_error(k, v, "valid unless v < 0 || v > 28 || v == 10");
    inf_decode_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "h_mfma") {  // 0: band H passes with the VALU convolution (k_resize_hb, A/B)
    h_mfma_ = v != 0;
    return DG_OK;
  }
  if (k == "band_dec") {  // 0: IDCT to planes + band H kernel (the split path, A/B)
    band_dec_ = v != 0;
    return DG_OK;
  }
  if (k == "dec_dbg") {  // timing experiments: skip k_band_dec phases (wrong pixels)
    dec_dbg_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "dec_strips") {
    if (v < 1 || v > 4096) return opt_error(k, v, "valid unless v < 1 || v > 4096");
    dec_strips_ = (uint32_t)v;
    return DG_OK;
  }
  if (k == "debug_flags") {
    debug_flags_ = (int)v;
    return DG_OK;
  }
  return opt_error(k, v, "unknown option");
}

int64_t Context::get_stat(const std::string &k) {
  if (k == "batches") return stat_batches_;
  if (k == "coalesced_batches") return stat_coalesced_batches_;
  if (k == "coalesced_images") return stat_coalesced_images_;
  if (k == "resync_rounds") return stat_resync_;
  if (k == "fix_workgroups") return stat_fix_;
  if (k == "write_mismatch") return stat_mismatch_;
  if (k == "unsettled_batches") return stat_unsettled_;
  if (k == "prog_items") return stat_prog_items_;
  if (k == "prog_aggregates") return stat_prog_aggs_;
  if (k == "prog_aggregate_images") return stat_prog_agg_images_;
  if (k == "prog_chains") return stat_prog_chains_;
  if (k == "pool_flushes") return stat_pool_flush_;
  if (k == "sync_iters_max") return stat_iters_;
  {  // wg_timing summaries, in nanoseconds: wg_{sync,write}_{span,mean,p90,max}
    static const char *kn[2] = {"sync", "write"}, *sn[4] = {"span", "mean", "p90", "max"};
    for (int a = 0; a < 2; a++)
      for (int q = 0; q < 4; q++)
        if (k == std::string("wg_") + kn[a] + "_" + sn[q]) return (int64_t)(wgstat_[a][q] * 1000.0);
  }
  if (k == "sub_bits") return last_sub_bits_;
  if (k == "sub_auto") return sub_auto_;
  if (k == "coalesce_inflight") return coalesce_inflight_;
  if (k == "meta_bytes") return (int64_t)last_meta_bytes_;
  if (k == "allocs") return stat_allocs_;
  if (k == "alloc_mb") return stat_alloc_mb_;
  if (k == "alloc_us") return (int64_t)stat_alloc_us_;
  if (k == "reclaims") return stat_reclaims_;
  if (k == "peak_device_mb") return stat_peak_dev_ >> 20;
  if (k == "device_mb") {
    std::lock_guard<std::mutex> lk(mu_);
    return (int64_t)(dev_footprint() >> 20);
  }
  if (k == "max_device_mb") return (int64_t)(max_dev_bytes_ >> 20);
  if (k == "budget_splits") return stat_budget_splits_;
  if (k == "budget_plan_mb") return (int64_t)(plan_arena_ >> 20);  // planned bytes per slot
  if (k == "budget_slots") return max_dev_bytes_ ? std::min<int64_t>(nslots_, stat_budget_slots_min_) : nslots_;
  if (k == "coef_cache_hits") return stat_ccache_hits_;
  if (k == "coef_cache_new") return stat_ccache_new_;
  if (k == "coef_cache_resets") return stat_ccache_resets_;
  if (k == "coef_cache_mb") return (int64_t)(ccache_off_ >> 20);
  if (k == "budget_frees") return stat_budget_frees_;
  if (k == "budget_oom") return stat_budget_oom_;
  if (k == "retire_syncs") return stat_retire_syncs_;
  if (k == "png_serial_fallbacks") return stat_png_serial_;
  if (k == "band_dec_images") return stat_band_dec_;
  if (k == "direct_d2h") return stat_direct_d2h_;
  if (k == "png_chunks") return stat_png_chunks_;
  if (k == "png_small_streams") return stat_png_small_;
  {  // host microseconds spent in dg_submit* since the last reset, per phase: wall and thread CPU
    static const char *pn[8] = {"plan", "pools", "layout", "lists", "upload", "h2d", "launch", "slotwait"};
    for (int q = 0; q < 8; q++) {
      if (k == std::string("host_us_") + pn[q]) return (int64_t)host_us_[q];
      if (q < 7 && k == std::string("host_cpu_us_") + pn[q]) return (int64_t)host_cpu_us_[q];
    }
  }
  if (k == "hpool") return (int64_t)hpool_.size();
  if (k == "qpool") return (int64_t)qpool_.size();
  set_error("dg_ctx_get_stat(\"" + k + "\"): unknown statistic");
  return -1;
}


int Context::timings(const char **names, float *ms, int cap) {
  int n = (int)last_ms_.size();
  for (int i = 0; i < n && i < cap; i++) {
    if (names) names[i] = kStageNames[i];
    if (ms) ms[i] = last_ms_[i];
  }
  return n;
}

// Grow a device buffer.  `user`: the only stream that can still be using it
// (a slot's own buffers); nullptr = shared by every stream (the table pools).
// Growing a buffer never frees the old one on the spot: hipFree / hipHostFree
// synchronise the whole device, which would make a baseline batch's growth
// wait for a ~1 s progressive aggregate on another slot (and serialised the
// aggregates).  The caller guarantees the old buffer is idle (a slot's
// previous batch is finished before its buffers are reused), so it is only
// retired and freed later: at destruction, or once retired buffers pass
// kRetiredMax, after a sync of every stream.
// Device and page-locked host memory have limits of their own: several ranks
// per host each keeping GiBs of grown-out buffers page-locked would pin a lot
// of the host's memory.  Retired buffers are also freed at the first idle
// moment (a wait that leaves no batch in flight, free_retired_if_idle).
// 32 GiB of retired device buffers at most before a device-wide sync frees
// them (growth happens while a workload sets new size maxima, i.e. in its
// first batches; a lower limit made those batches sync every few growths).
// Ranks sharing one device should set a budget (option "max_device_mb"):
// under a budget nothing is retired -- a grown-out buffer is freed at once.
static constexpr size_t kRetiredDevMax = (size_t)32 << 30;
static constexpr size_t kRetiredPinMax = (size_t)512 << 20;

void Context::retire(void *p, size_t bytes, bool pinned) {
  (pinned ? retired_pinned_ : retired_dev_).push_back(p);
  (pinned ? retired_pin_bytes_ : retired_dev_bytes_) += bytes;
  if ((retired_dev_bytes_ > kRetiredDevMax || retired_pin_bytes_ > kRetiredPinMax) && sync_all() == DG_OK) {
    stat_retire_syncs_++;
    free_retired();
  }
}

void Context::free_retired() {
  for (void *p : retired_dev_) hipFree(p);
  for (void *p : retired_pinned_) hipHostFree(p);
  retired_dev_.clear();
  retired_pinned_.clear();
  retired_dev_bytes_ = retired_pin_bytes_ = 0;
}

void Context::note_alloc(std::chrono::steady_clock::time_point t0, size_t bytes) {
  stat_allocs_++;
  stat_alloc_mb_ += (int64_t)(bytes >> 20);
  stat_alloc_us_ += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

size_t Context::grow_cap(size_t bytes, bool headroom) {
  return align_up(std::max(bytes, (size_t)1 << 20) + (headroom ? bytes / 2 : 0), 1 << 20);
}

// An allocation failed: free the retired buffers (after a sync of every
// stream; the failed call is about to fail the submit anyway) so the retry
// sees them.  True = worth retrying.
bool Context::reclaim() {
  (void)hipGetLastError();
  stat_reclaims_++;
  if (sync_all() != DG_OK) return false;
  free_retired();
  return true;
}

// mu_ held.  hipFree synchronises the device, so only when nothing is in flight.
void Context::free_retired_if_idle() {
  if (retired_dev_.empty() && retired_pinned_.empty()) return;
  for (const Slot &s : slots_)
    if (s.batch && !s.batch->done) return;
  free_retired();
}

// exact: no growth headroom and no reclaim on failure (prewarm_slots: a
// failed allocation there just leaves the slot to grow on first use)
dg_status Context::ensure(DevBuf &b, size_t bytes, hipStream_t user, bool exact) {
  (void)user;
  if (b.cap >= bytes) return DG_OK;
  if (b.p) {
    if (max_dev_bytes_) {  // under a budget the old buffer is gone now (budget_fit counted it so)
      hipFree(b.p);
    } else {
      retire(b.p, b.cap, false);
    }
    b.p = nullptr;
    b.cap = 0;
  }
  // 50% headroom: an allocation blocks on the driver (8 ranks sharing one
  // GPU measured 36-209 ms of wall time per step in the layout phase against
  // 0.3 ms of CPU while batches kept setting new size maxima,
  // profiles/r04/ranks), so growth must stay rare.  (Headroom on re-growth
  // only cost configs[1] 1.4 ms of submit time per batch: the extra growths
  // retired enough to trigger device-wide syncs.)  Under memory pressure the
  // retired buffers go first, then the headroom.
  // no headroom once the device is three quarters full (several ranks or
  // contexts sharing one device: 8 ranks x 4 slots x 1.5 ran a 288 GB device
  // out of memory, profiles/r04/ranks_r4f); under a budget, only the room
  // budget_fit left.
  size_t dfree = 0, dtotal = 0;
  const bool roomy = hipMemGetInfo(&dfree, &dtotal) != hipSuccess || dfree > dtotal / 4 + bytes;
  size_t cap = exact ? align_up(bytes, (size_t)1 << 20) : grow_cap(bytes, roomy);
  if (max_dev_bytes_) {
    const size_t lim = align_up(bytes, 1 << 20) + (budget_room_ / 3 & ~(((size_t)1 << 20) - 1));
    cap = std::min(cap, std::max(lim, align_up(bytes, 1 << 20)));
    budget_room_ -= std::min(budget_room_, cap - std::min(cap, bytes));
  }
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipMalloc(&b.p, cap);
  if (e != hipSuccess && !exact && reclaim()) {
    cap = grow_cap(bytes, false);
    e = hipMalloc(&b.p, cap);
  }
  note_alloc(t0, cap);
  if (e != hipSuccess) {
    if (exact) {
      (void)hipGetLastError();
      b.p = nullptr;
      return DG_ERR_OOM;
    }
    set_error("device allocation failed");
    b.p = nullptr;
    return DG_ERR_OOM;
  }
  b.cap = cap;
  stat_peak_dev_ = std::max<int64_t>(stat_peak_dev_, (int64_t)dev_footprint());
  return DG_OK;
}

// Device bytes the context holds: every slot's buffers, the table pools and
// the retired buffers not yet freed (`except`'s buffers left out).
size_t Context::dev_footprint(const Slot *except) const {
  size_t t = retired_dev_bytes_;
  for (const Slot &o : slots_) {
    if (&o == except) continue;
    for (const DevBuf *b : {&o.meta, &o.wgt, &o.arena}) t += b->cap;
    if (!o.views)
      for (const DevBuf *b : {&o.scratch, &o.input, &o.coef}) t += b->cap;
  }
  for (int g = 0; g < kPoolGens; g++) t += d_hpool_[g].cap + d_qpool_[g].cap;
  return t + d_ccache_.cap;
}

// The arena is nearly full: start it over once no batch in flight reads or
// writes it (finishing them first, as a pool flush does).  Runs before a
// batch's lookups, so a batch never mixes entries of two arena lifetimes.
void Context::ccache_maybe_reset(Slot &self) {
  if (!ccache_cap_ || (!ccache_full_ && ccache_off_ <= ccache_cap_ / 8 * 7)) return;
  for (Slot &o : slots_) {
    if (&o == &self || !o.batch || o.batch->done || !o.batch->uses_ccache) continue;
    if (finish(o)) return;  // keep the arena as it is; the next batch tries again
  }
  ccache_index_clear();
  ccache_.clear();
  ccache_off_ = 0;
  ccache_full_ = false;
  stat_ccache_resets_++;
}

void Context::ccache_index_clear() { ccache_slot_.assign((size_t)1 << kCIdxBits, -1); }

int Context::ccache_find(const CKey &k, uint32_t &slot) const {
  const uint32_t mask = (1u << kCIdxBits) - 1u;
  slot = (uint32_t)CKeyHash()(k) & mask;
  for (uint32_t probe = 0; probe <= mask; probe++, slot = (slot + 1) & mask) {
    const int32_t e = ccache_slot_[slot];
    if (e < 0) return -1;
    if (ccache_[e].key == k) return e;
  }
  return -1;
}

void Context::ccache_rollback(size_t n0, size_t off0) {
  if (ccache_.size() <= n0) return;
  ccache_.resize(n0);  // (rare: a submit that installed no batch) rebuild the index
  ccache_index_clear();
  for (size_t i = 0; i < ccache_.size(); i++) {
    uint32_t slot;
    ccache_find(ccache_[i].key, slot);
    ccache_slot_[slot] = (int32_t)i;
  }
  ccache_off_ = std::min(ccache_off_, off0);
}

int Context::ccache_lookup(const ResizePass &ps, Batch &b, bool &hit) {
  hit = false;
  if (!ccache_cap_ || max_dev_bytes_ && ccache_cap_ > max_dev_bytes_ / 8) return -1;
  CKey k;
  memcpy(&k.in0, &ps.in0, 8);
  memcpy(&k.in1, &ps.in1, 8);
  k.in_size = ps.in_size;
  k.out_size = ps.out_size;
  k.ksize = ps.ksize;
  if (ccache_slot_.empty()) ccache_index_clear();
  uint32_t slot;
  const int found = ccache_find(k, slot);
  if (found >= 0) {
    if (!ccache_[found].ready) return -1;  // a batch in flight is writing it: compute our own copy
    hit = true;
    b.uses_ccache = true;
    stat_ccache_hits_++;
    return found;
  }
  const size_t bytes = align_up((size_t)ps.out_size * 8 + (size_t)ps.out_size * ps.ksize * 2, 256);
  // full (arena, or the index at 3/4 load): the next submit starts the arena over
  if (ccache_off_ + bytes > ccache_cap_ || ccache_.size() >= ((size_t)3 << kCIdxBits) / 4) {
    ccache_full_ = true;
    return -1;
  }
  if (!d_ccache_.p) {
    if (hipMalloc(&d_ccache_.p, ccache_cap_) != hipSuccess) {
      (void)hipGetLastError();
      d_ccache_.p = nullptr;
      ccache_cap_ = 0;  // no cache on this device
      return -1;
    }
    d_ccache_.cap = ccache_cap_;
  }
  const int idx = (int)ccache_.size();
  ccache_.push_back(CEntry{k, ccache_off_, 0, false});
  ccache_slot_[slot] = idx;
  ccache_off_ += bytes;
  b.uses_ccache = true;
  stat_ccache_new_++;
  return idx;
}

// An idle slot's device buffers (no batch, or its batch finished).
void Context::free_slot_buffers(Slot &o) {
  if (o.views) {  // carved from the arena
    for (DevBuf *b : {&o.scratch, &o.input, &o.coef}) {
      b->p = nullptr;
      b->cap = 0;
    }
    o.views = false;
  }
  for (DevBuf *b : {&o.scratch, &o.meta, &o.input, &o.coef, &o.arena}) {
    if (!b->p) continue;
    hipFree(b->p);
    b->p = nullptr;
    b->cap = 0;
    stat_budget_frees_++;
  }
}

// mu_ held.  Planned budget (option "budget_plan"): the first baseline batch
// under the budget decides how many batches fit in flight and sizes every
// slot then -- an even share of the budget left after the table pools, the
// Lanczos cache and a 1/32 reserve for the descriptor buffers, split over
// scratch / coefficients / input in the first batch's proportions, at least
// 1.25x what that batch needs -- so that a loader sharing its GPU (ranks, or
// training) allocates and frees nothing after its first batch: hipMalloc took
// ~170 ms and hipFree synchronised the device inside the timed window of the
// 8-ranks-on-one-GPU rehearsal.  A later batch that does
// not fit its slot is split (kNeedSplit), never grown; its input arena
// (host-in submissions after device-in ones) is the one buffer added later.
dg_status Context::budget_planned_fit(Slot &sl, size_t rs, size_t rc, size_t ri) {
  const size_t MB = (size_t)1 << 20;
  budget_room_ = 0;
  // this batch's scratch / coefficient / input views of the slot's arena
  const size_t os = 0, oc = align_up(rs, 256), oi = oc + align_up(rc, 256), need = oi + ri;
  auto carve = [&]() {
    char *a = (char *)sl.arena.p;
    sl.scratch = DevBuf{a + os, rs};
    sl.coef = DevBuf{a + oc, rc};
    sl.input = DevBuf{ri ? a + oi : nullptr, ri};
    sl.views = true;
    const size_t fp = dev_footprint();
    budget_room_ = fp < max_dev_bytes_ ? (max_dev_bytes_ - fp) / 2 : 0;
  };
  if (budget_planned_) {
    if (need > plan_arena_) return kNeedSplit;
    if (!sl.arena.p) {  // a planned slot without its arena (a progressive batch took the room): take it back
      if (sl.scratch.p || sl.coef.p || sl.input.p) free_slot_buffers(sl);
      if (dev_footprint() + plan_arena_ > max_dev_bytes_ || ensure(sl.arena, plan_arena_, sl.st, true))
        return kNeedSplit;
    }
    carve();
    return DG_OK;
  }
  // first sizing: every other slot gives its buffers back (a budget set on a
  // context that ran without one), then the plan
  for (int j = 0; j < kAllSlots; j++) {
    Slot &o = slots_[j];
    if (&o == &sl) continue;
    if (o.batch && !o.batch->done && finish(o)) return DG_ERR_DEVICE;
    free_slot_buffers(o);
  }
  free_slot_buffers(sl);
  if (!retired_dev_.empty() && sync_all() == DG_OK) free_retired();
  const size_t others = dev_footprint(&sl) + sl.meta.cap + sl.wgt.cap;
  if (others >= max_dev_bytes_) return kNeedSplit;
  // descriptor / weight buffers of the planned slots grow into the reserve
  const size_t reserve =
      std::min<size_t>(std::max<size_t>(max_dev_bytes_ / 32, 64 * MB), (max_dev_bytes_ - others) / 4);
  size_t avail = max_dev_bytes_ - others - reserve;
  {  // a budget above what the device has free plans for what it has (less 1/8 for the others on it)
    size_t dfree = 0, dtotal = 0;
    if (hipMemGetInfo(&dfree, &dtotal) == hipSuccess) avail = std::min(avail, dfree - std::min(dfree, dtotal / 8));
  }
  if (need + need / 4 > avail) return kNeedSplit;  // the halves plan the budget
  const int ns = (int)std::max<size_t>(1, std::min<size_t>((size_t)nslots_, avail / (need + need / 4)));
  plan_arena_ = (avail / (size_t)ns) & ~(MB - 1);
  if (ensure(sl.arena, plan_arena_, sl.st, true)) {
    set_error("device allocation of the planned budget failed");
    return DG_ERR_OOM;
  }
  budget_slots_ = ns;
  stat_budget_slots_min_ = std::min<int64_t>(stat_budget_slots_min_, ns);
  budget_planned_ = true;
  next_slot_ = 1 % ns;
  carve();
  budget_room_ = reserve / 2;
  return DG_OK;
}

// mu_ held.  The device budget (option "max_device_mb"): make room for a
// batch of `self` whose scratch / coefficient / input arenas need rs / rc /
// ri bytes.  In order: keep self's buffers if they already fit; free the
// retired buffers; give back the buffers of baseline slots the budget took
// out of turn; then take the highest other baseline slot out of turn
// (budget_slots_: pick_slot cycles over fewer slots from now on), finishing
// its batch (waiting for its GPU work, as a dg_wait would) and freeing its
// buffers, and likewise the progressive slots; finally drop self's own
// oversized buffers (idle: the slot's previous batch is finished) for
// exact-size ones.  So a budget below what "slots" batches need settles on
// fewer batches in flight instead of trading buffers between slots batch
// after batch (each trade a hipFree + hipMalloc).  False: the batch alone
// does not fit -- the caller splits it (submit_split).  budget_room_: what
// growth may add on top.  (The descriptor buffer, a few MB, grows after this
// check.)
bool Context::budget_fit(Slot &self, size_t rs, size_t rc, size_t ri) {
  budget_room_ = 0;
  if (!max_dev_bytes_) return true;
  const size_t fixed = self.meta.cap + self.wgt.cap;
  const size_t keep = std::max(self.scratch.cap, rs) + std::max(self.coef.cap, rc) + std::max(self.input.cap, ri) + fixed;
  const size_t tight = rs + rc + ri + fixed;
  const int si = (int)(&self - slots_);
  auto others = [&] { return dev_footprint(&self); };
  auto give_back = [&](Slot &o) {
    if (o.batch && !o.batch->done && finish(o)) return;
    free_slot_buffers(o);
  };
  auto has_buffers = [](const Slot &o) { return o.scratch.p || o.coef.p || o.input.p || o.arena.p; };
  if (others() + keep > max_dev_bytes_ && !retired_dev_.empty() && sync_all() == DG_OK) free_retired();
  if (budget_planned_) {  // (a progressive slot) the planned baseline slots keep their buffers
    for (int j = kMaxInflight; j < kAllSlots && others() + keep > max_dev_bytes_; j++)
      if (j != si) give_back(slots_[j]);
    if (others() + keep <= max_dev_bytes_) {
      budget_room_ = max_dev_bytes_ - others() - keep;
      return true;
    }
    if (others() + tight > max_dev_bytes_) return false;
    free_slot_buffers(self);
    budget_room_ = max_dev_bytes_ - others() - tight;
    return true;
  }
  for (int j = std::max(1, budget_slots_); j < kMaxInflight && others() + keep > max_dev_bytes_; j++)
    if (j != si && has_buffers(slots_[j])) give_back(slots_[j]);
  while (others() + keep > max_dev_bytes_) {
    int j = kMaxInflight - 1;
    while (j >= 0 && (j == si || !has_buffers(slots_[j]))) j--;
    if (j < 0) break;
    give_back(slots_[j]);
    if (has_buffers(slots_[j])) break;  // its batch failed to finish: nothing more to take
    budget_slots_ = std::max(1, std::min(budget_slots_, std::max(j, si + 1)));
    stat_budget_slots_min_ = std::min<int64_t>(stat_budget_slots_min_, budget_slots_);
  }
  for (int j = kMaxInflight; j < kAllSlots && others() + keep > max_dev_bytes_; j++)
    if (j != si) give_back(slots_[j]);
  if (others() + keep <= max_dev_bytes_) {
    budget_room_ = max_dev_bytes_ - others() - keep;
    return true;
  }
  if (others() + tight > max_dev_bytes_) return false;
  free_slot_buffers(self);
  budget_room_ = max_dev_bytes_ - others() - tight;
  return true;
}

dg_status Context::ensure_pinned(PinBuf &b, size_t bytes, hipStream_t user, bool exact) {
  (void)user;
  if (b.cap >= bytes) return DG_OK;
  if (b.p) {
    retire(b.p, b.cap, true);
    b.p = nullptr;
    b.cap = 0;
  }
  size_t cap = exact ? align_up(bytes, (size_t)1 << 20) : grow_cap(bytes, true);
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e = hipHostMalloc(&b.p, cap, hipHostMallocDefault);
  if (e != hipSuccess && !exact && reclaim()) {
    cap = grow_cap(bytes, false);
    e = hipHostMalloc(&b.p, cap, hipHostMallocDefault);
  }
  note_alloc(t0, cap);
  if (e != hipSuccess && exact) {
    (void)hipGetLastError();
    b.p = nullptr;
    return DG_ERR_OOM;
  }
  if (e != hipSuccess) {
    set_error("pinned host allocation failed");
    b.p = nullptr;
    return DG_ERR_OOM;
  }
  b.cap = cap;
  return DG_OK;
}

// Table pools.  Huffman and quantisation tables are de-duplicated by content
// into per-context pools that the kernels index with 16-bit slots.  Pools are
// not grow-only: once a pool holds more than kPoolKeep tables (a long-running
// loader over per-image-optimised JPEGs adds ~4 new tables per image; a
// progressive file ~10-12, one per scan), the next submit starts the pools
// over in the next of kPoolGens device generations, waiting only for batches
// that still read that generation (round 2 drained every batch in flight
// here -- with progressive aggregates that was a ~1 s stall of every slot,
// and it serialised the aggregates).  Only a single batch that alone needs
// more than kPoolMax tables sends its overflow images back as
// DG_ERR_UNSUPPORTED (the caller's CPU path), never as CORRUPT.
static constexpr size_t kPoolKeep = 16384;
static constexpr size_t kPoolMax = 65535;

dg_status Context::flush_pools() {
  const int next = (pool_gen_ + 1) % kPoolGens;
  for (int s = 0; s < kAllSlots; s++) {  // batches in flight still reading (and may resync with) that generation
    Slot &o = slots_[s];
    if (o.batch && !o.batch->done && o.batch->pool_gen == next) {
      dg_status st = finish(o);
      if (st) return st;
    }
  }
  hpool_.clear();
  hpool_idx_.clear();
  qpool_.clear();
  qpool_idx_.clear();
  for (RecentTab &r : hrecent_) r.idx = -1;
  for (RecentTab &r : qrecent_) r.idx = -1;
  hpool_uploaded_ = qpool_uploaded_ = 0;
  pool_gen_ = next;
  stat_pool_flush_++;
  return DG_OK;
}

// Table de-duplication.  Loaders mostly see a handful of distinct tables
// (the encoder's standard ones), so a few recently pooled tables are compared
// byte for byte first; only a miss builds the key string and hashes it (the
// per-table string and hash were 0.65 ms of a 1,024-image WebDataset submit).
static int recent_find(RecentTab *r, int n, const uint8_t *key, uint32_t len) {
  for (int i = 0; i < n; i++)
    if (r[i].idx >= 0 && r[i].len == len && memcmp(r[i].key, key, len) == 0) return r[i].idx;
  return -1;
}

static void recent_put(RecentTab *r, int n, uint32_t &next, const uint8_t *key, uint32_t len, int idx) {
  RecentTab &e = r[next++ % (uint32_t)n];
  e.len = len;
  memcpy(e.key, key, len);
  e.idx = idx;
}

int Context::pool_huff(const HuffSpec &s) {
  uint8_t raw[17 + 256];
  memcpy(raw, s.bits, 17);
  const uint32_t len = 17 + (uint32_t)std::max(0, std::min(256, s.nvals));
  memcpy(raw + 17, s.vals, len - 17);
  int idx = recent_find(hrecent_, kRecentTabs, raw, len);
  if (idx >= 0) return idx;
  std::string key((const char *)raw, len);
  auto it = hpool_idx_.find(key);
  if (it != hpool_idx_.end()) {
    idx = it->second;
  } else {
    HuffTable t;
    if (!build_huff_table(s, t)) return -1;
    if (hpool_.size() >= kPoolMax) return -2;
    hpool_.push_back(t);
    idx = (int)hpool_.size() - 1;
    hpool_idx_[key] = idx;
  }
  recent_put(hrecent_, kRecentTabs, hrecent_next_, raw, len, idx);
  return idx;
}

int Context::pool_quant(const uint16_t *q) {
  int idx = recent_find(qrecent_, kRecentTabs, (const uint8_t *)q, 128);
  if (idx >= 0) return idx;
  std::string key((const char *)q, 128);
  auto it = qpool_idx_.find(key);
  if (it != qpool_idx_.end()) {
    idx = it->second;
  } else {
    QuantTable t;
    memcpy(t.q, q, 128);
    if (qpool_.size() >= kPoolMax) return -2;
    qpool_.push_back(t);
    idx = (int)qpool_.size() - 1;
    qpool_idx_[key] = idx;
  }
  recent_put(qrecent_, kRecentTabs, qrecent_next_, (const uint8_t *)q, 128, idx);
  return idx;
}

dg_status Context::upload_pools() {
  DevBuf &hb = d_hpool_[pool_gen_], &qb = d_qpool_[pool_gen_];
  if (!hb.p) {  // each generation is allocated once, at full capacity: no reallocation, no device sync
    if (dg_status st = ensure(hb, kPoolMax * sizeof(HuffTable))) return st;
    if (dg_status st = ensure(qb, kPoolMax * sizeof(QuantTable))) return st;
  }
  // appends only: entries below *_uploaded_ may be in use by batches in flight
  if (hpool_.size() != hpool_uploaded_) {
    HIPCHK(hipMemcpyAsync((char *)hb.p + hpool_uploaded_ * sizeof(HuffTable), &hpool_[hpool_uploaded_],
                          (hpool_.size() - hpool_uploaded_) * sizeof(HuffTable), hipMemcpyHostToDevice, stream_));
    HIPCHK(hipStreamSynchronize(stream_));  // the host vector may reallocate later
    hpool_uploaded_ = hpool_.size();
  }
  if (qpool_.size() != qpool_uploaded_) {
    HIPCHK(hipMemcpyAsync((char *)qb.p + qpool_uploaded_ * sizeof(QuantTable), &qpool_[qpool_uploaded_],
                          (qpool_.size() - qpool_uploaded_) * sizeof(QuantTable), hipMemcpyHostToDevice, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    qpool_uploaded_ = qpool_.size();
  }
  return DG_OK;
}

// Decide what the GPU will do with one image: header, bucket, output size.
dg_status Context::plan_image(const uint8_t *h, size_t len, int32_t forced, ImagePlan &p) {
  p = ImagePlan();
  if (!h || len == 0) {
    p.status = DG_ERR_CORRUPT;
    return DG_OK;
  }
  uint32_t W, H, C;
  if (is_png(h, len)) {
    p.fmt = kFmtPng;
    parse_png_header(h, len, p.png);
    if (p.png.status != PH_OK) {
      p.status = p.png.status == PH_UNSUPPORTED ? DG_ERR_UNSUPPORTED : DG_ERR_CORRUPT;
      return DG_OK;
    }
    // the decoder's working set (raw + unfiltered + expanded) must stay 32-bit addressable
    const uint64_t raw = p.png.rawlen;
    if (raw >= (1ull << 31) || (uint64_t)p.png.width * p.png.height * 4ull >= (1ull << 31) ||
        p.png.zlen >= (1ull << 28)) {
      p.status = DG_ERR_UNSUPPORTED;
      return DG_OK;
    }
    W = p.png.width;
    H = p.png.height;
    C = (uint32_t)p.png.out_c;
  } else {
    if (!is_jpeg(h, len)) {
      p.status = DG_ERR_CORRUPT;
      return DG_OK;
    }
    parse_jpeg_header(h, len, p.hdr);
    if (p.hdr.status != JH_OK) {
      p.status = p.hdr.status == JH_UNSUPPORTED ? DG_ERR_UNSUPPORTED : DG_ERR_CORRUPT;
      return DG_OK;
    }
    if (p.hdr.progressive && !progressive_) {  // see option "progressive"
      p.hdr.why = "progressive JPEG (context option \"progressive\" decodes it on the GPU)";
      p.status = DG_ERR_UNSUPPORTED;
      return DG_OK;
    }
    if (p.hdr.incomplete_refinement && decode_sem_ == 0) {
      // libjpeg-turbo would smooth these blocks (jdcoefct.c smoothing_ok); zune-jpeg does not
      p.hdr.why = "incomplete progressive refinement (libjpeg block smoothing; decodes with decode_semantics 1)";
      p.status = DG_ERR_UNSUPPORTED;
      return DG_OK;
    }
    W = p.hdr.width;
    H = p.hdr.height;
    C = p.hdr.ncomp == 1 ? 1 : 3;
    // component planes (padded to whole MCUs) must stay below 4 GiB: the
    // upsampling kernels address rows with 24-bit multiplies.  The reference's
    // decoder refuses far smaller images already (image's 512 MiB max_alloc).
    if ((uint64_t)(W + 32) * (H + 32) >= (1ull << 32)) {
      p.status = DG_ERR_UNSUPPORTED;
      return DG_OK;
    }
  }
  p.channels = (int32_t)C;  // pre-transform (image_processing.rs:349-351)
  p.bit_depth = 8;
  uint32_t ow = W, oh = H;
  if (has_cfg_) {
    int b = forced;
    if (b == -1) {
      b = buckets_->closest((int32_t)W, (int32_t)H);
    } else if (b < -1 || b >= (int)buckets_->buckets().size()) {  // -2: "NaN" key (dg_sample_align)
      p.status = DG_ERR_BAD_BUCKET;
      return DG_OK;
    }
    p.bucket = b;
    ow = buckets_->buckets()[b].w;
    oh = buckets_->buckets()[b].h;
  }
  p.out_w = ow;
  p.out_h = oh;
  p.out_c = cfg_.image_to_rgb8 ? 3 : C;  // convert_to_rgb8 (:163-186)
  if (cfg_.image_to_rgb8) p.channels = 3;  // image_processing.rs:367-372
  p.out_bytes = (uint64_t)ow * oh * p.out_c;
  p.img_bytes = p.out_bytes;
  if (cfg_.pre_encode_images) {  // image_processing.rs:374-419
    p.encode = true;
    p.enc_png = cfg_.encode_format == 0;
    // a resized LA image is a GrayImage over its LA bytes by now (image_to_dyn_image)
    p.enc_la_gray = p.out_c == 2 && has_cfg_ && !(W == p.out_w && H == p.out_h);
    p.out_bytes = p.enc_png ? png_enc_bound(ow, oh, p.enc_la_gray ? 1 : p.out_c) : jpeg_enc_bound(ow, oh, p.out_c);
    p.channels = -1;  // :416
    // the encoders count bits in 32-bit offsets (~400 MB of output): larger
    // images stay on the caller's CPU encoder
    if (p.out_bytes >= (1ull << 29)) {
      p.status = DG_ERR_UNSUPPORTED;
      return DG_OK;
    }
  }
  return DG_OK;
}

dg_status Context::output_size(const uint8_t *bytes, size_t len, int32_t forced, uint64_t *nbytes) {
  ImagePlan p;
  plan_image(bytes, len, forced, p);
  *nbytes = p.out_bytes;
  if (p.status) set_error(p.fmt == kFmtPng ? p.png.why : (p.hdr.why ? p.hdr.why : "unsupported"));
  return (dg_status)p.status;
}

namespace {
struct Layout {
  size_t off = 0;
  size_t take(size_t bytes, size_t align = 256) {
    off = align_up(off, align);
    size_t o = off;
    off += bytes;
    return o;
  }
};
}  // namespace

dg_status Context::submit(int n, const uint8_t *const *h_srcs, const uint8_t *const *d_srcs, const size_t *lens,
                          const int32_t *forced, uint8_t *const *outs, const uint64_t *caps,
                          dg_payload_meta *metas, bool host_io, uint64_t *ticket, dg_payload_meta *const *mptrs,
                          int force_slot, bool defer_meta) {
  const auto wait_t0 = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lk(mu_);
  if (n < 0 || (n > 0 && (!h_srcs || !lens || !outs || !caps || (!metas && !mptrs)))) {
    set_error("null argument");
    return DG_ERR_INVALID;
  }
  HIPCHK(hipSetDevice(device_));
  Slot &sl = slots_[force_slot >= 0 ? force_slot : pick_slot()];
  if (dg_status st = slot_streams(sl)) return st;
  // This slot's previous batch must complete first.  Its GPU work is waited
  // for without the context lock: a progressive slot's batch can run ~1 s,
  // and every other dg_submit / dg_wait / dg_poll of the context would stall
  // behind it.  Re-checked after relocking: another thread may
  // have finished that batch, or queued one of its own on the slot.
  while (sl.batch && !sl.batch->done) {
    if (hipEventQuery(sl.batch->fin->e) == hipErrorNotReady) {
      std::shared_ptr<BatchEvent> fin = sl.batch->fin;
      lk.unlock();
      const hipError_t e = hipEventSynchronize(fin->e);
      lk.lock();
      if (e != hipSuccess) {
        set_error(std::string("HIP error: ") + hipGetErrorString(e) + " waiting for a slot's batch");
        return DG_ERR_DEVICE;
      }
      continue;
    }
    dg_status st = finish(sl);
    if (st) return st;
  }
  // context lock + the slot's previous batch (stat "host_us_slotwait")
  host_us_[7] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - wait_t0).count();
  std::unique_ptr<Batch> bp(new Batch());
  Batch &b = *bp;
  b.ticket = next_ticket_++;
  b.fin = std::make_shared<BatchEvent>();
  HIPCHK(hipEventCreateWithFlags(&b.fin->e, hipEventDisableTiming));
  b.n = n;
  b.host_io = host_io;
  b.mptr.resize(n);
  for (int i = 0; i < n; i++) b.mptr[i] = mptrs ? mptrs[i] : &metas[i];
  if (defer_meta) {
    // A progressive aggregate's members: the callers' metas keep reading
    // DG_ERR_NOT_READY until finish() publishes the batch's own copies
    // (dg_wait_ready's contract; the GPU is still decoding while planning
    // fills in status and dimensions).
    b.pub = b.mptr;
    b.local_meta.assign(n, dg_payload_meta{});
    for (int i = 0; i < n; i++) b.mptr[i] = &b.local_meta[i];
  }
  b.plans.resize(n);
  b.desc_of.assign(n, -1);
  // host time per submit phase: wall ("host_us_<phase>") and this thread's CPU
  // time ("host_cpu_us_<phase>"); wall well above CPU = blocking (allocation,
  // copies, driver locks), not planning work
  auto phase_t0 = std::chrono::steady_clock::now();
  double cpu_t0 = thread_cpu_us();
  auto phase = [&](int k) {
    const auto now = std::chrono::steady_clock::now();
    const double c = thread_cpu_us();
    host_us_[k] += std::chrono::duration<double, std::micro>(now - phase_t0).count();
    host_cpu_us_[k] += c - cpu_t0;
    phase_t0 = now;
    cpu_t0 = c;
  };
  // ---- 1. plan every image (host, header only; on the planning workers)
  auto plan_one = [&](int i) {
    ImagePlan &p = b.plans[i];
    plan_image(h_srcs[i], lens[i], forced ? forced[i] : -1, p);
    dg_payload_meta &m = *b.mptr[i];
    memset(&m, 0, sizeof(m));
    m.status = p.status;
    m.bucket = p.bucket;
    if (p.fmt == kFmtJpeg && p.hdr.status == JH_OK) {
      m.original_width = p.hdr.width;
      m.original_height = p.hdr.height;
    } else if (p.fmt == kFmtPng && p.png.status == PH_OK) {
      m.original_width = p.png.width;
      m.original_height = p.png.height;
    }
    m.width = p.out_w;
    m.height = p.out_h;
    m.channels = p.channels;
    m.bit_depth = p.bit_depth;
    m.is_encoded = p.encode ? 1 : 0;
    m.nbytes = p.out_bytes;
    if (p.status == DG_OK && caps[i] < p.out_bytes) {
      p.status = DG_ERR_SMALL_BUFFER;
      m.status = DG_ERR_SMALL_BUFFER;
    }
    if (p.status == DG_OK && !outs[i]) {
      p.status = DG_ERR_INVALID;
      m.status = DG_ERR_INVALID;
    }
  };
  if (plan_threads_ > 1 && n >= 2 * kPlanGrain) {
    if (!plan_pool_ || plan_pool_->threads() != plan_threads_) plan_pool_.reset(new HostPool(plan_threads_));
    plan_pool_->run(n, kPlanGrain, plan_one);
  } else {
    for (int i = 0; i < n; i++) plan_one(i);
  }
  phase(0);
  // ---- 2. table pools
  size_t hneed = 0, qneed = 0;  // upper bound of the tables this batch adds
  for (int i = 0; i < n; i++) {
    const ImagePlan &p = b.plans[i];
    if (p.status || p.fmt != kFmtJpeg) continue;
    hneed += p.hdr.progressive ? p.hdr.tables.size() : 2u * (size_t)p.hdr.ncomp;
    qneed += (size_t)p.hdr.ncomp;
  }
  if (hpool_.size() > kPoolKeep || qpool_.size() > kPoolKeep ||
      (hpool_.size() && hpool_.size() + hneed > kPoolMax) || (qpool_.size() && qpool_.size() + qneed > kPoolMax)) {
    dg_status st = flush_pools();
    if (st) return st;
  }
  for (int i = 0; i < n; i++) {
    ImagePlan &p = b.plans[i];
    if (p.status || p.fmt != kFmtJpeg) continue;
    int worst = 0;  // -1: a table that does not build (corrupt), -2: pools full for this batch
    auto use = [&](int idx) { worst = std::min(worst, idx); };
    if (p.hdr.progressive) {  // the tables each scan uses
      for (const HuffSpec &t : p.hdr.tables) use(pool_huff(t));
      for (int c = 0; c < p.hdr.ncomp; c++) use(pool_quant(p.hdr.q[p.hdr.comp[c].tq]));
    } else {
      for (int c = 0; c < p.hdr.ncomp; c++) {
        use(pool_huff(p.hdr.dc[p.hdr.comp[c].td]));
        use(pool_huff(p.hdr.ac[p.hdr.comp[c].ta]));
        use(pool_quant(p.hdr.q[p.hdr.comp[c].tq]));
      }
    }
    if (worst == -2) {
      p.status = DG_ERR_UNSUPPORTED;
      b.mptr[i]->status = DG_ERR_UNSUPPORTED;
    } else if (worst < 0) {
      p.status = DG_ERR_CORRUPT;
      b.mptr[i]->status = DG_ERR_CORRUPT;
    }
  }
  dg_status st = upload_pools();
  if (st) return st;
  b.pool_gen = pool_gen_;
  b.hp = (const HuffTable *)d_hpool_[pool_gen_].p;
  b.qp = (const QuantTable *)d_qpool_[pool_gen_].p;

  phase(1);
  // Lanczos table cache: entries this submit creates are dropped again if it
  // returns before its batch is installed (budget split, allocation failure)
  ccache_maybe_reset(sl);
  struct CacheRoll {
    Context *c;
    size_t n0, off0;
    bool armed = true;
    ~CacheRoll() {
      if (armed) c->ccache_rollback(n0, off0);
    }
  } croll{this, ccache_.size(), ccache_off_};
  // ---- 3. layout
  // Subsequence size: the entropy kernels are latency-bound, so they want as
  // many lanes as the chip can keep resident, but every subsequence costs a
  // sync re-decode.  Measured on MI355X (profiles/r01/sweep_v4): 2048 bits
  // below 64 MiB of coded data (configs[2]'s 1,024 WebDataset members, ~25
  // MiB: 39.9 vs 38.5 Gpx/s with 4096, profiles/r04/wds_sub2); from 64 MiB
  // option "sub_auto"
  // (round 4: 8192, profiles/r04/ab -- the chip stays full with half the
  // lanes once the write pass no longer decodes, and the 6 kbit lead-in of a
  // 4:2:0 range costs 75% instead of 150% of its bits).
  // Small batches (dg_decode_one's few images, option "small_coded" bytes of
  // coded data) are latency-bound: a lane's chain of lead-in + range bits is
  // the batch's k_huff_sync time (0.87 ms of a ~3 ms coalesced batch in the
  // decode_one trace, profiles/r04/one_trace), so they take short ranges and
  // lead-ins ("sub_small", "lead_small") at the cost of more total decode.
  uint32_t sub_bits = sub_bits_;
  bool small = false;
  if (!sub_bits) {
    uint64_t coded = 0;
    for (int i = 0; i < n; i++)
      if (!b.plans[i].status && b.plans[i].fmt == kFmtJpeg && !b.plans[i].hdr.progressive)
        coded += b.plans[i].hdr.scan_end - b.plans[i].hdr.scan_off;
    small = coded < small_coded_;
    sub_bits = coded >= (64ull << 20) ? sub_auto_ : small ? sub_small_ : 2048u;
  }
  last_sub_bits_ = sub_bits;
  Layout L;        // scratch arena
  Layout CO;       // coefficient arena (zero-filled per batch)
  Layout IN;       // input arena (host path)
  // The chunk-parallel inflate's entries (CH, 2 bytes per output byte, most
  // of a PNG batch's memory) are dead once k_inf_resolve has turned them into
  // raw bytes, before anything writes the buffers of the unfilter / expand /
  // resize stages (LT).  Both regions are laid out from 0 and placed at the
  // same offset of the scratch arena (option "png_alias", default on).
  Layout LT, CH;
  const bool alias = png_alias_;
  std::vector<size_t> in_off(n, 0);
  size_t out_total = 0;
  uint64_t ckpt_total = 0;  // checkpoint records of the batch (per-image sub_bits)
  b.out_dev_off.assign(n, 0);
  b.out_direct.assign(n, 0);
  uint32_t sub_base = 0;
  b.descs.reserve(n);
  // first pass: sizes only (pointers are patched after allocation)
  struct Offs {
    size_t coef, ccnt, plane[3], pix, pass_dst[kStages], pass_coef[kStages], pass_bounds[kStages], pass_srcoff[kStages];
    int pass_cache[kStages];    // Lanczos table cache entry of the pass (-1: tables in the scratch arena)
    bool pass_hit[kStages];     // ... already computed (no k_coeffs item)
    size_t final_off, tmp, out, ds, mk, chunk, stage;
    size_t zs, raw, unf, pal;
    size_t tout, ecoef, ebits, ewords, hdr, eaux;  // JPEG / PNG re-encode
    // alpha programs: buffer = dst of pass `stage` (-1: the decoded image), byte offset
    int aop_stage[kAlphaPoints];
    size_t aop_off[kAlphaPoints];
    // offsets taken from the late region (LT): bit 0 unf, 1 pix, 2 out, 3 + s pass_dst[s]
    uint32_t late = 0;
    int img = -1;
  };
  std::vector<Offs> offs;
  for (int i = 0; i < n; i++) {
    ImagePlan &p = b.plans[i];
    if (p.status) continue;
    ImageDesc d;
    memset(&d, 0, sizeof(d));
    Offs o;
    memset(&o, 0, sizeof(o));
    o.late = 0;
    o.img = i;
    for (int s_ = 0; s_ < kStages; s_++) o.pass_cache[s_] = -1;
    uint32_t W, H, C;
    size_t cur_stride;
    bool colour = false;  // the source is the YCbCr planes of a colour JPEG
    if (p.fmt == kFmtPng) {
      const PngHeader &g = p.png;
      W = g.width;
      H = g.height;
      C = (uint32_t)g.out_c;
      d.fmt = kFmtPng;
      d.width = W;
      d.height = H;
      d.dec_c = (uint8_t)C;
      PngDesc &pd = d.png;
      pd.zlen = (uint32_t)g.zlen;
      pd.rowbytes = g.rowbytes;
      pd.ustride = (uint32_t)align_up(g.rowbytes, 16);
      pd.bpp = (uint32_t)g.bpp;
      pd.ctype = (uint32_t)g.ctype;
      pd.depth = (uint32_t)g.depth;
      pd.has_trns = (uint32_t)g.has_trns;
      for (int k = 0; k < 3; k++) pd.trns[k] = g.trns[k];
      pd.interlace = (uint32_t)g.interlace;
      pd.rawlen = (uint32_t)g.rawlen;
      pd.expand = g.ctype == 3 || g.depth < 8 || g.has_trns || g.interlace;  // k_png_expand also de-interlaces
      o.zs = L.take((size_t)g.zlen + 64, 256);
      // chunk-parallel inflate for streams of at least two chunks (small ones,
      // e.g. masks, inflate serially in one wave)
      {
        const uint64_t want = g.rawlen;
        const uint32_t span = inf_chunk_;
        const uint32_t nch = (uint32_t)((g.zlen + span - 1) / span);
        if (nch >= 2 && !chunked_off_) {
          pd.chunk0 = (uint32_t)b.ichunks.size();
          pd.nchunks = nch;
          // entries per chunk: inf_cap / 10 times the image's average expansion of a span (+64 Ki), at
          // most the whole image; a chunk that needs more sends the image to the serial kernel.  The
          // entries (2 bytes per output byte) are most of a PNG batch's device memory: 3x made them
          // 6x the raw image
          const double ratio = (double)want / (double)g.zlen;
          const uint64_t cap = std::min<uint64_t>(want, (uint64_t)(0.1 * inf_cap_ * ratio * span) + inf_pad_);
          for (uint32_t k = 0; k < nch; k++) {
            InfChunk c;
            memset(&c, 0, sizeof(c));
            c.image = (uint32_t)b.descs.size();
            c.idx = k;
            c.span = span;
            c.cap = (uint32_t)cap;
            c.start = k == 0 ? 16u : kInfNone;  // chunk 0: first block after the 2-byte zlib header
            c.out = (alias ? CH : L).take(cap * 2, 256);  // offsets: made absolute below
            c.tab = (alias ? CH : L).take(kInfTabBytes, 256);
            b.ichunks.push_back(c);
          }
        }
      }
      o.raw = L.take((size_t)g.rawlen + 16, 256);
      o.unf = (alias ? LT : L).take(g.interlace ? (size_t)g.unflen + 16 : (size_t)H * pd.ustride, 256);
      o.late |= alias ? 1u : 0u;
      if (pd.expand) {
        d.pix_stride = (uint32_t)align_up((size_t)W * C, 16);
        o.pix = (alias ? LT : L).take((size_t)d.pix_stride * H);
        o.late |= alias ? 2u : 0u;
      } else {
        d.pix_stride = pd.ustride;
      }
      if (g.ctype == 3) {
        o.pal = b.blob.size();
        b.blob.insert(b.blob.end(), &g.pal[0][0], &g.pal[0][0] + 1024);
      }
      if (host_io) in_off[i] = IN.take(lens[i] + 16, 16);
      cur_stride = d.pix_stride;
      b.any_png = true;
    } else {
    const JpegHeader &h = p.hdr;
    W = h.width;
    H = h.height;
    d.width = W;
    d.height = H;
    d.ncomp = (uint8_t)h.ncomp;
    d.colorspace = (uint8_t)h.colorspace;
    d.sem = (uint16_t)decode_sem_;
    d.ckpt = ckpt_ ? 1u : 0u;
    d.dec_c = h.ncomp == 1 ? 1 : 3;
    d.hmax = (uint32_t)h.hmax;
    d.vmax = (uint32_t)h.vmax;
    d.mcux = (W + 8 * d.hmax - 1) / (8 * d.hmax);
    d.mcuy = (H + 8 * d.vmax - 1) / (8 * d.vmax);
    uint32_t bpm = 0;
    for (int c = 0; c < h.ncomp; c++) {
      const JpegComponent &k = h.comp[c];
      d.ch[c] = (uint32_t)k.h;
      d.cv[c] = (uint32_t)k.v;
      d.cdsw[c] = (uint32_t)(((uint64_t)W * k.h + d.hmax - 1) / d.hmax);
      d.cdsh[c] = (uint32_t)(((uint64_t)H * k.v + d.vmax - 1) / d.vmax);
      if (h.ncomp == 1) {
        d.cbw[c] = (d.cdsw[c] + 7) / 8;
        d.cbh[c] = (d.cdsh[c] + 7) / 8;
        d.cfirst[c] = 0;
        d.blk_comp[0] = 0;
        bpm = 1;
      } else {
        d.cbw[c] = d.mcux * k.h;
        d.cbh[c] = d.mcuy * k.v;
        d.cfirst[c] = bpm;
        for (int j = 0; j < k.h * k.v; j++) d.blk_comp[bpm + j] = (uint8_t)c;
        bpm += (uint32_t)(k.h * k.v);
      }
    }
    d.bpm = bpm;
    d.comp_bits = 0;
    for (uint32_t k = 0; k < bpm; k++) d.comp_bits |= (uint32_t)d.blk_comp[k] << (2 * k);
    d.total_blocks = h.ncomp == 1 ? d.cbw[0] * d.cbh[0] : d.mcux * d.mcuy * bpm;
    d.restart = (uint32_t)h.restart;
    d.blocks_per_seg = d.restart * bpm;
    // Huffman slots: unique pool indices per image
    int nslots = 0;
    auto slot_of = [&](int pidx) {
      for (int s = 0; s < nslots; s++)
        if (d.hslot[s] == pidx) return s;
      d.hslot[nslots] = (uint16_t)pidx;
      return nslots++;
    };
    d.slotmap = 0;
    for (int c = 0; c < h.ncomp; c++) {
      if (!h.progressive) {
        d.slotmap |= (uint32_t)slot_of(pool_huff(h.dc[h.comp[c].td])) << ((2 * c) * 4);
        d.slotmap |= (uint32_t)slot_of(pool_huff(h.ac[h.comp[c].ta])) << ((2 * c + 1) * 4);
      }
      d.qpool[c] = (uint16_t)pool_quant(h.q[h.comp[c].tq]);
    }
    d.nslots = (uint8_t)nslots;
    b.max_slots = std::max<uint32_t>(b.max_slots, (uint32_t)nslots);
    if (!h.progressive) {  // distinct AC slots (k_huff_sync builds a multi-symbol lookup for each, up to 3)
      uint32_t acs = 0;
      for (int c = 0; c < h.ncomp; c++) acs |= 1u << ((d.slotmap >> ((2 * c + 1) * 4)) & 15u);
      b.max_ac = std::max<uint32_t>(b.max_ac, std::min<uint32_t>((uint32_t)__builtin_popcount(acs), kMultiLuts));
    }
    if (h.progressive) {  // scans decoded by k_prog_scan (records built once the source address is known)
      d.prog = (uint32_t)h.scans.size();
      if (host_io) in_off[i] = IN.take(lens[i] + 16, 16);
    } else {
    // entropy data
    d.scan_len = (uint32_t)(h.scan_end - h.scan_off);
    // Per-image subsequence size (option "sub_density" T > 0): a lane's
    // decode time follows its symbols and blocks, not its bits, so images
    // with few coded bits per block (flat, low quality: short EOB-heavy
    // codes, ~2x the symbols per bit) take shorter ranges -- half below T
    // bits per block, a quarter below T / 2 -- and their workgroups stop
    // forming the entropy kernels' tail.
    d.sub_bits = sub_bits;
    if (sub_density_ > 0 && sub_bits_ == 0) {
      const double bpb = (double)d.scan_len * 8.0 / (double)std::max<uint32_t>(1, d.total_blocks);
      if (bpb < sub_density_ * 0.5 && sub_bits >= 2048)
        d.sub_bits = sub_bits / 4;
      else if (bpb < sub_density_ && sub_bits >= 1024)
        d.sub_bits = sub_bits / 2;
    }
    // completed blocks go straight to plane pixels inside k_huff_write (not
    // with decode-once staging, whose k_huff_scatter writes coefficients)
    d.idct_fused = (idct_fused_ && !entropy_once_) ? 1u : 0u;
    // k_huff_write splits each range at the sync pass's half-way checkpoint
    // (option "write_split"): needs that checkpoint, no restart markers and
    // the plain write path
    if (write_split_ && d.ckpt && !d.idct_fused && !entropy_once_ && h.restart == 0 && d.sub_bits >= 1024 &&
        d.sub_bits / 2 / kCkptBits - 1 < num_ckpt(d.sub_bits))
      d.ckpt |= 2u;
    if (d.idct_fused) b.any_fused = true;
    // lead-in before each subsequence (lead_in in dg_entropy.h): covers the
    // self-synchronisation distance, which is longest for 6-block MCUs
    // (4:2:0; p99.9 ~7 kbit on the bench corpus, tools/sync_stats.cpp).
    // Option "lead_big" (4096): shorter than that tail, but a wrong entry
    // guess only costs a re-decode up to the first checkpoint where it merges
    // (6144 -> 4096: +1.3% on configs[1]; 2048 / 1024 slower on configs[2])
    d.lead_bits = lead_bits_ >= 0 ? (uint32_t)lead_bits_ : small ? lead_small_ : (bpm >= 4 ? lead_big_ : 2048u);
    // shorter ranges of symbol-dense images get a proportionally shorter lead-in (option
    // "lead_density"): their codes are short, so the decoder self-synchronises in fewer bits
    if (lead_density_ && lead_bits_ < 0 && d.sub_bits < sub_bits)
      d.lead_bits = std::max<uint32_t>(1024u, d.lead_bits / (sub_bits / d.sub_bits));
    d.nsub = std::max<uint32_t>(1, (uint32_t)(((uint64_t)d.scan_len * 8 + d.sub_bits - 1) / d.sub_bits));
    d.sub_base = sub_base;
    sub_base += d.nsub;
    d.ckpt_base = (uint32_t)ckpt_total;
    ckpt_total += (uint64_t)d.nsub * num_ckpt(d.sub_bits);
    d.nchunk = std::max<uint32_t>(1, (d.scan_len + kDestuffChunk - 1) / kDestuffChunk);
    uint32_t mcus = h.ncomp == 1 ? d.total_blocks : d.mcux * d.mcuy;
    d.mk_cap = (d.restart ? mcus / d.restart + 2 : 0) + 64;
    d.ds_lsw = 0;
    while ((32u << d.ds_lsw) < d.sub_bits) d.ds_lsw++;
    o.ds = L.take((size_t)ds_words_alloc(d.nsub, d.ds_lsw) * 4, 256);
    if (entropy_once_ && d.sub_bits <= 8192) {  // decode-once staging (dg_entropy.h StageCtx)
      d.stage_cap = (d.sub_bits / 2 + d.sub_bits / 8 + 64 + 3) / 4;
      o.stage = L.take((size_t)((d.nsub + 63) / 64) * d.stage_cap * 64 * 16, 256);
      b.stage_on = true;
    }
    o.mk = L.take((size_t)d.mk_cap * 4, 16);
    o.chunk = L.take((size_t)d.nchunk * 16, 16);
    if (host_io) in_off[i] = IN.take(lens[i] + 16, 16);
    }  // sequential
    // buffers
    o.coef = CO.take((size_t)d.total_blocks * 128);
    // sparse blocks: k_huff_write's cooperative flush + k_idct_t only (not the
    // fused / decode-once writers, k_idct or k_band_dec; progressive scans
    // write whole blocks)
    o.ccnt = (sparse_coef_ && idct_thread_ && !d.prog && !d.idct_fused && !entropy_once_)
                 ? CO.take((size_t)d.total_blocks, 64) + 1
                 : 0;
    for (int c = 0; c < 3; c++) o.plane[c] = (size_t)-1;  // allocated after the pass plan (not for k_band_dec)
    C = d.dec_c;
    colour = h.ncomp == 3;
    if (h.ncomp == 3) {
      d.pix_stride = (uint32_t)align_up((size_t)W * 3, 16);
      cur_stride = d.pix_stride;  // the RGB image is only materialised if no pass fuses it
    } else {
      cur_stride = (size_t)d.cbw[0] * 8;
    }
    }  // JPEG
    // resize plan (image_processing.rs:264-325)
    d.out_w = p.out_w;
    d.out_h = p.out_h;
    d.out_c = p.out_c;
    d.out_stride = p.out_w * p.out_c;
    // Passes (fast_image_resize semantics, B1): call 1 resizes W x H to the
    // scaled nw x nh, call 2 crops the bucket out of it with a possibly
    // fractional (x.5) offset.  An integral crop offset on an axis is only a
    // window of call 1's outputs on that axis, so call 1's pass computes just
    // that window (out0 / width) and call 2 needs no pass there; a fractional
    // offset keeps call 2's sub-pixel pass.  Without a call-1 pass on an axis
    // the window is a plain offset into the current image.
    uint32_t cw = W, chh = H;     // extent of the current image's valid window
    uint32_t xoff = 0, yoff = 0;  // window origin (pixels, rows) inside the current buffer
    int last_stage = -1;
    auto add_pass = [&](int stage, uint32_t kind, double in0, double in1, uint32_t in_size, uint32_t out_size,
                        uint32_t out0, uint32_t width, uint32_t rows, uint32_t row0) -> ResizePass & {
      ResizePass &ps = d.pass[stage];
      ps.kind = kind;
      ps.in0 = in0;
      ps.in1 = in1;
      ps.in_size = in_size;
      ps.out_size = out_size;
      ps.out0 = out0;
      ps.ksize = fir_ksize(in0, in1, out_size);
      ps.src_stride = (uint32_t)cur_stride;
      ps.width = width;
      ps.rows = rows;
      ps.row0 = row0;
      ps.bands = hb_bands_;
      ps.C = C;
      ps.dst_stride = (uint32_t)align_up((size_t)width * C, 16);
      o.pass_srcoff[stage] = (size_t)xoff * C;  // column window of the source (V passes)
      o.pass_dst[stage] = (alias ? LT : L).take((size_t)ps.dst_stride * ps.rows);
      o.late |= alias ? 8u << stage : 0u;
      o.pass_cache[stage] = ccache_lookup(ps, b, o.pass_hit[stage]);
      if (o.pass_cache[stage] < 0) {
        o.pass_coef[stage] = L.take((size_t)out_size * ps.ksize * 2);
        o.pass_bounds[stage] = L.take((size_t)out_size * 8);
      }
      cur_stride = ps.dst_stride;
      last_stage = stage;
      return ps;
    };
    if (has_cfg_ && !(W == p.out_w && H == p.out_h)) {
      uint32_t nw, nh;
      scaled_size(W, H, p.out_w, p.out_h, nw, nh);
      double l, t, bw, bh;
      fit_crop_box(nw, nh, p.out_w, p.out_h, l, t, bw, bh);
      // A window is exact for a scale-1 crop at an integral offset.  The crop box
      // comes out of f64 arithmetic (640x480 -> top 6.000000000000028, height
      // 431.99999999999994): deviations this small leave the i16 Lanczos
      // weights exactly one-hot (they are < 2^-15 off), so the sub-pixel pass
      // would copy pixel rint(offset) + i and the window is still bit-exact.
      auto near_int = [](double v, double tgt) { return std::fabs(v - tgt) <= 1e-6; };
      const bool fold_x = near_int(l, std::rint(l)) && near_int(bw, (double)p.out_w);
      const bool fold_y = near_int(t, std::rint(t)) && near_int(bh, (double)p.out_h);
      const uint32_t lx = fold_x ? (uint32_t)std::rint(l) : 0u, ty = fold_y ? (uint32_t)std::rint(t) : 0u;
      if (nw != W) {  // call 1, horizontal
        ResizePass &ps = add_pass(0, 1, 0.0, (double)W, W, nw, fold_x ? lx : 0u, fold_x ? p.out_w : nw, chh, 0);
        ps.mode = h_pass_mode(ps, colour);
        cw = ps.width;
      } else if (fold_x) {
        xoff = lx;
        cw = p.out_w;
      }
      if (nh != H) {  // call 1, vertical (reads the column window, absorbs xoff)
        ResizePass &ps = add_pass(1, 2, 0.0, (double)H, H, nh, fold_y ? ty : 0u, cw, fold_y ? p.out_h : nh, 0);
        chh = ps.rows;
        xoff = 0;
      } else if (fold_y) {
        yoff = ty;
        chh = p.out_h;
      }
      if (!fold_x) {  // call 2, horizontal sub-pixel crop (reads the row window, absorbs yoff)
        ResizePass &ps = add_pass(2, 1, l, l + bw, cw, p.out_w, 0, p.out_w, chh, yoff);
        ps.mode = h_pass_mode(ps, false);
        cw = p.out_w;
        yoff = 0;
      }
      if (!fold_y) {  // call 2, vertical sub-pixel crop (reads the column window, absorbs xoff)
        add_pass(3, 2, t, t + bh, chh, p.out_h, 0, cw, p.out_h, 0);
        chh = p.out_h;
        xoff = 0;
      }
      // U8x2 / U8x4: fast_image_resize multiplies colour by alpha before each
      // convolution call and divides after (mul_div_alpha); a call
      // whose crop box has the destination's size at integral offsets is a
      // copy and touches no alpha.  Programs run in place at three points.
      if (C == 2 || C == 4) {
        const bool call1 = !(nw == W && nh == H);
        const bool call2 = !(bw == (double)p.out_w && bh == (double)p.out_h && l == std::floor(l) &&
                             t == std::floor(t));
        const bool call2_passes = d.pass[2].kind || d.pass[3].kind;
        const int s1 = d.pass[1].kind ? 1 : 0;  // last call-1 pass (when call1)
        auto set = [&](int k, int stage, uint32_t w, uint32_t rows, uint32_t prog) {
          if (!prog) return;
          o.aop_stage[k] = stage;
          d.aop[k].width = w;
          d.aop[k].rows = rows;
          d.aop[k].prog = prog;
          b.any_alpha = true;
        };
        set(0, -1, W, H, call1 ? 1u : 0u);
        uint32_t prog1 = 0, sh = 0;
        auto push = [&](uint32_t op) {
          prog1 |= op << sh;
          sh += 2;
        };
        if (call1) push(2);
        if (call2) push(1);
        if (call2 && !call2_passes) push(2);
        if (call1)
          set(1, s1, d.pass[s1].width, d.pass[s1].rows, prog1);
        else
          set(1, -1, W, H, prog1);
        if (call2 && call2_passes) set(2, d.pass[3].kind ? 3 : 2, p.out_w, p.out_h, 2u);
      }
    }
    // colour images whose first pass is not a fused H pass need the RGB image
    d.color_fused = colour && d.pass[0].kind == 1 && (d.pass[0].mode & kHFused);
    if (hv_fused_ && hv_fusable(d.pass[0], d.pass[1])) d.pass[0].mode |= kHVFused;
    if (p.fmt == kFmtJpeg) {
      // k_band_dec decodes pass[0]'s source from the coefficients: no planes
      const uint32_t dm = band_dec_ ? band_dec_mode(d, d.pass[0]) : 0u;
      d.pass[0].mode |= dm;
      if (dm) stat_band_dec_++;
      if (!dm)
        for (uint32_t c = 0; c < d.ncomp; c++) {
          // half-rate chroma as 8-byte records (dg_plane.h, option "chroma_rec"): twice the bytes
          const bool rec = chroma_rec_ && d.ncomp == 3 && d.hmax == 2 * d.ch[c];
          if (rec) d.crec |= 1u << c;
          o.plane[c] = L.take((size_t)d.cbw[c] * 8 * d.cbh[c] * 8 * (rec ? 2 : 1));
        }
    }
    if (colour && !d.color_fused) o.pix = L.take((size_t)d.pix_stride * H);
    // final write: the last pass writes straight into the output when the
    // channel count is unchanged; otherwise (or with no pass) k_copy runs.
    if (last_stage >= 0 && d.out_c == C) {
      d.pass[last_stage].dst_stride = d.out_stride;
      o.pass_dst[last_stage] = (size_t)-1;  // -> out
      d.copy_needed = 0;
    } else {
      d.copy_needed = 1;
      d.final_src_c = C;
      d.final_src_stride = (uint32_t)cur_stride;
      o.final_off = (size_t)yoff * cur_stride + (size_t)xoff * C;  // an uncomputed integral crop
      if (d.out_c == C)
        d.copy_mode = 0;
      else if (C == 1)
        d.copy_mode = 1;  // L8 -> RGB8
      else if (C == 4)
        d.copy_mode = 2;  // RGBA8 -> RGB8 over gray
      else  // LA8 -> RGB8: resized images went through image_to_dyn_image's GrayImage (B3)
        d.copy_mode = (has_cfg_ && !(W == p.out_w && H == p.out_h)) ? 3 : 4;
    }
    if (host_io) {
      o.out = (alias ? LT : L).take(p.out_bytes, 16);
      o.late |= alias ? 4u : 0u;
      b.out_dev_off[i] = o.out;
      out_total += p.out_bytes;
    }
    if (p.encode && p.enc_png) {  // PNG re-encode (dg_penc.hip): the transform lands in tout
      EncDesc &e = d.enc;
      e.active = 1;
      e.png = 1;
      e.w = p.out_w;
      e.h = p.out_h;
      e.C = p.enc_la_gray ? 1 : p.out_c;
      e.src_stride = p.enc_la_gray ? p.out_w : d.out_stride;
      const uint64_t nf = (uint64_t)e.h * ((uint64_t)e.w * e.C + 1);
      e.nblocks = (uint32_t)((nf + 1023) / 1024);
      const std::vector<uint8_t> hdr = png_enc_header(e.w, e.h, e.C);
      e.hdr_len = (uint32_t)hdr.size();
      o.hdr = b.blob.size();
      b.blob.insert(b.blob.end(), hdr.begin(), hdr.end());
      o.tout = L.take(p.img_bytes + 16, 256);
      o.ecoef = L.take((size_t)nf + 16, 256);
      o.ebits = L.take((size_t)e.nblocks * 4, 256);
      o.eaux = L.take((size_t)e.nblocks * 8, 256);
      o.ewords = (size_t)((3 + 9 * nf + 7 + 64) / 8 + 64) / 4 * 4;  // size for now; placed after the loop
      b.any_enc = true;
    } else if (p.encode) {  // the transform lands in tout; the JPEG goes to the caller's buffer
      EncDesc &e = d.enc;
      e.active = 1;
      e.w = p.out_w;
      e.h = p.out_h;
      e.C = p.out_c;
      e.ncomp = p.out_c <= 2 ? 1 : 3;
      e.mode = p.enc_la_gray ? 1 : 0;
      e.src_stride = d.out_stride;
      e.nbx = (p.out_w + 7) / 8;
      e.nby = (p.out_h + 7) / 8;
      e.nblocks = e.nbx * e.nby * e.ncomp;
      int qual = cfg_.jpeg_quality;
      uint8_t q[2][64];
      jpeg_enc_qtables(qual, q);
      memcpy(e.q, q, sizeof(q));
      const std::vector<uint8_t> hdr = jpeg_enc_header(p.out_w, p.out_h, (int)e.ncomp, qual);
      e.hdr_len = (uint32_t)hdr.size();
      o.hdr = b.blob.size();
      b.blob.insert(b.blob.end(), hdr.begin(), hdr.end());
      o.tout = L.take(p.img_bytes + 16, 256);
      o.ecoef = L.take((size_t)e.nblocks * 128, 256);
      o.ebits = L.take((size_t)e.nblocks * 4, 256);
      o.ewords = (size_t)(e.nblocks * 210ull + 64) / 4 * 4 + 16;  // size for now; placed after the loop
      b.any_enc = true;
    }
    b.desc_of[i] = (int)b.descs.size();
    b.descs.push_back(d);
    offs.push_back(o);
    (void)last_stage;
  }
  if (alias) {  // the late buffers and the chunk entries share one region after the early ones
    const size_t r0 = align_up(L.off, 256);
    L.off = r0 + std::max(LT.off, CH.off);
    for (Offs &o : offs) {
      if (o.late & 1u) o.unf += r0;
      if (o.late & 2u) o.pix += r0;
      if (o.late & 4u) {
        o.out += r0;
        b.out_dev_off[o.img] = o.out;
      }
      for (int s = 0; s < kStages; s++)
        if ((o.late & (8u << s)) && o.pass_dst[s] != (size_t)-1) o.pass_dst[s] += r0;
    }
    for (InfChunk &c : b.ichunks) {
      c.out += r0;
      c.tab += r0;
    }
  }
  b.total_subs = sub_base;
  if (b.any_enc) {  // encoder bit buffers: one contiguous region, zeroed with one memset per batch
    size_t tot = 0;
    for (Offs &o : offs)
      if (o.ewords) {
        const size_t sz = o.ewords;
        o.ewords = tot;
        tot += (sz + 255) / 256 * 256;
      }
    b.words_off = L.take(tot, 256);
    b.words_bytes = tot;
    for (Offs &o : offs)
      if (o.tout) o.ewords += b.words_off;
    EncTables et;
    jpeg_enc_tables(et);
    while (b.blob.size() % 16) b.blob.push_back(0);
    b.enctab_off = b.blob.size();
    b.blob.insert(b.blob.end(), (const uint8_t *)&et, (const uint8_t *)&et + sizeof(et));
  }
  // PNG unfilter: one progress flag per 64-row band of every plane
  b.uf_n = 0;
  b.uf_maxbpp = 1;
  for (ImageDesc &dd : b.descs)
    if (dd.fmt == kFmtPng) {
      dd.png.uf_flag0 = b.uf_n;
      b.uf_n += png_bands(dd);
      b.uf_maxbpp = std::max(b.uf_maxbpp, dd.png.bpp);
    }
  b.uf_flags_off = b.uf_n ? L.take((size_t)(b.uf_n + 1) * 4) : 0;
  b.pf_n = 0;
  for (const ImageDesc &dd : b.descs)
    if (dd.fmt == kFmtJpeg) b.pf_n += dd.prog;
  b.pf_off = b.pf_n ? L.take((size_t)(b.pf_n + 2) * 4) : 0;  // AC ticket, progress words, DC ticket
  // k_destuff_one: a ticket word + one state word per destuff chunk (zeroed per batch)
  b.ds_n = 0;
  for (const ImageDesc &dd : b.descs)
    if (dd.fmt == kFmtJpeg && !dd.prog) b.ds_n += dd.nchunk;
  b.ds_state_off = (destuff_one_ && b.ds_n) ? L.take((size_t)(b.ds_n + 1) * 8) : 0;
  const size_t subs_off = L.take(b.total_subs * sizeof(SubState));
  const size_t ckpt_off = L.take(std::max<uint64_t>(1, ckpt_total) * sizeof(Ckpt));
  // fused IDCT leftovers: at most one carried-in block per subsequence, plus
  // the blocks of flushes with < 8 active lanes -- the tail of a wave, or
  // every block of an image with fewer subsequences than that.  Sized for
  // the worst case (all blocks of the fused images; 8 B each is small next
  // to their 128 B of coefficients); k_idct_list clamps to it and finish()
  // checks it.
  uint64_t fused_blocks = 0;
  for (const ImageDesc &dd : b.descs)
    if (dd.idct_fused) fused_blocks += dd.total_blocks;
  b.idct_cap = b.any_fused ? (uint32_t)std::min<uint64_t>(2 * b.total_subs + fused_blocks + 4096, 0xFFFFFFF0u) : 0u;
  const size_t idct_list_off = L.take((size_t)b.idct_cap * 8 + 16);
  // Device memory: under the budget (option "max_device_mb") a batch that
  // does not fit even with the other slots drained goes back to the caller
  // to be split (submit_split); without one, a failed allocation first
  // finishes the other slots' batches and frees their buffers, then splits.
  const size_t rs = L.off + 256, rc = CO.off + 256, ri = host_io ? IN.off + 64 : 0;
  const bool planned = max_dev_bytes_ && budget_plan_ && &sl - slots_ < kMaxInflight;
  if (planned) {
    st = budget_planned_fit(sl, rs, rc, ri);
    if (st) return st;
  } else {
    if (sl.views) free_slot_buffers(sl);  // (the budget plan was switched off)
    if (!budget_fit(sl, rs, rc, ri)) return kNeedSplit;
  }
  for (int attempt = 0; !planned; attempt++) {
    st = ensure(sl.scratch, rs, sl.st);
    if (!st) st = ensure(sl.coef, rc, sl.st);
    if (!st && host_io) st = ensure(sl.input, ri, sl.st);
    if (st != DG_ERR_OOM) break;
    if (attempt > 0) return kNeedSplit;
    for (Slot &o : slots_) {
      if (&o == &sl) continue;
      if (o.batch && !o.batch->done && finish(o)) continue;
      free_slot_buffers(o);
    }
    // the Lanczos table arena counts too (256 MiB by default): with every
    // other batch finished only this one could read it
    bool cache_busy = b.uses_ccache;
    for (const Slot &o : slots_)
      if (&o != &sl && o.batch && !o.batch->done && o.batch->uses_ccache) cache_busy = true;
    if (!cache_busy && d_ccache_.p) {
      ccache_index_clear();
      ccache_.clear();
      ccache_off_ = 0;
      ccache_full_ = false;
      hipFree(d_ccache_.p);
      d_ccache_.p = nullptr;
      d_ccache_.cap = 0;
    }
  }
  if (st) return st;
  sl.coef_bytes = CO.off;
  // ---- 4. patch device addresses
  char *S = (char *)sl.scratch.p;
  for (InfChunk &c : b.ichunks) {
    c.out = (uint64_t)(uintptr_t)(S + c.out);
    c.tab = (uint64_t)(uintptr_t)(S + c.tab);
  }
  int k = 0;
  for (int i = 0; i < n; i++) {
    if (b.desc_of[i] < 0) continue;
    ImageDesc &d = b.descs[b.desc_of[i]];
    const Offs &o = offs[k++];
    const JpegHeader &h = b.plans[i].hdr;
    const uint8_t *src = host_io ? (const uint8_t *)sl.input.p + in_off[i] : d_srcs[i];
    const uint64_t user_out = host_io ? (uint64_t)(uintptr_t)(S + o.out) : (uint64_t)(uintptr_t)outs[i];
    const uint64_t out = d.enc.active ? (uint64_t)(uintptr_t)(S + o.tout) : user_out;
    d.out = out;
    if (d.enc.active) {
      EncDesc &e = d.enc;
      e.src = out;
      e.out = user_out;
      e.coef = (uint64_t)(uintptr_t)(S + o.ecoef);
      e.bits = (uint64_t)(uintptr_t)(S + o.ebits);
      e.words = (uint64_t)(uintptr_t)(S + o.ewords);
      e.aux = o.eaux ? (uint64_t)(uintptr_t)(S + o.eaux) : 0;
      e.hdr = o.hdr + 1;  // blob offset + 1: made absolute with the meta buffer
    }
    if (d.fmt == kFmtPng) {
      const PngHeader &g = b.plans[i].png;
      PngDesc &pd = d.png;
      pd.zs = (uint64_t)(uintptr_t)(S + o.zs);
      pd.raw = (uint64_t)(uintptr_t)(S + o.raw);
      pd.unf = (uint64_t)(uintptr_t)(S + o.unf);
      d.pix = pd.expand ? (uint64_t)(uintptr_t)(S + o.pix) : pd.unf;
      pd.pal = g.ctype == 3 ? o.pal + 1 : 0;  // blob offset + 1, made absolute with the meta buffer
      uint64_t zo = 0;
      for (size_t c = 0; c < g.idat_off.size(); c++) {
        GatherJob j;
        j.src = (uint64_t)(uintptr_t)(src + g.idat_off[c]);
        j.dst = pd.zs + zo;
        j.len = g.idat_len[c];
        j.pad = 0;
        zo += g.idat_len[c];
        b.gjobs.push_back(j);
      }
    } else {
    d.scan = (uint64_t)(uintptr_t)(src + h.scan_off);
    d.coef = (uint64_t)(uintptr_t)((char *)sl.coef.p + o.coef);
    d.ccnt = (o.ccnt && !(d.pass[0].mode & kHDecode)) ? (uint64_t)(uintptr_t)((char *)sl.coef.p + o.ccnt - 1) : 0;
    if (d.prog) {
      // one record per scan; level = 1 + the highest level of an earlier scan
      // sharing a component and an overlapping coefficient band
      const size_t first = b.pscans.size();
      for (size_t j = 0; j < h.scans.size(); j++) {
        const JpegScan &sc = h.scans[j];
        ProgScan r;
        memset(&r, 0, sizeof(r));
        r.data = (uint64_t)(uintptr_t)(src + sc.off);
        r.len = (uint32_t)(sc.end - sc.off);
        r.image = (uint32_t)b.desc_of[i];
        r.ns = (uint32_t)sc.ns;
        for (int q = 0; q < sc.ns; q++) {
          r.comp[q] = (uint32_t)sc.comp[q];
          r.dc[q] = sc.dc_tab[q] >= 0 ? (uint16_t)pool_huff(h.tables[sc.dc_tab[q]]) : 0;
        }
        r.ac = sc.ac_tab >= 0 ? (uint16_t)pool_huff(h.tables[sc.ac_tab]) : 0;
        r.ss = (uint32_t)sc.ss;
        r.se = (uint32_t)sc.se;
        r.ah = (uint32_t)sc.ah;
        r.al = (uint32_t)sc.al;
        r.restart = (uint32_t)sc.restart;
        r.first = (uint32_t)first;
        r.next = kProgNoScan;
        r.pflags = 0;
        uint32_t lvl = 0;
        for (size_t e = 0; e < j; e++) {
          const JpegScan &pr = h.scans[e];
          if (pr.se < sc.ss || sc.se < pr.ss) continue;
          bool share = false;
          for (int x = 0; x < pr.ns; x++)
            for (int y = 0; y < sc.ns; y++) share |= pr.comp[x] == sc.comp[y];
          if (share) {
            lvl = std::max(lvl, b.pscans[first + e].level + 1);
            if (h.scans.size() <= kProgMaxDepScans) r.deps |= 1ull << e;  // larger files: chained only
          }
        }
        r.level = lvl;
        b.pscans.push_back(r);
      }
    } else {
    d.ds = (uint64_t)(uintptr_t)(S + o.ds);
    d.stage = d.stage_cap ? (uint64_t)(uintptr_t)(S + o.stage) : 0;
    d.mk = (uint64_t)(uintptr_t)(S + o.mk);
    d.chunk = (uint64_t)(uintptr_t)(S + o.chunk);
    }
    for (int c = 0; c < h.ncomp; c++) d.plane[c] = o.plane[c] == (size_t)-1 ? 0 : (uint64_t)(uintptr_t)(S + o.plane[c]);
    d.pix = h.ncomp == 3 && !d.color_fused ? (uint64_t)(uintptr_t)(S + o.pix) : 0;
    }  // JPEG
    uint64_t cur = (d.fmt == kFmtPng || h.ncomp == 3) ? d.pix : d.plane[0];
    const uint64_t decoded = cur;
    const uint32_t decoded_stride = d.fmt == kFmtPng ? d.pix_stride : (h.ncomp == 3 ? d.pix_stride : d.cbw[0] * 8);
    for (int s = 0; s < kStages; s++) {
      ResizePass &ps = d.pass[s];
      if (!ps.kind) continue;
      ps.src = cur + o.pass_srcoff[s];
      ps.dst = o.pass_dst[s] == (size_t)-1 ? out : (uint64_t)(uintptr_t)(S + o.pass_dst[s]);
      if (o.pass_cache[s] >= 0) {  // cached tables: bounds, then the weights
        const CEntry &e = ccache_[o.pass_cache[s]];
        char *cb = (char *)d_ccache_.p + e.off;
        ps.bounds = (uint64_t)(uintptr_t)cb;
        ps.coef = (uint64_t)(uintptr_t)(cb + (size_t)ps.out_size * 8);
        if (o.pass_hit[s]) {
          ps.precision = e.precision;
          b.coef_hit.resize(b.descs.size(), 0);
          b.coef_hit[b.desc_of[i]] |= (uint8_t)(1u << s);
        } else
          b.ccache_prod.push_back({b.desc_of[i], s, o.pass_cache[s]});
      } else {
        ps.coef = (uint64_t)(uintptr_t)(S + o.pass_coef[s]);
        ps.bounds = (uint64_t)(uintptr_t)(S + o.pass_bounds[s]);
      }
      cur = ps.dst;
    }
    d.final_src = cur + (d.copy_needed ? o.final_off : 0);
    for (uint32_t k = 0; k < kAlphaPoints; k++) {
      if (!d.aop[k].prog) continue;
      const int sg = o.aop_stage[k];
      if (sg < 0) {
        d.aop[k].buf = decoded;
        d.aop[k].stride = decoded_stride;
        d.aop[k].on_decoded = 1;
      } else {
        d.aop[k].buf = d.pass[sg].dst;
        d.aop[k].stride = d.pass[sg].dst_stride;
      }
    }
    (void)subs_off;
  }
  phase(2);
  // ---- 5. workgroup lists
  for (int l = 0; l < L_COUNT; l++) {  // sized from the previous batch: no regrowth copies
    b.lists[l].clear();
    b.lists[l].reserve(list_hint_[l] + list_hint_[l] / 4);
  }
  std::vector<WgItem> hb[2][2][4];  // band H items per (stage, fused fill, weight-count class)
  std::vector<WgItem> hvl[2];       // k_resize_hv items per H weight class
  std::vector<WgItem> decl[2];      // k_band_dec items per segment class
  std::vector<WgItem> hm[2][2][2];  // k_resize_hm items per (stage, fused fill, K steps)
  for (int di = 0; di < (int)b.descs.size(); di++) {
    const ImageDesc &d = b.descs[di];
    const uint32_t I = (uint32_t)di;
    for (uint32_t k = 0; k < kAlphaPoints; k++)
      if (d.aop[k].prog) {
        const uint32_t cnt = d.aop[k].width * d.aop[k].rows;
        for (uint32_t it = 0; it < cnt; it += 256) b.lists[L_ALPHA0 + k].push_back({I, it});
      }
    if (d.fmt == kFmtPng) {
      b.lists[L_PNG].push_back({I, 0});
      if (d.png.nchunks) {
        b.lists[L_INF_RES].push_back({I, 0});
        for (uint32_t k = 1; k < d.png.nchunks; k++) b.lists[L_INF_FIND].push_back({d.png.chunk0 + k, 0});
      }
      if (d.png.expand)
        for (uint32_t it = 0; it < d.width * d.height; it += 256) b.lists[L_EXPAND].push_back({I, it});
    } else {
    if (d.prog) {
      const uint64_t bytes = (uint64_t)d.total_blocks * 128;
      for (uint32_t c = 0; (uint64_t)c * kProgZeroBytes < bytes; c++) b.lists[L_PROG_ZERO].push_back({I, c});
    } else {
    // split ranges (write_split): 128 ranges per k_huff_write workgroup, two lanes each
    const uint32_t wstep = (d.ckpt & 2u) ? kSubPerWg / 2 : kSubPerWg;
    for (uint32_t w = 0; w < d.nsub; w += wstep) b.lists[L_HUFF].push_back({I, w});
    for (uint32_t w = 0; w < d.nsub; w += kSubPerWg - 1) b.lists[L_SYNC].push_back({I, w});
    b.descs[di].ds_state0 = (uint32_t)b.lists[L_DESTUFF].size();  // k_destuff_one's state words, list order
    for (uint32_t c = 0; c < d.nchunk; c++) b.lists[L_DESTUFF].push_back({I, c});
    b.lists[L_SCAN].push_back({I, 0});
    }
    uint32_t items = 0;
    for (uint32_t c = 0; c < d.ncomp; c++) items += d.cbh[c] * ((d.cbw[c] + 63) / 64);  // kIdctBlocks
    if (!d.idct_fused && !(d.pass[0].mode & kHDecode))  // fused: k_huff_write (+ k_idct_list) / k_band_dec
      for (uint32_t it = 0; it < items; it += idct_thread_ ? kIdctItemStride : 1u) b.lists[L_IDCT].push_back({I, it});
    if (d.ncomp == 3 && !d.color_fused) {
      uint32_t q = (d.width + 7) / 8 * d.height;
      for (uint32_t it = 0; it < q; it += 256) b.lists[L_COLOR].push_back({I, it});
    }
    }  // JPEG
    const bool hv = (d.pass[0].mode & kHVFused) != 0;
    if (hv) {  // one workgroup per (V segment of kHVRows rows, column tile)
      const uint32_t tiles = (d.pass[0].width + kHBandCols - 1) / kHBandCols;
      const uint32_t cnt = tiles * ((d.pass[1].rows + kHVRows - 1) / kHVRows);
      const int cls = d.pass[0].ksize + 1 <= 8 ? 0 : 1;
      for (uint32_t it = 0; it < cnt; it++) hvl[cls].push_back({I, it});
    }
    if (d.pass[0].mode & kHDecode) {  // one workgroup per (group of dec_strips 16-row strips, 128-column tile)
      const ResizePass &ps = d.pass[0];
      const uint32_t tiles = (ps.width + kDecCols - 1) / kDecCols;
      const uint32_t strips = (ps.row0 + ps.rows + 15) / 16 - ps.row0 / 16;
      const uint32_t cnt = tiles * ((strips + dec_strips_ - 1) / dec_strips_);
      for (uint32_t it = 0; it < cnt; it++) decl[(ps.mode & kHDecWide) ? 1 : 0].push_back({I, it});
    }
    for (int s = 0; s < kStages; s++) {
      const ResizePass &ps = d.pass[s];
      if (!ps.kind) continue;
      if (!(di < (int)b.coef_hit.size() && (b.coef_hit[di] >> s) & 1u)) b.lists[L_COEF].push_back({I, (uint32_t)s});
      if (hv && s < 2) continue;  // k_resize_hv runs both
      if (s == 0 && (ps.mode & kHDecode)) continue;  // k_band_dec runs it
      if (ps.kind == 1 && (ps.mode & kHDirect)) {  // one workgroup per (row, 512-column tile)
        uint32_t cnt = ps.rows * ((ps.width + 511) / 512);
        for (uint32_t it = 0; it < cnt; it++) b.lists[s == 0 ? L_RHX0 : L_RHX2].push_back({I, it});
      } else if (ps.kind == 1) {  // one workgroup per (band of rows, column tile)
        const uint32_t rows_per_wg = kHBandRows * ps.bands;
        uint32_t cnt = ((ps.rows + rows_per_wg - 1) / rows_per_wg) * ((ps.width + kHBandCols - 1) / kHBandCols);
        // k_resize_hb<K> reads taps in even-aligned pairs: a window starting
        // at an odd segment position spans ksize + 1 positions
        const uint32_t kk = ps.ksize + 1;
        int cls = kk <= 8 ? 0 : kk <= 16 ? 1 : kk <= 32 ? 2 : 3;
        // the 8- and 16-tap kernels stage narrower segments (hseg_px in kernels.hip)
        while (cls < 2 && h_pass_span(ps) > (cls == 0 ? 192.0 : 384.0)) cls++;
        const int fused = (ps.mode & kHFused) ? 1 : 0;
        const uint32_t ks = h_mfma_ ? h_mfma_steps(ps) : 0u;
        if (ks)
          for (uint32_t it = 0; it < cnt; it++) hm[s / 2][fused][ks - 1].push_back({I, it});
        else
          for (uint32_t it = 0; it < cnt; it++) hb[s / 2][fused][cls].push_back({I, it});
        if (fused && d.sem) b.h_zune = 1;  // the planar fused kernels of the zune fill classes
      } else if (v_tile_ && (ps.src_stride & 15) == 0) {  // k_resize_vt: 4 waves of (R rows x 1 KiB) tiles
        const uint32_t units = (ps.width * ps.C + 15) / 16;
        const uint32_t tiles = (units + 63) / 64 * ((ps.rows + v_tile_ - 1) / v_tile_);
        for (uint32_t it = 0; it < tiles; it += 4) b.lists[s == 1 ? L_RVT1 : L_RVT3].push_back({I, it});
        b.v_tile = v_tile_;
      } else {
        uint32_t cnt = (ps.width * ps.C + 15) / 16 * ps.rows;
        for (uint32_t it = 0; it < cnt; it += 256 * v_units_) b.lists[L_RH0 + s].push_back({I, it});
      }
    }
    if (d.copy_needed) {
      uint32_t cnt = d.out_w * d.out_h;
      for (uint32_t it = 0; it < cnt; it += 256) b.lists[L_COPY].push_back({I, it});
    }
    if (d.enc.active && d.enc.png) {
      const EncDesc &e = d.enc;
      for (uint32_t it = 0; it < e.h; it += 4) b.lists[L_PENC_ROW].push_back({I, it});
      for (uint32_t it = 0; it < e.nblocks; it += 256) b.lists[L_PENC_PIECE].push_back({I, it});
      b.lists[L_ENC_IMG].push_back({I, 0});  // k_enc_scan: piece offsets
      b.lists[L_PENC_IMG].push_back({I, 0});
    } else if (d.enc.active) {
      const EncDesc &e = d.enc;
      for (uint32_t it = 0; it < e.nbx * e.nby; it += 256) b.lists[L_ENC_MCU].push_back({I, it});
      for (uint32_t it = 0; it < e.nblocks; it += 256) b.lists[L_ENC_BLK].push_back({I, it});
      b.lists[L_ENC_IMG].push_back({I, 0});
    }
  }
  for (int l = 0; l < L_COUNT; l++) list_hint_[l] = b.lists[l].size();
  if (entropy_lpt_) {
    // Entropy workgroups decode a fixed number of bits, but their time follows
    // the symbol count: images with few coded bits per block (low quality,
    // flat content: short EOB-heavy codes) run up to 2x the mean.  Dispatch
    // those first (workgroups start in list order) so they do not form the
    // kernel's tail.
    auto cost_sort = [&](std::vector<WgItem> &l) {
      std::stable_sort(l.begin(), l.end(), [&](const WgItem &x, const WgItem &y) {
        const ImageDesc &a = b.descs[x.image], &c = b.descs[y.image];
        return (uint64_t)a.scan_len * c.total_blocks < (uint64_t)c.scan_len * a.total_blocks;
      });
    };
    cost_sort(b.lists[L_SYNC]);
    cost_sort(b.lists[L_HUFF]);
  }
  for (uint32_t j = 0; j < (uint32_t)b.gjobs.size(); j++)
    for (uint32_t pc = 0; pc * kGatherPiece < b.gjobs[j].len; pc++) b.lists[L_GATHER].push_back({j, pc});
  if (b.uf_n) {  // unfilter bands in ticket order: the j-th band of every plane, j = 0, 1, ...
    std::vector<std::vector<uint32_t>> per;  // per PNG image: pass << 24 | band, pass-major
    std::vector<uint32_t> who;
    for (uint32_t di = 0; di < (uint32_t)b.descs.size(); di++) {
      const ImageDesc &d = b.descs[di];
      if (d.fmt != kFmtPng) continue;
      std::vector<uint32_t> v;
      for (uint32_t p = 0; p < (d.png.interlace ? 7u : 1u); p++) {
        const uint32_t nb = png_pass_bands(d, p);
        for (uint32_t k = 0; k < nb; k++) v.push_back(p << 24 | k);
      }
      per.push_back(std::move(v));
      who.push_back(di);
    }
    for (size_t j = 0, more = 1; more; j++) {
      more = 0;
      for (size_t i = 0; i < per.size(); i++)
        if (j < per[i].size()) {
          b.lists[L_UNF].push_back({who[i], per[i][j]});
          more = 1;
        }
    }
  }
  b.prog_level_n.clear();
  for (uint32_t j = 0; j < (uint32_t)b.pscans.size(); j++) {  // L_PROG: scans grouped by level
    const uint32_t lv = b.pscans[j].level;
    if (lv >= b.prog_level_n.size()) b.prog_level_n.resize(lv + 1, 0);
    b.prog_level_n[lv]++;
  }
  b.prog_dc_n = 0;
  if (prog_pipe_) {
    plan_prog_items(b);
  } else {  // one launch per level: scans grouped by level
    std::vector<uint32_t> at(b.prog_level_n.size(), 0);
    for (size_t lv = 1; lv < at.size(); lv++) at[lv] = at[lv - 1] + b.prog_level_n[lv - 1];
    b.lists[L_PROG].resize(b.pscans.size());
    for (uint32_t j = 0; j < (uint32_t)b.pscans.size(); j++)
      b.lists[L_PROG][at[b.pscans[j].level]++] = WgItem{b.pscans[j].image, j};
  }
  for (int c = 0; c < 2; c++) {
    b.decclass[c] = (uint32_t)decl[c].size();
    b.lists[L_DEC].insert(b.lists[L_DEC].end(), decl[c].begin(), decl[c].end());
  }
  for (int c = 0; c < 2; c++) {
    b.hvclass[c] = (uint32_t)hvl[c].size();
    b.lists[L_RHV].insert(b.lists[L_RHV].end(), hvl[c].begin(), hvl[c].end());
  }
  for (int h = 0; h < 2; h++)
    for (int f = 1; f >= 0; f--)  // launch order (launch_resize_hm): fused KS 1, KS 2, byte-fill KS 1, KS 2
      for (int k = 0; k < 2; k++) {
        b.hmclass[h][f][k] = (uint32_t)hm[h][f][k].size();
        auto &l = b.lists[h ? L_RM2 : L_RM0];
        l.insert(l.end(), hm[h][f][k].begin(), hm[h][f][k].end());
      }
  for (int h = 0; h < 2; h++)
    for (int f = 1; f >= 0; f--)  // launch order: fused classes, then byte-fill classes
      for (int c = 0; c < 4; c++) {
        b.hclass[h][f][c] = (uint32_t)hb[h][f][c].size();
        auto &l = b.lists[h ? L_RH2 : L_RH0];
        l.insert(l.end(), hb[h][f][c].begin(), hb[h][f][c].end());
      }
  phase(3);
  // ---- 6. meta buffer: [flags][descs][lists...]
  Layout M;
  b.flags_off = M.take(sizeof(BatchFlags));
  b.desc_off = M.take(b.descs.size() * sizeof(ImageDesc));
  for (int l = 0; l < L_COUNT; l++) b.list_off[l] = M.take(b.lists[l].size() * sizeof(WgItem));
  b.gjob_off = M.take(b.gjobs.size() * sizeof(GatherJob));
  b.ichunk_off = M.take(b.ichunks.size() * sizeof(InfChunk));
  b.pscan_off = M.take(b.pscans.size() * sizeof(ProgScan));
  b.blob_off = M.take(b.blob.size());
  b.meta_bytes = align_up(M.off, 256);  // the host inputs follow, 16-byte aligned for k_meta_pull
  st = ensure(sl.meta, b.meta_bytes + 256, sl.st);
  if (st) return st;
  for (ImageDesc &d : b.descs) {
    if (d.fmt == kFmtPng && d.png.pal) d.png.pal = (uint64_t)(uintptr_t)((char *)sl.meta.p + b.blob_off + d.png.pal - 1);
    if (d.enc.active) {
      d.enc.hdr = (uint64_t)(uintptr_t)((char *)sl.meta.p + b.blob_off + d.enc.hdr - 1);
      d.enc.tab = (uint64_t)(uintptr_t)((char *)sl.meta.p + b.blob_off + b.enctab_off);
    }
  }
  size_t stage_bytes = b.meta_bytes + (host_io ? IN.off : 0);
  st = ensure_pinned(sl.stage, stage_bytes + 256, sl.st);
  if (st) return st;
  char *P = (char *)sl.stage.p;
  memset(P + b.flags_off, 0, sizeof(BatchFlags));
  b.ptime_off = 0;
  if (wg_timing_) {
    const size_t nrec = b.lists[L_SYNC].size() + b.lists[L_HUFF].size();
    b.ptime_off = b.pscans.empty() ? 0 : nrec * 16 + 64;  // per-scan {start, end} after the entropy records
    st = ensure(sl.wgt, nrec * 16 + 64 + b.pscans.size() * 16, sl.st);
    if (st) return st;
    BatchFlags *bf = (BatchFlags *)(P + b.flags_off);
    bf->wgtime = (uint64_t)(uintptr_t)sl.wgt.p;
    bf->wgtime_write = (uint32_t)b.lists[L_SYNC].size();
  }
  ((BatchFlags *)(P + b.flags_off))->debug = (uint32_t)(debug_flags_ >> 16) & 3u;
  ((BatchFlags *)(P + b.flags_off))->prio = (uint32_t)entropy_prio_;
  ((BatchFlags *)(P + b.flags_off))->idct_list = (uint64_t)(uintptr_t)((char *)sl.scratch.p + idct_list_off);
  ((BatchFlags *)(P + b.flags_off))->idct_cap = b.idct_cap;
  memcpy(P + b.desc_off, b.descs.data(), b.descs.size() * sizeof(ImageDesc));
  for (int l = 0; l < L_COUNT; l++)
    if (!b.lists[l].empty()) memcpy(P + b.list_off[l], b.lists[l].data(), b.lists[l].size() * sizeof(WgItem));
  if (!b.gjobs.empty()) memcpy(P + b.gjob_off, b.gjobs.data(), b.gjobs.size() * sizeof(GatherJob));
  if (!b.ichunks.empty()) memcpy(P + b.ichunk_off, b.ichunks.data(), b.ichunks.size() * sizeof(InfChunk));
  if (!b.pscans.empty()) memcpy(P + b.pscan_off, b.pscans.data(), b.pscans.size() * sizeof(ProgScan));
  if (!b.blob.empty()) memcpy(P + b.blob_off, b.blob.data(), b.blob.size());
  if (host_io) {
    std::vector<CopyJob> ins;
    for (int i = 0; i < n; i++)
      if (b.desc_of[i] >= 0) ins.push_back({P + b.meta_bytes + in_off[i], h_srcs[i], lens[i]});
    parallel_copy(ins, copy_threads_);
  }
  last_meta_bytes_ = b.meta_bytes;
  phase(4);
  if (timing_) HIPCHK(hipEventRecord(sl.ev[0], sl.st));
  if (meta_pull_ >= 1) {
    launch_meta_pull(sl.st, P, sl.meta.p, b.meta_bytes);
    HIPCHK(hipGetLastError());
  } else {
    HIPCHK(hipMemcpyAsync(sl.meta.p, P, b.meta_bytes, hipMemcpyHostToDevice, sl.st));
  }
  if (host_io && IN.off) {  // the coded inputs (dg_submit / dg_decode_one)
    if (meta_pull_ >= 2) {  // off by default: dg_decode_one 18.1 -> 16.6 Gpx/s with it (profiles/r04/one_r4i)
      launch_meta_pull(sl.st, P + b.meta_bytes, sl.input.p, IN.off);
      HIPCHK(hipGetLastError());
    } else {
      HIPCHK(hipMemcpyAsync(sl.input.p, P + b.meta_bytes, IN.off, hipMemcpyHostToDevice, sl.st));
    }
  }
  b.stage_ms.clear();
  sl.subs_off = subs_off;  // SubStates and checkpoints live in the scratch arena
  sl.ckpt_off = ckpt_off;
  if (host_io) {
    b.host_outs.assign(outs, outs + n);
    b.host_caps.assign(caps, caps + n);
    // outputs into page-locked caller memory go there by DMA, not via the staging buffer
    for (int i = 0; i < n; i++)
      if (b.desc_of[i] >= 0 && !b.plans[i].encode && b.plans[i].out_bytes && outs[i] &&
          host_pinned(outs[i], b.plans[i].out_bytes))
        b.out_direct[i] = 1;
  }
  sl.batch = std::move(bp);
  croll.armed = false;
  phase(5);
  st = launch_all(sl, false);
  if (st) {
    fail_batch(sl, st);
    return st;
  }
  phase(6);
  stat_batches_++;
  *ticket = sl.batch->ticket;
  if ((!max_dev_bytes_ || budget_planned_) && stat_batches_ <= 2 * kMaxInflight) prewarm_slots(sl);
  return DG_OK;
}

// The first batches (no budget): the idle baseline slots in turn take the
// buffers and streams the submitting slot has, exactly sized, while its batch
// runs -- so a slot's first batch does not pay for its streams, hipMalloc /
// hipHostMalloc and growth steps (the headline's fourth slot did, inside the
// first timed window: 110 vs 115-117 Gpx/s in the other four windows).
void Context::prewarm_slots(const Slot &self) {
  if (&self - slots_ >= kMaxInflight) return;
  const int ns = max_dev_bytes_ ? std::max(1, std::min(nslots_, budget_slots_)) : nslots_;
  for (int j = 0; j < ns; j++) {
    Slot &o = slots_[j];
    if (&o == &self || (o.batch && !o.batch->done)) continue;
    if (slot_streams(o)) return;
    if (self.views) {  // planned budget: the slot's arena
      if (ensure(o.arena, self.arena.cap, nullptr, true) || ensure(o.meta, self.meta.cap, nullptr, true) ||
          ensure(o.wgt, self.wgt.cap, nullptr, true) || ensure_pinned(o.stage, self.stage.cap, nullptr, true) ||
          ensure_pinned(o.out, self.out.cap, nullptr, true))
        return;
      continue;
    }
    if (ensure(o.scratch, self.scratch.cap, nullptr, true) || ensure(o.coef, self.coef.cap, nullptr, true) ||
        ensure(o.input, self.input.cap, nullptr, true) || ensure(o.meta, self.meta.cap, nullptr, true) ||
        ensure(o.wgt, self.wgt.cap, nullptr, true) || ensure_pinned(o.stage, self.stage.cap, nullptr, true) ||
        ensure_pinned(o.out, self.out.cap, nullptr, true))
      return;
  }
}

// A slot for the next batch: the next in turn, whose batch the caller then
// finishes first.  Progressive batches have slots of their own
// (pick_prog_slot), so every baseline slot cycles at the baseline pace.
int Context::pick_slot() {
  // the planned budget's first sizing runs on slot 0 (budget_planned_fit sizes
  // slots [0, budget_slots_)); submissions split before it keep that slot
  if (max_dev_bytes_ && budget_plan_ && !budget_planned_) {
    next_slot_ = 0;
    return 0;
  }
  const int ns = max_dev_bytes_ ? std::max(1, std::min(nslots_, budget_slots_)) : nslots_;
  const int i = next_slot_ % ns;
  next_slot_ = (i + 1) % ns;
  return i;
}

// A progressive slot: the first idle one, else the next in turn (whose batch
// the caller then waits for: backpressure on the progressive lane only).
int Context::pick_prog_slot() {
  for (int j = 0; j < kProgSlots; j++) {
    const int k = kMaxInflight + (next_pslot_ + j) % kProgSlots;
    const Slot &s = slots_[k];
    if (!s.batch || s.batch->done || hipEventQuery(s.done) == hipSuccess) {
      next_pslot_ = (next_pslot_ + j + 1) % kProgSlots;
      return k;
    }
  }
  const int k = kMaxInflight + next_pslot_;
  next_pslot_ = (next_pslot_ + 1) % kProgSlots;
  return k;
}

// Work items of the pipelined progressive launch (dg_prog.hip k_prog_scan).
// Scans of one image that share no (component, coefficient band) never wait
// on each other, so the connected groups of the dependency graph -- for a
// colour file the DC scans, and the AC scans of each component -- can each
// run back to back in one wave (a chain, ProgScan::next).  A chained scan
// never waits: its deps ran before it in the same wave.  That is the whole
// point: with one wave per scan, an image's later scans sit resident for its
// whole duration waiting on their producers' rows (10 waves per image for
// libjpeg's default script), and the batch's LDS-bound residency went to
// waiting waves.  A group whose decode costs more than prog_chain % of the
// batch's longest single scan (the long pole when every scan is pipelined)
// keeps one wave per scan and the row pipeline, so chaining never lengthens
// the batch.  Cost model: coded bytes + blocks / 2.  Items needing more than
// one Huffman table in LDS (DC-first scans of several components) go last
// (prog_dc_n) and run in a launch of their own with four tables.  Order:
// pipelined scans first (image by image, largest first, each in level order:
// a scan only ever waits on one with a lower ticket), then chains, costliest
// first.
void Context::plan_prog_items(Batch &b) {
  auto &list = b.lists[L_PROG];
  list.clear();
  const uint32_t n = (uint32_t)b.pscans.size();
  if (!n) return;
  std::vector<double> cost(n);
  double longest = 0;
  for (uint32_t j = 0; j < n; j++) {
    const ProgScan &sc = b.pscans[j];
    const ImageDesc &d = b.descs[sc.image];
    uint64_t blocks;
    if (sc.ns == 1) {
      const uint32_t c = sc.comp[0];
      blocks = (uint64_t)((d.cdsw[c] + 7) / 8) * ((d.cdsh[c] + 7) / 8);
    } else {
      blocks = (uint64_t)d.mcux * d.mcuy * d.bpm;
    }
    cost[j] = (double)sc.len + 0.5 * (double)blocks;
    longest = std::max(longest, cost[j]);
  }
  std::vector<uint32_t> par(n);
  for (uint32_t j = 0; j < n; j++) par[j] = j;
  auto find = [&](uint32_t x) {
    while (par[x] != x) x = par[x] = par[par[x]];
    return x;
  };
  // groups: scans of one image sharing a component and an overlapping band
  // (the deps relation, computed directly: files with more than
  // kProgMaxDepScans scans have no deps mask and run chained only)
  std::vector<uint8_t> nodeps(b.descs.size(), 0);
  for (uint32_t j = 0; j < n; j++) {
    const ProgScan &sj = b.pscans[j];
    if (sj.image < nodeps.size() && b.descs[sj.image].prog > kProgMaxDepScans) nodeps[sj.image] = 1;
    for (uint32_t e = sj.first; e < j; e++) {
      const ProgScan &se_ = b.pscans[e];
      if (se_.se < sj.ss || sj.se < se_.ss) continue;
      bool share = false;
      for (uint32_t x = 0; x < se_.ns && x < 4; x++)
        for (uint32_t y = 0; y < sj.ns && y < 4; y++) share |= se_.comp[x] == sj.comp[y];
      if (!share) continue;
      const uint32_t a = find(j), c = find(e);
      if (a != c) par[std::max(a, c)] = std::min(a, c);
    }
  }
  struct Group {
    std::vector<uint32_t> scans;  // ascending: every dep of a scan comes before it
    double cost = 0;
    bool dc = false;
  };
  std::vector<Group> groups;
  std::vector<int32_t> gi(n, -1);
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t r = find(j);
    if (gi[r] < 0) {
      gi[r] = (int32_t)groups.size();
      groups.emplace_back();
    }
    Group &g = groups[gi[r]];
    const ProgScan &sc = b.pscans[j];
    g.scans.push_back(j);
    g.cost += cost[j];
    g.dc |= (sc.ss == 0 && sc.ah == 0 ? sc.ns : (sc.ss == 0 ? 0u : 1u)) > 1;
  }
  const double limit = longest * (double)prog_chain_ / 100.0;
  std::vector<uint32_t> split[2];            // pipelined scans, AC / DC launch
  std::vector<std::pair<double, uint32_t>> chains[2];  // (cost, group)
  std::vector<double> img_cost(b.descs.size(), 0.0);
  for (uint32_t j = 0; j < n; j++) img_cost[b.pscans[j].image] += cost[j];
  for (uint32_t g = 0; g < (uint32_t)groups.size(); g++) {
    Group &G = groups[g];
    if ((prog_chain_ > 0 && G.cost <= limit) || nodeps[b.pscans[G.scans[0]].image]) {
      for (size_t i = 0; i < G.scans.size(); i++) {
        ProgScan &sc = b.pscans[G.scans[i]];
        sc.pflags |= kProgChained;
        sc.next = i + 1 < G.scans.size() ? G.scans[i + 1] : kProgNoScan;
      }
      chains[G.dc].push_back({G.cost, g});
    } else {
      for (uint32_t j : G.scans) split[G.dc].push_back(j);
    }
  }
  for (int dc = 0; dc < 2; dc++) {
    std::stable_sort(split[dc].begin(), split[dc].end(), [&](uint32_t x, uint32_t y) {
      const ProgScan &a = b.pscans[x], &c = b.pscans[y];
      if (a.image != c.image) {
        if (img_cost[a.image] != img_cost[c.image]) return img_cost[a.image] > img_cost[c.image];
        return a.image < c.image;
      }
      if (a.level != c.level) return a.level < c.level;
      return x < y;
    });
    std::stable_sort(chains[dc].begin(), chains[dc].end(),
                     [](const auto &x, const auto &y) { return x.first > y.first; });
  }
  for (int dc = 0; dc < 2; dc++) {
    for (uint32_t j : split[dc]) list.push_back(WgItem{b.pscans[j].image, j});
    for (const auto &c : chains[dc]) {
      const uint32_t j = groups[c.second].scans[0];
      list.push_back(WgItem{b.pscans[j].image, j});
    }
  }
  b.prog_dc_n = (uint32_t)(split[1].size() + chains[1].size());
  stat_prog_items_ += list.size();
  stat_prog_chains_ += chains[0].size() + chains[1].size();
}

dg_status Context::launch_all(Slot &sl, bool from_fix) {
  Batch &b = *sl.batch;
  char *M = (char *)sl.meta.p;
  const ImageDesc *dd = (const ImageDesc *)(M + b.desc_off);
  ImageDesc *dm = (ImageDesc *)(M + b.desc_off);
  BatchFlags *fl = (BatchFlags *)(M + b.flags_off);
  SubState *subs = (SubState *)((char *)sl.scratch.p + sl.subs_off);
  const HuffTable *hp = b.hp;  // the pool generation this batch was planned against
  const QuantTable *qp = b.qp;
  auto lst = [&](int l) { return (const WgItem *)(M + b.list_off[l]); };
  auto cnt = [&](int l) { return (uint32_t)b.lists[l].size(); };
  auto ev = [&](int i) -> dg_status {
    if (timing_) HIPCHK(hipEventRecord(sl.ev[i], sl.st));
    return DG_OK;
  };
  if (from_fix) HIPCHK(hipMemsetAsync(fl, 0, kFlagCounters, sl.st));
  int evi = 1;  // event i closes stage i-1 (kStageNames)
  auto next = [&]() -> dg_status { return ev(evi++); };
  // a resync round re-runs everything downstream of the entropy decode; the
  // decoded images themselves (PNG, alpha programs on them) are not redone
  const int alpha_flags = from_fix ? 1 : 0;
  if (next()) return DG_ERR_DEVICE;
  if (!from_fix && b.any_png) {
    launch_png_gather(sl.st, (const GatherJob *)(M + b.gjob_off), lst(L_GATHER), cnt(L_GATHER));
    if (!b.ichunks.empty()) {
      // streams too small to chunk (masks) inflate serially on the side stream,
      // beside the chunked kernels (which leave most CUs idle); chunked images
      // the resolve gives up on follow on the main stream
      const bool beside = side_stream_;
      if (beside) {
        HIPCHK(hipEventRecord(sl.ev_png0, sl.st));
        HIPCHK(hipStreamWaitEvent(sl.side, sl.ev_png0, 0));
        launch_png_inflate(sl.side, dm, lst(L_PNG), cnt(L_PNG), 0, fl, ncu_);
        HIPCHK(hipEventRecord(sl.ev_png1, sl.side));
      }
      InfChunk *ich = (InfChunk *)(M + b.ichunk_off);
      launch_inf_find(sl.st, dd, ich, lst(L_INF_FIND), cnt(L_INF_FIND), inf_stage3_);
      launch_inf_decode(sl.st, dd, ich, (uint32_t)b.ichunks.size(), inf_decode_);
      launch_inf_resolve(sl.st, dm, ich, lst(L_INF_RES), cnt(L_INF_RES));
      launch_png_inflate(sl.st, dm, lst(L_PNG), cnt(L_PNG), beside ? 1 : 2, fl, ncu_);
      if (beside) HIPCHK(hipStreamWaitEvent(sl.st, sl.ev_png1, 0));
    } else {
      launch_png_inflate(sl.st, dm, lst(L_PNG), cnt(L_PNG), 2, fl, ncu_);  // serial: every stream
    }
  }
  if (next()) return DG_ERR_DEVICE;
  if (!from_fix && b.any_png) {
    if (b.uf_n) {
      uint32_t *uf = (uint32_t *)((char *)sl.scratch.p + b.uf_flags_off);
      HIPCHK(hipMemsetAsync(uf, 0, (size_t)(b.uf_n + 1) * 4, sl.st));
      launch_png_unfilter(sl.st, dm, lst(L_UNF), cnt(L_UNF), uf, ncu_, b.uf_maxbpp, (uint32_t)(debug_flags_ >> 18) & 1u,
                          uf_units_, (uint32_t)uf_per_cu_);
    }
    launch_png_expand(sl.st, dd, lst(L_EXPAND), cnt(L_EXPAND));
  }
  if (next()) return DG_ERR_DEVICE;
  if (!from_fix) {
    // Lanczos coefficient tables depend only on the plan: compute them on a
    // side stream, overlapped with the entropy decode.
    hipStream_t cs = side_stream_ ? sl.side : sl.st;
    HIPCHK(hipEventRecord(sl.ev_meta, sl.st));
    HIPCHK(hipStreamWaitEvent(cs, sl.ev_meta, 0));

    launch_coeffs(cs, dm, lst(L_COEF), cnt(L_COEF));
    HIPCHK(hipEventRecord(sl.ev_coef, cs));
    if (b.ds_state_off) {  // one pass, decoupled look-back (option "destuff_one")
      uint64_t *dst = (uint64_t *)((char *)sl.scratch.p + b.ds_state_off);
      HIPCHK(hipMemsetAsync(dst, 0, (size_t)(b.ds_n + 1) * 8, sl.st));
      launch_destuff_one(sl.st, dm, lst(L_DESTUFF), cnt(L_DESTUFF), dst);
    } else {
      launch_destuff_count(sl.st, dd, lst(L_DESTUFF), cnt(L_DESTUFF));
      launch_destuff_scan(sl.st, dm, lst(L_SCAN), cnt(L_SCAN));
      launch_destuff_write(sl.st, dd, lst(L_DESTUFF), cnt(L_DESTUFF));
    }
  }
  if (next()) return DG_ERR_DEVICE;
  // progressive JPEG: zero, then the scans (one pipelined launch, or level by
  // level).  On the side stream, beside the baseline images' entropy decode
  // (the main stream waits for it before the IDCT), except with stage timing
  // on, where every stage runs on the main stream so its events bracket it.
  const bool pside = side_stream_ && prog_side_ && !timing_ && !b.pscans.empty();
  bool dc_side = false;  // DC items on the side stream, AC items on the main one
  if (!from_fix && !b.pscans.empty()) {
    hipStream_t pst = pside ? sl.side : sl.st;
    launch_prog_zero(pst, dd, lst(L_PROG_ZERO), cnt(L_PROG_ZERO));
    const ProgScan *ps = (const ProgScan *)(M + b.pscan_off);
    const uint32_t prog_dbg = ((uint32_t)(debug_flags_ >> 19) & 1u) << 1;  // forced wait timeouts (tests)
    uint64_t *pt = b.ptime_off ? (uint64_t *)((char *)sl.wgt.p + b.ptime_off) : nullptr;
    if (prog_pipe_) {
      // AC items (one Huffman table in LDS) and DC items (four) in launches of
      // their own; no scan of one waits on a scan of the other
      uint32_t *pf = (uint32_t *)((char *)sl.scratch.p + b.pf_off);
      HIPCHK(hipMemsetAsync(pf, 0, (size_t)(b.pf_n + 2) * 4, pst));
      const uint32_t nac = cnt(L_PROG) - b.prog_dc_n, sflags = (prog_serial_ ? 1u : 0u) | prog_dbg;
      hipStream_t dst = pst;
      if (!pside && side_stream_ && b.prog_dc_n && nac) {  // DC items beside the AC launch (also when timing:
                                                          // the IDCT stage then holds what the DC items outlast)
        HIPCHK(hipEventRecord(sl.ev_zero, pst));
        HIPCHK(hipStreamWaitEvent(sl.side, sl.ev_zero, 0));
        dst = sl.side;
        dc_side = true;
      }
      launch_prog_scan(pst, dd, ps, lst(L_PROG), nac, hp, sflags, pf, pf, pt, 1);
      launch_prog_scan(dst, dd, ps, lst(L_PROG) + nac, b.prog_dc_n, hp, sflags, pf, pf + b.pf_n + 1, pt, 4);
      if (dc_side) HIPCHK(hipEventRecord(sl.ev_prog, sl.side));
    } else {
      uint32_t at = 0;
      for (uint32_t nl : b.prog_level_n) {
        launch_prog_scan(pst, dd, ps, lst(L_PROG) + at, nl, hp, prog_serial_ ? 1u : 0u, nullptr, nullptr, pt, 4);
        at += nl;
      }
    }
    if (pside) HIPCHK(hipEventRecord(sl.ev_prog, sl.side));
  }
  if (next()) return DG_ERR_DEVICE;
  Ckpt *ck = (Ckpt *)((char *)sl.scratch.p + sl.ckpt_off);
  if (!from_fix)
    launch_huff_sync(sl.st, dd, lst(L_SYNC), cnt(L_SYNC), hp, subs, ck, fl, b.stage_on, b.max_slots,
                     multi_lead_ ? b.max_ac : 0u, sync_pair_, sync2_);
  if (next()) return DG_ERR_DEVICE;
  launch_huff_fix(sl.st, dd, lst(L_SYNC), cnt(L_SYNC), hp, subs, ck, fl, b.stage_on, b.max_slots);
  if (next()) return DG_ERR_DEVICE;
  launch_huff_scan(sl.st, dm, lst(L_SCAN), cnt(L_SCAN), subs);
  if (next()) return DG_ERR_DEVICE;
  if (b.stage_on)
    launch_huff_scatter(sl.st, dd, lst(L_HUFF), cnt(L_HUFF), subs);
  else
    launch_huff_write(sl.st, dm, lst(L_HUFF), cnt(L_HUFF), hp, subs, fl, b.max_slots, qp, (uint32_t)write_pair_, ck);
  if (next()) return DG_ERR_DEVICE;
  if (next()) return DG_ERR_DEVICE;  // coeffs (side stream)
  if (pside || dc_side) HIPCHK(hipStreamWaitEvent(sl.st, sl.ev_prog, 0));  // progressive coefficients
  if (b.any_fused) launch_idct_list(sl.st, dd, qp, fl, std::min<uint32_t>(2048u, (b.idct_cap + 31) / 32));
  if (idct_thread_)
    launch_idct_t(sl.st, dd, lst(L_IDCT), cnt(L_IDCT), qp);
  else
    launch_idct(sl.st, dd, lst(L_IDCT), cnt(L_IDCT), qp);
  if (next()) return DG_ERR_DEVICE;
  launch_color(sl.st, dd, lst(L_COLOR), cnt(L_COLOR));
  if (next()) return DG_ERR_DEVICE;
  HIPCHK(hipStreamWaitEvent(sl.st, sl.ev_coef, 0));
  launch_alpha(sl.st, dd, lst(L_ALPHA0), cnt(L_ALPHA0), 0 | (alpha_flags << 8));
  launch_band_dec(sl.st, dd, lst(L_DEC), b.decclass, qp, dec_strips_ | (dec_dbg_ << 16));
  launch_resize_hm(sl.st, dd, lst(L_RM0), b.hmclass[0], 0);
  launch_resize_hb(sl.st, dd, lst(L_RH0), b.hclass[0], 0, h_prefetch_, h_planar_, b.h_zune != 0);
  launch_resize_hv(sl.st, dd, lst(L_RHV), b.hvclass);
  launch_resize_h(sl.st, dd, lst(L_RHX0), cnt(L_RHX0), 0 | ((debug_flags_ & 0xFF) << 8));
  if (next()) return DG_ERR_DEVICE;
  launch_resize_v(sl.st, dd, lst(L_RV1), cnt(L_RV1), 1, v_units_);
  launch_resize_vt(sl.st, dd, lst(L_RVT1), cnt(L_RVT1), 1, b.v_tile);
  launch_alpha(sl.st, dd, lst(L_ALPHA1), cnt(L_ALPHA1), 1 | (alpha_flags << 8));
  if (next()) return DG_ERR_DEVICE;
  launch_resize_hm(sl.st, dd, lst(L_RM2), b.hmclass[1], 2);
  launch_resize_hb(sl.st, dd, lst(L_RH2), b.hclass[1], 2, h_prefetch_, h_planar_, b.h_zune != 0);
  launch_resize_h(sl.st, dd, lst(L_RHX2), cnt(L_RHX2), 2 | ((debug_flags_ & 0xFF) << 8));
  if (next()) return DG_ERR_DEVICE;
  launch_resize_v(sl.st, dd, lst(L_RV3), cnt(L_RV3), 3, v_units_);
  launch_resize_vt(sl.st, dd, lst(L_RVT3), cnt(L_RVT3), 3, b.v_tile);
  launch_alpha(sl.st, dd, lst(L_ALPHA2), cnt(L_ALPHA2), 2 | (alpha_flags << 8));
  if (next()) return DG_ERR_DEVICE;
  launch_copy(sl.st, dd, lst(L_COPY), cnt(L_COPY));
  if (next()) return DG_ERR_DEVICE;
  if (b.any_enc) {
    HIPCHK(hipMemsetAsync((char *)sl.scratch.p + b.words_off, 0, b.words_bytes, sl.st));
    launch_enc_fdct(sl.st, dd, lst(L_ENC_MCU), cnt(L_ENC_MCU));
    launch_enc_count(sl.st, dd, lst(L_ENC_BLK), cnt(L_ENC_BLK));
    launch_penc_filter(sl.st, dd, lst(L_PENC_ROW), cnt(L_PENC_ROW));
    launch_penc_count(sl.st, dd, lst(L_PENC_PIECE), cnt(L_PENC_PIECE));
    launch_enc_scan(sl.st, dm, lst(L_ENC_IMG), cnt(L_ENC_IMG));
    launch_enc_write(sl.st, dd, lst(L_ENC_BLK), cnt(L_ENC_BLK));
    launch_penc_write(sl.st, dd, lst(L_PENC_PIECE), cnt(L_PENC_PIECE));
    launch_enc_stuff(sl.st, dm, lst(L_ENC_IMG), cnt(L_ENC_IMG));
    launch_penc_final(sl.st, dm, lst(L_PENC_IMG), cnt(L_PENC_IMG));
  }
  if (next()) return DG_ERR_DEVICE;
  HIPCHK(hipGetLastError());
  // read back flags + per-image status (descs) for finish(), then outputs (host path)
  size_t back = b.desc_off + b.descs.size() * sizeof(ImageDesc);
  size_t total = align_up(back, 256);
  if (b.host_io)
    for (int i = 0; i < b.n; i++)
      if (b.desc_of[i] >= 0 && !b.plans[i].encode && !b.out_direct[i]) total += align_up(b.plans[i].out_bytes, 16);
  dg_status st = ensure_pinned(sl.out, total + 256, sl.st);
  if (st) return st;
  HIPCHK(hipMemcpyAsync(sl.out.p, M, back, hipMemcpyDeviceToHost, sl.st));
  if (b.host_io) {
    size_t off = align_up(back, 256);
    for (int i = 0; i < b.n; i++) {
      if (b.desc_of[i] < 0 || b.plans[i].encode) continue;  // encoded: exact size copied in finish()
      if (b.out_direct[i]) {  // DMA straight into the caller's page-locked buffer
        HIPCHK(hipMemcpyAsync(b.host_outs[i], (char *)sl.scratch.p + b.out_dev_off[i], b.plans[i].out_bytes,
                              hipMemcpyDeviceToHost, sl.st));
        continue;
      }
      HIPCHK(hipMemcpyAsync((char *)sl.out.p + off, (char *)sl.scratch.p + b.out_dev_off[i], b.plans[i].out_bytes,
                            hipMemcpyDeviceToHost, sl.st));
      off += align_up(b.plans[i].out_bytes, 16);
    }
  }
  if (next()) return DG_ERR_DEVICE;  // download
  HIPCHK(hipEventRecord(sl.done, sl.st));
  HIPCHK(hipEventRecord(b.fin->e, sl.st));
  return DG_OK;
}

// A batch that cannot complete (a launch, resync or copy-back failure): no
// kernel of it is left running, every image not already failed reads `st`,
// deferred metas are published, and the batch counts as done -- a later
// submit on the slot must not finish() it again and publish planning-time
// metas over the error.
void Context::fail_batch(Slot &sl, dg_status st) {
  if (!sl.batch || sl.batch->done) return;
  for (hipStream_t q : {sl.st, sl.side})
    if (q) (void)hipStreamSynchronize(q);
  (void)hipGetLastError();
  Batch &b = *sl.batch;
  for (int i = 0; i < b.n && i < (int)b.mptr.size(); i++)
    if (b.mptr[i] && b.mptr[i]->status == DG_OK) b.mptr[i]->status = st;
  for (size_t i = 0; i < b.pub.size(); i++) *b.pub[i] = b.local_meta[i];
  // Lanczos tables this batch was producing never become ready: retire their
  // keys (the index slot stays as a tombstone, probes pass it) so that a later
  // batch produces them again instead of recomputing its own copy every time
  // until the arena starts over
  for (const Batch::CProd &pr : b.ccache_prod)
    if (pr.entry < (int)ccache_.size() && !ccache_[pr.entry].ready) {
      ccache_[pr.entry].key.ksize = 0xFFFFFFFFu;
      ccache_[pr.entry].key.in_size = 0;
    }
  b.done = true;
}

dg_status Context::finish(Slot &sl) {
  const dg_status st = finish_body(sl);
  if (st) fail_batch(sl, st);
  return st;
}

dg_status Context::finish_body(Slot &sl) {
  Batch &b = *sl.batch;
  for (;;) {
    HIPCHK(hipEventSynchronize(sl.done));
    memcpy(&b.flags, (char *)sl.out.p + b.flags_off, sizeof(BatchFlags));
    stat_fix_ += b.flags.fix_count;
    stat_mismatch_ += b.flags.write_mismatch;
    stat_iters_ = std::max<int64_t>(stat_iters_, b.flags.sync_iters_max);
    if (b.flags.idct_late > b.idct_cap) {  // never seen; would leave blocks without pixels
      b.unsettled = true;
      set_error("fused IDCT list overflow: the batch's JPEGs are returned DG_ERR_UNSUPPORTED");
    }
    if (b.flags.chain_changed == 0) break;
    if (b.resync_rounds >= kMaxResyncRounds) {
      // The boundary repair did not settle: some entropy chain of this batch
      // may be wrong, and nothing tells which image it belongs to.  Every
      // sequential JPEG not already failed goes back to the caller's CPU
      // decoder (DG_ERR_UNSUPPORTED) instead of returning pixels that may
      // be wrong.
      stat_unsettled_++;
      b.unsettled = true;
      set_error("entropy resync did not converge: the batch's JPEGs are returned DG_ERR_UNSUPPORTED");
      break;
    }
    // a workgroup's last exit state changed during the boundary repair: repeat
    // repair + everything downstream until the chain is stable
    b.resync_rounds++;
    stat_resync_++;
    dg_status st = launch_all(sl, true);
    if (st) return st;
  }
  if (b.ptime_off) {  // debug: one line per progressive scan (option wg_timing, env DG_PROG_DUMP)
    std::vector<uint64_t> rec(2 * b.pscans.size());
    HIPCHK(hipMemcpy(rec.data(), (char *)sl.wgt.p + b.ptime_off, rec.size() * 8, hipMemcpyDeviceToHost));
    if (const char *dump = getenv("DG_PROG_DUMP")) {
      if (FILE *f = fopen(dump, "a")) {
        uint64_t lo = ~0ull;
        for (size_t i = 0; i < b.pscans.size(); i++) lo = std::min(lo, rec[2 * i]);
        for (size_t i = 0; i < b.pscans.size(); i++) {
          const ProgScan &sc = b.pscans[i];
          const ImageDesc &d = b.descs[sc.image];
          fprintf(f, "%zu %u %u %u %u %u %u %u %u %u %u %llu %llu %u %u\n", i, sc.image, sc.ns, sc.comp[0], sc.ss, sc.se,
                  sc.ah, sc.al, sc.len, sc.level, (uint32_t)sc.pflags, (unsigned long long)(rec[2 * i] - lo),
                  (unsigned long long)(rec[2 * i + 1] - lo), d.total_blocks, d.width * d.height);
        }
        fprintf(f, "end\n");
        fclose(f);
      }
    }
  }
  if (b.flags.wgtime) {
    const size_t ns = b.lists[L_SYNC].size(), nw = b.lists[L_HUFF].size();
    std::vector<uint64_t> rec(2 * (ns + nw));
    HIPCHK(hipMemcpy(rec.data(), sl.wgt.p, rec.size() * 8, hipMemcpyDeviceToHost));
    if (const char *dump = getenv("DG_WG_DUMP")) {  // debug: one line per entropy workgroup
      if (FILE *f = fopen(dump, "a")) {
        uint64_t lo = ~0ull;
        for (size_t i = 0; i < ns + nw; i++) lo = std::min(lo, rec[2 * i]);
        for (size_t i = 0; i < ns + nw; i++) {
          const WgItem &w = b.lists[i < ns ? L_SYNC : L_HUFF][i < ns ? i : i - ns];
          const ImageDesc &d = b.descs[w.image];
          fprintf(f, "%d %zu %u %u %llu %llu %u %u %u %u %u %u\n", i < ns ? 0 : 1, i, w.image, w.item0,
                  (unsigned long long)(rec[2 * i] - lo), (unsigned long long)(rec[2 * i + 1] - lo), d.scan_len,
                  d.total_blocks, d.sub_bits, d.nsub, d.lead_bits, d.width * d.height);
        }
        fprintf(f, "end\n");
        fclose(f);
      }
    }
    for (int a = 0; a < 2; a++) {
      const size_t r0 = a ? ns : 0, n = a ? nw : ns;
      if (!n) continue;
      uint64_t lo = ~0ull, hi = 0;
      std::vector<double> d(n);
      double sum = 0;
      for (size_t i = 0; i < n; i++) {
        const uint64_t t0 = rec[2 * (r0 + i)], t1 = rec[2 * (r0 + i) + 1];
        lo = std::min(lo, t0);
        hi = std::max(hi, t1);
        d[i] = (double)(t1 - t0) * 0.01;  // 100 MHz ticks -> us
        sum += d[i];
      }
      std::sort(d.begin(), d.end());
      wgstat_[a][0] = (double)(hi - lo) * 0.01;
      wgstat_[a][1] = sum / (double)n;
      wgstat_[a][2] = d[(size_t)(0.9 * (double)(n - 1))];
      wgstat_[a][3] = d.back();
    }
  }
  if (timing_) {
    last_ms_.assign(kNumStages, 0.f);
    for (int i = 0; i < kNumStages; i++) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, sl.ev[i], sl.ev[i + 1]) == hipSuccess) last_ms_[i] = ms;
    }
  }
  const ImageDesc *back = (const ImageDesc *)((char *)sl.out.p + b.desc_off);
  size_t off = align_up(b.desc_off + b.descs.size() * sizeof(ImageDesc), 256);
  if (b.host_io && b.any_enc) {
    // Re-encoded payloads are known in length only now: copy all of them
    // with one async D2H each into pinned staging behind the raw outputs and
    // wait once, instead of a synchronous hipMemcpy per image.
    size_t enc_total = 0;
    for (int i = 0; i < b.n; i++)
      if (b.desc_of[i] >= 0 && b.plans[i].encode && !back[b.desc_of[i]].status)
        enc_total += align_up(back[b.desc_of[i]].enc.enc_bytes, 16);
    if (enc_total) {
      size_t raw_end = off;
      for (int i = 0; i < b.n; i++)
        if (b.desc_of[i] >= 0 && !b.plans[i].encode) raw_end += align_up(b.plans[i].out_bytes, 16);
      if (sl.out.cap < raw_end + enc_total) {  // grow keeping the read-back descriptors and raw outputs
        std::vector<char> keep((char *)sl.out.p, (char *)sl.out.p + raw_end);
        dg_status st = ensure_pinned(sl.out, raw_end + enc_total + 256, sl.st);
        if (st) return st;
        memcpy(sl.out.p, keep.data(), keep.size());
        back = (const ImageDesc *)((char *)sl.out.p + b.desc_off);
      }
      size_t eo = raw_end;
      for (int i = 0; i < b.n; i++) {
        if (b.desc_of[i] < 0 || !b.plans[i].encode || back[b.desc_of[i]].status) continue;
        const uint32_t nb = back[b.desc_of[i]].enc.enc_bytes;
        HIPCHK(hipMemcpyAsync((char *)sl.out.p + eo, (char *)sl.scratch.p + b.out_dev_off[i], nb,
                              hipMemcpyDeviceToHost, sl.st));
        b.enc_host_off.resize(b.n, 0);
        b.enc_host_off[i] = eo;
        eo += align_up(nb, 16);
      }
      HIPCHK(hipStreamSynchronize(sl.st));
    }
  }
  for (const Batch::CProd &pr : b.ccache_prod) {  // tables this batch wrote into the cache: hits from now on
    if (pr.entry >= (int)ccache_.size()) continue;
    CEntry &e = ccache_[pr.entry];
    e.precision = back[pr.desc].pass[pr.stage].precision;
    e.ready = e.precision > 0;
  }
  std::vector<CopyJob> copies;
  for (int i = 0; i < b.n; i++) {
    if (b.desc_of[i] < 0) continue;
    int status = back[b.desc_of[i]].status;
    if (back[b.desc_of[i]].fmt == kFmtPng && back[b.desc_of[i]].png.nchunks) {
      stat_png_chunks_ += back[b.desc_of[i]].png.nchunks;
      stat_png_serial_ += back[b.desc_of[i]].png.serial ? 1 : 0;
    } else if (back[b.desc_of[i]].fmt == kFmtPng) {
      stat_png_small_++;
    }
    if (!status && b.unsettled && b.plans[i].fmt == kFmtJpeg && !b.plans[i].hdr.progressive)
      status = DG_ERR_UNSUPPORTED;
    if (status) b.mptr[i]->status = status;
    if (b.plans[i].encode) {
      const uint32_t nb = back[b.desc_of[i]].enc.enc_bytes;
      b.mptr[i]->nbytes = nb;
      if (b.host_io && !status && nb) copies.push_back({b.host_outs[i], (char *)sl.out.p + b.enc_host_off[i], nb});
      continue;
    }
    if (b.host_io && b.out_direct[i]) {
      stat_direct_d2h_++;
    } else if (b.host_io) {
      if (!status) copies.push_back({b.host_outs[i], (char *)sl.out.p + off, b.plans[i].out_bytes});
      off += align_up(b.plans[i].out_bytes, 16);
    }
  }
  parallel_copy(copies, copy_threads_);
  for (size_t i = 0; i < b.pub.size(); i++) *b.pub[i] = b.local_meta[i];  // defer_meta: publish now
  b.done = true;
  return DG_OK;
}

Slot *Context::find(uint64_t ticket) {
  for (Slot &sl : slots_)
    if (sl.batch && sl.batch->ticket == ticket) return &sl;
  return nullptr;
}

dg_status Context::wait(uint64_t ticket) {
  std::shared_ptr<BatchEvent> fin;
  {
    std::lock_guard<std::mutex> lk(mu_);
    HIPCHK(hipSetDevice(device_));
    Slot *sl = find(ticket);
    if (!sl) return ticket < next_ticket_ ? DG_OK : DG_ERR_INVALID;  // already recycled => completed
    if (sl->batch->done) return DG_OK;
    fin = sl->batch->fin;
  }
  // block on the GPU without holding the context lock, so other threads can
  // plan and submit meanwhile (the batch's own event: if the slot is
  // recycled first, the ticket then reads as completed)
  HIPCHK(hipEventSynchronize(fin->e));
  std::lock_guard<std::mutex> lk(mu_);
  Slot *sl = find(ticket);
  if (!sl) return ticket < next_ticket_ ? DG_OK : DG_ERR_INVALID;
  if (sl->batch->done) return DG_OK;
  const dg_status st = finish(*sl);
  if (!st) free_retired_if_idle();
  return st;
}

dg_status Context::flush_batch(std::vector<OneReq *> &batch, bool prog) {
  const int n = (int)batch.size();
  std::vector<const uint8_t *> srcs(n);
  std::vector<size_t> lens(n);
  std::vector<int32_t> forced(n);
  std::vector<uint8_t *> outs(n);
  std::vector<uint64_t> caps(n);
  std::vector<dg_payload_meta> metas(n);
  for (int i = 0; i < n; i++) {
    srcs[i] = batch[i]->src;
    lens[i] = batch[i]->len;
    forced[i] = batch[i]->forced;
    outs[i] = batch[i]->out;
    caps[i] = batch[i]->cap;
  }
  std::vector<dg_payload_meta *> mp(n);
  for (int i = 0; i < n; i++) mp[i] = &metas[i];
  std::vector<uint64_t> ts;
  dg_status st = submit_split(n, srcs.data(), nullptr, lens.data(), forced.data(), outs.data(), caps.data(), mp.data(),
                              true, ts, prog, false);
  for (uint64_t t : ts) {
    const dg_status s1 = wait(t);
    if (!st) st = s1;
  }
  for (int i = 0; i < n; i++) {
    *batch[i]->meta = metas[i];
    batch[i]->st = st ? st : (dg_status)metas[i].status;
  }
  return st;
}

dg_status Context::decode_one(const uint8_t *src, size_t len, int32_t forced, uint8_t *out, uint64_t cap,
                              dg_payload_meta *meta) {
  OneReq r{src, len, forced, out, cap, meta, false, DG_OK, false};
  if (coalesce_max_ <= 1) {
    std::vector<OneReq *> one{&r};
    flush_batch(one, false);
    return r.st;
  }
  // Progressive JPEGs decode their scans serially (one wave per scan, ~0.1-1 s
  // for a large file), so they coalesce into batches of their own: a
  // baseline caller never waits behind a progressive chain, and up to
  // prog_lanes progressive batches run beside the baseline ones.
  r.prog = progressive_ && prog_lanes_ > 0 && jpeg_sniff_progressive(src, len);
  std::unique_lock<std::mutex> lk(cmu_);
  callers_++;
  std::vector<OneReq *> &q = r.prog ? ppending_ : pending_;
  q.push_back(&r);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(coalesce_us_);
  for (;;) {
    if (r.done) break;
    // flush when the batch is full, when every caller in here is already
    // waiting (nobody else can add), or at the deadline; nslots baseline
    // batches (+ prog_lanes progressive ones) in flight at most
    const int waiting = callers_ - inflight_reqs_;
    const bool ready = !q.empty() && ((int)q.size() >= coalesce_max_ ||
                                      (int)(pending_.size() + ppending_.size()) >= waiting ||
                                      std::chrono::steady_clock::now() >= deadline);
    const bool room = r.prog ? pinflight_ < prog_lanes_ : inflight_ < (coalesce_inflight_ ? coalesce_inflight_ : nslots_);
    if (ready && room && std::find(q.begin(), q.end(), &r) != q.end()) {
      std::vector<OneReq *> batch;
      const size_t take = std::min(q.size(), (size_t)coalesce_max_);
      batch.assign(q.begin(), q.begin() + take);
      q.erase(q.begin(), q.begin() + take);
      (r.prog ? pinflight_ : inflight_)++;
      inflight_reqs_ += (int)batch.size();
      stat_coalesced_batches_++;
      stat_coalesced_images_ += (int64_t)batch.size();
      lk.unlock();
      flush_batch(batch, r.prog);
      lk.lock();
      for (OneReq *x : batch) x->done = true;
      (r.prog ? pinflight_ : inflight_)--;
      inflight_reqs_ -= (int)batch.size();
      ccv_.notify_all();
      continue;
    }
    if (ready)
      ccv_.wait(lk);
    else
      ccv_.wait_until(lk, deadline);
  }
  callers_--;
  ccv_.notify_all();
  return r.st;
}

dg_status Context::poll(uint64_t ticket) {
  std::lock_guard<std::mutex> lk(mu_);
  Slot *sl = find(ticket);
  if (!sl || sl->batch->done) return DG_OK;
  hipError_t e = hipEventQuery(sl->done);
  if (e == hipErrorNotReady) return DG_ERR_NOT_READY;
  return DG_OK;
}

// ---- progressive split (dg_submit / dg_submit_device / dg_wait / dg_poll / dg_wait_ready)
//
// A refinement scan is one serial chain (dg_prog.hip): a large progressive
// file takes ~0.1-1 s, and a batch lasts as long as its longest chain.  So a
// submission with progressive members is split: its other members run as a
// batch of their own (back at the baseline pace), and its progressive members
// join the open progressive aggregate, which is submitted as one batch on a
// progressive slot once it holds prog_batch images, once it is older than
// prog_flush_us at a submit / poll / wait_ready, or as soon as a caller blocks
// on one of its members (dg_wait).  An aggregate of ~1024 files keeps
// thousands of scan chains in flight at once, where a 256-image batch with a
// few progressive members idles the GPU behind one chain.  dg_wait(ticket)
// completes both parts (the ABI's contract is unchanged); dg_wait_ready
// returns once the non-progressive part is done and leaves the progressive
// members' metas at DG_ERR_NOT_READY until a later dg_wait(ticket).

// Launch the open aggregate early (before prog_batch images) only when it is
// older than prog_flush_us AND a progressive slot is idle: while both run,
// the aggregate keeps growing (a larger launch hides more of its long pole).
bool Context::pagg_stale_locked() {
  if (pagg_.empty() || std::chrono::steady_clock::now() - pagg_t0_ < std::chrono::microseconds(prog_flush_us_))
    return false;
  std::lock_guard<std::mutex> lk(mu_);
  for (int j = 0; j < kProgSlots; j++) {
    const Slot &sl = slots_[kMaxInflight + j];
    if (!sl.batch || sl.batch->done || hipEventQuery(sl.done) == hipSuccess) return true;
  }
  return false;
}

dg_status Context::submit_split(int n, const uint8_t *const *h_srcs, const uint8_t *const *d_srcs,
                                const size_t *lens, const int32_t *forced, uint8_t *const *outs,
                                const uint64_t *caps, dg_payload_meta *const *mptrs, bool host_io,
                                std::vector<uint64_t> &tickets, bool prog, bool defer_meta, bool whole_failed) {
  if (n <= 0) return DG_OK;
  int slot = -1;
  if (prog) {
    std::lock_guard<std::mutex> lk(mu_);
    slot = pick_prog_slot();
  }
  dg_status st = kNeedSplit;
  if (!whole_failed) {  // (the caller already planned the whole submission and saw kNeedSplit)
    uint64_t t = 0;
    st = submit(n, h_srcs, d_srcs, lens, forced, outs, caps, nullptr, host_io, &t, mptrs, slot, defer_meta);
    if (st != kNeedSplit) {
      if (!st) tickets.push_back(t);
      return st;
    }
  }
  if (n == 1) {  // one image larger than the device budget: that sample fails, not the worker
    dg_payload_meta &m = *mptrs[0];
    memset(&m, 0, sizeof(m));
    m.status = DG_ERR_OOM;
    m.bucket = -1;
    stat_budget_oom_++;
    set_error("image does not fit the device memory budget (max_device_mb)");
    return DG_OK;
  }
  stat_budget_splits_++;
  const int h = n / 2;
  st = submit_split(h, h_srcs, d_srcs, lens, forced, outs, caps, mptrs, host_io, tickets, prog, defer_meta);
  if (st) return st;
  if (debug_flags_ & (1 << 24)) {  // test switch: the second part fails after the first launched
    set_error("forced failure of a split submission's second part (debug_flags bit 24)");
    return DG_ERR_DEVICE;
  }
  return submit_split(n - h, h_srcs + h, d_srcs ? d_srcs + h : nullptr, lens + h, forced ? forced + h : nullptr,
                      outs + h, caps + h, mptrs + h, host_io, tickets, prog, defer_meta);
}

dg_status Context::flush_pagg_locked() {
  if (pagg_.empty()) return DG_OK;
  const int n = (int)pagg_.size();
  std::vector<const uint8_t *> h(n), d(n);
  std::vector<size_t> lens(n);
  std::vector<int32_t> forced(n);
  std::vector<uint8_t *> outs(n);
  std::vector<uint64_t> caps(n);
  std::vector<dg_payload_meta *> mp(n);
  for (int i = 0; i < n; i++) {
    const PEntry &e = pagg_[i];
    h[i] = e.host.data();
    d[i] = e.dsrc;
    lens[i] = e.len;
    forced[i] = e.forced;
    outs[i] = e.out;
    caps[i] = e.cap;
    mp[i] = e.meta;
  }
  std::vector<uint64_t> ts;
  dg_status st = submit_split(n, h.data(), pagg_host_ ? nullptr : d.data(), lens.data(), forced.data(), outs.data(),
                              caps.data(), mp.data(), pagg_host_, ts, true, true);
  if (st) {  // the members of parts that did not launch fail now; dg_wait on their tickets returns st
    for (PEntry &e : pagg_)
      if (e.meta->status == DG_ERR_NOT_READY) e.meta->status = st;
  }
  stat_prog_aggs_++;
  stat_prog_agg_images_ += n;
  pgen_[pagg_gen_] = PGen{ts, pagg_refs_, st};
  pagg_refs_ = 0;
  pagg_gen_++;
  pagg_.clear();
  return st;
}

// A split submission failed part-way: the parts that launched
// before the failure still write into the caller's outputs (and a host-out
// part copies to them at its finish), so they complete before the error is
// returned -- the caller may free its buffers as soon as this call fails.
dg_status Context::fail_split_parts(const std::vector<uint64_t> &launched, dg_status st) {
  const std::string why = g_last_error;
  for (uint64_t t : launched) wait(t);
  set_error(why);
  return st;
}

dg_status Context::submit_user(int n, const uint8_t *const *h_srcs, const uint8_t *const *d_srcs, const size_t *lens,
                               const int32_t *forced, uint8_t *const *outs, const uint64_t *caps,
                               dg_payload_meta *metas, bool host_io, uint64_t *ticket) {
  if (!ticket) return DG_ERR_INVALID;
  std::vector<uint8_t> isp(n > 0 ? n : 0, 0);
  int np = 0;
  if (progressive_ && prog_split_ && n > 0 && h_srcs && lens && outs && caps && metas && (host_io || d_srcs))
    for (int i = 0; i < n; i++) {
      isp[i] = h_srcs[i] && jpeg_sniff_progressive(h_srcs[i], lens[i]) ? 1 : 0;
      np += isp[i];
    }
  if (!np) {
    dg_status st = submit(n, h_srcs, d_srcs, lens, forced, outs, caps, metas, host_io, ticket);
    if (st == kNeedSplit) {  // over the device budget: parts under one user ticket
      std::vector<dg_payload_meta *> mp(n);
      for (int i = 0; i < n; i++) mp[i] = &metas[i];
      SplitRec rec;
      st = submit_split(n, h_srcs, d_srcs, lens, forced, outs, caps, mp.data(), host_io, rec.tbs, false, false, true);
      if (st) return fail_split_parts(rec.tbs, st);
      std::lock_guard<std::mutex> lk(pmu_);
      {
        std::lock_guard<std::mutex> lk2(mu_);
        *ticket = next_ticket_++;
      }
      split_[*ticket] = rec;
      return DG_OK;
    }
    // a stale aggregate is launched by whoever comes by, but a baseline
    // submitter never queues behind a thread that holds the aggregate (its
    // launch may wait for a busy progressive slot)
    std::unique_lock<std::mutex> lk(pmu_, std::try_to_lock);
    if (lk.owns_lock() && pagg_stale_locked()) flush_pagg_locked();
    return st;
  }
  SplitRec rec;
  if (np < n) {  // the other members: a batch of their own
    std::vector<const uint8_t *> h, d;
    std::vector<size_t> ln;
    std::vector<int32_t> fb;
    std::vector<uint8_t *> ou;
    std::vector<uint64_t> cp;
    std::vector<dg_payload_meta *> mp;
    for (int i = 0; i < n; i++) {
      if (isp[i]) continue;
      h.push_back(h_srcs[i]);
      d.push_back(d_srcs ? d_srcs[i] : nullptr);
      ln.push_back(lens[i]);
      fb.push_back(forced ? forced[i] : -1);
      ou.push_back(outs[i]);
      cp.push_back(caps[i]);
      mp.push_back(&metas[i]);
    }
    dg_status st = submit_split((int)h.size(), h.data(), host_io ? nullptr : d.data(), ln.data(), fb.data(),
                                ou.data(), cp.data(), mp.data(), host_io, rec.tbs, false, false);
    if (st) return fail_split_parts(rec.tbs, st);
  }
  std::lock_guard<std::mutex> lk(pmu_);
  if (!pagg_.empty() && pagg_host_ != host_io) flush_pagg_locked();  // an aggregate is host- or device-fed
  if (pagg_.empty()) pagg_t0_ = std::chrono::steady_clock::now();
  pagg_host_ = host_io;
  for (int i = 0; i < n; i++) {
    if (!isp[i]) continue;
    PEntry e;
    e.host.assign(h_srcs[i], h_srcs[i] + lens[i]);  // the caller's host bytes are only valid during the call
    e.dsrc = host_io ? nullptr : d_srcs[i];
    e.len = lens[i];
    e.forced = forced ? forced[i] : -1;
    e.out = outs[i];
    e.cap = caps[i];
    e.meta = &metas[i];
    memset(e.meta, 0, sizeof(*e.meta));
    e.meta->status = DG_ERR_NOT_READY;
    e.meta->bucket = -1;
    pagg_.push_back(std::move(e));
  }
  rec.gen = pagg_gen_;
  rec.nprog = np;
  pagg_refs_++;
  {
    std::lock_guard<std::mutex> lk2(mu_);
    *ticket = next_ticket_++;  // a ticket of its own, in the batch tickets' sequence
  }
  split_[*ticket] = rec;
  // The caller's members are queued and its ticket is live.  An aggregate
  // launch started here may carry other submissions' members too: its
  // failure is recorded for their dg_wait (pgen_) and in their metas, never
  // returned from this call, whose non-progressive part is already in flight.
  if ((int)pagg_.size() >= prog_batch_ || pagg_stale_locked()) flush_pagg_locked();
  return DG_OK;
}

// A user ticket of a split submission: its baseline part(s) (several when
// the device budget split them) and, when gen != 0, the progressive
// aggregate holding its progressive members.
dg_status Context::wait_user(uint64_t ticket) {
  SplitRec rec;
  std::vector<uint64_t> tps;
  dg_status agg_st = DG_OK;
  {
    std::lock_guard<std::mutex> lk(pmu_);
    auto it = split_.find(ticket);
    if (it == split_.end()) return wait(ticket);
    rec = it->second;
    if (rec.gen && rec.gen == pagg_gen_) flush_pagg_locked();  // someone blocks on the open aggregate: launch it now
    if (rec.gen) {
      const PGen &g = pgen_[rec.gen];
      tps = g.tickets;
      agg_st = g.st;
    }
  }
  dg_status st = DG_OK;
  for (uint64_t t : rec.tbs) {
    const dg_status s1 = wait(t);
    if (!st) st = s1;
  }
  dg_status st2 = agg_st;
  for (uint64_t t : tps) {
    const dg_status s1 = wait(t);
    if (!st2) st2 = s1;
  }
  std::lock_guard<std::mutex> lk(pmu_);
  if (split_.erase(ticket) && rec.gen) {
    auto g = pgen_.find(rec.gen);
    if (g != pgen_.end() && --g->second.refs <= 0) pgen_.erase(g);
  }
  return st ? st : st2;
}

dg_status Context::wait_ready(uint64_t ticket, int32_t *pending) {
  SplitRec rec;
  {
    std::lock_guard<std::mutex> lk(pmu_);
    if (pagg_stale_locked()) flush_pagg_locked();
    auto it = split_.find(ticket);
    if (it == split_.end()) {
      if (pending) *pending = 0;
      return wait(ticket);
    }
    rec = it->second;
  }
  dg_status st = DG_OK;
  for (uint64_t t : rec.tbs) {
    const dg_status s1 = wait(t);
    if (!st) st = s1;
  }
  if (pending) {  // progressive members not complete yet (their metas read DG_ERR_NOT_READY)
    std::vector<uint64_t> tps;
    bool busy = false;
    dg_status agg_st = DG_OK;
    if (rec.gen) {
      std::lock_guard<std::mutex> lk(pmu_);
      if (rec.gen != pagg_gen_) {
        auto g = pgen_.find(rec.gen);
        if (g != pgen_.end()) {
          tps = g->second.tickets;
          agg_st = g->second.st;
        }
      }
      busy = rec.gen == pagg_gen_;
      for (uint64_t t : tps) busy = busy || poll(t) == DG_ERR_NOT_READY;
    }
    // The aggregate's kernels are done: complete it (outputs copied to host
    // buffers, statuses written, metas published) before reporting 0 pending,
    // so pending == 0 means the progressive members are ready to read.  The
    // events have completed, so this does not block (bar a rare entropy
    // resync); it runs outside pmu_, like wait_user's, so polls and waits on
    // other tickets do not queue behind the aggregate's output copies.
    dg_status st2 = agg_st;
    if (!busy)
      for (uint64_t t : tps) {
        const dg_status s1 = wait(t);
        if (!st2) st2 = s1;
      }
    *pending = busy ? rec.nprog : 0;
    if (!st) st = st2;
  }
  return st;
}

dg_status Context::poll_user(uint64_t ticket) {
  SplitRec rec;
  std::vector<uint64_t> tps;
  {
    std::lock_guard<std::mutex> lk(pmu_);
    if (pagg_stale_locked()) flush_pagg_locked();
    auto it = split_.find(ticket);
    if (it == split_.end()) return poll(ticket);
    rec = it->second;
    if (rec.gen && rec.gen == pagg_gen_) return DG_ERR_NOT_READY;
    if (rec.gen) tps = pgen_[rec.gen].tickets;
  }
  for (uint64_t t : rec.tbs)
    if (poll(t) == DG_ERR_NOT_READY) return DG_ERR_NOT_READY;
  for (uint64_t t : tps)
    if (poll(t) == DG_ERR_NOT_READY) return DG_ERR_NOT_READY;
  return DG_OK;
}

}  // namespace dg
