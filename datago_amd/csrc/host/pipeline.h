// pipeline.h — per-device context and batch runtime behind the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/datago_hip.h"
#include "../dg_types.h"
#include "buckets.h"
#include "jpeg_header.h"
#include "png_header.h"
#include "jpeg_enc.h"
#include "host_pool.h"

namespace dg {

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
};

struct PinBuf {
  void *p = nullptr;
  size_t cap = 0;
};

// Per-image host-side plan (what the host knows before the GPU runs).
struct ImagePlan {
  int status = DG_OK;
  uint32_t fmt = kFmtJpeg;
  JpegHeader hdr;
  PngHeader png;
  int bucket = -1;
  uint32_t out_w = 0, out_h = 0, out_c = 0;
  uint64_t out_bytes = 0;
  int32_t channels = 0, bit_depth = 8;
  bool encode = false;     // pre_encode_images: out holds a JPEG / PNG of at most out_bytes
  bool enc_png = false;    // encode_format png (dg_penc.hip)
  bool enc_la_gray = false;  // resized LA: encoded as the GrayImage over its bytes
  uint64_t img_bytes = 0;  // transformed image bytes (out_w * out_h * out_c)
};

// The completion event of one batch (shared with waiters, so a slot recycled
// for a later batch never makes a waiter sync on that batch's work).
struct BatchEvent {
  hipEvent_t e = nullptr;
  ~BatchEvent() {
    if (e) hipEventDestroy(e);
  }
};

struct Batch {
  uint64_t ticket = 0;
  std::shared_ptr<BatchEvent> fin;
  int n = 0;
  bool host_io = false;
  std::vector<ImagePlan> plans;
  std::vector<ImageDesc> descs;
  std::vector<int> desc_of;           // image -> desc index or -1
  // workgroup lists (host copies) and their offsets in the device meta buffer
  std::vector<WgItem> lists[40];
  size_t list_off[40] = {0};
  // PNG: IDAT gather jobs and palettes, uploaded with the descriptors
  std::vector<GatherJob> gjobs;
  size_t gjob_off = 0;
  std::vector<InfChunk> ichunks;  // chunk-parallel inflate records (kernels fill start/len/stop/status)
  size_t ichunk_off = 0;
  uint32_t uf_n = 0;        // PNG unfilter bands (progress flags, L_UNF tasks)
  uint32_t uf_maxbpp = 1;   // widest filter unit of the batch's PNGs (k_png_unfilter's LDS)
  size_t uf_flags_off = 0;  // their flags + ticket in the scratch arena (zeroed per batch)
  uint32_t ds_n = 0;          // destuff chunks of the batch (k_destuff_one state words)
  size_t ds_state_off = 0;    // their ticket + state words in the scratch arena (zeroed per batch), 0 = three-pass destuff
  uint32_t pf_n = 0;        // progressive scans (progress words, one pipelined k_prog_scan launch)
  size_t pf_off = 0;        // AC ticket, progress words, DC ticket in the scratch arena (zeroed per batch)
  size_t ptime_off = 0;     // debug (wg_timing): per-scan {start, end} in the wgt buffer, 0 = none
  uint32_t prog_dc_n = 0;   // the last prog_dc_n items of L_PROG need four Huffman tables (DC-first scans)
  std::vector<uint8_t> blob;
  size_t blob_off = 0;
  bool any_png = false, any_alpha = false, any_enc = false;
  bool any_fused = false;  // some image's IDCT runs inside k_huff_write
  uint32_t idct_cap = 0;   // entries of BatchFlags::idct_list
  uint32_t v_tile = 0;     // rows per k_resize_vt tile the V lists were built for
  uint32_t h_zune = 0;     // fused H items in zune decode semantics: k_resize_hbp's zune-class kernels
  bool stage_on = false;  // decode-once staging (option "entropy_once")
  uint32_t max_slots = 1; // largest Huffman table count of an image (dynamic LDS of k_huff_sync/fix)
  uint32_t max_ac = 0;    // most distinct AC tables of a baseline JPEG (k_huff_sync multi-symbol lookups)
  size_t words_off = 0, words_bytes = 0;  // contiguous encoder bit buffers (zeroed per batch)
  size_t enctab_off = 0;                  // EncTables in the blob
  std::vector<ProgScan> pscans;           // progressive JPEG scans of the batch
  size_t pscan_off = 0;
  std::vector<uint32_t> prog_level_n;     // L_PROG holds the scans level by level: counts
  // band H lists (L_RH0, L_RH2) are grouped by weight-count class (<=8, <=16,
  // <=32, more): hclass[stage/2][k] items of class k, in that order
  uint32_t hclass[2][2][4] = {{{0}}};  // [stage/2][fused][class]
  uint32_t hvclass[2] = {0, 0};        // L_RHV items of H weight class <= 8, <= 16 (k_resize_hv)
  uint32_t decclass[2] = {0, 0};       // L_DEC items of the 320- / 640-pixel segment class (k_band_dec)
  uint32_t hmclass[2][2][2] = {{{0}}};  // L_RM0 / L_RM2 items [stage/2][fused][K steps - 1] (k_resize_hm)
  size_t desc_off = 0, flags_off = 0;
  size_t meta_bytes = 0;
  size_t total_subs = 0;
  // host outputs
  std::vector<uint8_t *> host_outs;
  std::vector<uint64_t> host_caps;
  std::vector<size_t> out_dev_off;    // offset of each output in the scratch arena (host path)
  std::vector<uint8_t> out_direct;    // host path: output DMA'd straight into the caller's pinned buffer
  std::vector<dg_payload_meta *> mptr;  // each image's meta (the caller's; a split submission's are scattered)
  std::vector<dg_payload_meta> local_meta;  // defer_meta: the metas planning and finish() write ...
  std::vector<dg_payload_meta *> pub;       // ... copied to the callers' (pub) only when finish() completes
  const HuffTable *hp = nullptr;       // the table pools (generation pool_gen) this batch's kernels read
  const QuantTable *qp = nullptr;
  int pool_gen = 0;
  bool done = false;
  int resync_rounds = 0;
  bool unsettled = false;             // resync hit kMaxResyncRounds: JPEGs go back as DG_ERR_UNSUPPORTED
  std::vector<size_t> enc_host_off;  // host_io + encode: offset of image i's payload in the pinned read-back
  BatchFlags flags = {0, 0, 0, 0};
  std::vector<float> stage_ms;
  // Lanczos table cache (Context::ccache_*): this batch reads cached tables
  // or writes new ones (desc, stage, entry) that become hits once it finishes
  bool uses_ccache = false;
  std::vector<uint8_t> coef_hit;  // per descriptor: bit s = pass s reads cached tables (no k_coeffs item)
  struct CProd {
    int desc, stage, entry;
  };
  std::vector<CProd> ccache_prod;
};

// One in-flight batch's device/pinned buffers.  Three (option "slots", 1 to
// kMaxInflight) slots let the host plan and upload batch k+1 while the GPU
// still runs batches k and k-1.  kProgSlots more run progressive batches only
// (dg_submit's progressive aggregates, dg_decode_one's progressive lanes), so a
// ~0.1-1 s refinement chain never holds a baseline slot.
constexpr int kMaxInflight = 6;
#ifndef DG_PROG_SLOTS
#define DG_PROG_SLOTS 2
#endif
constexpr int kProgSlots = DG_PROG_SLOTS;  // (-DDG_PROG_SLOTS=n: experiment builds)
constexpr int kAllSlots = kMaxInflight + kProgSlots;
struct Slot {
  DevBuf scratch, meta, input;
  DevBuf wgt;  // debug: per-workgroup timestamps of the entropy kernels (option "wg_timing")
  DevBuf coef;  // coefficient arena of the batch (k_huff_write -> k_idct)
  // planned budget: one allocation per slot, scratch / coef / input carved
  // from it per batch (views: never allocated or freed on their own)
  DevBuf arena;
  bool views = false;
  size_t coef_bytes = 0;
  PinBuf stage, out;
  std::vector<hipEvent_t> ev;  // per-stage timing events
  hipEvent_t done = nullptr;   // recorded after the batch's last copy
  // Each slot has its own streams, so batch k+1's entropy kernels can run
  // beside batch k's pixel kernels (the entropy kernels leave most CUs idle
  // in their tails).
  hipStream_t st = nullptr, side = nullptr;
  hipEvent_t ev_meta = nullptr, ev_coef = nullptr, ev_zero = nullptr, ev_prog = nullptr;
  hipEvent_t ev_png0 = nullptr, ev_png1 = nullptr;  // PNG: serial inflate on the side stream
  std::unique_ptr<Batch> batch;
  size_t subs_off = 0, ckpt_off = 0;
};

enum ListId {
  L_HUFF = 0, L_SYNC, L_DESTUFF, L_SCAN, L_IDCT, L_COLOR, L_COEF, L_RH0, L_RV1, L_RH2, L_RV3, L_COPY,
  L_RHX0, L_RHX2,  // H passes whose source segment is too wide for the band kernel
  L_GATHER, L_PNG, L_EXPAND, L_ALPHA0, L_ALPHA1, L_ALPHA2,  // PNG decode, alpha programs
  L_INF_FIND, L_INF_RES,                                    // chunk-parallel inflate
  L_ENC_MCU, L_ENC_BLK, L_ENC_IMG,                          // JPEG re-encode
  L_PROG_ZERO, L_PROG,                                      // progressive JPEG
  L_PENC_ROW, L_PENC_PIECE, L_PENC_IMG,                     // PNG re-encode
  L_UNF,                                                    // PNG unfilter bands (ticket order)
  L_RHV,                                                    // fused first H + V pass (k_resize_hv)
  L_DEC,                                                    // IDCT + colour + first H pass (k_band_dec)
  L_RM0, L_RM2,                                             // band H passes on the matrix cores (k_resize_hm)
  L_RVT1, L_RVT3,                                           // V passes on column tiles (k_resize_vt)
  L_COUNT
};
static_assert((int)L_COUNT <= 40, "Batch::lists");

// A recently pooled table (pool_huff / pool_quant): its key bytes and slot.
struct RecentTab {
  uint8_t key[17 + 256];
  uint32_t len = 0;
  int idx = -1;
};

class Context {
 public:
  Context(int device, const dg_image_config *cfg);
  ~Context();
  dg_status init();

  // One batch in one slot (mptrs: per-image meta pointers instead of the
  // metas array; force_slot: a progressive slot instead of the next in turn).
  dg_status submit(int n, const uint8_t *const *h_srcs, const uint8_t *const *d_srcs, const size_t *lens,
                   const int32_t *forced, uint8_t *const *outs, const uint64_t *caps, dg_payload_meta *metas,
                   bool host_io, uint64_t *ticket, dg_payload_meta *const *mptrs = nullptr, int force_slot = -1,
                   bool defer_meta = false);
  dg_status wait(uint64_t ticket);
  dg_status poll(uint64_t ticket);
  // The C ABI's dg_submit / dg_submit_device / dg_wait / dg_poll /
  // dg_wait_ready: a submission with progressive members is split (option
  // "prog_split"): the rest run as a batch of their own, the progressive
  // members join an aggregate batch on a progressive slot.
  dg_status submit_user(int n, const uint8_t *const *h_srcs, const uint8_t *const *d_srcs, const size_t *lens,
                        const int32_t *forced, uint8_t *const *outs, const uint64_t *caps, dg_payload_meta *metas,
                        bool host_io, uint64_t *ticket);
  dg_status wait_user(uint64_t ticket);
  dg_status poll_user(uint64_t ticket);
  dg_status wait_ready(uint64_t ticket, int32_t *pending);
  // One image, coalesced with concurrent callers into shared GPU batches
  // (SURVEY §8(b).6): returns the image's status.
  dg_status decode_one(const uint8_t *src, size_t len, int32_t forced, uint8_t *out, uint64_t cap,
                       dg_payload_meta *meta);
  dg_status output_size(const uint8_t *bytes, size_t len, int32_t forced, uint64_t *nbytes);

  const BucketTable *buckets() const { return buckets_.get(); }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }
  dg_status sync_all();  // every stream of the context
  dg_status host_register(void *ptr, size_t bytes);
  dg_status host_unregister(void *ptr);
  bool host_pinned(const void *ptr, size_t bytes);  // inside a registered range, or runtime-pinned memory
  dg_status set_option(const std::string &k, int64_t v);
  int64_t get_stat(const std::string &k);
  int timings(const char **names, float *ms, int cap);

 private:
  dg_status plan_image(const uint8_t *h, size_t len, int32_t forced, ImagePlan &p);
  int pool_huff(const HuffSpec &s);
  dg_status flush_pools();
  int pool_quant(const uint16_t *q);
  dg_status ensure(DevBuf &b, size_t bytes, hipStream_t user = nullptr, bool exact = false);
  void prewarm_slots(const Slot &self);
  void retire(void *p, size_t bytes, bool pinned);
  void free_retired();
  static size_t grow_cap(size_t bytes, bool headroom);
  void note_alloc(std::chrono::steady_clock::time_point t0, size_t bytes);
  int64_t stat_allocs_ = 0, stat_alloc_mb_ = 0, stat_reclaims_ = 0;  // stats "allocs", "alloc_mb", "reclaims"
  int64_t stat_retire_syncs_ = 0;  // stat "retire_syncs": device-wide syncs to free retired buffers
  double stat_alloc_us_ = 0;                                          // stat "alloc_us"
  bool reclaim();
  void free_retired_if_idle();
  std::vector<void *> retired_dev_, retired_pinned_;  // grown-out buffers, freed later (ensure)
  size_t retired_dev_bytes_ = 0, retired_pin_bytes_ = 0;
  dg_status ensure_pinned(PinBuf &b, size_t bytes, hipStream_t user = nullptr, bool exact = false);
  dg_status upload_pools();
  dg_status launch_all(Slot &sl, bool from_fix);
  void plan_prog_items(Batch &b);
  dg_status flush_pagg_locked();  // pmu_ held
  bool pagg_stale_locked();       // the open aggregate is older than prog_flush_us
  // submit(), split into halves while a part's plan exceeds the device
  // budget (option "max_device_mb"); tickets of the parts that run are
  // appended.  prog: the parts go to progressive slots.  whole_failed: the
  // caller planned all n already and got kNeedSplit (start with the halves).
  dg_status submit_split(int n, const uint8_t *const *h_srcs, const uint8_t *const *d_srcs, const size_t *lens,
                         const int32_t *forced, uint8_t *const *outs, const uint64_t *caps,
                         dg_payload_meta *const *mptrs, bool host_io, std::vector<uint64_t> &tickets, bool prog,
                         bool defer_meta, bool whole_failed = false);
  dg_status fail_split_parts(const std::vector<uint64_t> &launched, dg_status st);
  size_t dev_footprint(const Slot *except = nullptr) const;  // device bytes this context holds
  bool budget_fit(Slot &self, size_t rs, size_t rc, size_t ri);  // mu_ held: room for self's next batch
  void free_slot_buffers(Slot &o);
  // Lanczos tables cached across batches (option "coef_cache_mb"): a pass's
  // i16 weights and bounds depend only on (box, in/out size, taps), and
  // sources of one size recur (ImageNet-like shards, a cycled pool), so
  // k_coeffs computes each once into a device arena; later batches point
  // their passes at it.  An entry turns into a hit once the batch that wrote
  // it has finished (its precision read back with the descriptors).
  struct CKey {
    uint64_t in0, in1;
    uint32_t in_size, out_size, ksize;
    bool operator==(const CKey &o) const {
      return in0 == o.in0 && in1 == o.in1 && in_size == o.in_size && out_size == o.out_size && ksize == o.ksize;
    }
  };
  struct CKeyHash {
    size_t operator()(const CKey &k) const {
      uint64_t h = k.in0 * 0x9E3779B97F4A7C15ull ^ (k.in1 + 0x632BE59BD9B4E019ull);
      h ^= ((uint64_t)k.in_size << 40) ^ ((uint64_t)k.out_size << 20) ^ k.ksize;
      h *= 0xBF58476D1CE4E5B9ull;
      return (size_t)(h ^ (h >> 31));
    }
  };
  struct CEntry {
    CKey key;
    size_t off;         // bounds at off, weights at off + out_size * 8 (arena offsets)
    int32_t precision;  // read back from the producing batch
    bool ready;
  };
  // open-addressed index over ccache_ (linear probing, -1 = empty): a
  // node-based map cost ~0.8 us per lookup, 0.5 ms of planning per
  // configs[1] batch (profiles/r05/ab5); this one is a few cache lines
  static constexpr uint32_t kCIdxBits = 16;
  std::vector<int32_t> ccache_slot_;  // 1 << kCIdxBits slots
  int ccache_find(const CKey &k, uint32_t &slot) const;  // entry index or -1; slot: where it is / would go
  void ccache_index_clear();
  std::vector<CEntry> ccache_;
  DevBuf d_ccache_;
  size_t ccache_off_ = 0, ccache_cap_ = (size_t)256 << 20;
  bool ccache_full_ = false;  // an entry did not fit: start over at the next submit
  int64_t stat_ccache_hits_ = 0, stat_ccache_new_ = 0, stat_ccache_resets_ = 0;
  int ccache_lookup(const ResizePass &ps, Batch &b, bool &hit);  // mu_ held; -1 = not cached
  void ccache_maybe_reset(Slot &self);                            // mu_ held, before a batch's lookups
  void ccache_rollback(size_t n0, size_t off0);                   // a submit that installs no batch
  size_t max_dev_bytes_ = 0;        // option "max_device_mb" (0: no budget)
  size_t budget_room_ = 0;          // headroom the current submit's growth may take under the budget
  int budget_slots_ = kMaxInflight;  // baseline slots in turn under the budget (budget_fit lowers it)
  int64_t stat_budget_slots_min_ = kMaxInflight;
  // Planned budget (option "budget_plan", default 1): the
  // first baseline batch under a budget decides the slot count and each
  // slot's buffer sizes from the budget, and every planned slot is sized
  // then; later batches that do not fit their slot are split, never grown.
  bool budget_plan_ = true;
  bool budget_planned_ = false;
  size_t plan_arena_ = 0;  // planned bytes per slot (scratch + coefficients + input, one allocation)
  bool queue_set_ = false;  // slot_queue / side_queue set explicitly (else a budget shares the process queues)
  dg_status budget_planned_fit(Slot &sl, size_t rs, size_t rc, size_t ri);
  int64_t stat_peak_dev_ = 0, stat_budget_splits_ = 0, stat_budget_frees_ = 0, stat_budget_oom_ = 0;
  dg_status finish(Slot &sl);       // finish_body, or fail_batch on its error
  dg_status finish_body(Slot &sl);
  void fail_batch(Slot &sl, dg_status st);
  Slot *find(uint64_t ticket);
  int pick_slot();
  int pick_prog_slot();
  dg_status make_prog_streams();
  dg_status make_streams(int first, int count, int mode, int cus, int side_mode, int limit = -1);
  dg_status slot_streams(Slot &sl);

  int device_;
  bool has_cfg_ = false;
  dg_image_config cfg_{};
  std::unique_ptr<BucketTable> buckets_;
  hipStream_t stream_ = nullptr, side_ = nullptr;
  hipEvent_t ev_meta_ = nullptr, ev_coef_ = nullptr;
  std::mutex mu_;

  // decode_one coalescing (options "coalesce_max", "coalesce_us")
  struct OneReq {
    const uint8_t *src;
    size_t len;
    int32_t forced;
    uint8_t *out;
    uint64_t cap;
    dg_payload_meta *meta;
    bool done;
    dg_status st;
    bool prog;  // progressive JPEG: coalesced apart (option "prog_lanes")
  };
  std::mutex cmu_;
  std::condition_variable ccv_;
  std::vector<OneReq *> pending_, ppending_;  // baseline / progressive callers waiting for a batch
  int callers_ = 0, inflight_ = 0, inflight_reqs_ = 0, pinflight_ = 0;
  int prog_lanes_ = 1;  // option "prog_lanes": progressive batches in flight beside the baseline ones
  // progressive aggregate of split submissions (options "prog_split", "prog_batch", "prog_flush_us")
  struct PEntry {
    std::vector<uint8_t> host;  // the coded file (the header parser walks every scan at flush time)
    const uint8_t *dsrc;        // device copy (dg_submit_device) or null
    size_t len;
    int32_t forced;
    uint8_t *out;
    uint64_t cap;
    dg_payload_meta *meta;
  };
  struct SplitRec {
    std::vector<uint64_t> tbs;  // internal tickets of the non-progressive members (a device-budget split: several)
    uint64_t gen = 0;  // aggregate generation holding the progressive members
    int32_t nprog = 0;
  };
  std::mutex pmu_;
  std::vector<PEntry> pagg_;
  bool pagg_host_ = true;
  uint64_t pagg_gen_ = 1;
  std::chrono::steady_clock::time_point pagg_t0_;
  struct PGen {
    std::vector<uint64_t> tickets;  // the aggregate's batches (several after a device-budget split; none: launch failed)
    int refs = 0;         // split records still referring to it
    dg_status st = DG_OK; // launch status, returned by dg_wait of its members
  };
  std::unordered_map<uint64_t, PGen> pgen_;  // flushed generation -> aggregate
  std::unordered_map<uint64_t, SplitRec> split_;                 // user ticket -> parts
  int pagg_refs_ = 0;      // split records referring to the open aggregate
  int next_pslot_ = 0;
  bool prog_split_ = true;
  int prog_batch_ = 2048;
  int prog_flush_us_ = 20000;
  int slot_queue_ = 1;      // option "slot_queue" (make_streams for the baseline slots): high priority
  int side_queue_ = 3;      // option "side_queue": the baseline slots' side streams (-1: as slot_queue; 3: own queues)
  int prog_cus_ = 0;        // option "prog_cus" (prog_queue 3: CU mask width, 0 = all)
  int prog_queue_ = 2;      // option "prog_queue" (make_prog_streams): low priority, a queue of its own
  int64_t stat_prog_aggs_ = 0, stat_prog_agg_images_ = 0;
  bool multi_lead_ = true;   // option "multi_lead": multi-symbol AC steps in k_huff_sync's state-only decodes
  int write_pair_ = 3;       // option "write_pair": up to this many more AC symbols per k_huff_write step from one peek
  bool sync2_ = false;       // option "sync2": k_huff_sync with two chains per lane (k_huff_sync2)
  bool sync_pair_ = false;   // option "sync_pair": the same in k_huff_sync (measured slower beside multi_lead: off)
  bool prog_side_ = false;  // option "prog_side": progressive scans on the side stream (measured slower: off)
  int coalesce_max_ = 64, coalesce_us_ = 500;
  // option "coalesce_inflight": coalesced batches in flight (0 = nslots_); 3 fills the batches better
  // (7.6 vs 5.4 images) and measured 5-20% faster than 4 from 32 callers (profiles/r04/one_r4*)
  int coalesce_inflight_ = 3;
  int64_t stat_coalesced_batches_ = 0, stat_coalesced_images_ = 0;
  dg_status flush_batch(std::vector<OneReq *> &batch, bool prog);

  std::vector<HuffTable> hpool_;
  std::unordered_map<std::string, int> hpool_idx_;
  static constexpr int kRecentTabs = 8;  // recently pooled tables, compared before the hash map
  RecentTab hrecent_[kRecentTabs], qrecent_[kRecentTabs];
  uint32_t hrecent_next_ = 0, qrecent_next_ = 0;
  std::vector<QuantTable> qpool_;
  std::unordered_map<std::string, int> qpool_idx_;
  size_t hpool_uploaded_ = 0, qpool_uploaded_ = 0;
  // Device copies of the pools: kPoolGens generations, each allocated once at
  // full capacity.  Starting the pools over moves to the next generation and
  // waits only for batches still reading that (oldest) one, never for the
  // batches in flight on the current ones.
  static constexpr int kPoolGens = 4;
  DevBuf d_hpool_[kPoolGens], d_qpool_[kPoolGens];
  int pool_gen_ = 0;

  Slot slots_[kAllSlots];  // [0, kMaxInflight): baseline batches; then kProgSlots progressive ones
  uint32_t ncu_ = 256;  // compute units: persistent-worker grids
  int entropy_prio_ = 0;  // option "entropy_prio"
  int uf_per_cu_ = 0;     // option "uf_per_cu"
  int nslots_ = 4;  // option "slots": batches in flight (each slot: own streams + scratch; 4 measured +2% over 3 with own queues)
  int next_slot_ = 0;
  uint64_t next_ticket_ = 1;

  uint32_t sub_bits_ = 0;  // 0 = auto per batch (see submit)
  uint32_t sub_auto_ = 8192;  // the auto size of large batches
  int64_t lead_bits_ = -1;  // -1 = auto per image (see submit)
  uint32_t last_sub_bits_ = kDefaultSubBits;
  bool timing_ = false;
  bool side_stream_ = true;
  int debug_flags_ = 0;
  bool wg_timing_ = false;
  bool chunked_off_ = false;  // option "png_chunked" = 0
  uint32_t inf_chunk_ = kInfChunk;  // option "inf_chunk"
  uint32_t inf_cap_ = 30;           // option "inf_cap": chunk entries, tenths of the expansion of a span
  bool png_alias_ = true;           // option "png_alias": chunk entries alias the unfilter/resize buffers
  uint32_t inf_pad_ = 65536;        // option "inf_pad": chunk entries on top of inf_cap's
  uint32_t inf_stage3_ = 32;        // option "inf_stage3"
  int plan_threads_ = 4;            // option "plan_threads"
  int meta_pull_ = 1;               // option "meta_pull"
  size_t list_hint_[L_COUNT] = {};  // work-list sizes of the previous batch (reserve)
  bool write_split_ = true;         // option "write_split"
  uint32_t lead_big_ = 4096;        // option "lead_big" (6144 -> 4096 with 8192-bit ranges: +1.3%, profiles/r04/lead_big)
  uint64_t small_coded_ = 0;        // option "small_coded" (0: off)
  uint32_t sub_small_ = 512, lead_small_ = 1024;  // options "sub_small", "lead_small"
  uint32_t v_tile_ = 4;             // option "v_tile": V pass on R-row column tiles (k_resize_vt<R>; 0 = k_resize_v)
  uint32_t v_units_ = 2;            // option "v_units" (profiles/r04/v_units: 1 / 2 / 4 -> V traffic 1.95 / ? / 3.91 GB per batch)
  static constexpr int kPlanGrain = 32;  // images per planning work piece
  std::unique_ptr<HostPool> plan_pool_;
  uint32_t hb_bands_ = kHBandsDefault;  // option "hb_bands"
  int decode_sem_ = 0;                  // option "decode_semantics"
  bool ckpt_ = true;                    // option "ckpt"
  double host_us_[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // submit phases + slot wait (stats "host_us_*"; option "reset_host_us")
  double host_cpu_us_[7] = {0, 0, 0, 0, 0, 0, 0};
  size_t last_meta_bytes_ = 0;  // stat "meta_bytes": the last batch's descriptor/list upload  // the same phases' thread CPU time (stats "host_cpu_us_*")
  int copy_threads_ = 8;                // option "copy_threads": host threads for a host-out batch's output copies
  bool hv_fused_ = false;               // option "hv_fused": first H + V pass fused (k_resize_hv) when it fits
  bool idct_thread_ = true;             // option "idct_thread": one lane per block (k_idct_t) instead of 8 (k_idct)
  bool sparse_coef_ = true;             // option "sparse_coef": k_huff_write stores, k_idct_t loads, only the
                                        // 16-byte parts through each block's last nonzero (ImageDesc::ccnt)
  bool h_prefetch_ = true;              // option "h_prefetch": specialised fused fills load the next band before the convolution
  bool h_planar_ = true;                // option "h_planar": fused 8/16-tap band passes over planar u16-pair segments (k_resize_hbp)
  bool destuff_one_ = false;            // option "destuff_one": single-pass destuff with decoupled look-back
                                        // (configs[1] 0.66 vs 0.43 ms three-pass: off)
  bool chroma_rec_ = true;              // option "chroma_rec": half-rate chroma planes as 8-byte records (dg_plane.h)
  bool band_dec_ = false;               // option "band_dec": IDCT + colour + first H pass in k_band_dec
  uint32_t uf_units_ = 1;               // option "uf_units": PNG unfilter units per lane per step (1 or 2; round 5: 1)
  uint32_t inf_decode_ = 25;            // option "inf_decode": k_inf_decode shape (25 = 7/5 lookup bits, 20 KiB LDS
                                        // per wave, 16 stream words per lane in registers)
  bool h_mfma_ = false;                 // option "h_mfma": band H passes on the matrix cores (k_resize_hm; measured slower: off)
  double sub_density_ = 0;              // option "sub_density": bits per block below which subsequences shrink
  bool lead_density_ = false;           // option "lead_density": their lead-in shrinks by the same factor
  uint32_t dec_dbg_ = 0;                // option "dec_dbg": k_band_dec phase switches (timing experiments only)
  uint32_t dec_strips_ = kDecStripsDefault;  // option "dec_strips"
  bool idct_fused_ = false;             // option "idct_fused" (measured 7x slower k_huff_write: off)
  bool progressive_ = true;             // option "progressive"
  bool prog_serial_ = false;            // option "prog_serial": serial reader for every scan (A/B)
  bool prog_pipe_ = true;               // option "prog_pipe": all scans in one pipelined launch (0: one launch per level)
  int prog_chain_ = 100;                // option "prog_chain": chain dependency groups costing <= this % of the longest scan
  bool entropy_lpt_ = true;             // option "entropy_lpt": slow entropy workgroups first
  bool entropy_once_ = false;           // option "entropy_once": decode-once staging + k_huff_scatter
  int64_t stat_png_serial_ = 0, stat_png_chunks_ = 0, stat_png_small_ = 0;
  int64_t stat_band_dec_ = 0;  // images whose first H pass ran in k_band_dec (stat "band_dec_images")
  // "wg_timing" summaries of the last batch (microseconds): per kernel {span, mean, p90, max}
  double wgstat_[2][4] = {{0}};
  // stats
  int64_t stat_batches_ = 0, stat_resync_ = 0, stat_fix_ = 0, stat_mismatch_ = 0, stat_iters_ = 0;
  int64_t stat_unsettled_ = 0, stat_pool_flush_ = 0;
  int64_t stat_prog_items_ = 0, stat_prog_chains_ = 0;  // pipelined progressive launches: work items, chains
  std::vector<float> last_ms_;
  std::mutex reg_mu_;
  std::vector<std::pair<uintptr_t, size_t>> registered_;  // dg_host_register ranges
  int64_t stat_direct_d2h_ = 0;                           // outputs copied straight into caller memory
};

}  // namespace dg
