// capi.cpp — extern "C" entry points declared in include/datago_hip.h.
#include <string.h>

#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <unistd.h>

#include <mutex>
#include <new>
#include <set>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../../include/datago_hip.h"
#include "buckets.h"
#include "jpeg_header.h"
#include "pipeline.h"
#include "png_header.h"

namespace dg {
extern thread_local std::string g_last_error;
void set_error(const std::string &s);
}  // namespace dg

struct dg_bucket_table {
  dg::BucketTable t;
  dg_bucket_table(uint32_t a, uint32_t b, double c, double d) : t(a, b, c, d) {}
};

// A context behind the C ABI.  Entry points hold `gate` shared while they
// use the context; dg_ctx_destroy (and the exit hook) take it exclusively.
// The exit hook tears down the contexts a process leaves alive -- before
// the HIP runtime's own static destructors run -- when no thread is inside
// one of their calls; a context it ran down stays `dead` (later calls
// return DG_ERR_INVALID) instead of being freed under a caller.
struct dg_ctx {
  std::shared_mutex gate;
  bool dead = false;
  dg::Context *c;
  dg_bucket_table view;
  dg_ctx(int dev, const dg_image_config *cfg)
      : c(new dg::Context(dev, cfg)),
        view(cfg && cfg->crop_and_resize && cfg->default_image_size && cfg->downsampling_ratio
                 ? cfg->default_image_size
                 : 224,
             cfg && cfg->crop_and_resize && cfg->default_image_size && cfg->downsampling_ratio
                 ? cfg->downsampling_ratio
                 : 16,
             cfg && cfg->crop_and_resize ? cfg->min_aspect_ratio : 0.5,
             cfg && cfg->crop_and_resize ? cfg->max_aspect_ratio : 2.0) {}
  ~dg_ctx() { delete c; }
};

namespace {

// Live contexts (never destroyed itself: the exit hook may run after other
// static destructors of this library).
std::mutex &reg_mu() {
  static std::mutex *m = new std::mutex;
  return *m;
}
std::set<dg_ctx *> &registry() {
  static std::set<dg_ctx *> *r = new std::set<dg_ctx *>;
  return *r;
}

// Registered with atexit at the first dg_ctx_create, i.e. after the HIP
// runtime (loaded with this library) registered its destructors, so it runs
// before them.  DG_NO_EXIT_HOOK=1 leaves everything to the runtime.
void exit_hook() {
  std::vector<dg_ctx *> live;
  {
    std::lock_guard<std::mutex> lk(reg_mu());
    live.assign(registry().begin(), registry().end());
  }
  for (dg_ctx *x : live) {
    if (!x->gate.try_lock()) continue;  // a thread is still inside a call: leave it to the runtime
    if (!x->dead) {
      delete x->c;
      x->c = nullptr;
      x->dead = true;
    }
    x->gate.unlock();
  }
}

// Debug (DG_SEGV_TRACE=1): a host fault prints the native stack to stderr
// (symbolised from the dynamic symbol tables) before the default action.
void segv_trace(int sig) {
  void *fr[64];
  const int n = backtrace(fr, 64);
  static const char msg[] = "datago_amd: fatal signal, native stack:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void install_exit_hook() {
  static std::once_flag once;
  std::call_once(once, [] {
    const char *e = getenv("DG_NO_EXIT_HOOK");
    if (!(e && e[0] == '1')) atexit(exit_hook);
    const char *t = getenv("DG_SEGV_TRACE");
    if (t && t[0] == '1') {
      signal(SIGSEGV, segv_trace);
      signal(SIGABRT, segv_trace);
    }
  });
}

// Shared use of a live context for one entry point.
struct CtxUse {
  dg_ctx *x;
  bool ok = false;
  explicit CtxUse(dg_ctx *c) : x(c) {
    if (!c) return;
    c->gate.lock_shared();
    ok = !c->dead;
    if (!ok) c->gate.unlock_shared();
  }
  ~CtxUse() {
    if (ok) x->gate.unlock_shared();
  }
  CtxUse(const CtxUse &) = delete;
  CtxUse &operator=(const CtxUse &) = delete;
};

}  // namespace

#define DG_USE(ctx, fail)                                             \
  CtxUse use_(ctx);                                                   \
  if (!use_.ok) {                                                     \
    dg::set_error(ctx ? "context already destroyed" : "null context"); \
    return fail;                                                      \
  }

extern "C" {

const char *dg_last_error(void) { return dg::g_last_error.c_str(); }
int32_t dg_abi_version(void) { return DG_ABI_VERSION; }

dg_status dg_bucket_table_build(uint32_t size, uint32_t ratio, double min_ar, double max_ar,
                                dg_bucket_table **out) {
  if (!out) return DG_ERR_INVALID;
  *out = nullptr;
  // assert!s of image_processing.rs:78-93, reported instead of aborting
  if (size == 0 || ratio == 0 || !(min_ar > 0.0) || !(max_ar >= min_ar)) {
    dg::set_error("invalid bucket parameters");
    return DG_ERR_INVALID;
  }
  dg_bucket_table *t = new (std::nothrow) dg_bucket_table(size, ratio, min_ar, max_ar);
  if (!t) return DG_ERR_OOM;
  *out = t;
  return DG_OK;
}

void dg_bucket_table_free(dg_bucket_table *t) { delete t; }

int32_t dg_bucket_count(const dg_bucket_table *t) { return t ? (int32_t)t->t.buckets().size() : 0; }

dg_status dg_bucket_get(const dg_bucket_table *t, int32_t i, uint32_t *w, uint32_t *h, char *key, size_t cap) {
  if (!t || i < 0 || i >= (int32_t)t->t.buckets().size()) return DG_ERR_BAD_BUCKET;
  const dg::Bucket &b = t->t.buckets()[i];
  if (w) *w = b.w;
  if (h) *h = b.h;
  if (key && cap) {
    strncpy(key, b.key.c_str(), cap - 1);
    key[cap - 1] = 0;
  }
  return DG_OK;
}

int32_t dg_closest_bucket(const dg_bucket_table *t, int32_t w, int32_t h) {
  if (!t || w <= 0 || h <= 0) return -1;
  return t->t.closest(w, h);
}

int32_t dg_bucket_find_key(const dg_bucket_table *t, const char *key) {
  if (!t || !key) return -1;
  return t->t.find_key(key);
}

dg_status dg_aspect_ratio_to_str(uint32_t w, uint32_t h, char *out, size_t cap) {
  if (!out || !cap || h == 0) return DG_ERR_INVALID;
  std::string s = dg::aspect_ratio_to_str(w, h);
  strncpy(out, s.c_str(), cap - 1);
  out[cap - 1] = 0;
  return DG_OK;
}

dg_status dg_probe(const uint8_t *bytes, size_t len, dg_probe_info *out) {
  if (!out) return DG_ERR_INVALID;
  memset(out, 0, sizeof(*out));
  if (!bytes || !len) return DG_ERR_CORRUPT;
  if (dg::is_png(bytes, len)) {
    dg::PngHeader h;
    dg::parse_png_header(bytes, len, h);
    out->format = DG_FMT_PNG;
    out->width = h.width;
    out->height = h.height;
    out->components = h.out_c;   // channels after EXPAND (L8 1, La8 2, Rgb8 3, Rgba8 4)
    out->bit_depth = h.depth;
    out->precision = h.depth;
    out->progressive = h.interlace;  // Adam7
    out->gpu_supported = h.status == dg::PH_OK;
    if (h.status == dg::PH_CORRUPT) {
      dg::set_error(h.why);
      return DG_ERR_CORRUPT;
    }
    return DG_OK;
  }
  if (!dg::is_jpeg(bytes, len)) {
    dg::set_error("unknown image format");
    return DG_ERR_CORRUPT;
  }
  dg::JpegHeader h;
  dg::parse_jpeg_header(bytes, len, h);
  out->format = DG_FMT_JPEG;
  out->width = h.width;
  out->height = h.height;
  out->components = h.ncomp;
  out->bit_depth = h.precision;
  for (int c = 0; c < h.ncomp && c < 4; c++) {
    out->h_samp[c] = h.comp[c].h;
    out->v_samp[c] = h.comp[c].v;
  }
  out->progressive = h.progressive;
  out->arithmetic = h.arithmetic;
  out->precision = h.precision;
  out->restart_interval = h.restart;
  // (a context with decode_semantics 1 also decodes incompletely refined progressive files)
  out->gpu_supported = h.status == dg::JH_OK && !h.incomplete_refinement;
  if (h.status == dg::JH_CORRUPT) {
    dg::set_error(h.why);
    return DG_ERR_CORRUPT;
  }
  return DG_OK;
}

dg_status dg_ctx_create(int32_t device, const dg_image_config *cfg, dg_ctx **out) {
  if (!out) return DG_ERR_INVALID;
  *out = nullptr;
  dg_ctx *c = new (std::nothrow) dg_ctx(device, cfg);
  if (!c) return DG_ERR_OOM;
  dg_status st = c->c->init();
  if (st) {
    delete c;
    return st;
  }
  install_exit_hook();
  {
    std::lock_guard<std::mutex> lk(reg_mu());
    registry().insert(c);
  }
  *out = c;
  return DG_OK;
}

void dg_ctx_destroy(dg_ctx *ctx) {
  if (!ctx) return;
  {
    std::lock_guard<std::mutex> lk(reg_mu());
    registry().erase(ctx);
  }
  { std::unique_lock<std::shared_mutex> lk(ctx->gate); }  // every call on it has returned
  delete ctx;
}

const dg_bucket_table *dg_ctx_buckets(const dg_ctx *ctx) {
  if (!ctx || ctx->dead || !ctx->c->buckets()) return nullptr;
  return &ctx->view;
}

dg_status dg_sample_align(const dg_bucket_table *t, int32_t n, const uint8_t *const *srcs, const size_t *lens,
                          int32_t forced_first, int32_t *forced_out) {
  if (n < 0 || (n > 0 && (!srcs || !lens || !forced_out))) return DG_ERR_INVALID;
  for (int32_t i = 0; i < n; i++) forced_out[i] = -1;
  if (!t) return DG_OK;  // no image_config: the aspect ratio is never used
  const dg::BucketTable *bt = &t->t;
  // the reference payload: the first one whose header gives dimensions (a payload
  // that fails to load is skipped, worker_wds.rs:134-137)
  int32_t ref = -1;
  uint32_t w = 0, h = 0;
  for (int32_t i = 0; i < n && ref < 0; i++) {
    dg_probe_info pi;
    if (dg_probe(srcs[i], lens[i], &pi) == DG_OK && pi.width && pi.height) {
      ref = i;
      w = pi.width;
      h = pi.height;
    }
  }
  if (ref < 0) return DG_OK;
  const int nb = (int)bt->buckets().size();
  if (forced_first >= nb || forced_first < -1) return DG_ERR_BAD_BUCKET;
  const int b = forced_first >= 0 ? forced_first : bt->closest((int32_t)w, (int32_t)h);
  forced_out[ref] = forced_first;
  // aspect_ratio_to_str(first payload's output size) -> the key the others are forced to
  const dg::Bucket &bk = bt->buckets()[b];
  const int k = bt->find_key(dg::aspect_ratio_to_str(bk.w, bk.h));
  for (int32_t i = ref + 1; i < n; i++) forced_out[i] = k < 0 ? -2 : k;
  return DG_OK;
}

dg_status dg_output_size(dg_ctx *ctx, const uint8_t *bytes, size_t len, int32_t forced, uint64_t *nbytes) {
  if (!nbytes) return DG_ERR_INVALID;
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->output_size(bytes, len, forced, nbytes);
}

dg_status dg_submit(dg_ctx *ctx, int32_t n, const uint8_t *const *srcs, const size_t *lens, const int32_t *forced,
                    uint8_t *const *outs, const uint64_t *caps, dg_payload_meta *metas, uint64_t *ticket) {
  if (!ticket) return DG_ERR_INVALID;
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->submit_user(n, srcs, nullptr, lens, forced, outs, caps, metas, true, ticket);
}

dg_status dg_submit_device(dg_ctx *ctx, int32_t n, const uint8_t *const *h_srcs, const uint8_t *const *d_srcs,
                           const size_t *lens, const int32_t *forced, uint8_t *const *d_outs,
                           const uint64_t *caps, dg_payload_meta *metas, uint64_t *ticket) {
  if (!ticket || (n > 0 && !d_srcs)) return DG_ERR_INVALID;
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->submit_user(n, h_srcs, d_srcs, lens, forced, d_outs, caps, metas, false, ticket);
}

dg_status dg_wait(dg_ctx *ctx, uint64_t ticket) {
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->wait_user(ticket);
}
dg_status dg_poll(dg_ctx *ctx, uint64_t ticket) {
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->poll_user(ticket);
}
dg_status dg_wait_ready(dg_ctx *ctx, uint64_t ticket, int32_t *pending) {
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->wait_ready(ticket, pending);
}

dg_status dg_decode_one(dg_ctx *ctx, const uint8_t *src, size_t len, int32_t forced, uint8_t *out, uint64_t cap,
                        dg_payload_meta *meta) {
  if (!meta) return DG_ERR_INVALID;
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->decode_one(src, len, forced, out, cap, meta);
}

dg_status dg_device_alloc(dg_ctx *ctx, size_t bytes, void **dptr) {
  if (!dptr) return DG_ERR_INVALID;
  DG_USE(ctx, DG_ERR_INVALID);
  hipSetDevice(ctx->c->device());
  if (hipMalloc(dptr, bytes ? bytes : 1) != hipSuccess) return DG_ERR_OOM;
  return DG_OK;
}
dg_status dg_device_free(dg_ctx *ctx, void *dptr) {
  DG_USE(ctx, DG_ERR_INVALID);
  hipSetDevice(ctx->c->device());
  return hipFree(dptr) == hipSuccess ? DG_OK : DG_ERR_DEVICE;
}
dg_status dg_memcpy_h2d(dg_ctx *ctx, void *dst, const void *src, size_t bytes) {
  DG_USE(ctx, DG_ERR_INVALID);
  hipSetDevice(ctx->c->device());
  return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess ? DG_OK : DG_ERR_DEVICE;
}
dg_status dg_memcpy_d2h(dg_ctx *ctx, void *dst, const void *src, size_t bytes) {
  DG_USE(ctx, DG_ERR_INVALID);
  hipSetDevice(ctx->c->device());
  return hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost) == hipSuccess ? DG_OK : DG_ERR_DEVICE;
}
dg_status dg_host_register(dg_ctx *ctx, void *ptr, size_t bytes) {
  if (!ptr || !bytes) return DG_ERR_INVALID;
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->host_register(ptr, bytes);
}
dg_status dg_host_unregister(dg_ctx *ctx, void *ptr) {
  if (!ptr) return DG_ERR_INVALID;
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->host_unregister(ptr);
}
dg_status dg_synchronize(dg_ctx *ctx) {
  DG_USE(ctx, DG_ERR_INVALID);
  hipSetDevice(ctx->c->device());
  return ctx->c->sync_all();
}

int32_t dg_last_batch_timings(dg_ctx *ctx, const char **names, float *ms, int32_t cap) {
  DG_USE(ctx, 0);
  return ctx->c->timings(names, ms, cap);
}

dg_status dg_ctx_set_option(dg_ctx *ctx, const char *key, int64_t value) {
  if (!key) {
    dg::set_error("dg_ctx_set_option: null key");
    return DG_ERR_INVALID;
  }
  DG_USE(ctx, DG_ERR_INVALID);
  return ctx->c->set_option(key, value);
}

int64_t dg_ctx_get_stat(dg_ctx *ctx, const char *key) {
  if (!key) {
    dg::set_error("dg_ctx_get_stat: null key");
    return -1;
  }
  DG_USE(ctx, -1);
  return ctx->c->get_stat(key);
}

}  // extern "C"
