// dg_decode_one from native threads: the integration path of INTEGRATION.md
// (the Rust glue's tokio workers call the library from native threads, one
// image per call; bench.py's Python threads also contend for the interpreter
// lock between calls).  Host JPEG bytes in -> host RGB out, one reused
// page-locked output buffer per thread (dg_host_register), as in bench.py's
// e2e_decode_one.  Prints one JSON object.
//
//   one_bench POOL THREADS IMAGES SIZE RATIO SEM [key=value context options...]
//   POOL: u32 n, then n x (u64 len, len bytes)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/datago_hip.h"

int main(int argc, char **argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s POOL THREADS IMAGES SIZE RATIO SEM [key=value ...]\n", argv[0]);
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  uint32_t n = 0;
  if (fread(&n, 4, 1, f) != 1 || n == 0) return 2;
  std::vector<std::vector<uint8_t>> pool(n);
  for (uint32_t i = 0; i < n; i++) {
    uint64_t len = 0;
    if (fread(&len, 8, 1, f) != 1) return 2;
    pool[i].resize(len);
    if (fread(pool[i].data(), 1, len, f) != len) return 2;
  }
  fclose(f);
  const int threads = atoi(argv[2]), images = atoi(argv[3]);
  dg_image_config cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.crop_and_resize = 1;
  cfg.default_image_size = (uint32_t)atoi(argv[4]);
  cfg.downsampling_ratio = (uint32_t)atoi(argv[5]);
  cfg.min_aspect_ratio = 0.5;
  cfg.max_aspect_ratio = 2.0;
  cfg.encode_format = 1;
  cfg.jpeg_quality = 92;
  cfg.decode_semantics = atoi(argv[6]);
  dg_ctx *ctx = nullptr;
  if (dg_ctx_create(0, &cfg, &ctx) != DG_OK) return 3;
  for (int a = 7; a < argc; a++) {
    std::string kv(argv[a]);
    const size_t e = kv.find('=');
    if (e == std::string::npos || dg_ctx_set_option(ctx, kv.substr(0, e).c_str(), atoll(kv.c_str() + e + 1))) return 2;
  }
  uint64_t cap = 16;
  for (const auto &d : pool) {
    uint64_t nb = 0;
    if (dg_output_size(ctx, d.data(), d.size(), -1, &nb) == DG_OK && nb > cap) cap = nb;
  }
  std::vector<std::vector<uint8_t>> bufs(threads, std::vector<uint8_t>(cap));
  for (auto &b : bufs)
    if (dg_host_register(ctx, b.data(), b.size()) != DG_OK) return 3;
  std::atomic<int> next{0};
  std::atomic<int64_t> px{0}, fails{0};
  auto work = [&](int t, int count) {
    for (int i; (i = next.fetch_add(1)) < count;) {
      const auto &d = pool[(size_t)i % n];
      dg_payload_meta m;
      if (dg_decode_one(ctx, d.data(), d.size(), -1, bufs[t].data(), cap, &m) == DG_OK)
        px += (int64_t)m.original_width * m.original_height;
      else
        fails++;
    }
  };
  // warm-up: one untimed pass over every image (buffer growth, table pools;
  // bench.py's Python leg runs on a context the whole bench has warmed)
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) ts.emplace_back(work, t, images);
    for (auto &t : ts) t.join();
  }
  next = 0;
  px = 0;
  fails = 0;
  const int64_t b0 = dg_ctx_get_stat(ctx, "coalesced_batches"), i0 = dg_ctx_get_stat(ctx, "coalesced_images");
  const auto t0 = std::chrono::steady_clock::now();
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; t++) ts.emplace_back(work, t, images);
    for (auto &t : ts) t.join();
  }
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const int64_t nb = dg_ctx_get_stat(ctx, "coalesced_batches") - b0, ni = dg_ctx_get_stat(ctx, "coalesced_images") - i0;
  printf("{\"threads\": %d, \"images\": %d, \"failed\": %lld, \"mpix_s\": %.2f, \"images_per_s\": %.1f, "
         "\"gpu_batches\": %lld, \"mean_images_per_batch\": %.1f}\n",
         threads, images, (long long)fails.load(), (double)px.load() / s / 1e6, images / s, (long long)nb,
         nb ? (double)ni / (double)nb : 0.0);
  for (auto &b : bufs) dg_host_unregister(ctx, b.data());
  dg_ctx_destroy(ctx);
  return 0;
}
