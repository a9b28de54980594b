// Persistent host worker pool for the data-parallel loops of dg_submit*
// planning (per-image header parsing).  A 1024-image WebDataset batch spent
// ~0.6 ms of its ~2.6 ms submit in header parsing on the calling thread
// (profiles/r04/wds); spawning threads per submit would cost about as much as
// the work, so the workers persist and sleep between jobs.  The calling thread
// takes part; one job runs at a time.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace dg {

class HostPool {
 public:
  explicit HostPool(int nthreads) {
    for (int t = 1; t < nthreads; t++) ts_.emplace_back([this] { worker(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      quit_ = true;
    }
    cv_.notify_all();
    for (std::thread &t : ts_) t.join();
  }
  int threads() const { return (int)ts_.size() + 1; }

  // fn(i) for every i in [0, n), in pieces of `grain`; returns when all are done.
  void run(int n, int grain, const std::function<void(int)> &fn) {
    if (n <= 0) return;
    if (ts_.empty() || n <= grain) {
      for (int i = 0; i < n; i++) fn(i);
      return;
    }
    std::lock_guard<std::mutex> one(run_m_);
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      n_ = n;
      grain_ = std::max(1, grain);
      next_.store(0);
      busy_ = (int)ts_.size();
      gen_++;
    }
    cv_.notify_all();
    take();
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void take() {
    for (int k; (k = next_.fetch_add(grain_)) < n_;) {
      const int e = std::min(n_, k + grain_);
      for (int i = k; i < e; i++) (*fn_)(i);
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
      }
      take();
      {
        std::lock_guard<std::mutex> lk(m_);
        if (--busy_ == 0) done_cv_.notify_one();
      }
    }
  }

  std::vector<std::thread> ts_;
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)> *fn_ = nullptr;
  std::atomic<int> next_{0};
  int n_ = 0, grain_ = 1, busy_ = 0;
  uint64_t gen_ = 0;
  bool quit_ = false;
};

}  // namespace dg
