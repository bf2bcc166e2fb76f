// A persistent host worker pool shared by the packer (kad_pack.cpp) and the upload / download checks
// (kad_api.hip). Creating 16 threads per parallel call cost ~0.3 ms each time, ~9 ms per batch upload over
// its ~20 parallel checks — the fixed cost that made small batches slower end to end than the CPU
// baseline. Workers are created once (the first parallel call). A job of T tasks is split statically:
// thread j (the caller is thread 0) runs tasks j, j + P, j + 2P, ... (P = min(T, threads)), so every
// range runs on its own thread as with per-call threads. Between jobs a worker spins for ~0.2 ms before it
// sleeps on a condition variable: the packer's and the checks' back-to-back parallel loops do not pay a
// wake-up each. A parallel call made from inside a task runs serially (no nested jobs).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace kadpool {

class Pool {
 public:
  explicit Pool(int workers) {
    for (int i = 0; i < workers; i++) th_.emplace_back([this, i] { loop(i + 1); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_.store(true);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int threads() const { return (int)th_.size() + 1; }
  // f(t) for every t in [0, n); returns when all have run
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (n == 1 || in_task() || th_.empty()) {
      for (int t = 0; t < n; t++) f(t);
      return;
    }
    std::lock_guard<std::mutex> rg(run_mu_);  // one job at a time
    const int P = std::min(n, threads());
    pending_.store(P - 1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(mu_);  // a worker reads (gen, job) together under mu_
      job_ = &f;
      ntask_ = n;
      nthr_ = P;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    in_task() = true;
    for (int t = 0; t < n; t += P) f(t);
    in_task() = false;
    while (pending_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }

 private:
  static bool& in_task() {
    static thread_local bool flag = false;
    return flag;
  }
  void loop(int j) {
    uint64_t seen = 0;
    for (;;) {
      // spin ~0.2 ms for the next job, then sleep
      const auto t0 = std::chrono::steady_clock::now();
      uint64_t g = gen_.load(std::memory_order_acquire);
      while (g == seen && std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200)) {
        std::this_thread::yield();
        g = gen_.load(std::memory_order_acquire);
      }
      const std::function<void(int)>* job;
      int ntask, nthr;
      {
        // the latest job, consistently (a job this worker skipped did not include it: the job after one
        // cannot start before all of its workers are done)
        std::unique_lock<std::mutex> lk(mu_);
        if (g == seen) cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
        seen = gen_.load(std::memory_order_acquire);
        if (stop_.load()) return;
        job = job_;
        ntask = ntask_;
        nthr = nthr_;
      }
      if (j < nthr && job) {
        in_task() = true;
        for (int t = j; t < ntask; t += nthr) (*job)(t);
        in_task() = false;
        pending_.fetch_sub(1, std::memory_order_acq_rel);
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> stop_{false};
  // written by run() before gen_ is bumped (release), read by workers after they see the bump (acquire)
  const std::function<void(int)>* job_ = nullptr;
  int ntask_ = 0, nthr_ = 0;
};

// up to 16 threads (the GPU box's CPU share), created on first use
inline Pool& pool() {
  static Pool p((int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency())) - 1);
  return p;
}

}  // namespace kadpool
