// A persistent host worker pool shared by the packer (kad_pack.cpp) and the upload / download checks
// (kad_api.hip). Creating 16 threads per parallel call cost ~0.3 ms each time, ~9 ms per batch upload over
// its ~20 parallel checks — the fixed cost that made small batches slower end to end than the CPU
// baseline. Workers are created once (the first parallel call). A job of T tasks is split statically:
// thread j (the caller is thread 0) runs tasks j, j + P, j + 2P, ... (P = min(T, threads)), so every
// range runs on its own thread as with per-call threads. Between jobs a worker spins for ~0.2 ms before it
// sleeps on a condition variable: the packer's and the checks' back-to-back parallel loops do not pay a
// wake-up each. A parallel call made from inside a task runs serially (no nested jobs).
//
// fork(): a child has none of the parent's workers (and may have inherited a locked mutex), so a
// pthread_atfork child handler drops the pool (it is leaked, never touched again) and the child's first
// parallel call builds a fresh one.
// Exceptions: a task that throws (e.g. std::bad_alloc in the packer) is caught on whichever thread ran it;
// run() still waits for every worker to finish the job before it rethrows the first one, so no worker
// can touch the caller's unwound frame. The extern "C" entry points turn it into an error code.
#pragma once
#include <pthread.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <functional>
#include <mutex>
#include <new>
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
  // f(t) for every t in [0, n); returns when all have run; rethrows the first exception a task threw
  void run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return;
    if (n == 1 || in_task() || th_.empty()) {
      for (int t = 0; t < n; t++) f(t);
      return;
    }
    std::lock_guard<std::mutex> rg(run_mu_);  // one job at a time
    run_locked(n, f);
  }
  // run() if no other thread's job holds the pool; false (nothing run) if one does
  bool try_run(int n, const std::function<void(int)>& f) {
    if (n <= 0) return true;
    if (n == 1 || in_task() || th_.empty()) {
      for (int t = 0; t < n; t++) f(t);
      return true;
    }
    std::unique_lock<std::mutex> rg(run_mu_, std::try_to_lock);
    if (!rg.owns_lock()) return false;
    run_locked(n, f);
    return true;
  }

 private:
  void run_locked(int n, const std::function<void(int)>& f) {
    const int P = std::min(n, threads());
    err_ = nullptr;
    pending_.store(P - 1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(mu_);  // a worker reads (gen, job) together under mu_
      job_ = &f;
      ntask_ = n;
      nthr_ = P;
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    {
      struct InTask {  // reset even when a task throws
        InTask() { in_task() = true; }
        ~InTask() { in_task() = false; }
      } guard;
      run_tasks(f, 0, n, P);
    }
    while (pending_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    if (err_) {
      std::exception_ptr e = err_;
      err_ = nullptr;
      std::rethrow_exception(e);
    }
  }
  static bool& in_task() {
    static thread_local bool flag = false;
    return flag;
  }
  void run_tasks(const std::function<void(int)>& f, int j, int ntask, int nthr) {
    try {
      for (int t = j; t < ntask; t += nthr) f(t);
    } catch (...) {
      std::lock_guard<std::mutex> g(err_mu_);
      if (!err_) err_ = std::current_exception();
    }
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
        run_tasks(*job, j, ntask, nthr);
        in_task() = false;
        pending_.fetch_sub(1, std::memory_order_acq_rel);
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_, err_mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> stop_{false};
  // written by run() before gen_ is bumped (release), read by workers after they see the bump (acquire)
  const std::function<void(int)>* job_ = nullptr;
  int ntask_ = 0, nthr_ = 0;
  std::exception_ptr err_;
};

struct Holder {
  std::mutex mu;
  Pool* p = nullptr;
};

inline Holder& holder() {
  static Holder h;
  return h;
}

// the second pool (side_pool): 8 threads for the upload / download checks while another thread's job (a
// packer's, in a pipelined caller) holds the main one
inline Holder& side_holder() {
  static Holder h;
  return h;
}

// fork() child: only the forking thread exists; forget the parent's pools and reset the creation locks
inline void on_fork_child() {
  for (Holder* h : {&holder(), &side_holder()}) {
    new (&h->mu) std::mutex();
    h->p = nullptr;
  }
}

inline Pool& make(Holder& h, unsigned max_threads) {
  static std::once_flag once;
  std::call_once(once, [] { pthread_atfork(nullptr, nullptr, &on_fork_child); });
  std::lock_guard<std::mutex> g(h.mu);
  if (!h.p) h.p = new Pool((int)std::min<unsigned>(max_threads, std::max(1u, std::thread::hardware_concurrency())) - 1);
  return *h.p;
}

// up to 16 threads (the GPU box's CPU share), created on first use (per process)
inline Pool& pool() { return make(holder(), 16u); }
inline Pool& side_pool() { return make(side_holder(), 8u); }

// a checks job: on the main pool when it is free, else on the side pool (created on first need) rather than
// waiting behind the other thread's job
inline void run_checks(int n, const std::function<void(int)>& f) {
  if (!pool().try_run(n, f)) side_pool().run(n, f);
}

}  // namespace kadpool
