// parallel.h -- a persistent host thread pool for the per-user scalar math of
// the weighted models (ComputeUserWeights, the per-sample terms of the
// smoothed-quantile objective).  The reference spawns hardware_concurrency()
// threads per call (safer2.h:745-794); here the pool lives for the process
// and is sized to the CPU share the process actually has: OMP_NUM_THREADS
// when set (the GPU boxes give one GPU 16 CPUs of a larger machine), else
// the affinity mask.  Work is split into contiguous index ranges, so every
// result that is written per index is identical to the serial loop's.
#pragma once

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace frecsys {

class ThreadPool {
 public:
  static ThreadPool& Get() {
    static ThreadPool pool(DefaultThreads());
    return pool;
  }

  static int DefaultThreads() {
    if (const char* e = getenv("OMP_NUM_THREADS")) {
      const int v = atoi(e);
      if (v > 0) return std::min(v, 64);
    }
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::clamp(CPU_COUNT(&set), 1, 64);
    return (int)std::clamp(std::thread::hardware_concurrency(), 1u, 64u);
  }

  int size() const { return (int)workers_.size() + 1; }

  // fn(lo, hi) over [0, n) in contiguous ranges; the caller runs one range.
  // Small n runs inline, and so does a call made while the pool serves
  // another caller (models trained from two host threads, or a nested call
  // from inside a task): the pool holds one job at a time, and the per-index
  // results do not depend on the split.
  //
  // The smoothed-quantile Newton issues ~12 jobs of ~30 us each back to
  // back per epoch; a condition-variable hand-off per job (futex wake of
  // every worker, then a futex wait for the last one) cost more than the
  // work.  So the hand-off is lock-free: workers spin on the job generation
  // for up to kSpinUs after their last task before they sleep, and the
  // caller spins until the job is drained.
  //
  // Job lifetime.  gen_ is odd while a job is open, even between jobs.  The
  // caller writes the job (job_, n_, tasks_, next_), opens it (gen_ odd),
  // runs tasks until none is left, closes it (gen_ even) and then waits for
  // active_ == 0.  A worker that saw open generation g joins it by
  // incrementing active_ and only then re-reads gen_: if g is no longer open
  // it backs off without touching the job.  The two seq_cst pairs
  // (worker: active_++ then gen_ load; caller: gen_++ then active_ load)
  // guarantee that either the worker sees the job closed or the caller sees
  // the worker counted, so a job's fields are never rewritten while a worker
  // that joined it still reads them.
  void ParallelFor(int64_t n, int64_t min_per_task,
                   const std::function<void(int64_t, int64_t)>& fn) {
    const int64_t tasks =
        std::max<int64_t>(1, std::min<int64_t>(size(), n / std::max<int64_t>(1, min_per_task)));
    bool idle = false;
    if (tasks <= 1 || workers_.empty() ||
        !busy_.compare_exchange_strong(idle, true, std::memory_order_acquire,
                                       std::memory_order_relaxed)) {
      if (n > 0) fn(0, n);
      return;
    }
    job_ = &fn;
    n_ = n;
    tasks_ = tasks;
    next_.store(1, std::memory_order_relaxed);
    gen_.fetch_add(1, std::memory_order_seq_cst);  // open (odd)
    if (sleepers_.load(std::memory_order_seq_cst) > 0) {
      std::lock_guard<std::mutex> lk(mu_);
      cv_.notify_all();
    }
    fn(0, n / tasks);  // task 0 on the caller
    // then any task no worker has taken yet
    for (int64_t t; (t = next_.fetch_add(1, std::memory_order_relaxed)) < tasks;)
      fn(n * t / tasks, n * (t + 1) / tasks);
    gen_.fetch_add(1, std::memory_order_seq_cst);  // close (even): no new worker joins
    // every worker that joined has finished its tasks and left the job
    while (active_.load(std::memory_order_seq_cst) > 0) Relax();
    job_ = nullptr;
    busy_.store(false, std::memory_order_release);
  }

  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true);
      cv_.notify_all();
    }
    for (auto& t : workers_) t.join();
  }

 private:
  static constexpr int kSpinUs = 300;

  static void Relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
  }

  explicit ThreadPool(int n) {
    for (int i = 1; i < n; ++i) workers_.emplace_back([this] { Loop(); });
  }

  // an open job this worker has not joined yet
  static bool Joinable(uint64_t g, uint64_t seen) { return (g & 1) && g != seen; }

  void Loop() {
    uint64_t seen = 0;
    for (;;) {
      // wait for a new job: spin, then sleep
      auto t0 = std::chrono::steady_clock::now();
      int spins = 0;
      uint64_t g;
      while (!Joinable(g = gen_.load(std::memory_order_acquire), seen)) {
        if (stop_.load(std::memory_order_acquire)) return;
        Relax();
        if ((++spins & 255) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs)) {
          std::unique_lock<std::mutex> lk(mu_);
          sleepers_.fetch_add(1, std::memory_order_seq_cst);
          cv_.wait(lk, [&] {
            return stop_.load(std::memory_order_acquire) ||
                   Joinable(gen_.load(std::memory_order_seq_cst), seen);
          });
          sleepers_.fetch_sub(1, std::memory_order_relaxed);
          t0 = std::chrono::steady_clock::now();
        }
      }
      seen = g;
      active_.fetch_add(1, std::memory_order_seq_cst);
      if (gen_.load(std::memory_order_seq_cst) == g) {  // still open: joined
        const std::function<void(int64_t, int64_t)>& job = *job_;
        const int64_t n = n_, tasks = tasks_;
        for (int64_t t; (t = next_.fetch_add(1, std::memory_order_relaxed)) < tasks;)
          job(n * t / tasks, n * (t + 1) / tasks);
      }
      active_.fetch_sub(1, std::memory_order_release);
    }
  }

  std::vector<std::thread> workers_;
  std::atomic<bool> busy_{false};  // a caller's job owns the pool
  std::mutex mu_;                  // sleeping workers only
  std::condition_variable cv_;
  const std::function<void(int64_t, int64_t)>* job_ = nullptr;
  int64_t n_ = 0, tasks_ = 0;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int64_t> next_{0};
  std::atomic<int> active_{0}, sleepers_{0};
  std::atomic<bool> stop_{false};
};

}  // namespace frecsys
