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
  // another caller (models trained from two host threads, or a nested call):
  // the pool holds one job at a time, and the per-index results do not
  // depend on the split.
  void ParallelFor(int64_t n, int64_t min_per_task,
                   const std::function<void(int64_t, int64_t)>& fn) {
    const int64_t tasks =
        std::max<int64_t>(1, std::min<int64_t>(size(), n / std::max<int64_t>(1, min_per_task)));
    std::unique_lock<std::mutex> owner(call_mu_, std::try_to_lock);
    if (tasks <= 1 || workers_.empty() || !owner.owns_lock()) {
      if (n > 0) fn(0, n);
      return;
    }
    {
      std::unique_lock<std::mutex> lk(mu_);
      job_ = &fn;
      n_ = n;
      tasks_ = tasks;
      next_ = 1;
      pending_ = tasks - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0, n / tasks);  // task 0 on the caller
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

  ~ThreadPool() {
    {
      std::unique_lock<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  explicit ThreadPool(int n) {
    for (int i = 1; i < n; ++i) workers_.emplace_back([this] { Loop(); });
  }

  void Loop() {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || (gen_ != seen && next_ < tasks_); });
      if (stop_) return;
      seen = gen_;
      while (next_ < tasks_) {
        const int64_t t = next_++;
        const auto* job = job_;
        const int64_t lo = n_ * t / tasks_, hi = n_ * (t + 1) / tasks_;
        lk.unlock();
        (*job)(lo, hi);
        lk.lock();
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }

  std::vector<std::thread> workers_;
  std::mutex call_mu_;  // held by the caller whose job the pool runs
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t, int64_t)>* job_ = nullptr;
  int64_t n_ = 0, tasks_ = 0, next_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace frecsys
