// plan_pool.hpp — the host planner's worker threads (plan.cpp, tiles.cpp).
#pragma once

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>

namespace dynohip {

// The planner's workers: threads created once per process and reused by
// every plan (a plan runs a dozen parallel sections; creating 16 threads for
// each cost milliseconds). run(nw, body) calls body(0..nw-1), body(0) on the
// calling thread, and returns when all are done. A plan's sections come back
// to back, so an idle worker spins on the section counter for a while before
// it blocks on the condition variable (waking a blocked thread costs tens of
// microseconds per section), and the caller spins until its helpers are
// done. An exception in a body (any worker's) reaches the caller of run()
// after every helper has finished. Never destroyed: the threads block until
// the process exits.
class PlanPool {
 public:
  static PlanPool& get() {
    // a forked child has none of the parent's threads: it starts its own pool
    static PlanPool* p = nullptr;
    static pid_t owner = 0;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (!p || owner != getpid()) {
      p = new PlanPool();
      owner = getpid();
    }
    return *p;
  }
  // (a PlanCap on the calling thread lowers both: a section sized by
  // workers() never asks run() for more workers than it gets)
  int workers() const { return cap() > 0 ? std::min(nmax_, cap()) : nmax_; }
  static int& cap() {
    static thread_local int c = 0;
    return c;
  }
  template <typename Body>
  void run(int nw, Body&& body) {
    nw = std::max(1, std::min(nw, workers()));
    if (nw == 1) {
      body(0);
      return;
    }
    std::unique_lock<std::mutex> call(call_mu_);   // one parallel section at a time
    std::function<void(int)> fn = [&body](int r) { body(r); };
    fn_ = &fn;
    pending_.store(nw - 1, std::memory_order_relaxed);
    {
      // the section word carries its worker count: a worker decides from the
      // word it saw, never from a later section's
      std::lock_guard<std::mutex> lk(mu_);
      gen_.store(((gen_.load(std::memory_order_relaxed) >> 8) + 1) << 8 | static_cast<uint64_t>(nw),
                 std::memory_order_release);
    }
    if (sleepers_.load(std::memory_order_acquire) > 0) cv_.notify_all();
    // the helpers call through fn_, which lives in this frame: wait for them
    // however body(0) ends, then rethrow the first exception of any worker
    std::exception_ptr mine;
    try {
      body(0);
    } catch (...) {
      mine = std::current_exception();
    }
    while (pending_.load(std::memory_order_acquire) != 0) pause();
    fn_ = nullptr;
    std::exception_ptr theirs;
    {
      std::lock_guard<std::mutex> lk(mu_);
      theirs = err_;
      err_ = nullptr;
    }
    if (mine) std::rethrow_exception(mine);
    if (theirs) std::rethrow_exception(theirs);
  }

 private:
  static void pause() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  }
  PlanPool() {
    const unsigned hc = std::thread::hardware_concurrency();
    nmax_ = static_cast<int>(std::max(1u, std::min(16u, hc ? hc : 1u)));
    // DYNOHIP_PLAN_WORKERS caps the pool (1 = the single-threaded build the
    // parallel sections must reproduce bit for bit; tests/test_plan_digest.py)
    if (const char* e = std::getenv("DYNOHIP_PLAN_WORKERS"))
      nmax_ = std::max(1, std::min(nmax_, std::atoi(e)));
    // DYNOHIP_PLAN_SPIN_US: how long an idle worker spins before it blocks
    if (const char* e = std::getenv("DYNOHIP_PLAN_SPIN_US")) spin_us_ = std::max(0, std::atoi(e));
    for (int r = 1; r < nmax_; ++r) std::thread([this, r] { loop(r); }).detach();
  }
  void loop(int r) {
    uint64_t seen = 0;
    for (;;) {
      // spin for the next section a while, then block
      uint64_t g = gen_.load(std::memory_order_acquire);
      if (g == seen && spin_us_ > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 1; (g = gen_.load(std::memory_order_acquire)) == seen; ++k) {
          pause();
          if ((k & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) break;
        }
      }
      if (g == seen) {
        std::unique_lock<std::mutex> lk(mu_);
        sleepers_.fetch_add(1, std::memory_order_acq_rel);
        cv_.wait(lk, [&] { return (g = gen_.load(std::memory_order_acquire)) != seen; });
        sleepers_.fetch_sub(1, std::memory_order_acq_rel);
      }
      seen = g;
      if (r >= static_cast<int>(g & 255)) continue;
      try {
        (*fn_)(r);
      } catch (...) {   // handed to the caller of run(); the worker lives on
        std::lock_guard<std::mutex> lk(mu_);
        if (!err_) err_ = std::current_exception();
      }
      pending_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  int nmax_ = 1, spin_us_ = 500;
  std::mutex call_mu_, mu_;
  std::condition_variable cv_;
  std::function<void(int)>* fn_ = nullptr;
  std::exception_ptr err_;   // first exception of a helper in the current section
  std::atomic<int> pending_{0}, sleepers_{0};
  std::atomic<uint64_t> gen_{0};
};

// Caps the parallel sections of the calling thread at `c` workers (0: none)
// for its lifetime. A sliding window's plan (a few thousand factors) is
// faster on one thread than with the pool's wake-ups per section (set_values
// 1.26-1.29 against 1.37-1.43 ms per C2-stream window in one A/B run,
// profiles/r05/window/plan_cap_ab.log); the plan is the same either way
// (tests/test_plan_digest.py compares the capped small plans with the same
// plans built threaded, DYNOHIP_SMALL_PLAN_ITEMS=0).
struct PlanCap {
  int prev;
  explicit PlanCap(int c) : prev(PlanPool::cap()) { PlanPool::cap() = c; }
  ~PlanCap() { PlanPool::cap() = prev; }
  PlanCap(const PlanCap&) = delete;
  PlanCap& operator=(const PlanCap&) = delete;
};

// body(b, e) over [0, n) in contiguous ranges on the planner's workers
template <typename Body>
void parallel_for(int64_t n, Body&& body) {
  const int nw = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(PlanPool::get().workers(), n / 8192 + 1)));
  PlanPool::get().run(nw, [&](int r) { body(n * r / nw, n * (r + 1) / nw); });
}

// body(b, e) over chunks of [0, n) handed out one at a time (work of uneven
// size per item, e.g. chains sorted longest first)
template <typename Body>
void parallel_chunks(int64_t n, int64_t chunk, Body&& body) {
  const int64_t nch = (n + chunk - 1) / chunk;
  const int nw = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(PlanPool::get().workers(), nch)));
  std::atomic<int64_t> next{0};
  PlanPool::get().run(nw, [&](int) {
    for (int64_t k; (k = next.fetch_add(1, std::memory_order_relaxed)) < nch;)
      body(k * chunk, std::min(n, (k + 1) * chunk));
  });
}

}  // namespace dynohip
