// thread_pool.h -- the host worker pool of a libfgv context (block parse / policy fold in
// fgv_block.cpp; block data hashing in fgv_integrity.cpp, which owns a second pool so the
// deliver-side hash can run concurrently with a committer call, as in a pipelined peer).
#pragma once
#include <stddef.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

struct ThreadPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::function<void(size_t)> job;
  size_t njobs = 0;
  std::atomic<size_t> next{0};
  size_t active = 0;
  std::atomic<uint64_t> gen{0};
  bool stop = false;
  // A worker that finished a run may spin this long for the next one before sleeping (a
  // futex wake-up of 16 threads costs tens of microseconds).  Off: the committer's device
  // path issues one run per call, and spinning threads only compete with the caller when
  // the host's CPU share is tight.
  static constexpr auto kSpin = std::chrono::microseconds(0);
  explicit ThreadPool(unsigned n) {
    for (unsigned i = 0; i < n; i++)
      th.emplace_back([this] {
        uint64_t seen = 0;
        for (;;) {
          const auto t0 = std::chrono::steady_clock::now();
          while (gen.load(std::memory_order_acquire) == seen && std::chrono::steady_clock::now() - t0 < kSpin)
            std::this_thread::yield();
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return stop || gen.load() != seen; });
          if (stop) return;
          seen = gen.load();
          lk.unlock();
          for (size_t i; (i = next.fetch_add(1)) < njobs;) job(i);
          lk.lock();
          if (--active == 0) done_cv.notify_all();
        }
      });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  // run f(j) for every job j in [0, njobs) on the pool (dynamic assignment); the calling
  // thread takes jobs too while the workers wake up
  void run(size_t nj, const std::function<void(size_t)> &f) {
    if (nj == 0) return;
    if (th.empty() || nj == 1) {
      for (size_t i = 0; i < nj; i++) f(i);
      return;
    }
    std::unique_lock<std::mutex> lk(mu);
    job = f;
    njobs = nj;
    next = 0;
    active = th.size();
    gen.fetch_add(1, std::memory_order_release);
    lk.unlock();
    cv.notify_all();
    for (size_t i; (i = next.fetch_add(1)) < nj;) f(i);
    lk.lock();
    done_cv.wait(lk, [&] { return active == 0; });
  }
  // run f(i) for i in [0, n) in chunks
  void parallel_for(size_t n, const std::function<void(size_t)> &f) {
    if (n == 0) return;
    if (th.empty() || n < 64) {
      for (size_t i = 0; i < n; i++) f(i);
      return;
    }
    const size_t chunk = std::max<size_t>(16, n / (th.size() * 8));
    run((n + chunk - 1) / chunk, [&](size_t c) {
      size_t lo = c * chunk, hi = std::min(n, lo + chunk);
      for (size_t i = lo; i < hi; i++) f(i);
    });
  }
};

