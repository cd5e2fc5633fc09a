// copy_pool.h -- parallel host memcpy for the page-locked bounce ring (host_stage.h).
//
// A copy is cut into 1 MiB chunks claimed from one atomic word; the calling thread copies
// too, and the pool's threads join when they wake up.  The caller waits only for chunks
// already claimed by a worker, never for a worker that has not woken up yet: round 4's pool
// split a copy into one part per thread and waited for every thread, so a thread the host
// scheduled late stalled the whole call (pageable one-frame calls: 8-9 ms stalls in 3 of 7
// rounds, tools/e2e_probe.py enqueue_ms, round 5).  The claim word carries the job's
// generation, so a worker that wakes up after its job has ended (or while a later one runs)
// claims nothing of a job whose parameters it did not read.  No HIP dependency
// (tests/cpp/test_copy_pool.cpp).  The workers run on the CPUs of the engine's NUMA place
// when one is given (numa_place.h).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "numa_place.h"

namespace mipgpu {

class CopyPool {
 public:
  static constexpr size_t kChunk = 1u << 20;
  static constexpr size_t kMinParallel = 4u << 20;  // smaller copies: one memcpy on the caller

  explicit CopyPool(int n, const NumaPlace &place = NumaPlace()) {
    for (int i = 0; i < n; i++)
      th_.emplace_back([this, place] {
        (void)bind_current_thread(place);
        run();
      });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  int threads() const { return (int)th_.size(); }

  // memcpy(dst, src, n) over the caller and the pool; returns when done.
  void copy(void *dst, const void *src, size_t n) {
    if (n < kMinParallel || th_.empty()) {
      memcpy(dst, src, n);
      return;
    }
    Job j{(char *)dst, (const char *)src, n, (uint32_t)((n + kChunk - 1) / kChunk), 0};
    {
      std::lock_guard<std::mutex> lk(mu_);
      j.gen = ++gen_;
      job_ = j;
      done_.store(0, std::memory_order_relaxed);
      claim_.store((uint64_t)j.gen << 32, std::memory_order_release);
    }
    cv_.notify_all();
    work(j);
    while (done_.load(std::memory_order_acquire) < j.nchunks) std::this_thread::yield();
  }

 private:
  struct Job {
    char *dst;
    const char *src;
    size_t n;
    uint32_t nchunks, gen;
  };

  // Claim and copy chunks of job j until none is left (or the job is no longer current).
  void work(const Job &j) {
    uint64_t st = claim_.load(std::memory_order_acquire);
    for (;;) {
      if ((uint32_t)(st >> 32) != j.gen || (uint32_t)st >= j.nchunks) return;
      if (!claim_.compare_exchange_weak(st, st + 1, std::memory_order_acq_rel)) continue;
      const size_t o = (size_t)(uint32_t)st * kChunk;
      memcpy(j.dst + o, j.src + o, std::min(kChunk, j.n - o));
      done_.fetch_add(1, std::memory_order_release);
      st = claim_.load(std::memory_order_acquire);
    }
  }

  void run() {
    uint32_t seen = 0;
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        j = job_;
      }
      work(j);
    }
  }

  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  uint32_t gen_ = 0;
  Job job_{};
  std::atomic<uint64_t> claim_{0};  // (generation << 32) | next chunk
  std::atomic<uint32_t> done_{0};   // chunks of the current job copied
};

}  // namespace mipgpu
