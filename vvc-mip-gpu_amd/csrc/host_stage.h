// host_stage.h -- page-locked bounce ring for pageable (malloc'd) host buffers of the host
// pipeline (mip_search_frames[_async]).
//
// DMA from / to pageable memory is staged by the HIP runtime at ~8 GB/s (measured on MI355X,
// profiles/r03_pageable_probe.txt); a copy engine moves ~57 GB/s from page-locked memory and
// eight host threads copy page-locked -> pageable at ~117 GB/s.  So pageable transfers go
// through a ring of page-locked pieces:
//   upload    host memcpy (parallel) pageable -> piece, then the piece's DMA on the upload
//             stream; the piece is free again once that DMA has completed;
//   download  the piece's DMA on the download stream, then host memcpy (parallel) piece ->
//             pageable, done by the ring's own completion thread as soon as the DMA has
//             completed (round 5; before, the copy-out ran on the caller's thread when the
//             piece was reused or the call waited for, so for one-frame calls it piled up at
//             mip_wait after the GPU had finished).
// Pieces are used round robin, in the order they were enqueued; the completion thread
// finishes them in that order (waits for the piece's DMA, copies a download out) and the
// caller reuses the oldest piece once it is finished.  The DMAs stay on the pipeline's
// streams, so the per-slot events that order the device buffers are unchanged: a device
// buffer is free once the DMA has run, whether or not the host copy-out has.  The public
// calls are made by one host thread at a time (the engine's rule); the completion thread
// shares the piece queue with it under a mutex.
//
// The ring is a template over its device operations (page-locked allocation, async copies,
// events), so the queue / thread logic is unit-tested on the CPU with a simulated device
// (tests/cpp/test_host_stage.cpp); host_stage_hip.h binds it to HIP.
#pragma once
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

#include "copy_pool.h"

namespace mipgpu {

// Dev provides: types Err, Stream, Event; static constexpr Err kOk; and
//   Err host_alloc(char **p, size_t n);        void host_free(char *p);
//   Err event_create(Event *e);                void event_destroy(Event e);
//   Err copy_h2d(void *dev, const void *host, size_t n, Stream s);
//   Err copy_d2h(void *host, const void *dev, size_t n, Stream s);
//   Err record(Event e, Stream s);             Err sync(Event e);
//   void bind_thread(int device);             (the completion thread's device)
template <class Dev>
class BounceRing {
 public:
  using Err = typename Dev::Err;
  using Stream = typename Dev::Stream;
  using Event = typename Dev::Event;

  // Ring pieces: a chunk's downloads must fit the ring with room for the next chunk's
  // uploads (kMaxChunkPieces), else enqueueing them would wait on the host for the chunk's
  // own search and the next upload could not be queued behind it (mipgpu.cpp caps pageable
  // chunks accordingly).
  static constexpr int kRing = 16;
  static constexpr int kMaxChunkPieces = kRing - 4;
  static constexpr size_t kMaxPiece = 64u << 20;
  static constexpr size_t kMinPiece = 1u << 20;

  explicit BounceRing(Dev dev = Dev()) : dev_(dev) {}
  ~BounceRing() {
    if (getenv("MIPGPU_STAGE_STATS"))  // diagnostic: where the staging time goes
      fprintf(stderr, "mipgpu stage: %d threads; upload copies %.1f ms (%.2f GB), download copies %.1f ms (%.2f GB), "
              "DMA waits %.1f ms\n", threads_, t_up_ * 1e3, b_up_ / 1e9, t_down_ * 1e3, b_down_ / 1e9, t_wait_ * 1e3);
    abandon();
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_work_.notify_all();
    if (worker_.joinable()) worker_.join();
    release();
  }
  void set_device(int device) { device_ = device; }
  Dev &dev() { return dev_; }

  // Allocate the ring (pieces of `piece` bytes) if it is not there or smaller.
  Err reserve(size_t piece) {
    piece = std::max(piece, kMinPiece);
    if (piece_ >= piece) return Dev::kOk;
    Err e = drain(~0ull);
    if (e != Dev::kOk) return e;
    release();
    for (int i = 0; i < kRing; i++) {
      if ((e = dev_.host_alloc(&buf_[i], piece)) != Dev::kOk) return e;
      if ((e = dev_.event_create(&ev_[i])) != Dev::kOk) return e;
      have_ev_[i] = true;
    }
    piece_ = piece;
    if (!pool_) {
      const char *t = getenv("MIPGPU_COPY_THREADS");  // tuning knob: host copy threads
      threads_ = t && atoi(t) >= 1 && atoi(t) <= 64 ? atoi(t) : 8;
      pool_.reset(new CopyPool(threads_));
    }
    if (!worker_.joinable()) worker_ = std::thread([this] { complete_loop(); });
    return Dev::kOk;
  }

  size_t piece() const { return piece_; }

  // Pageable host -> device on stream s (the source is copied before this returns).
  Err upload(void *dst_dev, const void *src, size_t n, Stream s, uint64_t call) {
    for (size_t o = 0; o < n; o += piece_) {
      const size_t len = std::min(piece_, n - o);
      int j = 0;
      Err e = take(&j);
      if (e != Dev::kOk) return e;
      const double t0 = now();
      pool_copy(buf_[j], (const char *)src + o, len);
      t_up_ += now() - t0;
      b_up_ += len;
      if ((e = dev_.copy_h2d((char *)dst_dev + o, buf_[j], len, s)) != Dev::kOk ||
          (e = dev_.record(ev_[j], s)) != Dev::kOk)
        return e;
      push({j, nullptr, len, call, false});
    }
    return Dev::kOk;
  }

  // Device -> pageable host on stream s; the host side is written by the completion thread
  // (complete for every call <= c once drain(c) returns).
  Err download(void *dst, const void *src_dev, size_t n, Stream s, uint64_t call) {
    for (size_t o = 0; o < n; o += piece_) {
      const size_t len = std::min(piece_, n - o);
      int j = 0;
      Err e = take(&j);
      if (e != Dev::kOk) return e;
      if ((e = dev_.copy_d2h(buf_[j], (const char *)src_dev + o, len, s)) != Dev::kOk ||
          (e = dev_.record(ev_[j], s)) != Dev::kOk)
        return e;
      push({j, (char *)dst + o, len, call, false});
    }
    return Dev::kOk;
  }

  // Wait until every piece of calls <= `call` (and the pieces enqueued before them) is
  // finished, and retire them.
  Err drain(uint64_t call) {
    std::unique_lock<std::mutex> lk(mu_);
    while (!fifo_.empty() && fifo_.front().call <= call) {
      cv_done_.wait(lk, [&] { return fifo_.front().done; });
      pop_front();
    }
    return take_error();
  }

  bool idle() {
    std::lock_guard<std::mutex> lk(mu_);
    return fifo_.empty();
  }

  // Drop every piece after its DMA has finished, without copying downloads out (engine
  // teardown, failed calls: the caller's buffers of calls never waited for may be gone).
  // A download piece the completion thread is copying out already is finished first.
  void abandon() {
    std::unique_lock<std::mutex> lk(mu_);
    skip_copy_ = true;
    cv_done_.wait(lk, [&] { return fifo_.empty() || fifo_.back().done; });
    while (!fifo_.empty()) pop_front();
    skip_copy_ = false;
    err_ = Dev::kOk;
  }

 private:
  struct Piece {
    int ring;
    char *dst;  // download: pageable destination; upload: nullptr
    size_t bytes;
    uint64_t call;
    bool done;
  };

  void push(Piece p) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      fifo_.push_back(p);
    }
    cv_work_.notify_one();
  }

  // The completion thread: finishes pieces in queue order.  Pieces are numbered by their
  // position in the whole sequence (fifo_.front() is number popped_), so the thread's next
  // piece, finished_, stays valid while the caller retires finished pieces at the front.
  void complete_loop() {
    dev_.bind_thread(device_);
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_work_.wait(lk, [&] { return stop_ || finished_ - popped_ < fifo_.size(); });
      if (finished_ - popped_ >= fifo_.size()) return;  // stop_, nothing left
      const Piece p = fifo_[finished_ - popped_];
      lk.unlock();
      const double t0 = now();
      const Err e = dev_.sync(ev_[p.ring]);
      const double t1 = now();
      bool copied = false;
      if (e == Dev::kOk && p.dst) {
        lk.lock();
        const bool skip = skip_copy_;  // read after the DMA: abandon() may have come meanwhile
        lk.unlock();
        if (!skip) {
          pool_copy(p.dst, buf_[p.ring], p.bytes);
          copied = true;
        }
      }
      const double t2 = now();
      lk.lock();
      t_wait_ += t1 - t0;
      if (copied) {
        t_down_ += t2 - t1;
        b_down_ += p.bytes;
      }
      if (e != Dev::kOk && err_ == Dev::kOk) err_ = e;
      fifo_[finished_ - popped_].done = true;  // (the caller pops only finished pieces)
      finished_++;
      cv_done_.notify_all();
    }
  }

  void pop_front() {  // (mu_ held; the front piece is finished)
    fifo_.pop_front();
    popped_++;
  }

  Err take_error() {  // (mu_ held)
    const Err e = err_;
    err_ = Dev::kOk;
    return e;
  }

  // The next ring piece (the oldest one, once it is finished, when all are in use).
  Err take(int *j) {
    std::unique_lock<std::mutex> lk(mu_);
    if ((int)fifo_.size() == kRing) {
      cv_done_.wait(lk, [&] { return fifo_.front().done; });
      pop_front();
      const Err e = take_error();
      if (e != Dev::kOk) return e;
    }
    *j = next_;
    next_ = (next_ + 1) % kRing;
    return Dev::kOk;
  }

  void pool_copy(void *d, const void *s, size_t n) {
    std::lock_guard<std::mutex> lk(pool_mu_);  // one copy job at a time (caller and completion thread)
    pool_->copy(d, s, n);
  }

  void release() {
    for (int i = 0; i < kRing; i++) {
      if (buf_[i]) dev_.host_free(buf_[i]);
      if (have_ev_[i]) dev_.event_destroy(ev_[i]);
      buf_[i] = nullptr;
      have_ev_[i] = false;
    }
    piece_ = 0;
    next_ = 0;
  }

  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  Dev dev_;
  int device_ = 0;
  int threads_ = 0;
  double t_up_ = 0, t_down_ = 0, t_wait_ = 0, b_up_ = 0, b_down_ = 0;
  char *buf_[kRing] = {};
  Event ev_[kRing] = {};
  bool have_ev_[kRing] = {};
  size_t piece_ = 0;
  int next_ = 0;
  std::mutex mu_, pool_mu_;
  std::condition_variable cv_work_, cv_done_;
  std::deque<Piece> fifo_;
  uint64_t popped_ = 0, finished_ = 0;  // pieces retired from the front of fifo_ / finished
  bool stop_ = false, skip_copy_ = false;
  Err err_ = Dev::kOk;
  std::unique_ptr<CopyPool> pool_;
  std::thread worker_;
};

}  // namespace mipgpu
