// host_stage.h -- page-locked bounce ring for pageable (malloc'd) host buffers of the host
// pipeline (mip_search_frames[_async]).
//
// DMA from / to pageable memory is staged by the HIP runtime at ~8 GB/s (measured on MI355X,
// profiles/r03_pageable_probe.txt); a copy engine moves ~57 GB/s from page-locked memory and
// eight host threads copy page-locked -> pageable at ~117 GB/s.  So pageable transfers go
// through a ring of page-locked pieces:
//   upload    host memcpy (parallel) pageable -> piece, then the piece's DMA on the upload
//             stream; the piece is free again once that DMA has completed;
//   download  the piece's DMA on the download stream, then -- when a later operation needs
//             the piece, or the call is waited for -- host memcpy (parallel) piece -> pageable.
// Pieces are used round robin, in the order they were enqueued, so the oldest piece in flight
// is always the next one to reuse; `complete_front` finishes it (waits for its DMA, copies a
// download out).  The DMAs stay on the pipeline's streams, so the per-slot events that order
// the device buffers are unchanged: a device buffer is free once the DMA has run, whether or
// not the host copy-out has.  Not thread safe (the engine is used by one host thread at a
// time).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "copy_pool.h"

namespace mipgpu {

class HostStage {
 public:
  // Ring pieces: a chunk's downloads must fit the ring with room for the next chunk's
  // uploads (kMaxChunkPieces), else enqueueing them would wait on the host for the chunk's
  // own search and the next upload could not be queued behind it (mipgpu.cpp caps pageable
  // chunks accordingly).
  static constexpr int kRing = 16;
  static constexpr int kMaxChunkPieces = kRing - 4;
  static constexpr size_t kMaxPiece = 64u << 20;

  ~HostStage() {
    if (getenv("MIPGPU_STAGE_STATS"))  // diagnostic: where the staging time goes
      fprintf(stderr, "mipgpu stage: %d threads; upload copies %.1f ms (%.2f GB), download copies %.1f ms (%.2f GB), "
              "DMA waits %.1f ms\n", threads_, t_up_ * 1e3, b_up_ / 1e9, t_down_ * 1e3, b_down_ / 1e9, t_wait_ * 1e3);
    release();
  }

  // Page-locked host memory (mip_host_alloc / hipHostRegister) or device memory: transfers
  // run at DMA rate without staging.
  static bool pinned(const void *p) {
    hipPointerAttribute_t at{};
    const hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
      (void)hipGetLastError();  // unregistered host memory reports an error: clear it
      return false;
    }
    return at.type == hipMemoryTypeHost || at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
  }

  // Allocate the ring (pieces of `piece` bytes) if it is not there or smaller.
  hipError_t reserve(size_t piece) {
    piece = std::max<size_t>(piece, 1u << 20);
    if (piece_ >= piece) return hipSuccess;
    hipError_t e = drain(~0ull);
    if (e != hipSuccess) return e;
    release();
    for (int i = 0; i < kRing; i++) {
      if ((e = hipHostMalloc((void **)&buf_[i], piece, hipHostMallocDefault)) != hipSuccess) return e;
      if ((e = hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming)) != hipSuccess) return e;
    }
    piece_ = piece;
    if (!pool_) {
      const char *t = getenv("MIPGPU_COPY_THREADS");  // tuning knob: host copy threads
      threads_ = t && atoi(t) >= 1 && atoi(t) <= 64 ? atoi(t) : 8;
      pool_.reset(new CopyPool(threads_));
    }
    return hipSuccess;
  }

  size_t piece() const { return piece_; }

  // Pageable host -> device on stream s (the source is copied before this returns).
  hipError_t upload(void *dst_dev, const void *src, size_t n, hipStream_t s, uint64_t call) {
    for (size_t o = 0; o < n; o += piece_) {
      const size_t len = std::min(piece_, n - o);
      int j;
      hipError_t e = take(&j);
      if (e != hipSuccess) return e;
      const double t0 = now();
      pool_->copy(buf_[j], (const char *)src + o, len);
      t_up_ += now() - t0;
      b_up_ += len;
      if ((e = hipMemcpyAsync((char *)dst_dev + o, buf_[j], len, hipMemcpyHostToDevice, s)) != hipSuccess ||
          (e = hipEventRecord(ev_[j], s)) != hipSuccess)
        return e;
      fifo_.push_back({j, nullptr, len, call});
    }
    return hipSuccess;
  }

  // Device -> pageable host on stream s; the host side is written by complete_front / drain.
  hipError_t download(void *dst, const void *src_dev, size_t n, hipStream_t s, uint64_t call) {
    for (size_t o = 0; o < n; o += piece_) {
      const size_t len = std::min(piece_, n - o);
      int j;
      hipError_t e = take(&j);
      if (e != hipSuccess) return e;
      if ((e = hipMemcpyAsync(buf_[j], (const char *)src_dev + o, len, hipMemcpyDeviceToHost, s)) != hipSuccess ||
          (e = hipEventRecord(ev_[j], s)) != hipSuccess)
        return e;
      fifo_.push_back({j, (char *)dst + o, len, call});
    }
    return hipSuccess;
  }

  // Finish every piece of calls <= `call` (and the pieces enqueued before them).
  hipError_t drain(uint64_t call) {
    while (!fifo_.empty() && fifo_.front().call <= call) {
      const hipError_t e = complete_front();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }

  bool idle() const { return fifo_.empty(); }

  // Drop every piece after its DMA has finished, without copying downloads out (engine
  // teardown: the caller's buffers of calls never waited for may be gone).
  void abandon() {
    for (const Piece &p : fifo_) (void)hipEventSynchronize(ev_[p.ring]);
    fifo_.clear();
  }

 private:
  struct Piece {
    int ring;
    char *dst;  // download: pageable destination; upload: nullptr
    size_t bytes;
    uint64_t call;
  };

  hipError_t complete_front() {
    const Piece p = fifo_.front();
    const double t0 = now();
    const hipError_t e = hipEventSynchronize(ev_[p.ring]);
    const double t1 = now();
    t_wait_ += t1 - t0;
    if (e != hipSuccess) return e;
    if (p.dst) {
      pool_->copy(p.dst, buf_[p.ring], p.bytes);
      t_down_ += now() - t1;
      b_down_ += p.bytes;
    }
    fifo_.pop_front();
    return hipSuccess;
  }

  hipError_t take(int *j) {
    if ((int)fifo_.size() == kRing) {
      const hipError_t e = complete_front();
      if (e != hipSuccess) return e;
    }
    *j = next_;
    next_ = (next_ + 1) % kRing;
    return hipSuccess;
  }

  void release() {
    for (int i = 0; i < kRing; i++) {
      if (buf_[i]) (void)hipHostFree(buf_[i]);
      if (ev_[i]) (void)hipEventDestroy(ev_[i]);
      buf_[i] = nullptr;
      ev_[i] = nullptr;
    }
    piece_ = 0;
    next_ = 0;
  }

  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  int threads_ = 0;
  double t_up_ = 0, t_down_ = 0, t_wait_ = 0, b_up_ = 0, b_down_ = 0;
  char *buf_[kRing] = {};
  hipEvent_t ev_[kRing] = {};
  size_t piece_ = 0;
  int next_ = 0;
  std::deque<Piece> fifo_;
  std::unique_ptr<CopyPool> pool_;
};

}  // namespace mipgpu
