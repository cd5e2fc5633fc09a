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
// Parts are taken from the ring in the order they are enqueued; the completion thread
// finishes them in that order (waits for the part's DMA, copies a download out) and the
// caller reuses the oldest part's bytes once it is finished.  The DMAs stay on the pipeline's
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
#include <vector>

#include "copy_pool.h"

namespace mipgpu {

// Dev provides: types Err, Stream, Event; static constexpr Err kOk, kNotReady (a transfer
// before reserve()); and
//   Err host_alloc(char **p, size_t n, bool numa_user);   void host_free(char *p);
//                                             (numa_user: the pages follow the calling
//                                             thread's memory policy, numa_place.h)
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

  // The ring is one page-locked arena of kRing pieces' worth of bytes; a transfer is cut into
  // parts of at most one piece, and each part takes only its own bytes (rounded to kAlign) at
  // the arena's head, so small transfers (decisions-only outputs, one frame's upload) do not
  // each hold a whole piece (round 5: with fixed pieces a decisions-only one-frame call held
  // three 4 MB pieces for 4 MB of data and a few KB of results, and 8 queued calls stalled on
  // the ring).  Parts are retired in the order they were enqueued; at most kEvents are in
  // flight (one event each).  A chunk's downloads must fit the ring with room for the next
  // chunk's uploads (kMaxChunkPieces pieces of downloads; the wasted tail of a wrap is less
  // than one piece), else enqueueing them would wait on the host for the chunk's own search
  // and the next upload could not be queued behind it (mipgpu.cpp caps pageable chunks by
  // footprint()).
  static constexpr int kRing = 16;
  static constexpr int kMaxChunkPieces = kRing - 5;
  static constexpr int kMaxChunkUploadPieces = 4;
  static constexpr int kEvents = 64;
  static constexpr size_t kMaxPiece = 64u << 20;
  static constexpr size_t kMinPiece = 1u << 20;
  static constexpr size_t kAlign = 4096;  // default part alignment (MIPGPU_RING_ALIGN: tuning knob)

  explicit BounceRing(Dev dev = Dev()) : dev_(dev), trace_path_(getenv("MIPGPU_STAGE_TRACE")) {}
  ~BounceRing() {
    if (getenv("MIPGPU_STAGE_STATS"))  // diagnostic: where the staging time goes
      fprintf(stderr, "mipgpu stage: %d threads; upload copies %.1f ms (%.2f GB), download copies %.1f ms (%.2f GB), "
              "DMA waits %.1f ms, ring-full waits %.1f ms\n", threads_, t_up_ * 1e3, b_up_ / 1e9, t_down_ * 1e3,
              b_down_ / 1e9, t_wait_ * 1e3, t_full_ * 1e3);
    abandon();
    dump_trace();
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_work_.notify_all();
    if (worker_.joinable()) worker_.join();
    release();
  }
  void set_device(int device) { device_ = device; }
  // NUMA placement of the ring (numa_place.h): the arena's pages, the copy pool's and the
  // completion thread's CPUs.  Before the first reserve().
  void set_place(const NumaPlace &p) { place_ = p; }

  // Allocate the ring (kRing pieces of `piece` bytes) if it is not there or smaller.
  Err reserve(size_t piece) {
    if (const char *a = getenv("MIPGPU_RING_ALIGN")) {
      const size_t v = strtoull(a, nullptr, 0);
      if (v >= kAlign && v <= kMaxPiece && !(v & (v - 1))) align_ = v;
    }
    piece = round_up(std::max(piece, kMinPiece));
    if (piece_ >= piece) return Dev::kOk;
    Err e = drain(~0ull);
    if (e != Dev::kOk) return e;
    release();
    {
      const ScopedNodePolicy pol(place_);  // (the arena's pages on the GPU's node)
      e = dev_.host_alloc(&arena_, piece * kRing, pol.applied());
    }
    if (e != Dev::kOk) {
      arena_ = nullptr;
      return e;
    }
    for (int i = 0; i < kEvents; i++) {
      if ((e = dev_.event_create(&ev_[i])) != Dev::kOk) return e;
      have_ev_[i] = true;
    }
    piece_ = piece;
    cap_ = piece * kRing;
    if (const char *r = getenv("MIPGPU_RING_PIECES")) {  // tuning knob: ring bytes in use (pieces)
      const int v = atoi(r);
      if (v >= 4 && v < kRing) cap_ = piece * v;
    }
    if (!pool_) {
      const char *t = getenv("MIPGPU_COPY_THREADS");  // tuning knob: host copy threads
      threads_ = t && atoi(t) >= 1 && atoi(t) <= 64 ? atoi(t) : 8;
      pool_.reset(new CopyPool(threads_, place_));
    }
    if (!worker_.joinable()) worker_ = std::thread([this] { complete_loop(); });
    return Dev::kOk;
  }

  size_t piece() const { return piece_; }
  uint64_t bad_takes() const { return bad_takes_; }  // (MIPGPU_RING_CHECK builds)
  // Ring bytes a transfer of `bytes` takes (0 for none).
  size_t footprint(size_t bytes) const { return round_up(bytes); }

  // Pageable host -> device on stream s (the source is copied before this returns).
  Err upload(void *dst_dev, const void *src, size_t n, Stream s, uint64_t call) {
    if (!piece_) return Dev::kNotReady;
    for (size_t o = 0; o < n; o += piece_) {
      const size_t len = std::min(piece_, n - o);
      Piece p{0, len, nullptr, call, 0, false};
      Err e = take(&p);
      if (e != Dev::kOk) return e;
      const double t0 = now();
      pool_copy(arena_ + p.off, (const char *)src + o, len);
      t_up_ += now() - t0;
      b_up_ += len;
      if ((e = dev_.copy_h2d((char *)dst_dev + o, arena_ + p.off, len, s)) != Dev::kOk ||
          (e = dev_.record(ev_[p.ev], s)) != Dev::kOk)
        return e;
      push(p);
    }
    return Dev::kOk;
  }

  // Device -> pageable host on stream s; the host side is written by the completion thread
  // (complete for every call <= c once drain(c) returns).
  Err download(void *dst, const void *src_dev, size_t n, Stream s, uint64_t call) {
    if (!piece_) return Dev::kNotReady;
    for (size_t o = 0; o < n; o += piece_) {
      const size_t len = std::min(piece_, n - o);
      Piece p{0, len, (char *)dst + o, call, 0, false};
      Err e = take(&p);
      if (e != Dev::kOk) return e;
      if ((e = dev_.copy_d2h(arena_ + p.off, (const char *)src_dev + o, len, s)) != Dev::kOk ||
          (e = dev_.record(ev_[p.ev], s)) != Dev::kOk)
        return e;
      push(p);
    }
    return Dev::kOk;
  }

  // Wait until every part of calls <= `call` (and the parts enqueued before them) is
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

  // Drop every part after its DMA has finished, without copying downloads out (engine
  // teardown, failed calls: the caller's buffers of calls never waited for may be gone).
  // A download part the completion thread is copying out already is finished first.
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
    size_t off;  // arena offset
    size_t bytes;
    char *dst;  // download: pageable destination; upload: nullptr
    uint64_t call;
    int ev;
    bool done;
  };

  size_t round_up(size_t n) const { return (n + align_ - 1) / align_ * align_; }

  void push(const Piece &p) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      fifo_.push_back(p);
      trace('P', popped_ + fifo_.size() - 1, p);
    }
    cv_work_.notify_one();
  }

  // The completion thread: finishes parts in queue order.  Parts are numbered by their
  // position in the whole sequence (fifo_.front() is number popped_), so the thread's next
  // part, finished_, stays valid while the caller retires finished parts at the front.
  void complete_loop() {
    dev_.bind_thread(device_);
    (void)bind_current_thread(place_);
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_work_.wait(lk, [&] { return stop_ || finished_ - popped_ < fifo_.size(); });
      if (finished_ - popped_ >= fifo_.size()) return;  // stop_, nothing left
      const Piece p = fifo_[finished_ - popped_];
      lk.unlock();
      const double t0 = now();
      const Err e = dev_.sync(ev_[p.ev]);
      const double t1 = now();
      bool copied = false;
      if (e == Dev::kOk && p.dst) {
        lk.lock();
        const bool skip = skip_copy_;  // read after the DMA: abandon() may have come meanwhile
        lk.unlock();
        if (!skip) {
          pool_copy(p.dst, arena_ + p.off, p.bytes);
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
      if (trace_path_) {
        trace('D', finished_, p, t1);
        trace('C', finished_, p, t2);
      }
      fifo_[finished_ - popped_].done = true;  // (the caller pops only finished parts)
      finished_++;
      cv_done_.notify_all();
    }
  }

  void pop_front() {  // (mu_ held; the front part is finished)
    fifo_.pop_front();
    popped_++;
    if (fifo_.empty()) head_ = 0;  // (an empty ring starts again at its beginning)
  }

  Err take_error() {  // (mu_ held)
    const Err e = err_;
    err_ = Dev::kOk;
    return e;
  }

  // Arena bytes and an event for part p (p->bytes <= piece_): at the head, or at the start
  // of the arena when the tail end is too short; retires the oldest parts, once finished,
  // while there is no room.  The live bytes run from the oldest part's offset to head_
  // (wrapping at most once); head_ never catches up with the oldest part from behind (the
  // strict comparisons), so a non-empty ring is never mistaken for an empty one.
  Err take(Piece *p) {
    const size_t n = round_up(p->bytes);
    std::unique_lock<std::mutex> lk(mu_);
    double t0 = 0;
    for (;;) {
      if ((int)fifo_.size() < kEvents) {
        if (fifo_.empty()) {
          p->off = 0;
          break;
        }
        const size_t t = fifo_.front().off;
        if (head_ > t) {  // live [t, head_)
          if (cap_ - head_ >= n) {
            p->off = head_;
            break;
          }
          if (n < t) {
            p->off = 0;
            break;
          }
        } else if (t - head_ > n) {  // live [t, cap_) and [0, head_)
          p->off = head_;
          break;
        }
      }
      if (t0 == 0) {
        t0 = now();
        trace('W', popped_, fifo_.front(), t0);  // (waiting for the oldest part)
      }
      cv_done_.wait(lk, [&] { return fifo_.front().done; });
      pop_front();
      const Err e = take_error();
      if (e != Dev::kOk) return e;
    }
    if (t0 != 0) t_full_ += now() - t0;
#ifdef MIPGPU_RING_CHECK  // (tests/cpp/test_host_stage.cpp: no live part is overlapped)
    if (p->off + n > cap_) bad_takes_++;
    for (const Piece &q : fifo_)
      if (p->off < q.off + round_up(q.bytes) && q.off < p->off + n) bad_takes_++;
#endif
    head_ = p->off + n;
    trace('T', popped_ + fifo_.size(), *p);
    p->ev = (int)((popped_ + fifo_.size()) % kEvents);  // (its sequence number's event: free)
    return Dev::kOk;
  }

  // Diagnostic (MIPGPU_STAGE_TRACE=path): one line per event -- time, kind (T part taken,
  // W caller waits for the oldest part, P part enqueued, D its DMA seen complete, C finished),
  // part number, arena offset, bytes, call, download? -- written at teardown.
  struct TraceRec {
    double t;
    char kind;
    uint64_t seq, call;
    size_t off, bytes;
    bool down;
  };
  void trace(char kind, uint64_t seq, const Piece &p, double t = 0) {  // (mu_ held)
    if (trace_path_ && trace_.size() < (1u << 22))
      trace_.push_back({t ? t : now(), kind, seq, p.call, p.off, p.bytes, p.dst != nullptr});
  }
  void dump_trace() {
    if (!trace_path_ || trace_.empty()) return;
    char path[512];
    snprintf(path, sizeof path, "%s.%p.txt", trace_path_, (void *)this);
    if (FILE *f = fopen(path, "w")) {
      fprintf(f, "# piece %zu cap %zu\n", piece_, cap_);
      for (const TraceRec &r : trace_)
        fprintf(f, "%.6f %c %llu %zu %zu %llu %d\n", r.t, r.kind, (unsigned long long)r.seq, r.off, r.bytes,
                (unsigned long long)r.call, (int)r.down);
      fclose(f);
    }
    trace_.clear();
  }

  void pool_copy(void *d, const void *s, size_t n) {
    std::lock_guard<std::mutex> lk(pool_mu_);  // one copy job at a time (caller and completion thread)
    pool_->copy(d, s, n);
  }

  void release() {
    if (arena_) dev_.host_free(arena_);
    arena_ = nullptr;
    for (int i = 0; i < kEvents; i++) {
      if (have_ev_[i]) dev_.event_destroy(ev_[i]);
      have_ev_[i] = false;
    }
    piece_ = 0;
    cap_ = 0;
    head_ = 0;
  }

  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  Dev dev_;
  int device_ = 0;
  NumaPlace place_;
  int threads_ = 0;
  double t_up_ = 0, t_down_ = 0, t_wait_ = 0, t_full_ = 0, b_up_ = 0, b_down_ = 0;
  char *arena_ = nullptr;
  Event ev_[kEvents] = {};
  bool have_ev_[kEvents] = {};
  size_t piece_ = 0, cap_ = 0, head_ = 0, align_ = kAlign;
  std::mutex mu_, pool_mu_;
  std::condition_variable cv_work_, cv_done_;
  std::deque<Piece> fifo_;
  uint64_t bad_takes_ = 0;
  uint64_t popped_ = 0, finished_ = 0;  // parts retired from the front of fifo_ / finished
  bool stop_ = false, skip_copy_ = false;
  Err err_ = Dev::kOk;
  std::unique_ptr<CopyPool> pool_;
  std::thread worker_;
  const char *trace_path_;
  std::vector<TraceRec> trace_;
};

}  // namespace mipgpu
