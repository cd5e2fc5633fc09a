// queue_ring.h -- bookkeeping of the persistent search kernel's item-counter pairs.
//
// Each launch of mip_search_kernel takes its items from a device counter pair {next item,
// workgroups done} that must be zero at launch; the kernel's last workgroup leaves it zero
// again.  An engine owns kSlots pairs, used round robin.  A pair is reused only after the
// launch that last used it has completed (stream wait on its event), so launches on
// different streams never share one.  A launch that fails (launch error, or an error
// between taking the slot and recording its event) may leave its pair non-zero, or the
// pair's event unrecorded: the slot is then marked dirty and the next launch that takes it
// first clears the pair with an asynchronous memset on its own stream.
//
// Ops (host-side effects, so the logic is unit-testable without a GPU,
// tests/cpp/test_queue_ring.cpp):
//   int wait(int slot, Stream s)      stream s waits for the slot's last recorded event
//   int record(int slot, Stream s)    record the slot's event on s
//   int clear(int slot, Stream s)     zero the slot's counter pair on s (memset)
//   int sync(Stream s)                wait on the host until everything queued on s is done
// each returning 0 on success.
// A launch that was enqueued but whose event could not be recorded is still running with
// its pair: no event can order the pair's reuse, so launched() waits for the stream on the
// host (then the pair is cleared before its next use like a failed launch's); if even that
// fails, the slot is retired for good -- a later launch on another stream could otherwise
// clear or share the pair under the running kernel.
#pragma once

template <class Ops, int kSlots>
class QueueRing {
 public:
  explicit QueueRing(Ops ops) : ops_(ops) {}

  // Take the next slot for a launch on stream s (waits / clears as needed): the slot index,
  // or -1 if an op failed (the slot is then dirty).
  template <class Stream>
  int acquire(Stream s) {
    int slot = (int)(seq_++ % kSlots);
    for (int i = 0; i < kSlots && retired_[slot]; i++) slot = (int)(seq_++ % kSlots);
    if (retired_[slot]) return -1;  // every slot retired
    // the last launch recorded on the slot (a failed one may have recorded nothing: then
    // this waits for an earlier one, which is harmless)
    if (used_[slot] && ops_.wait(slot, s) != 0) {
      dirty_[slot] = true;
      return -1;
    }
    if (dirty_[slot]) {  // zero the pair behind everything queued on this stream
      if (ops_.clear(slot, s) != 0) return -1;
      dirty_[slot] = false;
    }
    pending_ = slot;
    return slot;
  }

  // The launch on the slot was enqueued: record its completion event.
  template <class Stream>
  int launched(int slot, Stream s) {
    pending_ = -1;
    if (ops_.record(slot, s) != 0) {
      // the kernel was enqueued: wait for it here, since no event orders the pair's reuse
      if (ops_.sync(s) != 0) retired_[slot] = true;
      dirty_[slot] = true;
      return -1;
    }
    used_[slot] = true;
    return 0;
  }

  // The launch on the slot failed (nothing reliable recorded): clear before its next use.
  void failed(int slot) {
    pending_ = -1;
    dirty_[slot] = true;
  }

  bool dirty(int slot) const { return dirty_[slot]; }
  bool retired(int slot) const { return retired_[slot]; }
  bool used(int slot) const { return used_[slot]; }

 private:
  Ops ops_;
  unsigned seq_ = 0;
  int pending_ = -1;
  bool used_[kSlots] = {};
  bool dirty_[kSlots] = {};
  bool retired_[kSlots] = {};
};
