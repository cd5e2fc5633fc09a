// CPU unit test of the pageable bounce ring (csrc/host_stage.h) over a simulated device:
// three in-order "streams", each run by its own thread, execute the ring's copies and event
// records after random delays, like DMA engines.  Checks that every download reaches its
// pageable destination by the time drain(call) returns, that no piece is refilled before its
// DMA has read it and no two live parts overlap in the arena (uploads arrive intact), that a failing event wait is reported once by the
// next drain, and that abandon() / teardown with work in flight return with the ring idle
// and reusable.  Built and run by tests/test_host_stage.py (g++, no GPU; also under
// ThreadSanitizer when the compiler has it).
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#define MIPGPU_RING_CHECK 1
#include "host_stage.h"

namespace {

struct Sim {
  static constexpr int kStreams = 3;
  struct Ev {
    uint64_t target = 0, reached = 0;
    bool fail_next = false, failed = false;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q[kStreams];
  std::vector<Ev> ev;
  bool stop = false;
  std::atomic<int> max_delay_us{200};
  std::vector<std::thread> th;
  std::mt19937 rng{7};

  Sim() {
    for (int s = 0; s < kStreams; s++) th.emplace_back([this, s] { run(s); });
  }
  ~Sim() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  void run(int s) {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || !q[s].empty(); });
      if (q[s].empty()) return;
      auto op = q[s].front();
      q[s].pop_front();
      const int d = (int)(rng() % (unsigned)(max_delay_us.load() + 1));
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::microseconds(d));
      op();
      lk.lock();
      cv.notify_all();
    }
  }
  void enqueue(int s, std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu);
      q[s].push_back(std::move(f));
    }
    cv.notify_all();
  }
};

struct SimDev {
  using Err = int;
  using Stream = int;
  using Event = int;
  static constexpr Err kOk = 0;
  static constexpr Err kNotReady = 3;
  Sim *sim;
  std::atomic<int> *allocs;
  Err host_alloc(char **p, size_t n, bool) {
    *p = new char[n];
    allocs->fetch_add(1);
    return kOk;
  }
  void host_free(char *p) {
    delete[] p;
    allocs->fetch_sub(1);
  }
  Err event_create(Event *e) {
    std::lock_guard<std::mutex> lk(sim->mu);
    sim->ev.emplace_back();
    *e = (int)sim->ev.size() - 1;
    return kOk;
  }
  void event_destroy(Event) {}
  Err copy_h2d(void *dev, const void *host, size_t n, Stream s) {
    sim->enqueue(s, [=] { std::memcpy(dev, host, n); });
    return kOk;
  }
  Err copy_d2h(void *host, const void *dev, size_t n, Stream s) {
    sim->enqueue(s, [=] { std::memcpy(host, dev, n); });
    return kOk;
  }
  Err record(Event e, Stream s) {
    uint64_t t;
    {
      std::lock_guard<std::mutex> lk(sim->mu);
      t = ++sim->ev[e].target;
    }
    Sim *m = sim;
    sim->enqueue(s, [m, e, t] {
      std::lock_guard<std::mutex> lk(m->mu);  // (run() holds no lock while an op executes)
      Sim::Ev &v = m->ev[e];
      v.reached = t;
      if (v.fail_next) {
        v.fail_next = false;
        v.failed = true;
      }
    });
    return kOk;
  }
  Err sync(Event e) {
    std::unique_lock<std::mutex> lk(sim->mu);
    const uint64_t t = sim->ev[e].target;
    sim->cv.wait(lk, [&] { return sim->ev[e].reached >= t; });
    if (sim->ev[e].failed) {
      sim->ev[e].failed = false;
      return 700;  // an illegal-address-like error
    }
    return kOk;
  }
  void bind_thread(int) {}
};

using Ring = mipgpu::BounceRing<SimDev>;

int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
      fails++;                                                      \
    }                                                               \
  } while (0)

void fill(std::vector<char> &v, uint32_t seed) {
  std::mt19937 r(seed);
  for (auto &c : v) c = (char)r();
}

// Calls of random sizes: upload a pageable source into the call's "device" buffer, then
// download it (same stream, so in order) into a pageable destination; the caller drains
// calls a few behind, as mip_wait does, and checks each destination right after its drain.
void round_trips(Sim &sim, std::atomic<int> &allocs, int ncalls, size_t piece, int lag, size_t max_bytes = 0) {
  Ring ring(SimDev{&sim, &allocs});
  CHECK(ring.reserve(piece) == 0);
  std::mt19937 r(11);
  struct Call {
    std::vector<char> src, dev, dst;
  };
  std::vector<Call> calls(ncalls);
  for (int c = 0; c < ncalls; c++) {
    Call &k = calls[c];
    const size_t n = 1 + r() % (max_bytes ? max_bytes : 3 * ring.piece() + 12345);  // 1 .. several pieces
    k.src.resize(n);
    k.dev.assign(n, 0);
    k.dst.assign(n, 0);
    fill(k.src, 100 + c);
    const int s = (int)(r() % Sim::kStreams);
    CHECK(ring.upload(k.dev.data(), k.src.data(), n, s, (uint64_t)c + 1) == 0);
    std::fill(k.src.begin(), k.src.end(), 0x5a);  // the source may be reused once upload() returns
    CHECK(ring.download(k.dst.data(), k.dev.data(), n, s, (uint64_t)c + 1) == 0);
    if (c >= lag) {
      const int w = c - lag;
      CHECK(ring.drain((uint64_t)w + 1) == 0);
      std::vector<char> want(calls[w].dst.size());
      fill(want, 100 + w);
      CHECK(calls[w].dst == want);
      calls[w] = Call();
    }
  }
  CHECK(ring.drain(~0ull) == 0);
  CHECK(ring.bad_takes() == 0);
  for (int w = std::max(0, ncalls - lag); w < ncalls; w++) {
    std::vector<char> want(calls[w].dst.size());
    fill(want, 100 + w);
    CHECK(calls[w].dst == want);
  }
  CHECK(ring.idle());
}

}  // namespace

int main(int argc, char **argv) {
  const int q = argc > 1 && !std::strcmp(argv[1], "quick") ? 6 : 1;  // (ThreadSanitizer build)
  Sim sim;
  std::atomic<int> allocs{0};

  round_trips(sim, allocs, 60 / q, 1, 0);   // drain each call at once
  round_trips(sim, allocs, 120 / q, 1, 5);  // several calls in flight (ring wraps many times)
  sim.max_delay_us = 0;
  round_trips(sim, allocs, 200 / q, 1, 3);  // fast device: the completion thread races the caller
  sim.max_delay_us = 200;
  round_trips(sim, allocs, 300 / q, 1, 40, 64u << 10);  // small parts: more in flight than events
  round_trips(sim, allocs, 300 / q, 1, 12, 700u << 10);  // parts of mixed sizes: the arena wraps
  round_trips(sim, allocs, 200 / q, 1, 30, 5u << 19);    // calls waiting for room (the ring retires parts)
  CHECK(allocs.load() == 0);

  {
    // a transfer before reserve() is refused (no ring to stage through)
    Ring ring(SimDev{&sim, &allocs});
    std::vector<char> buf(100), dev(100);
    CHECK(ring.upload(dev.data(), buf.data(), buf.size(), 0, 1) == SimDev::kNotReady);
    CHECK(ring.download(buf.data(), dev.data(), dev.size(), 0, 1) == SimDev::kNotReady);
    CHECK(ring.idle());
  }

  {
    // a failing event wait: reported once, by the drain that covers it; the ring goes on
    Ring ring(SimDev{&sim, &allocs});
    CHECK(ring.reserve(1) == 0);
    std::vector<char> src(3u << 20, 1), dev(3u << 20), dst(3u << 20);
    {
      std::lock_guard<std::mutex> lk(sim.mu);
      sim.ev[sim.ev.size() - Ring::kEvents + 2].fail_next = true;  // the upload's last piece
    }
    CHECK(ring.upload(dev.data(), src.data(), src.size(), 0, 1) == 0);
    CHECK(ring.download(dst.data(), dev.data(), dst.size(), 0, 2) == 0);
    CHECK(ring.drain(2) == 700);
    CHECK(ring.drain(2) == 0);
    CHECK(ring.idle());
    CHECK(ring.upload(dev.data(), src.data(), src.size(), 1, 3) == 0);
    CHECK(ring.download(dst.data(), dev.data(), dst.size(), 1, 3) == 0);
    CHECK(ring.drain(3) == 0);
    CHECK(dst == src);
  }

  {
    // abandon() with slow DMAs in flight: returns with the ring idle, nothing written to
    // destinations after it returned, and the ring reusable
    Ring ring(SimDev{&sim, &allocs});
    CHECK(ring.reserve(1) == 0);
    sim.max_delay_us = 3000;
    std::vector<char> dev(8u << 20, 7);
    std::vector<char> *dst = new std::vector<char>(8u << 20, 0);
    CHECK(ring.download(dst->data(), dev.data(), dev.size(), 2, 1) == 0);
    ring.abandon();
    CHECK(ring.idle());
    std::fill(dst->begin(), dst->end(), 3);
    std::this_thread::sleep_for(std::chrono::milliseconds(30));
    CHECK(std::all_of(dst->begin(), dst->end(), [](char c) { return c == 3; }));
    delete dst;
    sim.max_delay_us = 200;
    std::vector<char> out(dev.size(), 0);
    CHECK(ring.download(out.data(), dev.data(), dev.size(), 0, 2) == 0);
    CHECK(ring.drain(2) == 0);
    CHECK(out == dev);
  }

  {
    // teardown with downloads in flight
    std::vector<char> dev(5u << 20, 9), dst(5u << 20, 0);
    {
      Ring ring(SimDev{&sim, &allocs});
      CHECK(ring.reserve(2u << 20) == 0);
      CHECK(ring.piece() == (2u << 20));
      CHECK(ring.download(dst.data(), dev.data(), dev.size(), 1, 1) == 0);
    }
    CHECK(allocs.load() == 0);
  }

  {
    // growing the ring drains what is queued first
    Ring ring(SimDev{&sim, &allocs});
    CHECK(ring.reserve(1) == 0);
    std::vector<char> dev(3u << 20, 4), dst(3u << 20, 0);
    CHECK(ring.download(dst.data(), dev.data(), dev.size(), 0, 1) == 0);
    CHECK(ring.reserve(4u << 20) == 0);
    CHECK(dst == dev);
    CHECK(allocs.load() == 1);  // (one arena)
  }
  CHECK(allocs.load() == 0);

  if (fails) return 1;
  std::printf("host_stage: ok\n");
  return 0;
}
