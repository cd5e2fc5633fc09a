// CPU unit test of the search kernel's item-counter bookkeeping (csrc/queue_ring.h): every
// slot is waited for before reuse, a failed launch / event record makes the next use of its
// slot clear the counter pair, failing ops are reported.  Built and run by
// tests/test_queue_ring.py (g++, no GPU).
#include <cstdio>
#include <string>
#include <vector>

#include "queue_ring.h"

struct Log {
  std::vector<std::string> ev;
  int fail_wait = -1, fail_record = -1, fail_clear = -1;  // slot whose next op fails
  bool fail_sync = false;                                  // the next sync fails
};

struct MockOps {
  Log *log;
  int wait(int slot, int s) const { return op("wait", slot, s, log->fail_wait); }
  int record(int slot, int s) const { return op("record", slot, s, log->fail_record); }
  int clear(int slot, int s) const { return op("clear", slot, s, log->fail_clear); }
  int sync(int s) const {
    log->ev.push_back((log->fail_sync ? "sync!@" : "sync@") + std::to_string(s));
    const bool f = log->fail_sync;
    log->fail_sync = false;
    return f ? 1 : 0;
  }
  int op(const char *what, int slot, int s, int &fail) const {
    if (fail == slot) {
      fail = -1;
      log->ev.push_back(std::string(what) + "!" + std::to_string(slot));
      return 1;
    }
    log->ev.push_back(std::string(what) + std::to_string(slot) + "@" + std::to_string(s));
    return 0;
  }
};

static int failures = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
      failures++;                                                  \
    }                                                              \
  } while (0)

static bool has(const Log &l, const std::string &e) {
  for (const auto &x : l.ev)
    if (x == e) return true;
  return false;
}

int main() {
  {  // normal use: no wait before a slot's first launch, a wait on the same slot afterwards
    Log l;
    QueueRing<MockOps, 4> q{MockOps{&l}};
    for (int i = 0; i < 4; i++) {
      const int s = q.acquire(i % 2);
      CHECK(s == i);
      CHECK(q.launched(s, i % 2) == 0);
    }
    CHECK(l.ev.size() == 4);  // four records, no waits
    const int s = q.acquire(7);
    CHECK(s == 0 && has(l, "wait0@7") && !has(l, "clear0@7"));
  }
  {  // a failed launch: the next use of its slot waits for the last recorded launch and clears
    Log l;
    QueueRing<MockOps, 2> q{MockOps{&l}};
    int s = q.acquire(0);
    q.launched(s, 0);  // slot 0 used once
    s = q.acquire(0);
    CHECK(s == 1);
    q.failed(s);  // slot 1 never recorded
    CHECK(q.dirty(1));
    s = q.acquire(1);  // slot 0: clean
    CHECK(s == 0 && !has(l, "clear0@1"));
    q.launched(s, 1);
    s = q.acquire(3);  // slot 1: dirty, never recorded -> no wait, a clear
    CHECK(s == 1 && has(l, "clear1@3") && !has(l, "wait1@3") && !q.dirty(1));
  }
  {  // a failed event record: dirty; the next use waits (earlier recording) and clears
    Log l;
    QueueRing<MockOps, 2> q{MockOps{&l}};
    int s = q.acquire(0);
    q.launched(s, 0);
    s = q.acquire(0);
    q.launched(s, 0);  // both used
    s = q.acquire(0);
    l.fail_record = 0;
    CHECK(s == 0 && q.launched(s, 0) != 0 && q.dirty(0));
    q.launched(q.acquire(0), 0);  // slot 1
    s = q.acquire(5);
    CHECK(s == 0 && has(l, "wait0@5") && has(l, "clear0@5") && !q.dirty(0));
  }
  {  // launch failed vs launched but its record failed: only the latter (a kernel in
     // flight on the pair) waits for its stream on the host before the slot is reused
    Log l;
    QueueRing<MockOps, 2> q{MockOps{&l}};
    int s = q.acquire(4);
    q.failed(s);
    CHECK(!has(l, "sync@4") && q.dirty(s));
    s = q.acquire(6);
    l.fail_record = s;
    CHECK(q.launched(s, 6) != 0 && has(l, "sync@6") && q.dirty(s) && !q.retired(s));
    q.launched(q.acquire(0), 0);  // slot 0 (cleared first)
    s = q.acquire(7);             // slot 1: dirty after the sync -> cleared, usable
    CHECK(s == 1 && has(l, "clear1@7"));
    // the sync fails too: the slot is retired and skipped from then on
    l.fail_record = s;
    l.fail_sync = true;
    CHECK(q.launched(s, 7) != 0 && q.retired(1));
    for (int i = 0; i < 4; i++) {
      const int t = q.acquire(8);
      CHECK(t == 0);
      q.launched(t, 8);
    }
  }
  {  // every slot retired: acquire fails
    Log l;
    QueueRing<MockOps, 1> q{MockOps{&l}};
    const int s = q.acquire(0);
    l.fail_record = s;
    l.fail_sync = true;
    q.launched(s, 0);
    CHECK(q.acquire(0) == -1);
  }
  {  // failing wait / clear are reported and keep the slot dirty
    Log l;
    QueueRing<MockOps, 1> q{MockOps{&l}};
    q.launched(q.acquire(0), 0);
    l.fail_wait = 0;
    CHECK(q.acquire(0) == -1 && q.dirty(0));
    l.fail_clear = 0;
    CHECK(q.acquire(0) == -1 && q.dirty(0));
    CHECK(q.acquire(0) == 0 && !q.dirty(0));
  }
  std::printf(failures ? "queue_ring: %d failures\n" : "queue_ring: ok\n", failures);
  return failures ? 1 : 0;
}
