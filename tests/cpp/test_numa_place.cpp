// CPU unit test of the engine's NUMA placement (csrc/numa_place.h) over a fake sysfs tree made
// by tests/test_numa_place.py: argv[1] = the tree's root.  Expected: device 0000:c1:00.0 on
// node 1 (cpulist "2-3,6-7"), 0000:41:00.0 on node 0, 0000:05:00.0 with numa_node -1, an
// unknown device; the memory policy scope applies and restores.
#include <cstdio>
#include <string>
#include <vector>

#include "numa_place.h"

static int fails = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      fails++;                                \
      std::printf("FAIL %s: ", #c);           \
      std::printf(__VA_ARGS__);               \
      std::printf("\n");                      \
    }                                         \
  } while (0)

int main(int argc, char **argv) {
  using namespace mipgpu;
  CHECK((parse_cpulist("0-3,8,10-11") == std::vector<int>{0, 1, 2, 3, 8, 10, 11}), "cpulist");
  CHECK(parse_cpulist("").empty(), "empty cpulist");
  CHECK((parse_cpulist("5\n") == std::vector<int>{5}), "single");
  if (argc < 2) return 1;
  const std::string root = argv[1];
  const std::vector<int> ok = allowed_cpus();
  auto allowed = [&](int c) {
    for (int a : ok)
      if (a == c) return true;
    return false;
  };
  const NumaPlace p1 = numa_place_of_pci("0000:C1:00.0", root);  // (upper case, as HIP prints it)
  std::vector<int> want1;
  for (int c : {2, 3, 6, 7})
    if (allowed(c)) want1.push_back(c);
  CHECK(p1.node == (want1.empty() ? -1 : 1), "node %d", p1.node);
  CHECK(p1.cpus == want1, "node 1 cpus (%zu)", p1.cpus.size());
  const NumaPlace p0 = numa_place_of_pci("0000:41:00.0", root);
  CHECK(p0.node == (allowed(0) || allowed(1) ? 0 : -1), "node %d", p0.node);
  CHECK(!numa_place_of_pci("0000:05:00.0", root).active(), "numa_node -1");
  CHECK(!numa_place_of_pci("0000:99:00.0", root).active(), "unknown device");
  CHECK(!numa_place_of_pci("0000:c1:00.0", root + "/one_node").active(), "one-node host");
  if (p1.active()) {
    CHECK(bind_current_thread(p1), "bind");
    const std::vector<int> now = allowed_cpus();
    CHECK(now == p1.cpus, "affinity after bind (%zu cpus)", now.size());
  }
  {  // the scope sets a preferred node (node 0 exists on every Linux host) and restores the policy
    NumaPlace real;
    real.node = 0;
    real.cpus = {0};
    int mode_before = -1, mode_after = -1;
    unsigned long mask[16] = {};
    (void)syscall(SYS_get_mempolicy, &mode_before, mask, 1024UL, nullptr, 0UL);
    {
      const ScopedNodePolicy pol(real);
      if (pol.applied()) {
        int mode = -1;
        (void)syscall(SYS_get_mempolicy, &mode, mask, 1024UL, nullptr, 0UL);
        CHECK(mode == ScopedNodePolicy::kMpolPreferred && (mask[0] & 1), "preferred node 0 (mode %d)", mode);
      }
    }
    (void)syscall(SYS_get_mempolicy, &mode_after, mask, 1024UL, nullptr, 0UL);
    CHECK(mode_after == mode_before, "policy restored (%d -> %d)", mode_before, mode_after);
  }
  if (fails) return 1;
  std::printf("numa_place: ok (node1 cpus %zu)\n", p1.cpus.size());
  return 0;
}
