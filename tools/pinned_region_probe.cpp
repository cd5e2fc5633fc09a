// Device -> page-locked host DMA rate per 64 MB region of one large hipHostMalloc block
// (the bounce ring's arena, csrc/host_stage.h) and of separate 64 MB blocks, alone and with
// host threads copying out of another region at the same time (as the ring's completion
// thread does).  Also prints the NUMA node of each region's first page.
//   hipcc -O2 -o /tmp/prp tools/pinned_region_probe.cpp  (NUMA node via the move_pages syscall)
//   /tmp/prp [arena_MB=1024] [reps=3]
#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

static int node_of(void *p) {
  void *pages[1] = {p};
  int status[1] = {-1};
  if (syscall(SYS_move_pages, 0, 1, pages, nullptr, status, 0) != 0) return -2;
  return status[0];
}

int main(int argc, char **argv) {
  const size_t MB = 1u << 20;
  const size_t arena_mb = argc > 1 ? atoi(argv[1]) : 1024;
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  const size_t region = 64 * MB;
  const int nreg = (int)(arena_mb * MB / region);
  char *dev;
  CK(hipMalloc(&dev, region));
  CK(hipMemset(dev, 1, region));
  char *arena;
  CK(hipHostMalloc((void **)&arena, nreg * region, hipHostMallocDefault));
  std::vector<char *> blocks(nreg);
  for (auto &b : blocks) CK(hipHostMalloc((void **)&b, region, hipHostMallocDefault));
  std::vector<char> pageable(region);
  memset(pageable.data(), 0, region);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto d2h = [&](char *dst) {
    CK(hipEventRecord(a, s));
    CK(hipMemcpyAsync(dst, dev, region, hipMemcpyDeviceToHost, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return region / (ms * 1e-3) / 1e9;
  };
  // background host copy out of a region (8 threads, like the ring's copy pool)
  std::atomic<int> bg_region{-1};
  std::atomic<bool> stop{false};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; t++)
    th.emplace_back([&, t] {
      while (!stop) {
        const int r = bg_region.load();
        if (r < 0) {
          std::this_thread::yield();
          continue;
        }
        const size_t part = region / 8;
        memcpy(pageable.data() + t * part, arena + (size_t)r * region + t * part, part);
      }
    });
  for (int rep = 0; rep < reps; rep++) {
    printf("rep %d\nregion node  arena_GB/s  arena+bg_GB/s  block_node block_GB/s\n", rep);
    for (int r = 0; r < nreg; r++) {
      char *dst = arena + (size_t)r * region;
      const double g0 = d2h(dst);
      bg_region = (r + 1) % nreg;  // host threads read the next region meanwhile
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
      const double g1 = d2h(dst);
      bg_region = -1;
      const double g2 = d2h(blocks[r]);
      printf("%6d %4d %11.1f %14.1f %10d %10.1f\n", r, node_of(dst), g0, g1, node_of(blocks[r]), g2);
    }
  }
  stop = true;
  for (auto &t : th) t.join();
  return 0;
}
