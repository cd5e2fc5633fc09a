// free_repro.hip -- standalone reproducer of round 5's "transfers run at half speed after a
// large device free" (profiles/r05_engine_sequence.txt), no engine involved.
//
// Phases (each measures D2H and H2D of one 1080p frame's full cost table, 52.8 MB, from / to
// page-locked host memory on one stream, 20 copies, HIP events; plus the buffers' addresses):
//   A  fresh device + host buffers
//   B  the same buffers while a 20 GB hipMalloc is held, and after it is freed
//   C  buffers allocated after the free: new device + old host, old device + new host, both new
//   D  after 6.8 GB of page-locked host memory was allocated and freed (round 5: restores)
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/bin/free_repro tools/free_repro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../vvc-mip-gpu_amd/csrc/numa_place.h"

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

static const size_t kBytes = (size_t)135 * 97840 * 4;  // one 1080p cost table

static double rate(void *dst, const void *src, hipMemcpyKind kind, hipStream_t s) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipMemcpyAsync(dst, src, kBytes, kind, s));  // warm
  CK(hipEventRecord(a, s));
  const int n = 20;
  for (int i = 0; i < n; i++) CK(hipMemcpyAsync(dst, src, kBytes, kind, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return n * kBytes / (ms * 1e-3) / 1e9;
}

static void report(const char *phase, void *d, void *h, hipStream_t s) {
  void *hd = nullptr;
  (void)hipHostGetDevicePointer(&hd, h, 0);
  const double d2h = rate(h, d, hipMemcpyDeviceToHost, s), h2d = rate(d, h, hipMemcpyHostToDevice, s);
  printf("{\"phase\": \"%s\", \"d2h_GBps\": %.1f, \"h2d_GBps\": %.1f, \"dev\": \"%p\", \"host\": \"%p\", \"host_dev_va\": \"%p\", "
         "\"dev_align_2M\": %d, \"host_align_2M\": %d}\n",
         phase, d2h, h2d, d, h, hd, (int)(((uintptr_t)d & ((2u << 20) - 1)) == 0),
         (int)(((uintptr_t)hd & ((2u << 20) - 1)) == 0));
  fflush(stdout);
}

// Mode "remedy": fresh buffers, then page-locked host allocations of 128 MB are made and freed
// in growing batches (1, 2, 4, ..., 64 x 128 MB) and the same buffers measured after each; also
// four fresh streams (each may map to another copy engine).
static int remedy() {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *d0, *h0;
  CK(hipMalloc(&d0, kBytes));
  CK(hipHostMalloc(&h0, kBytes, hipHostMallocDefault));
  CK(hipMemset(d0, 1, kBytes));
  report("R fresh buffers", d0, h0, s);
  for (int i = 0; i < 4; i++) {
    hipStream_t t;
    CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
    char name[64];
    snprintf(name, sizeof name, "R another stream %d", i);
    report(name, d0, h0, t);
  }
  for (int n = 1; n <= 64; n *= 2) {
    std::vector<void *> v;
    for (int i = 0; i < n; i++) {
      void *p;
      CK(hipHostMalloc(&p, 128u << 20, hipHostMallocDefault));
      v.push_back(p);
    }
    for (void *p : v) CK(hipHostFree(p));
    char name[64];
    snprintf(name, sizeof name, "R after %d x 128 MB page-locked alloc + free", n);
    report(name, d0, h0, s);
  }
  return 0;
}

// Mode "cure": after the big free (half speed), which cheap step restores the rate?  Each step
// is measured with the same buffers; the big allocation is made and freed again before each.
static void cure_step(const char *name, void *d, void *h, hipStream_t s, size_t big, void (*step)()) {
  void *bigp;
  CK(hipMalloc(&bigp, big));
  CK(hipMemset(bigp, 0, big));
  CK(hipFree(bigp));
  char n1[96], n2[96];
  snprintf(n1, sizeof n1, "X after the free, before: %s", name);
  report(n1, d, h, s);
  step();
  snprintf(n2, sizeof n2, "X after: %s", name);
  report(n2, d, h, s);
}
static void host_cycle(int n, size_t mb) {
  std::vector<void *> v;
  for (int i = 0; i < n; i++) {
    void *p;
    CK(hipHostMalloc(&p, mb << 20, hipHostMallocDefault));
    v.push_back(p);
  }
  for (void *p : v) CK(hipHostFree(p));
}
static int cure(size_t big) {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *d0, *h0;
  CK(hipMalloc(&d0, kBytes));
  CK(hipHostMalloc(&h0, kBytes, hipHostMallocDefault));
  CK(hipMemset(d0, 1, kBytes));
  report("X fresh", d0, h0, s);
  cure_step("nothing", d0, h0, s, big, [] {});
  cure_step("hipDeviceSynchronize", d0, h0, s, big, [] { CK(hipDeviceSynchronize()); });
  cure_step("small device malloc + free", d0, h0, s, big, [] { void *p; CK(hipMalloc(&p, 1 << 20)); CK(hipFree(p)); });
  cure_step("64 MB device malloc + free", d0, h0, s, big, [] { void *p; CK(hipMalloc(&p, 64 << 20)); CK(hipFree(p)); });
  cure_step("1 x 128 MB page-locked", d0, h0, s, big, [] { host_cycle(1, 128); });
  cure_step("8 x 128 MB page-locked", d0, h0, s, big, [] { host_cycle(8, 128); });
  cure_step("1 x 2 GB page-locked", d0, h0, s, big, [] { host_cycle(1, 2048); });
  cure_step("54 x 128 MB page-locked", d0, h0, s, big, [] { host_cycle(54, 128); });
  cure_step("256 x 4 MB page-locked", d0, h0, s, big, [] { host_cycle(256, 4); });
  cure_step("a 20 GB device malloc held", d0, h0, s, big, [] { void *p; CK(hipMalloc(&p, 20ull << 30)); CK(hipMemset(p, 0, 1 << 20)); });
  return 0;
}

// Mode "split": the same bytes as 1, 2 or 4 concurrent copies on as many streams (in the
// half-speed state: are the copies bound to one copy engine?).  Before and after a big free.
static double rate_split(void *dst, const void *src, hipMemcpyKind kind, hipStream_t *st, int ns) {
  hipEvent_t a, b[4];
  CK(hipEventCreate(&a));
  for (int i = 0; i < ns; i++) CK(hipEventCreate(&b[i]));
  CK(hipEventRecord(a, st[0]));
  for (int i = 1; i < ns; i++) CK(hipStreamWaitEvent(st[i], a, 0));
  const int n = 20;
  const size_t part = kBytes / ns;
  for (int r = 0; r < n; r++)
    for (int i = 0; i < ns; i++)
      CK(hipMemcpyAsync((char *)dst + i * part, (const char *)src + i * part, part, kind, st[i]));
  for (int i = 0; i < ns; i++) CK(hipEventRecord(b[i], st[i]));
  float ms = 0;
  for (int i = 0; i < ns; i++) {
    CK(hipEventSynchronize(b[i]));
    float m = 0;
    CK(hipEventElapsedTime(&m, a, b[i]));
    if (m > ms) ms = m;
  }
  return n * (part * ns) / (ms * 1e-3) / 1e9;
}
static int split() {
  CK(hipSetDevice(0));
  hipStream_t st[4];
  for (auto &x : st) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  void *d0, *h0;
  CK(hipMalloc(&d0, kBytes));
  CK(hipHostMalloc(&h0, kBytes, hipHostMallocDefault));
  CK(hipMemset(d0, 1, kBytes));
  for (int phase = 0; phase < 2; phase++) {
    if (phase == 1) {
      void *bigp;
      CK(hipMalloc(&bigp, 20ull << 30));
      CK(hipMemset(bigp, 0, 20ull << 30));
      CK(hipFree(bigp));
    }
    for (int ns : {1, 2, 4})
      printf("{\"phase\": \"%s, %d stream(s)\", \"d2h_GBps\": %.1f, \"h2d_GBps\": %.1f}\n", phase ? "after a 20 GB free" : "start", ns,
             rate_split(h0, d0, hipMemcpyDeviceToHost, st, ns), rate_split(d0, h0, hipMemcpyHostToDevice, st, ns));
  }
  return 0;
}

// Mode "numa": page-locked buffers placed on the GPU's NUMA node vs the other node vs the
// default policy, with the allocating thread on either node's CPUs (numa_place.h), before and
// after a big free.
static int numa() {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  char bus[64] = {};
  CK(hipDeviceGetPCIBusId(bus, sizeof bus, 0));
  mipgpu::NumaPlace gpu = mipgpu::numa_place_of_pci(bus);
  printf("{\"pci\": \"%s\", \"gpu_node\": %d, \"node_cpus\": %zu}\n", bus, gpu.node, gpu.cpus.size());
  if (!gpu.active()) return 0;
  std::string online;
  mipgpu::read_text(mipgpu::sysfs_root() + "/devices/system/node/online", &online);
  const std::vector<int> nodes = mipgpu::parse_cpulist(online);
  mipgpu::NumaPlace other;
  for (int n : nodes)
    if (n != gpu.node) {
      std::string cl;
      if (mipgpu::read_text(mipgpu::sysfs_root() + "/devices/system/node/node" + std::to_string(n) + "/cpulist", &cl)) {
        other.node = n;
        for (int c : mipgpu::parse_cpulist(cl))
          for (int a : mipgpu::allowed_cpus())
            if (a == c) other.cpus.push_back(c);
      }
      if (other.active()) break;
    }
  void *d0;
  CK(hipMalloc(&d0, kBytes));
  CK(hipMemset(d0, 1, kBytes));
  auto alloc_on = [&](const mipgpu::NumaPlace &p) {
    void *h = nullptr;
    mipgpu::ScopedNodePolicy pol(p);
    CK(hipHostMalloc(&h, kBytes, pol.applied() ? hipHostMallocNumaUser : hipHostMallocDefault));
    memset(h, 0, kBytes);
    return h;
  };
  for (int phase = 0; phase < 2; phase++) {
    if (phase == 1) {
      void *bigp;
      CK(hipMalloc(&bigp, 20ull << 30));
      CK(hipMemset(bigp, 0, 20ull << 30));
      CK(hipFree(bigp));
    }
    const char *ph = phase ? "after a 20 GB free" : "start";
    char name[160];
    mipgpu::bind_current_thread(gpu);
    void *hl = alloc_on(gpu), *hd = alloc_on(mipgpu::NumaPlace());
    snprintf(name, sizeof name, "%s: thread on the GPU node, host buffer on the GPU node %d", ph, gpu.node);
    report(name, d0, hl, s);
    snprintf(name, sizeof name, "%s: thread on the GPU node, host buffer by default policy", ph);
    report(name, d0, hd, s);
    if (other.active()) {
      void *hr = alloc_on(other);
      snprintf(name, sizeof name, "%s: thread on the GPU node, host buffer on the other node %d", ph, other.node);
      report(name, d0, hr, s);
      mipgpu::bind_current_thread(other);
      snprintf(name, sizeof name, "%s: thread on the other node, host buffer on the GPU node", ph);
      report(name, d0, hl, s);
      snprintf(name, sizeof name, "%s: thread on the other node, host buffer on the other node", ph);
      report(name, d0, hr, s);
    }
  }
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1 && std::string(argv[1]) == "numa") return numa();
  if (argc > 1 && std::string(argv[1]) == "split") return split();
  if (argc > 1 && std::string(argv[1]) == "remedy") return remedy();
  if (argc > 1 && std::string(argv[1]) == "cure") return cure(20ull << 30);
  const size_t big = (size_t)(argc > 1 ? atof(argv[1]) : 20.0) * (1ull << 30);
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *d0, *h0;
  CK(hipMalloc(&d0, kBytes));
  CK(hipHostMalloc(&h0, kBytes, hipHostMallocDefault));
  CK(hipMemset(d0, 1, kBytes));
  report("A fresh buffers", d0, h0, s);
  void *bigp;
  CK(hipMalloc(&bigp, big));
  CK(hipMemset(bigp, 0, big));
  report("B holding the big allocation", d0, h0, s);
  CK(hipFree(bigp));
  report("B after freeing it (old buffers)", d0, h0, s);
  void *d1, *h1;
  CK(hipMalloc(&d1, kBytes));
  CK(hipMemset(d1, 1, kBytes));
  CK(hipHostMalloc(&h1, kBytes, hipHostMallocDefault));
  report("C new device, old host", d1, h0, s);
  report("C old device, new host", d0, h1, s);
  report("C new device, new host", d1, h1, s);
  {
    std::vector<void *> v;
    for (int i = 0; i < 54; i++) {
      void *p;
      CK(hipHostMalloc(&p, 128u << 20, hipHostMallocDefault));
      v.push_back(p);
    }
    for (void *p : v) CK(hipHostFree(p));
  }
  report("D after 6.8 GB page-locked host (C buffers)", d1, h1, s);
  void *d2, *h2;
  CK(hipMalloc(&d2, kBytes));
  CK(hipMemset(d2, 1, kBytes));
  CK(hipHostMalloc(&h2, kBytes, hipHostMallocDefault));
  report("D new device, new host", d2, h2, s);
  report("D new device, C host", d2, h1, s);
  report("D C device, new host", d1, h2, s);
  return 0;
}
