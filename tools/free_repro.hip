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
#include <string>
#include <vector>

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

int main(int argc, char **argv) {
  if (argc > 1 && std::string(argv[1]) == "remedy") return remedy();
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
