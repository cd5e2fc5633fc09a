// pageable_probe.cpp -- GPU box: host-transfer options for pageable (malloc'd) buffers.
// (1) hipMemcpy D2H into pageable memory (runtime staging), (2) hipHostRegister + D2H +
// unregister, (3) D2H into a pinned bounce buffer + memcpy to pageable on T threads.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void pmemcpy(char *dst, const char *src, size_t n, int T) {
  std::vector<std::thread> th;
  const size_t per = (n / T + 4095) & ~(size_t)4095;
  for (int t = 0; t < T; t++) {
    const size_t o = (size_t)t * per;
    if (o >= n) break;
    th.emplace_back([=] { memcpy(dst + o, src + o, std::min(per, n - o)); });
  }
  for (auto &x : th) x.join();
}

int main() {
  const size_t N = (size_t)1 << 30;  // 1 GiB
  char *d;
  hipMalloc(&d, N);
  hipMemset(d, 1, N);
  char *pg = (char *)malloc(N);
  memset(pg, 0, N);
  hipDeviceSynchronize();
  double t0 = now();
  hipMemcpy(pg, d, N, hipMemcpyDeviceToHost);
  printf("pageable D2H: %.1f GB/s\n", N / (now() - t0) / 1e9);
  t0 = now();
  hipHostRegister(pg, N, hipHostRegisterDefault);
  const double treg = now() - t0;
  t0 = now();
  hipMemcpy(pg, d, N, hipMemcpyDeviceToHost);
  const double tcp = now() - t0;
  t0 = now();
  hipHostUnregister(pg);
  printf("register %.1f GB/s, registered D2H %.1f GB/s, unregister %.1f GB/s\n", N / treg / 1e9, N / tcp / 1e9,
         N / (now() - t0) / 1e9);
  char *pin;
  hipHostMalloc(&pin, N, hipHostMallocDefault);
  t0 = now();
  hipMemcpy(pin, d, N, hipMemcpyDeviceToHost);
  printf("pinned D2H: %.1f GB/s\n", N / (now() - t0) / 1e9);
  for (int T : {1, 2, 4, 8, 16}) {
    pmemcpy(pg, pin, N, T);
    t0 = now();
    pmemcpy(pg, pin, N, T);
    printf("memcpy pinned->pageable T=%d: %.1f GB/s\n", T, N / (now() - t0) / 1e9);
  }
  // overlapped: D2H of half i+1 while memcpy of half i (64 MB pieces, 8 threads)
  for (int T : {4, 8, 16}) {
    const size_t P = 64 << 20;
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t ev[2];
    hipEventCreate(&ev[0]);
    hipEventCreate(&ev[1]);
    t0 = now();
    const int np = (int)(N / P);
    hipMemcpyAsync(pin, d, P, hipMemcpyDeviceToHost, s);
    hipEventRecord(ev[0], s);
    for (int i = 0; i < np; i++) {
      if (i + 1 < np) {
        hipMemcpyAsync(pin + ((i + 1) % 2) * P, d + (i + 1) * P, P, hipMemcpyDeviceToHost, s);
        hipEventRecord(ev[(i + 1) % 2], s);
      }
      hipEventSynchronize(ev[i % 2]);
      pmemcpy(pg + i * P, pin + (i % 2) * P, P, T);
    }
    printf("pipelined D2H + memcpy (64 MB pieces, T=%d): %.1f GB/s\n", T, N / (now() - t0) / 1e9);
  }
  return 0;
}
