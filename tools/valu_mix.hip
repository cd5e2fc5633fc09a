// valu_rate.hip -- VALU issue-rate probe for gfx950: cycles per wave64 vector instruction on
// one SIMD with 1..8 waves resident per SIMD, for the instruction kinds the search kernel's
// pair loops are made of (packed 16-bit ops, 32-bit adds).  Each wave runs NACC independent
// accumulator chains so issue, not latency, limits a single wave.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int kIters = 2048 * 8;

template <int OP, int NACC>
__global__ __launch_bounds__(256) void probe(unsigned *out, unsigned long long *cyc, unsigned seed) {
  unsigned a[NACC];
#pragma unroll
  for (int i = 0; i < NACC; i++) a[i] = seed + threadIdx.x * 7 + i;
  const unsigned b = seed * 3 + 1;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; it++) {
    if constexpr (OP == 0) { asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[7]) : "v"(b)); }
    else if constexpr (OP == 1) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[7]) : "v"(b)); }
    else if constexpr (OP == 2) { asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[7]) : "v"(b)); }
    else if constexpr (OP == 3) { asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[7]) : "v"(b)); }
    else if constexpr (OP == 4) { asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[7]) : "v"(b)); }
    else if constexpr (OP == 5) { asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[7]) : "v"(b)); }
    else if constexpr (OP == 6) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[1]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[2]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[3]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[4]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[5]) : "v"(b)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[6]) : "v"(b)); asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[7]) : "v"(b)); }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < NACC; i++) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

static const char *kNames[] = {"S8", "F8", "SF x4", "SSFF x2", "SFF", "SSSF x2", "FFFS x2"};

template <int OP, int NACC>
void run(int cus) {
  for (int wps : {4}) {  // waves per SIMD (4 waves per block, 1 per SIMD)
    const int blocks = cus * wps;
    unsigned *out;
    unsigned long long *cyc;
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    CHECK(hipMalloc(&cyc, (size_t)blocks * 4 * 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL((probe<OP, NACC>), dim3(blocks), dim3(256), 0, 0, out, cyc, 1u);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((probe<OP, NACC>), dim3(blocks), dim3(256), 0, 0, out, cyc, 2u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long *h = (unsigned long long *)malloc((size_t)blocks * 4 * 8);
    CHECK(hipMemcpy(h, cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost));
    double mean = 0;
    for (int i = 0; i < blocks * 4; i++) mean += (double)h[i];
    mean /= blocks * 4;
    const double insts = (double)kIters * NACC;  // per wave
    // per-SIMD throughput: wps waves each issuing `insts` in ~`mean` cycles (concurrent)
    const double simd_cpi = mean / (insts * wps);
    const double gips = (double)blocks * 4 * insts / (ms * 1e-3) / 1e9;
    printf("%-22s nacc=%2d waves/SIMD=%d  wave-cycles/inst=%.2f  SIMD cycles/inst=%.2f  %.0f G wave-inst/s (%.3f ms, memtime %.2f GHz)\n",
           kNames[OP], NACC, wps, mean / insts, simd_cpi, gips, ms, mean / (ms * 1e6));
    free(h);
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
  }
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  printf("CUs: %d\n", cus);
  run<0, 8>(cus);
  run<1, 8>(cus);
  run<2, 8>(cus);
  run<3, 8>(cus);
  run<4, 8>(cus);
  run<5, 8>(cus);
  run<6, 8>(cus);
  return 0;
}
