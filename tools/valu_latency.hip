// valu_latency.hip -- dependent-issue behaviour of gfx950 VALU ops: cycles per instruction
// per SIMD with C independent chains per wave and W waves per SIMD (C*W instructions
// between two dependent ones in a round-robin schedule).
//   hipcc --offload-arch=gfx950 -O3 tools/valu_latency.hip -o /tmp/vl && /tmp/vl
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kInsts = 32768;  // per wave

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  return x ^ (x >> 16);
}

template <int OP, int C>
__global__ __launch_bounds__(64) void probe(unsigned *out, unsigned long long *cyc) {
  unsigned a[C];
  const unsigned t = blockIdx.x * 64 + threadIdx.x;
  for (int i = 0; i < C; i++) a[i] = hash(t * 8 + i) & 0x03ff03ffu;
  const unsigned b = hash(t ^ 0x1234567u) & 0x00ff00ffu;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kInsts / (C * 8); it++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
#pragma unroll
      for (int i = 0; i < C; i++) {
        if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        else if constexpr (OP == 1) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        else if constexpr (OP == 2) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        else if constexpr (OP == 3) asm volatile("v_add_u32 %0, %0, %1\n v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        else asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = 0;
  for (int i = 0; i < C; i++) s ^= a[i];
  out[t] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static const char *kNames[] = {"v_add_u32", "v_pk_add_u16", "v_max_u32", "add_u32+pk_add_u16 (x2 insts)", "v_add3_u32"};

template <int OP, int C>
void run(int cus, int w) {
  const int blocks = cus * 4 * w;  // 1 wave per block: w waves per SIMD
  unsigned *out;
  unsigned long long *cyc;
  CHECK(hipMalloc(&out, (size_t)blocks * 64 * 4));
  CHECK(hipMalloc(&cyc, (size_t)blocks * 8));
  for (int r = 0; r < 2; r++) hipLaunchKernelGGL((probe<OP, C>), dim3(blocks), dim3(64), 0, 0, out, cyc);
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(blocks);
  CHECK(hipMemcpy(h.data(), cyc, blocks * 8, hipMemcpyDeviceToHost));
  double m = 0;
  for (auto v : h) m += (double)v;
  m /= blocks;
  const double insts = (double)(kInsts / (C * 8)) * C * 8 * (OP == 3 ? 2 : 1);
  printf("%-32s chains=%d waves/SIMD=%d  wave cyc/inst %.2f  SIMD cyc/inst %.2f\n", kNames[OP], C, w, m / insts, m / insts / w);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
}

template <int OP>
void sweep(int cus) {
  for (int w : {1, 2, 4, 8}) {
    run<OP, 1>(cus, w);
    run<OP, 2>(cus, w);
    run<OP, 4>(cus, w);
    run<OP, 8>(cus, w);
  }
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  sweep<0>(cus);
  sweep<1>(cus);
  sweep<2>(cus);
  sweep<3>(cus);
  sweep<4>(cus);
  return 0;
}
