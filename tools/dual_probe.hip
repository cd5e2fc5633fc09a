// dual_probe.hip -- which neighbours of a VALU stream stop gfx950 from issuing two VALU
// instructions per SIMD quad-cycle (SQ_ACTIVE_INST_VALU2)?  Every probe runs 2 workgroups
// of 8 waves per CU (4 waves per SIMD, like the search kernel) over the same VALU stream
// -- 8 independent chains, half v_add_u32, half v_pk_add_u16 -- and adds one kind of
// neighbour per variant (LDS reads + waits, MFMAs, DPP, SALU, s_nop, ...).  Reported: VALU
// instructions per SIMD quad-cycle from the event time at the measured shader clock.
//   hipcc --offload-arch=gfx950 -O3 tools/dual_probe.hip -o /tmp/dp && /tmp/dp
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

constexpr int kIters = 1024;  // x 64 VALU per iteration per wave

typedef _Float16 __attribute__((ext_vector_type(4))) h4;
typedef float __attribute__((ext_vector_type(4))) f4;

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  return x ^ (x >> 16);
}

#define F(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define S(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define G8 F(0) S(1) F(2) S(3) F(4) S(5) F(6) S(7)

// VAR: 0 plain, 1 + ds_read_b64 and wait every 16 VALU, 2 + ds_write_b16 every 8, 3 + MFMA every 32,
// 4 + DPP add every 8, 5 + SALU every 8, 6 + s_nop 1 every 16, 7 + v_cvt_u32_f32 every 8,
// 8 + VOP3 v_add3_u32 instead of F, 9 + global store every 64, 10 + wave barrier every 64,
// 11 all-F stream, 12 all-S stream, 13 + ds_read_b64 (no wait until the end of 64)
template <int VAR>
__global__ __launch_bounds__(512, 2) void probe(unsigned *out, unsigned long long *cyc) {
  __shared__ uint2 lds[4096];
  unsigned a[8];
  const unsigned t = blockIdx.x * 512 + threadIdx.x;
  for (int i = 0; i < 8; i++) a[i] = hash(t * 8 + i) & 0x03ff03ffu;
  const unsigned b = hash(t ^ 0x1234567u) & 0x00ff00ffu;
  for (int i = threadIdx.x; i < 4096; i += 512) lds[i] = make_uint2(hash(i), hash(i + 7));
  __syncthreads();
  h4 av = {(_Float16)1, (_Float16)2, (_Float16)3, (_Float16)4}, bv = av;
  f4 acc = {0, 0, 0, 0};
  unsigned s0 = __builtin_amdgcn_readfirstlane(t);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < kIters; it++) {
#pragma unroll
    for (int g = 0; g < 8; g++) {
      if constexpr (VAR == 11) {
        F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7)
      } else if constexpr (VAR == 12) {
        S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)
      } else if constexpr (VAR == 8) {
        asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[0]) : "v"(b));
        S(1)
        asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[2]) : "v"(b));
        S(3)
        asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[4]) : "v"(b));
        S(5)
        asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[6]) : "v"(b));
        S(7)
      } else {
        G8
      }
      if constexpr (VAR == 1) {
        if (g & 1) {
          uint2 v = lds[(threadIdx.x + it * 8 + g) & 4095];
          a[g & 7] ^= v.x;
        }
      } else if constexpr (VAR == 13) {
        uint2 v = lds[(threadIdx.x * 3 + it * 8 + g) & 4095];
        a[(g + 3) & 7] += v.y;
      } else if constexpr (VAR == 2) {
        reinterpret_cast<unsigned short *>(lds)[(threadIdx.x * 2 + g) & 16383] = (unsigned short)a[g];
      } else if constexpr (VAR == 3) {
        if ((g & 3) == 3) acc = __builtin_amdgcn_mfma_f32_16x16x16f16(av, bv, acc, 0, 0, 0);
      } else if constexpr (VAR == 4) {
        a[g] += (unsigned)__builtin_amdgcn_update_dpp(0, (int)a[(g + 1) & 7], 0x111, 0xf, 0xf, true);
      } else if constexpr (VAR == 5) {
        asm volatile("s_add_u32 %0, %0, 3" : "+s"(s0));
      } else if constexpr (VAR == 6) {
        if (g & 1) asm volatile("s_nop 1");
      } else if constexpr (VAR == 7) {
        a[g] = (unsigned)(float)a[g];
      } else if constexpr (VAR == 10) {
        if (g == 7) __builtin_amdgcn_wave_barrier();
      }
    }
    if constexpr (VAR == 9) out[t + (it & 7) * 1024 * 512] = a[it & 7];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  unsigned s = s0 + (unsigned)acc[0];
  for (int i = 0; i < 8; i++) s ^= a[i];
  out[t] = s;
  if ((threadIdx.x & 63) == 0) {
    cyc[2 * (t / 64)] = t1 - t0;
    cyc[2 * (t / 64) + 1] = r1 - r0;
  }
}

static const char *kNames[] = {"plain F/S mix", "+ds_read_b64+wait /16", "+ds_write_b16 /8", "+MFMA16 /32",
                               "+DPP add /8", "+SALU /8", "+s_nop 1 /16", "+cvt_u32_f32 /8", "VOP3 add3 for F",
                               "+global store /64", "+wave_barrier /64", "all F", "all S", "+ds_read_b64 /8 lazy"};

template <int VAR>
void run(int cus) {
  const int blocks = cus * 2;
  unsigned *out;
  unsigned long long *cyc;
  CHECK(hipMalloc(&out, (size_t)8 * 1024 * 512 * 4 + (size_t)blocks * 512 * 4));
  CHECK(hipMalloc(&cyc, (size_t)blocks * 8 * 16));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(probe<VAR>, dim3(blocks), dim3(512), 0, 0, out, cyc);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(probe<VAR>, dim3(blocks), dim3(512), 0, 0, out, cyc);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h((size_t)blocks * 16);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  double cy = 0, rt = 0;
  for (int i = 0; i < blocks * 8; i++) cy += (double)h[2 * i], rt += (double)h[2 * i + 1];
  cy /= blocks * 8;
  rt /= blocks * 8;
  const double ghz = cy / (rt / 100e6) / 1e9;
  const double valu = 64.0 * kIters;  // the counted VALU stream per wave (extras not counted)
  // per SIMD: 4 waves; quad-cycles over the wave's own elapsed clock
  printf("%-24s VALU/quad %.3f (wave clock)  %.3f (event time @%.2f GHz)  %.3f ms\n", kNames[VAR], 4 * valu / (cy / 4),
         4 * valu / (ms * 1e-3 * ghz * 1e9 / 4),
         ghz, ms);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  run<0>(cus);
  run<11>(cus);
  run<12>(cus);
  run<1>(cus);
  run<13>(cus);
  run<2>(cus);
  run<3>(cus);
  run<4>(cus);
  run<5>(cus);
  run<6>(cus);
  run<7>(cus);
  run<8>(cus);
  run<9>(cus);
  run<10>(cus);
  run<0>(cus);
  return 0;
}
