// valu_census.hip -- issue-rate census of single VALU instruction forms on gfx950.
// Each probe: 4 waves per SIMD (16 per CU), every wave runs 8 independent chains
// a[i] = OP(a[i], b, c) with per-lane pseudo-random b, c.  Reports wave-instructions per
// second over the whole chip, the shader clock (s_memtime delta over s_memrealtime's
// 100 MHz) and SIMD cycles per instruction at that clock.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_census.hip -o /tmp/vc && /tmp/vc
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

constexpr int kIters = 4096;

struct Probe {
  const char *name;
  void (*fn)(unsigned *, unsigned long long *, unsigned);
};
std::vector<Probe> &probes() {
  static std::vector<Probe> v;
  return v;
}
struct Reg {
  Reg(const char *n, void (*f)(unsigned *, unsigned long long *, unsigned)) { probes().push_back({n, f}); }
};

__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

#define ONE(I) asm volatile(OPSTR : "+v"(a[I]) : "v"(b), "v"(c));
#define PROBE(ID, OPSTR_)                                                                          \
  __global__ __launch_bounds__(256) void probe_##ID(unsigned *out, unsigned long long *cyc, unsigned seed) { \
    unsigned a[8];                                                                                 \
    const unsigned t = blockIdx.x * 256 + threadIdx.x;                                             \
    for (int i = 0; i < 8; i++) a[i] = hash(seed + t * 8 + i);                                     \
    const unsigned b = hash(t ^ 0x1234567u), c = hash(t ^ 0x7654321u) & 0x03ff03ffu;               \
    __syncthreads();                                                                               \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                    \
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();                                \
    for (int it = 0; it < kIters; it++) {                                                          \
      _Pragma("unroll") for (int i = 0; i < 8; i++) asm volatile(OPSTR_ : "+v"(a[i]) : "v"(b), "v"(c)); \
    }                                                                                              \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                    \
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();                                \
    unsigned s = 0;                                                                                \
    for (int i = 0; i < 8; i++) s ^= a[i];                                                         \
    out[t] = s;                                                                                    \
    if ((threadIdx.x & 63) == 0) {                                                                 \
      cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64)] = t1 - t0;                                      \
      cyc[2 * (blockIdx.x * 4 + threadIdx.x / 64) + 1] = r1 - r0;                                  \
    }                                                                                              \
  }                                                                                                \
  static Reg reg_##ID(OPSTR_, probe_##ID);

// 32-bit
PROBE(add_u32, "v_add_u32 %0, %0, %1")
PROBE(add_u32_rev, "v_add_u32 %0, %1, %0")
PROBE(sub_u32, "v_sub_u32 %0, %0, %1")
PROBE(subrev_u32, "v_subrev_u32 %0, %1, %0")
PROBE(add_co_u32, "v_add_co_u32 %0, vcc, %0, %1")
PROBE(add3_u32, "v_add3_u32 %0, %0, %1, %2")
PROBE(lshl_add_u32, "v_lshl_add_u32 %0, %0, 1, %1")
PROBE(add_lshl_u32, "v_add_lshl_u32 %0, %0, %1, 1")
PROBE(and_b32, "v_and_b32 %0, %0, %1")
PROBE(or_b32, "v_or_b32 %0, %0, %1")
PROBE(xor_b32, "v_xor_b32 %0, %0, %1")
PROBE(and_or_b32, "v_and_or_b32 %0, %0, %1, %2")
PROBE(lshlrev_b32, "v_lshlrev_b32 %0, %1, %0")
PROBE(lshrrev_b32, "v_lshrrev_b32 %0, %1, %0")
PROBE(lshlrev_b32_c, "v_lshlrev_b32 %0, 1, %0")
PROBE(lshrrev_b32_c, "v_lshrrev_b32 %0, 1, %0")
PROBE(max_u32, "v_max_u32 %0, %0, %1")
PROBE(min_u32, "v_min_u32 %0, %0, %1")
PROBE(max_i32, "v_max_i32 %0, %0, %1")
PROBE(max3_u32, "v_max3_u32 %0, %0, %1, %2")
PROBE(med3_i32, "v_med3_i32 %0, %0, %1, %2")
PROBE(mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
PROBE(mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
PROBE(mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
PROBE(bfe_u32, "v_bfe_u32 %0, %0, 4, 16")
PROBE(alignbit_b32, "v_alignbit_b32 %0, %0, %1, 16")
PROBE(perm_b32, "v_perm_b32 %0, %0, %1, %2")
PROBE(sad_u16, "v_sad_u16 %0, %1, %2, %0")
PROBE(sad_u32, "v_sad_u32 %0, %1, %2, %0")
PROBE(sad_u8, "v_sad_u8 %0, %1, %2, %0")
PROBE(msad_u8, "v_msad_u8 %0, %1, %2, %0")
PROBE(cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
PROBE(mov_b32, "v_mov_b32 %0, %1")
PROBE(not_b32, "v_not_b32 %0, %0")
PROBE(dot2_u32_u16, "v_dot2_u32_u16 %0, %1, %2, %0")
// 16-bit scalar
PROBE(add_u16, "v_add_u16 %0, %0, %1")
PROBE(sub_u16, "v_sub_u16 %0, %0, %1")
PROBE(max_i16, "v_max_i16 %0, %0, %1")
PROBE(max_u16, "v_max_u16 %0, %0, %1")
PROBE(lshrrev_b16, "v_lshrrev_b16 %0, 1, %0")
PROBE(mad_u16, "v_mad_u16 %0, %0, %1, %2")
// packed 16-bit
PROBE(pk_add_u16, "v_pk_add_u16 %0, %0, %1")
PROBE(pk_sub_u16, "v_pk_sub_u16 %0, %0, %1")
PROBE(pk_sub_i16, "v_pk_sub_i16 %0, %0, %1")
PROBE(pk_sub_u16_clamp, "v_pk_sub_u16 %0, %0, %1 clamp")
PROBE(pk_add_i16_opsel, "v_pk_add_i16 %0, %1, %0 op_sel_hi:[0,1]")
PROBE(pk_max_i16, "v_pk_max_i16 %0, %0, %1")
PROBE(pk_max_u16, "v_pk_max_u16 %0, %0, %1")
PROBE(pk_min_u16, "v_pk_min_u16 %0, %0, %1")
PROBE(pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %2")
PROBE(pk_mad_u16_c, "v_pk_mad_u16 %0, %0, 3, %1 op_sel_hi:[1,0,1]")
PROBE(pk_lshrrev_b16, "v_pk_lshrrev_b16 %0, 1, %0 op_sel_hi:[0,1]")
PROBE(pk_lshlrev_b16, "v_pk_lshlrev_b16 %0, 1, %0 op_sel_hi:[0,1]")
PROBE(pk_mul_lo_u16, "v_pk_mul_lo_u16 %0, %0, %1")
// float
PROBE(add_f32, "v_add_f32 %0, %0, %1")
PROBE(fma_f32, "v_fma_f32 %0, %0, %1, %2")
PROBE(add_f16, "v_add_f16 %0, %0, %1")
PROBE(pk_add_f16, "v_pk_add_f16 %0, %0, %1")
PROBE(pk_fma_f16, "v_pk_fma_f16 %0, %0, %1, %2")
PROBE(cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
PROBE(cvt_u32_f32, "v_cvt_u32_f32 %0, %0")
// DPP / SDWA forms
PROBE(add_u32_dpp, "v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf")
PROBE(add_u32_sdwa, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0")
PROBE(max_i16_sdwa, "v_max_i16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1")

template <class F>
void run(const char *name, F fn, int cus, int wps) {
  const int blocks = cus * wps;  // 4 waves per block: wps waves per SIMD
  unsigned *out;
  unsigned long long *cyc;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CHECK(hipMalloc(&cyc, (size_t)blocks * 4 * 16));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 2; w++) hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, out, cyc, 1u);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, out, cyc, 2u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h((size_t)blocks * 8);
  CHECK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  double cy = 0, rt = 0;
  for (int i = 0; i < blocks * 4; i++) cy += (double)h[2 * i], rt += (double)h[2 * i + 1];
  cy /= blocks * 4;
  rt /= blocks * 4;
  const double ghz = cy / (rt / 100e6) / 1e9;  // s_memrealtime: 100 MHz
  const double insts = (double)kIters * 8;     // per wave
  const double gips = (double)blocks * 4 * insts / (ms * 1e-3) / 1e9;
  printf("%-70s wps=%d  %7.1f G inst/s  clk %.2f GHz  SIMD cyc/inst %.2f\n", name, wps, gips, ghz, cy / (insts * wps));
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
}

int main(int argc, char **argv) {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int wps = argc > 1 ? atoi(argv[1]) : 4;
  printf("CUs: %d\n", cus);
  for (auto &p : probes()) run(p.name, p.fn, cus, wps);
  return 0;
}
