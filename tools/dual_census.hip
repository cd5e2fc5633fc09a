// dual_census.hip -- which VALU encodings can gfx950 issue two at a time?  One kernel per
// instruction form (probe_<id>), each wave running 8 independent chains of it; run under
//   rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -- /tmp/dc [waves/SIMD]
// and read VALU instructions per SIMD quad-cycle and the dual-issued share per kernel.
//   hipcc --offload-arch=gfx950 -O3 tools/dual_census.hip -o /tmp/dc
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

constexpr int kIters = 2048;
typedef void (*Fn)(unsigned *);
std::vector<std::pair<const char *, Fn>> &probes() {
  static std::vector<std::pair<const char *, Fn>> v;
  return v;
}
struct Reg {
  Reg(const char *n, Fn f) { probes().push_back({n, f}); }
};
__device__ __forceinline__ unsigned hash(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  return x ^ (x >> 16);
}
// OPA on chains 0..3, OPB on chains 4..7, issued in the order given by ORDER (0: ABAB.., 1: AABB..)
#define PROBE2(ID, OPA, OPB, ORDER)                                                                   \
  __global__ __launch_bounds__(256) void probe_##ID(unsigned *out) {                                  \
    unsigned a[8];                                                                                    \
    const unsigned t = blockIdx.x * 256 + threadIdx.x;                                                \
    for (int i = 0; i < 8; i++) a[i] = hash(t * 8 + i) & 0x03ff03ffu;                                 \
    const unsigned b = hash(t ^ 0x1234567u) & 0x00ff00ffu, c = hash(t ^ 0x7654321u) & 0x00ff00ffu;    \
    for (int it = 0; it < kIters; it++) {                                                             \
      if (ORDER == 0) {                                                                               \
        asm volatile(OPA : "+v"(a[0]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[4]) : "v"(b), "v"(c));                                              \
        asm volatile(OPA : "+v"(a[1]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[5]) : "v"(b), "v"(c));                                              \
        asm volatile(OPA : "+v"(a[2]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[6]) : "v"(b), "v"(c));                                              \
        asm volatile(OPA : "+v"(a[3]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[7]) : "v"(b), "v"(c));                                              \
      } else {                                                                                        \
        asm volatile(OPA : "+v"(a[0]) : "v"(b), "v"(c));                                              \
        asm volatile(OPA : "+v"(a[1]) : "v"(b), "v"(c));                                              \
        asm volatile(OPA : "+v"(a[2]) : "v"(b), "v"(c));                                              \
        asm volatile(OPA : "+v"(a[3]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[4]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[5]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[6]) : "v"(b), "v"(c));                                              \
        asm volatile(OPB : "+v"(a[7]) : "v"(b), "v"(c));                                              \
      }                                                                                               \
    }                                                                                                 \
    unsigned s = 0;                                                                                   \
    for (int i = 0; i < 8; i++) s ^= a[i];                                                            \
    out[t] = s;                                                                                       \
  }                                                                                                   \
  static Reg reg_##ID(#ID ": " OPA " | " OPB, probe_##ID);
#define PROBE(ID, OP) PROBE2(ID, OP, OP, 0)

PROBE(add_u32, "v_add_u32 %0, %0, %1")
PROBE(sub_u32, "v_sub_u32 %0, %0, %1")
PROBE(subrev_u32, "v_subrev_u32 %0, %1, %0")
PROBE(and_b32, "v_and_b32 %0, %0, %1")
PROBE(or_b32, "v_or_b32 %0, %0, %1")
PROBE(xor_b32, "v_xor_b32 %0, %0, %1")
PROBE(lshrrev_b32, "v_lshrrev_b32 %0, %1, %0")
PROBE(lshlrev_b32, "v_lshlrev_b32 %0, %1, %0")
PROBE(ashrrev_i32, "v_ashrrev_i32 %0, %1, %0")
PROBE(max_u32, "v_max_u32 %0, %0, %1")
PROBE(min_u32, "v_min_u32 %0, %0, %1")
PROBE(max_i32, "v_max_i32 %0, %0, %1")
PROBE(mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
PROBE(mov_b32, "v_mov_b32 %0, %1")
PROBE(not_b32, "v_not_b32 %0, %0")
PROBE(add_u16, "v_add_u16 %0, %0, %1")
PROBE(sub_u16, "v_sub_u16 %0, %0, %1")
PROBE(max_u16, "v_max_u16 %0, %0, %1")
PROBE(max_i16, "v_max_i16 %0, %0, %1")
PROBE(lshrrev_b16, "v_lshrrev_b16 %0, %1, %0")
PROBE(add_f32, "v_add_f32 %0, %0, %1")
PROBE(mul_f32, "v_mul_f32 %0, %0, %1")
PROBE(max_f32, "v_max_f32 %0, %0, %1")
PROBE(fmac_f32, "v_fmac_f32 %0, %1, %2")
PROBE(add_f16, "v_add_f16 %0, %0, %1")
PROBE(cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
PROBE(cvt_u32_f32, "v_cvt_u32_f32 %0, %0")
PROBE(add_co_u32, "v_add_co_u32 %0, vcc, %0, %1")
PROBE(cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
PROBE(add_u32_e64, "v_add_u32_e64 %0, %0, %1")
PROBE(add_u32_e64_clamp, "v_add_u32_e64 %0, %0, %1 clamp")
PROBE(add_u32_inl, "v_add_u32 %0, 7, %0")
PROBE(add_u32_lit, "v_add_u32 %0, 0x12345, %0")
PROBE(add_u32_dpp, "v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf")
PROBE(add_u32_sdwa, "v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0")
PROBE(add3_u32, "v_add3_u32 %0, %0, %1, %2")
PROBE(lshl_add_u32, "v_lshl_add_u32 %0, %0, 1, %1")
PROBE(bfe_u32, "v_bfe_u32 %0, %0, 4, 16")
PROBE(perm_b32, "v_perm_b32 %0, %0, %1, %2")
PROBE(sad_u16, "v_sad_u16 %0, %1, %2, %0")
PROBE(pk_add_u16, "v_pk_add_u16 %0, %0, %1")
PROBE(pk_fma_f16, "v_pk_fma_f16 %0, %0, %1, %2")
PROBE(dot2_u32_u16, "v_dot2_u32_u16 %0, %1, %2, %0")
PROBE(dot2c_f32_f16, "v_dot2c_f32_f16 %0, %1, %2")
PROBE2(mix_add_pk_abab, "v_add_u32 %0, %0, %1", "v_pk_add_u16 %0, %0, %1", 0)
PROBE2(mix_add_pk_aabb, "v_add_u32 %0, %0, %1", "v_pk_add_u16 %0, %0, %1", 1)
PROBE2(mix_add_and_abab, "v_add_u32 %0, %0, %1", "v_and_b32 %0, %0, %1", 0)
PROBE2(mix_add_max_abab, "v_add_u32 %0, %0, %1", "v_max_u32 %0, %0, %1", 0)
PROBE2(mix_add_add3_abab, "v_add_u32 %0, %0, %1", "v_add3_u32 %0, %0, %1, %2", 0)
PROBE2(mix_add_add3_aabb, "v_add_u32 %0, %0, %1", "v_add3_u32 %0, %0, %1, %2", 1)

int main(int argc, char **argv) {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int wps = argc > 1 ? atoi(argv[1]) : 4;  // waves per SIMD (256-thread blocks = 1 wave per SIMD)
  unsigned *out;
  CHECK(hipMalloc(&out, (size_t)cus * wps * 256 * 4));
  for (auto &p : probes()) {
    hipLaunchKernelGGL(p.second, dim3(cus * wps), dim3(256), 0, 0, out);
    CHECK(hipDeviceSynchronize());
    printf("%s\n", p.first);
  }
  return 0;
}
