// mip_search.hip -- fused MIP mode search for gfx950 (MI355X).
//
// One kernel does what the reference splits over initBoundaries, MIP_ReducedPred and
// three upsampleDistortion builds (intra.cl:17-1171): boundary downsampling, the MIP
// matrix-vector products, linear upsampling, SAD and 4x4-Hadamard SATD and the
// min(2*SAD, SATD) cost -- without any intermediate in HBM (the reference round-trips
// ~1.2 GB of reduced predictions per 1080p frame, main.cpp:443-444).
//
// Work decomposition
//   workgroup = persistent, 12 waves (two per CU: six waves per SIMD, MIP_SIX_WAVES 3; 16 in
//               small launches, one per CU); takes items = (frame, CTU, quadrant, slice) from a
//               device-wide queue (one counter per XCD chunk, take_item).  No CU of the 47 shapes straddles a 64x64 quadrant, so
//               an item stages only its quadrant (+1 row above, +4 columns left: the
//               reference samples) in LDS; the MIP matrices are staged once per workgroup.
//               CTUs cut by the frame border have their own lists (CUs outside the frame
//               get MIP_COST_UNAVAILABLE and no work).
//   wave      = a list of tasks (host-built, load balanced).  A task is up to 64/(S*V) CUs
//               of ONE size class W x H (S = W/4 column strips, V = row parts) and a range
//               of mode pairs; every loop bound is a compile-time constant of the class.
//   lane      = (CU, row part, strip), CU-stationary: it loads its boundaries and original
//               samples once and walks the mode pairs of the task one after another.  The
//               two modes of a pair ride in the two 16-bit halves of each VGPR (packed
//               v_pk_* int16 ops; all intermediates provably fit 16 bits).
//   per pair  phase A: the reduced predictions of all CUs of the task for the pair, as
//               16x16x16 f16 MFMAs (exact: integer inputs < 2^11, sums < 2^24), into a
//               wave-private LDS scratch; phase B: every lane upsamples its strip window by
//               window and computes SAD + SATD 4x4 block by 4x4 block; strips and row parts
//               of a CU are combined with xor shuffles, one lane stores the two costs.
//
// Bit-exactness: every step restates the reference integer semantics (citations inline);
// tests/test_gpu_parity.py checks the tables bit for bit against the C oracle, which is
// pinned to the reference kernels' own outputs (tests/golden/).
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include <hip/hip_ext.h>

// The four-wave twin (round 6): this file compiled a second time with -DMIP_SIX_WAVES=0
// -DMIP_FOUR_WAVE_TWIN=1 (Makefile: build/mip_search_four.o) exports the 8-wave search as
// launch_search_four / search_resident_groups_four, which the host pipeline uses for its small
// alternating chunks (mipgpu.cpp search_device_impl).  The helper kernels live in the
// primary compilation only.
#ifndef MIP_FOUR_WAVE_TWIN
#define MIP_FOUR_WAVE_TWIN 0
#endif
#if MIP_FOUR_WAVE_TWIN
#define launch_search launch_search_four
#define search_resident_groups search_resident_groups_four
#define search_lds_bytes search_lds_bytes_four
#endif

#include "mip_kernels.h"
#include "mip_tables.h"

namespace mipgpu {
namespace {

typedef short __attribute__((ext_vector_type(2))) s2;
typedef unsigned short __attribute__((ext_vector_type(2))) u2;
typedef _Float16 __attribute__((ext_vector_type(2))) h2;
typedef _Float16 __attribute__((ext_vector_type(4))) h4;
typedef float __attribute__((ext_vector_type(4))) f4;

[[maybe_unused]] __constant__ mip_shape_desc c_shapes[MIP_NUM_SHAPES] = MIP_SHAPE_TABLE;  // (helper kernels)
// first CU (reference order inside a CTU) of every shape, for the decision-list kernel
struct ShapeStarts {
  uint16_t v[MIP_NUM_SHAPES + 1];
};
constexpr mip_shape_desc kShapesC[MIP_NUM_SHAPES] = MIP_SHAPE_TABLE;
constexpr ShapeStarts make_shape_starts() {
  ShapeStarts st{};
  for (int i = 0; i < MIP_NUM_SHAPES; i++) st.v[i + 1] = (uint16_t)(st.v[i] + kShapesC[i].ncu);
  return st;
}
static_assert(make_shape_starts().v[MIP_NUM_SHAPES] == MIP_CUS_PER_CTU, "shape table");
[[maybe_unused]] __constant__ ShapeStarts c_shape_start = make_shape_starts();

#ifndef MIP_PREFETCH_MIN_ITEMS
#define MIP_PREFETCH_MIN_ITEMS 32  // items per workgroup from which a launch prefetches (A/B knob)
#endif
#ifndef MIP_PF_BATCH
#define MIP_PF_BATCH 10  // window loads in flight per lane in the prefetching wave (6: -0.3 %)
#endif
#ifndef MIP_PHASEA_BATCH_NCS
#define MIP_PHASEA_BATCH_NCS 2  // column sets from which phase A reads its B operands up front (A/B knob)
#endif
#ifndef MIP_ACC_PAIR
#define MIP_ACC_PAIR 1  // blocks accumulated in pairs before unpacking (A/B knob)
#endif
#ifndef MIP_UV2_UNROLL
#define MIP_UV2_UNROLL 2  // blocks per loop iteration, UV = 2 classes with H > 8 (A/B knob)
#endif
#ifndef MIP_WIN_UNROLL
#define MIP_WIN_UNROLL 2  // windows of the vertical pass per loop iteration (A/B knob)
#endif
#ifndef MIP_PAIR_BLOCKS
#define MIP_PAIR_BLOCKS 1  // classes with an even block count per lane walk block pairs (A/B knob)
#endif
#ifndef MIP_PRIO_BALANCE
#define MIP_PRIO_BALANCE 0  // wave priority follows the item's remaining tasks (A/B knob; measured
                            // -1.7 % at 384 frames / -1.5 % at 32, 1 frame 0.184 -> 0.177 ms: off)
#endif
#ifndef MIP_ONLY_CLASS
#define MIP_ONLY_CLASS -1  // resource census of one size class (tools/vgpr_census.sh)
#endif
#ifndef MIP_SKIP_CLASSES
#define MIP_SKIP_CLASSES 0  // bit mask of size classes compiled out (occupancy experiments; wrong tables)
#endif

constexpr int kPitch = 68;       // LDS row pitch in samples (34 dwords: conflict-free rows)
constexpr int kColOff = 4;       // LDS column of quadrant column 0 (-4..-1: left halo)
constexpr int kTileElems = (65 * kPitch + 7) / 8 * 8;  // quadrant rows -1..63
// Alternative references (ALT): CU boundaries only read quadrant rows 4i-1 (top) and
// columns 4i-1 (left), so only that lattice of the reference frame is staged.
constexpr int kLatRowPitch = kPitch, kLatColPitch = 66;
constexpr int kLatElems = (16 * kLatRowPitch + 16 * kLatColPitch + 7) / 8 * 8;
// Wave-private LDS: per-CU MFMA inputs + reduced-prediction scratch.
constexpr int kEntryBytes = 16;                         // 8 f16 MFMA inputs per CU
constexpr int kCuTableBytes = 64 * kEntryBytes;
#ifndef MIP_SCRATCH_WORDS
// 1152 with six waves per SIMD: two 12-wave workgroups per CU in 160 KB of LDS
// (MIP_SIX_WAVES 3, round 6: 768, the MIP tables kept in LDS, the 64-slot 4xN and the 8xH
// tasks' reduced predictions produced in chunks of two rows, see Geo)
#define MIP_SCRATCH_WORDS \
  (MIP_SIX_WAVES == 1 ? 1152 : (MIP_SIX_WAVES == 2 ? 1144 : (MIP_SIX_WAVES == 3 ? 768 : 1280)))
#endif
// Chunks that end inside a CU's block pair or 4x4 block (MIP_SIX_WAVES 3): phase A of the next
// chunk runs in the middle of the lane's walk (walk_pairs_chunked, walk_4x4_chunked).
constexpr bool kSpanChunks = MIP_SIX_WAVES == 3;
constexpr int kScratchWords = MIP_SCRATCH_WORDS;        // [slot][position] packed mode pairs
constexpr int kWaveBytes = kCuTableBytes + kScratchWords * 4;
constexpr int kWaveStride = kWaveBytes;  // LDS bytes between waves' private areas
constexpr int kZeroBytes = 7 * 8 * kEntryBytes + 16;    // > every uniform B offset + 8 B
constexpr int kUnavailable = 0x7fffffff;

// Biased residuals.  The Hadamard butterflies of the SATD run as plain 32-bit adds /
// subtracts on both 16-bit halves at once (v_add_u32 / v_sub_u32 can be dual-issued on
// gfx950, the packed v_pk_* ops cannot: tools/dual_census.sh), which is exact only while no
// half ever goes negative or past 65535.  So every value carries a bias: the original
// samples are staged into LDS as o + kBiasD[y & 1][x & 3] (the 4x4 block position), so the
// residual o - p arrives biased, and the biases propagate through the butterflies to
//   row stage 1 (s):  >= 2046,  row stage 2 (t): >= 4092,  column stage (u): >= 8184
// -- each exactly the magnitude bound of that stage (|d| <= 1023 doubles per stage) -- with
// every biased value below 40920.  The last column butterfly is folded as
// |a+b| + |a-b| = 2 max(|a|, |b|) on pairs that share a bias: u0/u2 of column k carry
// kBiasP[k], u1/u3 carry kBiasQ (2 * bias < 65536, see block_finish).
constexpr uint32_t kBiasD[2][4] = {{15345, 1023, 3069, 1023}, {7161, 1023, 3069, 1023}};  // [row & 1][col]
constexpr uint32_t kBiasP[4] = {32736, 24552, 16368, 16368};
constexpr uint32_t kBiasQ = 8184;
constexpr uint32_t splat32(uint32_t v) { return v | v << 16; }
// a staged dword holds columns (x, x+1), x even: the biases of a block row's column pair
constexpr uint32_t bias_word(int y, int x) { return kBiasD[y & 1][x & 3] | kBiasD[y & 1][(x + 1) & 3] << 16; }

__device__ __forceinline__ int tidx(int x, int y) { return (y + 1) * kPitch + x + kColOff; }
__device__ __forceinline__ s2 as_s2(uint32_t v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ u2 as_u2(s2 v) { return __builtin_bit_cast(u2, v); }
__device__ __forceinline__ s2 as_s2(u2 v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ s2 splat(int v) { return s2{(short)v, (short)v}; }
__device__ __forceinline__ s2 smax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }

constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v / 2); }

// (a + b + 1) >> 1 on both halves of non-negative 10-bit samples: one 32-bit three-input add
// (a + b + 1 <= 2047, so no carry crosses the halves) and one packed shift.
__device__ __forceinline__ s2 avg_round(s2 a, s2 b) {
  const uint32_t t = __builtin_bit_cast(uint32_t, a) + __builtin_bit_cast(uint32_t, b) + 0x00010001u;
  return __builtin_bit_cast(s2, __builtin_bit_cast(u2, t) >> (u2){1, 1});
}

// Compile-time loop: f(integral_constant<int, I>) for I = 0..N-1.
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F &f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// a * O + c on both 16-bit halves as ONE v_pk_mad_u16 (the compiler splits small constant
// multipliers into shift + add).
template <int O>
__device__ __forceinline__ u2 pk_mad_c(u2 a, u2 c) {
  if constexpr (O == 1) {
    return a + c;
  } else {
    u2 d;
    asm("v_pk_mad_u16 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(a), "i"(O), "v"(c));
    return d;
  }
}
// a * O + C on both halves, O and C constants
template <int O, int C>
__device__ __forceinline__ u2 pk_mad_cc(u2 a) {
  u2 d;
  asm("v_pk_mad_u16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(a), "i"(O), "i"(C));
  return d;
}

// LDS fence for data handed between lanes of ONE wave (wave-private scratch).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Compile-time geometry of a size class (W x H, VP row parts; default: the base class).
template <int W, int H, int VP = kClassV[size_class(W, H)]>
struct Geo {
  static constexpr int SID = class_size_id(W, H);
  static constexpr int R = SID == 2 ? 8 : 4;          // reduced prediction side
  static constexpr int RBS = SID == 0 ? 2 : 4;        // reduced boundary length per side
  static constexpr int NOUT = R * R;
  static constexpr int UH = W / R, UV = H / R;        // upsampling factors
  static constexpr int LH = ilog2c(UH), LV = ilog2c(UV);
  static constexpr int S = W / 4;                     // column strips per CU
  static constexpr int V = VP;                        // row parts per CU
  static constexpr int SLOTS = 64 / (S * V);          // CUs per task
  static constexpr int KV = R / V;                    // upsampling windows per row part
  // Classes without horizontal interpolation whose reduced predictions for all the task's CUs
  // do not fit the scratch produce them in chunks of CROWS reduced rows: 8xH in two halves
  // (four quarters with MIP_SIX_WAVES 3), the 64-slot 4x4 / 4x8 tasks (MIP_SIX_WAVES 3) in two.
  // With horizontal interpolation (padded rows, MIP_SIX_WAVES 3: 16x16, 16x8) in halves.
  static constexpr int CROWS = UH != 1 ? (kSpanChunks && 64 / (S * V) * (R * (R + 1) + 1) > kScratchWords ? R / 2 : R)
                               : 64 / (S * V) * (NOUT + 4) <= kScratchWords ? R
                               : !kSpanChunks ? (SID == 2 ? R / 2 : R)
                               : 64 / (S * V) * (NOUT / 2 + 4) > kScratchWords ? R / 4 : R / 2;
  static constexpr bool CHUNKED = CROWS < R;
  static constexpr int NCH = R / CROWS;               // chunks
  static constexpr int CPOS = CROWS * R;              // scratch positions per chunk (UH == 1: rows of R)
  // Scratch rows: classes with horizontal interpolation (UH > 1) keep the anchor row's left
  // boundary sample in front of each reduced row (position k*RP, reduced (k, kx) at
  // k*RP + kx + 1), so the interpolation reads "the sample before" without a select.
  static constexpr bool PAD = UH > 1;
  static constexpr int RP = PAD ? R + 1 : R;
  // scratch: [slot][PITCH] dwords; UH == 1 classes read 4 consecutive positions (16-B aligned)
  // (the 64-slot 4xN classes drop the 4-word pad when it does not fit: 64 x 20 > kScratchWords)
  static constexpr int PITCH = UH == 1 ? (SLOTS * (CPOS + 4) <= kScratchWords ? CPOS + 4 : CPOS) : CROWS * RP + 1;
  static constexpr int WBASE = SID == 2 ? 0 : (SID == 1 ? kWeightRowOffS1 : kWeightRowOffS0);
  static constexpr int MODES = SID == 2 ? 6 : (SID == 1 ? 8 : 16);
  static_assert(SLOTS * S * V == 64, "lanes");
  static_assert(SLOTS * PITCH <= kScratchWords, "scratch");
  // a row part is whole upsampling windows and whole 4x4 blocks
  static_assert(V == 1 || (!CHUNKED && SID != 0 && (UV >= 4 || KV % (4 / UV) == 0)), "row parts");
  static_assert(!CHUNKED || (CROWS >= 2 && (kSpanChunks || (SID == 2 && NCH == 2))), "chunks");
};

// ---- reference samples -------------------------------------------------------------
// Full quadrant tile (original references): any (x, y) of rows -1..63, columns -4..63.
// Its samples carry the residual bias (kBiasD), removed here: reference rows lie at
// y = 4i - 1 (bias row 1) and reference columns at x = 4i - 1 (bias column 3 = 1023).
// Lattice (ALT): rows y = 4i-1 and columns x = 4i-1 only -- all a CU boundary reads; unbiased.
template <bool LAT>
struct RefTile {
  const uint16_t *t;
  template <int PH>  // PH = x & 3
  __device__ __forceinline__ int top(int x, int y) const {      // y = 4i - 1
    return LAT ? t[((y + 1) >> 2) * kLatRowPitch + x + kColOff] : t[tidx(x, y)] - (int)kBiasD[1][PH];
  }
  __device__ __forceinline__ uint2 top4(int x, int y) const {   // y = 4i - 1, x = 4k
    const uint2 v = *reinterpret_cast<const uint2 *>(t + (LAT ? ((y + 1) >> 2) * kLatRowPitch + x + kColOff : tidx(x, y)));
    return LAT ? v : make_uint2(v.x - bias_word(3, 0), v.y - bias_word(3, 2));
  }
  __device__ __forceinline__ int left(int x, int y) const {     // x = 4i - 1
    return LAT ? t[16 * kLatRowPitch + ((x + 1) >> 2) * kLatColPitch + y + 1] : t[tidx(x, y)] - (int)kBiasD[0][3];
  }
  template <int PH>  // PH = y & 3 (the bias of a reference column does not depend on it)
  __device__ __forceinline__ int left_ph(int x, int y) const { return left(x, y); }
};

// Transposed view of a reference tile, for classes searched as their transpose (TR tasks,
// see run_task): (x, y) here is (y, x) in the tile, so this view's top row is the tile's left
// column and its left column the tile's top row.
template <bool LAT>
struct RefTileT {
  RefTile<LAT> r;
  template <int PH>
  __device__ __forceinline__ int top(int x, int y) const { return r.left(y, x); }
  __device__ __forceinline__ uint2 top4(int x, int y) const {
    return make_uint2((uint32_t)r.left(y, x) | (uint32_t)r.left(y, x + 1) << 16,
                      (uint32_t)r.left(y, x + 2) | (uint32_t)r.left(y, x + 3) << 16);
  }
  template <int PH>  // PH = y & 3: the tile column y & 3 of the tile row's bias
  __device__ __forceinline__ int left_ph(int x, int y) const { return r.template top<PH>(y, x); }
  __device__ __forceinline__ int left(int x, int y) const {  // runtime bias (PAD classes only)
    const int ph = y & 3;
    return ph == 0 ? left_ph<0>(x, y) : ph == 1 ? left_ph<1>(x, y) : ph == 2 ? left_ph<2>(x, y) : left_ph<3>(x, y);
  }
};

__device__ __forceinline__ uint2 lds_row4(const uint16_t *tile, int x, int y) {
  return *reinterpret_cast<const uint2 *>(tile + tidx(x, y));
}

// Per-CU geometry + boundary padding, quadrant-relative.
struct CuPos {
  int lx, ly;      // CU origin inside the quadrant
  bool top, left;  // reference row above / column left lies inside the frame
  int padT, padL;  // padding values, intra.cl:102-106, 238-242
};

// TR: the CU's transpose -- origin (ly, lx) in the transposed view (fx0 / fy0 swapped too).
template <bool TR, class RT>
__device__ __forceinline__ CuPos cu_pos(const Job &j, int fx0, int fy0, const RT &rt) {
  CuPos c;
  c.lx = TR ? j.ly : j.lx;
  c.ly = TR ? j.lx : j.ly;
  c.top = (TR ? fx0 : fy0) + c.ly > 0;
  c.left = (TR ? fy0 : fx0) + c.lx > 0;
  c.padT = c.left ? rt.template left_ph<0>(c.lx - 1, c.ly) : 512;  // top edge: sample (x-1, 0)
  c.padL = c.top ? rt.template top<0>(c.lx, c.ly - 1) : 512;    // left edge: sample (0, y-1)
  return c;
}

// Reduced boundaries (intra.cl:71-73, 127-141, 202-204, 259-279: box downsampling; a
// factor of 1 is a copy) -> the CU's MFMA input entry: f16 values 1024 + b for the
// boundary vector b = (redT, redL) (f16 bit pattern 0x6400 | b, exact for b < 1024).  The
// transposed orientation (redL, redT) (intra.cl:417-418) is the same entry read with its
// two 8-byte halves swapped; sizeId 0 stores (T0 T1 L0 L1 | L0 L1 T0 T1) for that.
// The coefficient tables (mip_kernels.h) absorb p = b - b0, p_0 and the bias.
template <int W, int H, class RT>
__device__ __forceinline__ void write_inputs(const CuPos &c, const RT &rt, uint8_t *entry) {
  using G = Geo<W, H>;
  constexpr int dfT = W / G::RBS, l2T = ilog2c(dfT), rndT = dfT > 1 ? dfT / 2 : 0;
  constexpr int dfL = H / G::RBS, l2L = ilog2c(dfL), rndL = dfL > 1 ? dfL / 2 : 0;
  uint32_t redT[G::RBS], redL[G::RBS];
  static_for<G::RBS>([&](auto i_c) {
    constexpr int i = decltype(i_c)::value;
    uint32_t s = 0;
    if constexpr (dfT >= 4) {
#pragma unroll
      for (int t = 0; t < dfT; t += 4) {
        const uint2 v = rt.top4(c.lx + i * dfT + t, c.ly - 1);
        s += (v.x & 0xffff) + (v.x >> 16) + (v.y & 0xffff) + (v.y >> 16);
      }
    } else {
      static_for<dfT>([&](auto t_c) {
        constexpr int off = i * dfT + decltype(t_c)::value;
        s += rt.template top<off & 3>(c.lx + off, c.ly - 1);
      });
    }
    redT[i] = c.top ? (s + rndT) >> l2T : c.padT;
    uint32_t l = 0;
    static_for<dfL>([&](auto t_c) {  // c.ly % 4 == 0: the row phase is i * dfL + t
      constexpr int off = i * dfL + decltype(t_c)::value;
      l += rt.template left_ph<off & 3>(c.lx - 1, c.ly + off);
    });
    redL[i] = c.left ? (l + rndL) >> l2L : c.padL;
  });
  constexpr uint32_t kBias = 0x64006400u;  // f16 1024.0 in both halves
  uint4 e;
  if constexpr (G::RBS == 4) {
    e = make_uint4(redT[0] | redT[1] << 16, redT[2] | redT[3] << 16, redL[0] | redL[1] << 16, redL[2] | redL[3] << 16);
  } else {
    const uint32_t t01 = redT[0] | redT[1] << 16, l01 = redL[0] | redL[1] << 16;
    e = make_uint4(t01, l01, l01, t01);
  }
  e.x |= kBias;
  e.y |= kBias;
  e.z |= kBias;
  e.w |= kBias;
  *reinterpret_cast<uint4 *>(entry) = e;
}

struct BlockAcc {
  uint32_t t[16];  // row-transformed biased residual (both modes, 16-bit halves)
  uint32_t pos;    // sum of max(d, 0), both modes packed (see block_finish for the bound)
};

__device__ __forceinline__ uint32_t as_u32(s2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t as_u32(u2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u2 as_u2(uint32_t v) { return __builtin_bit_cast(u2, v); }

// One residual row i of a 4x4 block: d' = o' - p = d + kBiasD[i & 1][c] (o' is the biased
// staged sample, splat over both modes), the positive-part sum max(d, 0) = sat(d' - bias)
// (v_pk_sub_u16 clamp), and the row butterflies as carry-free 32-bit adds / subtracts.
template <int I>
__device__ __forceinline__ void block_row(BlockAcc &b, const s2 (&prow)[4], uint2 orow) {
  constexpr const uint32_t *B = kBiasD[I & 1];
  const s2 o01 = as_s2(orow.x), o23 = as_s2(orow.y);
  const uint32_t d0 = as_u32(s2{o01.x, o01.x} - prow[0]), d1 = as_u32(s2{o01.y, o01.y} - prow[1]);
  const uint32_t d2 = as_u32(s2{o23.x, o23.x} - prow[2]), d3 = as_u32(s2{o23.y, o23.y} - prow[3]);
  const uint32_t p0 = as_u32(__builtin_elementwise_sub_sat(as_u2(d0), (u2){(unsigned short)B[0], (unsigned short)B[0]}));
  const uint32_t p1 = as_u32(__builtin_elementwise_sub_sat(as_u2(d1), (u2){(unsigned short)B[1], (unsigned short)B[1]}));
  const uint32_t p2 = as_u32(__builtin_elementwise_sub_sat(as_u2(d2), (u2){(unsigned short)B[2], (unsigned short)B[2]}));
  const uint32_t p3 = as_u32(__builtin_elementwise_sub_sat(as_u2(d3), (u2){(unsigned short)B[3], (unsigned short)B[3]}));
  b.pos = I == 0 ? p0 + p1 + p2 + p3 : b.pos + p0 + p1 + p2 + p3;
  const uint32_t s0 = d0 + d1, s1 = d0 - d1, s2_ = d2 + d3, s3 = d2 - d3;
  b.t[4 * I + 0] = s0 + s2_;
  b.t[4 * I + 1] = s1 + s3;
  b.t[4 * I + 2] = s0 - s2_;
  b.t[4 * I + 3] = s1 - s3;
}

// max(|a|, |b|) of two column-stage values sharing the bias `beta` (both halves):
// max(max(a', b'), 2 beta - min(a', b')) - beta, unsigned compares on the biased values.
template <uint32_t BETA>
__device__ __forceinline__ uint32_t fold_pair(uint32_t a, uint32_t b) {
  static_assert(2 * BETA < 65536, "bias");
  const u2 mx = __builtin_elementwise_max(as_u2(a), as_u2(b)), mn = __builtin_elementwise_min(as_u2(a), as_u2(b));
  const uint32_t ng = splat32(2 * BETA) - as_u32(mn);
  return as_u32(__builtin_elementwise_max(mx, as_u2(ng))) - splat32(BETA);
}

// SAD and SATD of the block for both modes (packed 16-bit).
// d = orig - pred in [-1023, 1023].  Hadamard intermediates: rows <= 4092, column sums
// <= 8184, DC <= 16368.  SATD per block (kernel_aux_functions.cl:142-249):
//   (sum_k |c_k| - |c_0| + (|c_0| >> 2) + 1) >> 1.
// The last butterfly is folded with |a+b| + |a-b| = 2 max(|a|, |b|), so with T = sum of
// the seven non-DC pair maxima and U = |AC0| + (|DC| >> 2):  satd = T + ((U + 1) >> 1),
// where |AC0| = 2 max(|u0|, |u2|) - |DC| for the column-0 pair (DC = u0 + u2, AC0 = u0 - u2).
// By Parseval (||c||_2 = 4 ||d||_2) satd <= 32736 and T <= satd, so u16 holds both.
// SAD = sum |d| = 2 * sum max(d, 0) - DC <= 16368, exact in 16 bits for the same reason.
// Sums of non-negative packed halves that stay below 2^16 are plain 32-bit adds.
__device__ __forceinline__ void block_finish(const BlockAcc &b, u2 &sad, u2 &satd) {
  uint32_t T = 0, m0 = 0;
  s2 dc = splat(0);
  static_for<4>([&](auto c_c) {
    constexpr int c = decltype(c_c)::value;
    const uint32_t u0 = b.t[c] + b.t[4 + c], u1 = b.t[c] - b.t[4 + c];
    const uint32_t u2_ = b.t[8 + c] + b.t[12 + c], u3 = b.t[8 + c] - b.t[12 + c];
    T += fold_pair<kBiasQ>(u1, u3);
    if constexpr (c == 0) {
      m0 = fold_pair<kBiasP[0]>(u0, u2_);
      dc = as_s2(u0) - as_s2(splat32(2 * kBiasP[0]) - u2_);  // u0 + u2 - 2 bias, signed
    } else {
      T += fold_pair<kBiasP[c]>(u0, u2_);
    }
  });
  const s2 adc = smax(dc, splat(0) - dc);
  const uint32_t U = m0 + m0 - as_u32(adc) + as_u32(as_u2(adc) >> (u2){2, 2});
  satd = as_u2(T + as_u32(as_u2(U + 0x00010001u) >> (u2){1, 1}));
  sad = as_u2(as_s2(b.pos + b.pos) - dc);
}

// ---- paired blocks ---------------------------------------------------------------------
// Classes whose lanes walk an even number of 4x4 blocks per mode pair (H >= 8) process two
// blocks of the strip at once -- A = rows r..r+3, B = rows r+4..r+7 -- and, per mode, keep the
// two blocks in the two 16-bit halves of a register (the unpaired path keeps the two modes
// there).  Sums over the two halves then belong to one mode, so the absolute values of the
// SATD coefficients and of the SAD residuals are single v_sad_u16 instructions accumulating
// straight into 32-bit per-mode sums:
//   |x - y| = sad(x', y') for two values sharing a bias, |x + y| = sad(x', 2b - y'),
// replacing the unpaired path's max/min folds, packed positive-part sums and unpacking dot2s.
// The residual rows are computed as before (both modes packed) and transposed once per row
// (two v_perm_b32 per column).  The per-block SATD rounding (kernel_aux_functions.cl:238-246)
//   satd_b = (S_b + (|c0| >> 2) + 1) >> 1,  S_b = sum of the 15 non-DC |c_k|,
// is exact on the pair's sum because S_b and |c0| have the same parity (the 16 coefficients
// sum to 16 d_0, so sum |c_k| is even): satd_b = (S_b + D_b) / 2 with
// D_b = (|c0| >> 2) + ((|c0| + (|c0| >> 2)) & 1), and the lane accumulates S_b + D_b (even)
// over its blocks; the CU's SATD is that sum / 2.
struct PairAcc {
  uint32_t sad0 = 0, sad1 = 0;  // per-mode SAD
  uint32_t t0 = 0, t1 = 0;      // per-mode 2 * SATD
};

// Biased residual row I of one block, both modes packed (as block_row).
template <int I>
__device__ __forceinline__ void residual_row(const s2 (&prow)[4], uint2 orow, uint32_t (&d)[4]) {
  const s2 o01 = as_s2(orow.x), o23 = as_s2(orow.y);
  d[0] = as_u32(s2{o01.x, o01.x} - prow[0]);
  d[1] = as_u32(s2{o01.y, o01.y} - prow[1]);
  d[2] = as_u32(s2{o23.x, o23.x} - prow[2]);
  d[3] = as_u32(s2{o23.y, o23.y} - prow[3]);
}

// Row I of block B: transpose with block A's row I into per-mode (A, B) registers, SAD, row
// butterflies (carry-free 32-bit adds on the biased values, as block_row).
template <int I>
__device__ __forceinline__ void pair_row(const uint32_t *dA, const uint32_t (&dB)[4], uint32_t (&t0)[16],
                                         uint32_t (&t1)[16], PairAcc &acc) {
  constexpr const uint32_t *B = kBiasD[I & 1];
  uint32_t m0[4], m1[4];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    m0[c] = __builtin_amdgcn_perm(dB[c], dA[c], 0x05040100u);  // (A.mode0, B.mode0)
    m1[c] = __builtin_amdgcn_perm(dB[c], dA[c], 0x07060302u);  // (A.mode1, B.mode1)
    acc.sad0 = __builtin_amdgcn_sad_u16(m0[c], splat32(B[c]), acc.sad0);  // |d| = |d' - bias|
    acc.sad1 = __builtin_amdgcn_sad_u16(m1[c], splat32(B[c]), acc.sad1);
  }
  auto rowbf = [&](const uint32_t (&m)[4], uint32_t (&t)[16]) {
    const uint32_t s0 = m[0] + m[1], s1 = m[0] - m[1], s2_ = m[2] + m[3], s3 = m[2] - m[3];
    t[4 * I + 0] = s0 + s2_;
    t[4 * I + 1] = s1 + s3;
    t[4 * I + 2] = s0 - s2_;
    t[4 * I + 3] = s1 - s3;
  };
  rowbf(m0, t0);
  rowbf(m1, t1);
}

// Column butterflies and magnitudes of one mode's block pair (halves = blocks A, B):
// T += sum over both blocks of S_b + D_b (see above).  Column stage values u0/u2 of column c
// carry kBiasP[c], u1/u3 kBiasQ (block_finish); 2 * bias - u' = bias - u stays in [0, 65536).
__device__ __forceinline__ uint32_t pair_finish(const uint32_t (&t)[16], uint32_t T) {
  static_for<4>([&](auto c_c) {
    constexpr int c = decltype(c_c)::value;
    const uint32_t u0 = t[c] + t[4 + c], u1 = t[c] - t[4 + c];
    const uint32_t u2_ = t[8 + c] + t[12 + c], u3 = t[8 + c] - t[12 + c];
    const uint32_t n2 = splat32(2 * kBiasP[c]) - u2_, n3 = splat32(2 * kBiasQ) - u3;
    T = __builtin_amdgcn_sad_u16(u0, u2_, T);  // |u0 - u2|
    T = __builtin_amdgcn_sad_u16(u1, u3, T);   // |u1 - u3|
    T = __builtin_amdgcn_sad_u16(u1, n3, T);   // |u1 + u3|
    if constexpr (c > 0) {
      T = __builtin_amdgcn_sad_u16(u0, n2, T);  // |u0 + u2|
    } else {
      // DC c0 = u0 + u2: |c0| per block = max(u0', n2) - min(u0', n2), then D_b
      const u2 mx = __builtin_elementwise_max(as_u2(u0), as_u2(n2)), mn = __builtin_elementwise_min(as_u2(u0), as_u2(n2));
      const uint32_t a = as_u32(mx) - as_u32(mn);
      const uint32_t q = as_u32(as_u2(a) >> (u2){2, 2});
      const uint32_t d = q + ((a + q) & 0x00010001u);
      T = __builtin_amdgcn_sad_u16(d, 0u, T);  // both halves
    }
  });
  return T;
}

// Packed block results -> 32-bit per-mode accumulators.
struct Acc {
  uint32_t sad0 = 0, sad1 = 0, satd0 = 0, satd1 = 0;
#if MIP_ACC_PAIR
  // blocks are added in pairs: two blocks' packed sums still fit 16 bits per mode
  // (SAD <= 32736, SATD <= 65472), so a pair costs two adds + the four unpacking dot2
  u2 ps{0, 0}, pt{0, 0};
  bool have = false;
  __device__ __forceinline__ void unpack(u2 sad, u2 satd) {
    sad0 = __builtin_amdgcn_udot2(sad, (u2){1, 0}, sad0, false);
    sad1 = __builtin_amdgcn_udot2(sad, (u2){0, 1}, sad1, false);
    satd0 = __builtin_amdgcn_udot2(satd, (u2){1, 0}, satd0, false);
    satd1 = __builtin_amdgcn_udot2(satd, (u2){0, 1}, satd1, false);
  }
  __device__ __forceinline__ void add(u2 sad, u2 satd) {
    if (have) unpack(as_u2(as_u32(ps) + as_u32(sad)), as_u2(as_u32(pt) + as_u32(satd)));
    else ps = sad, pt = satd;
    have = !have;
  }
  __device__ __forceinline__ void flush() {
    if (have) unpack(ps, pt);
    have = false;
  }
#else
  __device__ __forceinline__ void add(u2 sad, u2 satd) {
    sad0 = __builtin_amdgcn_udot2(sad, (u2){1, 0}, sad0, false);
    sad1 = __builtin_amdgcn_udot2(sad, (u2){0, 1}, sad1, false);
    satd0 = __builtin_amdgcn_udot2(satd, (u2){1, 0}, satd0, false);
    satd1 = __builtin_amdgcn_udot2(satd, (u2){0, 1}, satd1, false);
  }
  __device__ __forceinline__ void flush() {}
#endif
};

// Both modes' sums in the two 16-bit halves of one register, for CUs of at most two 4x4
// blocks (4x4, 8x4, 4x8): per mode SAD <= 2 * 16368 and SATD <= 2 * 32736 < 2^16, so plain
// 32-bit adds (and the DPP group sums) never carry across the halves, and
// min(2 * SAD, SATD) is one packed shift and one packed min.
struct PackedAcc {
  uint32_t sad = 0, satd = 0;
  __device__ __forceinline__ void add(u2 s, u2 t) {
    sad += as_u32(s);
    satd += as_u32(t);
  }
};

// ---- transposed classes (TR) ----------------------------------------------------------------
// A wide CU W x H is searched as its transpose H x W (run_task): the transposed view's 4x4 block
// row I is the tile's block column I, so the original samples arrive one per register (OrigT)
// and carry the staged bias of the TILE position, kBiasD[c & 1][I] at view position (I, c).
// The block transform is the same 2-D Hadamard with the two butterfly stages swapped: the
// residual rows are kept raw and the butterflies of the tile's rows (view columns) run first
// (block_finish / pair_finish for BlockAccTr), which reproduces exactly the biased values the
// untransposed path builds, so the folds and the SATD rounding are unchanged.  SAD and SATD
// of a block are invariant under transposition.
struct OrigT {
  uint32_t v[4];  // view row: columns x..x+3 = tile rows, one staged (biased) sample each
};

struct BlockAccTr {
  uint32_t t[16];  // raw biased residuals, view position (I, c) at 4 * I + c
  uint32_t pos;
};

template <int I>
__device__ __forceinline__ void residual_row(const s2 (&prow)[4], const OrigT &o, uint32_t (&d)[4]) {
#pragma unroll
  for (int c = 0; c < 4; c++) d[c] = as_u32(s2{(short)o.v[c], (short)o.v[c]} - prow[c]);
}

template <int I>
__device__ __forceinline__ void block_row(BlockAccTr &b, const s2 (&prow)[4], const OrigT &o) {
  uint32_t d[4];
  residual_row<I>(prow, o, d);
  uint32_t p = 0;
  static_for<4>([&](auto c_c) {
    constexpr int c = decltype(c_c)::value;
    constexpr unsigned short B = (unsigned short)kBiasD[c & 1][I];
    p += as_u32(__builtin_elementwise_sub_sat(as_u2(d[c]), (u2){B, B}));
    b.t[4 * I + c] = d[c];
  });
  b.pos = I == 0 ? p : b.pos + p;
}

// The tile-row butterflies (view columns) of raw residuals -> the row-transformed layout of
// block_row (tile row r at 4 * r + k).
__device__ __forceinline__ void rows_transform_tr(const uint32_t (&raw)[16], uint32_t (&t)[16]) {
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const uint32_t e0 = raw[r], e1 = raw[4 + r], e2 = raw[8 + r], e3 = raw[12 + r];
    const uint32_t s0 = e0 + e1, s1 = e0 - e1, s2_ = e2 + e3, s3 = e2 - e3;
    t[4 * r + 0] = s0 + s2_;
    t[4 * r + 1] = s1 + s3;
    t[4 * r + 2] = s0 - s2_;
    t[4 * r + 3] = s1 - s3;
  }
}

__device__ __forceinline__ void block_finish(const BlockAccTr &b, u2 &sad, u2 &satd) {
  BlockAcc r;
  rows_transform_tr(b.t, r.t);
  r.pos = b.pos;
  block_finish(r, sad, satd);
}

// Paired walk, TR: as pair_row with the tile-position biases; rows kept raw.
template <int I>
__device__ __forceinline__ void pair_row_tr(const uint32_t *dA, const uint32_t (&dB)[4], uint32_t (&t0)[16],
                                            uint32_t (&t1)[16], PairAcc &acc) {
  static_for<4>([&](auto c_c) {
    constexpr int c = decltype(c_c)::value;
    const uint32_t m0 = __builtin_amdgcn_perm(dB[c], dA[c], 0x05040100u);  // (A.mode0, B.mode0)
    const uint32_t m1 = __builtin_amdgcn_perm(dB[c], dA[c], 0x07060302u);  // (A.mode1, B.mode1)
    acc.sad0 = __builtin_amdgcn_sad_u16(m0, splat32(kBiasD[c & 1][I]), acc.sad0);
    acc.sad1 = __builtin_amdgcn_sad_u16(m1, splat32(kBiasD[c & 1][I]), acc.sad1);
    t0[4 * I + c] = m0;
    t1[4 * I + c] = m1;
  });
}

__device__ __forceinline__ uint32_t pair_finish_tr(const uint32_t (&raw)[16], uint32_t T) {
  uint32_t t[16];
  rows_transform_tr(raw, t);
  return pair_finish(t, T);
}

// Reduced prediction of the lane's CU in the wave scratch: both modes of the pair per dword,
// stored position (k, kx) at k*R + kx (rows offset by `k0` for the second half of a chunked
// class).
template <int R, int RP = R>
struct Red {
  static constexpr int OFF = RP > R ? 1 : 0;  // padded rows: the left sample at kx = -1
  const uint32_t *p;
  int k0;
  // phase A stores floor(D) saturated at 0 only; the clip to 1023 is applied here, to
  // both modes of a pair at once
  static __device__ __forceinline__ s2 clip(uint32_t v) {
    return __builtin_bit_cast(s2, __builtin_elementwise_min(__builtin_bit_cast(u2, v), (u2){1023, 1023}));
  }
  __device__ __forceinline__ s2 operator()(int k, int kx) const { return clip(p[(k + k0) * RP + kx + OFF]); }
  __device__ __forceinline__ void row4(int k, int kx, s2 (&out)[4]) const {  // kx % 4 == 0
    static_assert(RP == R, "row4 reads unpadded rows");
    const uint4 v = *reinterpret_cast<const uint4 *>(p + (k + k0) * R + kx);
    out[0] = clip(v.x);
    out[1] = clip(v.y);
    out[2] = clip(v.z);
    out[3] = clip(v.w);
  }
};

// Horizontal pass of anchor row k (CU row k*UV + UV-1) at strip columns x0..x0+3,
// intra.cl:816-843; the first UH columns interpolate from the left boundary sample, which
// the padded scratch row holds at kx = -1.
// ((UH-o)*before + o*after + UH/2) >> LH == (base + o*delta) >> LH with
// base = (before << LH) + UH/2; the sum equals the reference numerator, in [0, 8188].
template <int W, int H, class RED>
__device__ __forceinline__ void anchor_row(const RED &red, int k, int x0, s2 (&a)[4]) {
  using G = Geo<W, H>;
  if constexpr (G::UH == 1) {
    red.row4(k, x0, a);
  } else if constexpr (G::UH == 2) {
    const int kx = x0 >> 1;  // covers kx, kx+1
    const s2 r0 = red(k, kx), r1 = red(k, kx + 1);
    const s2 before = red(k, kx - 1);
    a[0] = avg_round(before, r0);
    a[1] = r0;
    a[2] = avg_round(r0, r1);
    a[3] = r1;
  } else {
    const int kx = x0 >> G::LH;
    const s2 after = red(k, kx);
    const s2 before = red(k, kx - 1);
    // Numerators n_o = base + o*delta walked incrementally: `delta` is the exact 32-bit
    // difference of the packed pairs (after - before), so n += delta is one v_add_u32 that
    // is exact on both halves (every n_o per half lies in [0, 8188]: no carry or borrow
    // leaves the low half of the true sum).  v_add_u32 dual-issues on gfx950, the
    // v_pk_mad_u16 it replaces does not (tools/dual_census.hip).
    const uint32_t delta = as_u32(after) - as_u32(before);
    const u2 base = pk_mad_cc<G::UH, G::UH / 2>(as_u2(before));
    // the strip's 4 columns are phases o0+1..o0+4 of one window (o0 = 0 or 4 for UH = 8:
    // it differs between neighbouring lanes, so it enters as data, base += o0 * delta,
    // not as a branch)
    uint32_t n = as_u32(base);
    if constexpr (G::UH == 8) {
      // per-half differences for the packed multiply (the 32-bit difference carries the
      // low half's borrow in its high half)
      const u2 hdelta = as_u2(after - before);
      const uint32_t o0 = splat32(x0 & (G::UH - 1));
      u2 base0;
      asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(base0) : "v"(hdelta), "v"(o0), "v"(base));
      n = as_u32(base0);
    }
    static_for<4>([&](auto oc) {  // (o*delta + base) >> LH, o = oc + 1 + o0
      constexpr int c = decltype(oc)::value;
      if constexpr (G::UH == 4 && c == 3) {
        a[c] = after;  // o = UH: the anchor itself
      } else {
        n += delta;
        a[c] = as_s2(as_u2(n) >> (u2){G::LH, G::LH});
      }
    });
  }
}

// Original samples of a lane's strip (rows [y0, y0 + N)): kept in VGPRs across the mode
// pairs for 4-row CUs, re-read from LDS otherwise (register budget).
template <int H>
struct OrigRows {
  static constexpr bool TR = false;
  using Block = BlockAcc;
  static constexpr bool CACHED = H <= 4;
  uint2 r[CACHED ? H : 1];
  const uint16_t *row0;  // the strip's first sample (row y, column x)
  __device__ __forceinline__ void load(const uint16_t *t, int xx, int yy) {
    row0 = t + tidx(xx, yy);
    if constexpr (CACHED) {
#pragma unroll
      for (int i = 0; i < H; i++) r[i] = lds_row4(t, xx, yy + i);
    }
  }
  // Row i as a constant stride from row0: a runtime block-pair base (walk_pairs' yb) plus a
  // constant row becomes one address per block pair and immediate offsets (through tidx the
  // compiler emitted an add and a v_mad_u32_u24 per row read).
  __device__ __forceinline__ uint2 operator()(int i) const {
    if constexpr (CACHED) return r[i];
    else return *reinterpret_cast<const uint2 *>(row0 + i * kPitch);
  }
};

// Original samples of a TR lane's strip: view row i = tile column, re-read per mode pair.
template <int H>
struct OrigRowsT {
  static constexpr bool TR = true;
  using Block = BlockAccTr;
  const uint16_t *tile;
  int x, y;  // view coordinates of the strip's first sample
  __device__ __forceinline__ void load(const uint16_t *t, int xx, int yy) {
    tile = t;
    x = xx;
    y = yy;
  }
  __device__ __forceinline__ OrigT operator()(int i) const {
    OrigT o;
#pragma unroll
    for (int k = 0; k < 4; k++) o.v[k] = tile[tidx(y + i, x + k)];
    return o;
  }
};

// Walk one strip of one CU for one mode pair over upsampling windows [k0, k1) (rows for
// UV == 1 and 4x4): prediction rows (upsampling, intra.cl:815-912) streamed through the
// block transform.  `prev` is the anchor row above window k0 (vertical pass state).
template <int W, int H, int V, class ORIG, class RED, class ACC>
__device__ __forceinline__ void walk_strip(const ORIG &orig, const RED &red, int x0, int k0, int k1, s2 (&prev)[4],
                                           ACC &acc) {
  using G = Geo<W, H, V>;
  if constexpr (G::SID == 0) {
    // 4x4 CU: the reduced prediction is the prediction (intra.cl:934-936, 995).
    typename ORIG::Block b;
    static_for<4>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      s2 prow[4];
      red.row4(i, 0, prow);
      block_row<i>(b, prow, orig(i));
    });
    u2 sad, satd;
    block_finish(b, sad, satd);
    acc.add(sad, satd);
  } else if constexpr (G::UV == 1) {
    // every row is an anchor row (horizontal pass only); [k0, k1) are rows
    (void)k1;
#pragma unroll
    for (int bi = 0; bi < G::KV / 4; bi++) {
      const int by = k0 / 4 + bi;
      typename ORIG::Block b;
      static_for<4>([&](auto i_c) {
        constexpr int i = decltype(i_c)::value;
        s2 prow[4];
        anchor_row<W, H>(red, 4 * by + i, x0, prow);
        block_row<i>(b, prow, orig(4 * by + i));
      });
      u2 sad, satd;
      block_finish(b, sad, satd);
      acc.add(sad, satd);
    }
  } else if constexpr (G::UV == 2) {
    // Vertical pass (intra.cl:867-893) with two windows per 4x4 block: the row between
    // anchors k-1 and k is (prev + next + 1) >> 1.
    constexpr int kUnroll = H <= 8 ? 2 : MIP_UV2_UNROLL;
    constexpr int NBLK = (G::CHUNKED ? 4 : G::KV) / 2;  // blocks in [k0, k1)
    (void)k1;
#pragma unroll kUnroll
    for (int bi = 0; bi < NBLK; bi++) {
      const int by = k0 / 2 + bi;
      typename ORIG::Block b;
      static_for<2>([&](auto hh_c) {
        constexpr int hh = decltype(hh_c)::value;
        const int k = 2 * by + hh;
        s2 next[4], mid[4];
        anchor_row<W, H>(red, k, x0, next);
#pragma unroll
        for (int cc = 0; cc < 4; cc++) mid[cc] = avg_round(prev[cc], next[cc]);
        block_row<2 * hh>(b, mid, orig(2 * k));
        block_row<2 * hh + 1>(b, next, orig(2 * k + 1));
#pragma unroll
        for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
      });
      u2 sad, satd;
      block_finish(b, sad, satd);
      acc.add(sad, satd);
    }
  } else {
    // Vertical pass: row o (1..UV) of window k is n_o >> LV with n_o = base + o*delta,
    // base = (prev << LV) + UV/2: the reference numerator, in [0, 8188] on both halves.  It
    // is walked incrementally, n_o = n_{o-1} + delta, with delta the exact 32-bit
    // difference of the packed pairs (see anchor_row); o = UV gives the anchor itself.
    constexpr int NB = G::UV / 4;  // blocks per window
    constexpr int NW = G::CHUNKED ? 4 : G::KV;  // windows in [k0, k1)
    (void)k1;
#pragma unroll MIP_WIN_UNROLL
    for (int kk = 0; kk < NW; kk++) {
      const int k = k0 + kk;
      s2 next[4];
      anchor_row<W, H>(red, k, x0, next);
      uint32_t delta[4], num[4];
#pragma unroll
      for (int cc = 0; cc < 4; cc++) {
        delta[cc] = as_u32(next[cc]) - as_u32(prev[cc]);
        num[cc] = as_u32(pk_mad_cc<G::UV, G::UV / 2>(as_u2(prev[cc])));
      }
      static_for<NB>([&](auto bi_c) {
        constexpr int bi = decltype(bi_c)::value;
        typename ORIG::Block b;
        static_for<4>([&](auto i_c) {
          constexpr int i = decltype(i_c)::value, o = 4 * bi + i + 1;
          s2 prow[4];
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            if constexpr (o == G::UV) {
              prow[cc] = next[cc];
            } else {
              num[cc] += delta[cc];
              prow[cc] = as_s2(as_u2(num[cc]) >> (u2){G::LV, G::LV});
            }
          }
          block_row<i>(b, prow, orig(k * G::UV + 4 * bi + i));
        });
        u2 sad, satd;
        block_finish(b, sad, satd);
        acc.add(sad, satd);
      });
#pragma unroll
      for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
    }
  }
}

// Paired walk (see PairAcc): the lane's blocks in [k0, k0 + windows) two at a time, rows
// generated exactly as in walk_strip; block A's residual rows wait for block B's.
#ifndef MIP_PAIR_MIN_AREA
#define MIP_PAIR_MIN_AREA 32  // smallest CU area walked in block pairs (A/B knob; 33: 4x8 unpaired, -0.6 %)
#endif
template <int W, int H, int V>
constexpr bool kPaired = Geo<W, H, V>::SID != 0 && W * H >= MIP_PAIR_MIN_AREA && V == kClassV[size_class(W, H)] &&
                         ((Geo<W, H, V>::CHUNKED && !kSpanChunks ? Geo<W, H, V>::CROWS * Geo<W, H, V>::UV
                                                                 : Geo<W, H, V>::KV * Geo<W, H, V>::UV) / 4) % 2 == 0;

template <int W, int H, int V, class ORIG, class RED>
__device__ __forceinline__ void walk_pairs(const ORIG &orig, const RED &red, int x0, int k0, s2 (&prev)[4],
                                           PairAcc &acc) {
  using G = Geo<W, H, V>;
  constexpr int ROWS = G::CHUNKED ? 4 * G::UV : G::KV * G::UV;  // CU rows of this call
  constexpr int NBP = ROWS / 8;                                   // block pairs
  const int y0 = k0 * G::UV;                                      // first CU row
  // per block pair: 4 rows of A -> dA, 4 rows of B -> pair_row.  (Unrolling two block pairs,
  // which drops the loop-carried copies of the top boundary and the zeroed accumulators --
  // 8 v_mov per pair -- measured flat: 7544 -> 7532 frames/s, and spills in the ALT kernels.)
#pragma unroll 1
  for (int bp = 0; bp < NBP; bp++) {
    uint32_t dA[16], t0[16], t1[16];
    const int yb = y0 + 8 * bp;  // CU row of A's first row
    // emit(i, prow): CU row yb + i (i = 0..7)
    auto emit = [&](auto i_c, const s2 (&prow)[4]) {
      constexpr int i = decltype(i_c)::value;
      if constexpr (i < 4) {
        uint32_t d[4];
        residual_row<i>(prow, orig(yb + i), d);
#pragma unroll
        for (int c = 0; c < 4; c++) dA[4 * i + c] = d[c];
      } else {
        uint32_t dB[4];
        residual_row<i - 4>(prow, orig(yb + i), dB);
        if constexpr (ORIG::TR) pair_row_tr<i - 4>(dA + 4 * (i - 4), dB, t0, t1, acc);
        else pair_row<i - 4>(dA + 4 * (i - 4), dB, t0, t1, acc);
      }
    };
    if constexpr (G::UV == 1) {
      static_for<8>([&](auto i_c) {
        s2 prow[4];
        anchor_row<W, H>(red, yb + decltype(i_c)::value, x0, prow);
        emit(i_c, prow);
      });
    } else if constexpr (G::UV == 2) {
      const int kb = yb / 2;  // windows kb..kb+3
      static_for<4>([&](auto w_c) {
        constexpr int w = decltype(w_c)::value;
        s2 next[4], mid[4];
        anchor_row<W, H>(red, kb + w, x0, next);
#pragma unroll
        for (int cc = 0; cc < 4; cc++) mid[cc] = avg_round(prev[cc], next[cc]);
        emit(std::integral_constant<int, 2 * w>{}, mid);
        emit(std::integral_constant<int, 2 * w + 1>{}, next);
#pragma unroll
        for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
      });
    } else {
      // UV = 4: windows yb/4, yb/4 + 1; UV = 8: rows o = 1..8 of window yb/8
      constexpr int NWIN = G::UV == 4 ? 2 : 1;
      static_for<NWIN>([&](auto w_c) {
        constexpr int w = decltype(w_c)::value;
        const int k = yb / G::UV + w;
        s2 next[4];
        anchor_row<W, H>(red, k, x0, next);
        uint32_t delta[4], num[4];
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
          delta[cc] = as_u32(next[cc]) - as_u32(prev[cc]);
          num[cc] = as_u32(pk_mad_cc<G::UV, G::UV / 2>(as_u2(prev[cc])));
        }
        static_for<G::UV>([&](auto r_c) {
          constexpr int r = decltype(r_c)::value, o = r + 1;
          s2 prow[4];
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            if constexpr (o == G::UV) {
              prow[cc] = next[cc];
            } else {
              num[cc] += delta[cc];
              prow[cc] = as_s2(as_u2(num[cc]) >> (u2){G::LV, G::LV});
            }
          }
          emit(std::integral_constant<int, w * G::UV + r>{}, prow);
        });
#pragma unroll
        for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
      });
    }
    if constexpr (ORIG::TR) {
      acc.t0 = pair_finish_tr(t0, acc.t0);
      acc.t1 = pair_finish_tr(t1, acc.t1);
    } else {
      acc.t0 = pair_finish(t0, acc.t0);
      acc.t1 = pair_finish(t1, acc.t1);
    }
  }
}

// MIP_SIX_WAVES 3 (kSpanChunks): walks whose chunks of reduced rows end inside a block or a
// block pair.  sw(c) runs phase A of chunk c (wave-synchronised on both sides); the partial
// block / block A's residuals and the vertical-pass state stay in registers across it.
// 4x4: rows 0, 1 from chunk 0, rows 2, 3 from chunk 1.
template <int W, int H, int V, class ORIG, class RED, class SW, class ACC>
__device__ __forceinline__ void walk_4x4_chunked(const ORIG &orig, RED red, SW &sw, ACC &acc) {
  static_assert(Geo<W, H, V>::SID == 0 && Geo<W, H, V>::CROWS == 2, "4x4 chunks");
  typename ORIG::Block b;
  static_for<4>([&](auto i_c) {
    constexpr int i = decltype(i_c)::value;
    if constexpr (i == 2) {
      sw(1);
      red.k0 = -2;
    }
    s2 prow[4];
    red.row4(i, 0, prow);
    block_row<i>(b, prow, orig(i));
  });
  u2 sad, satd;
  block_finish(b, sad, satd);
  acc.add(sad, satd);
}

// Paired walk over all of the lane's rows (V = 1) with a chunk switch before every anchor row
// k that starts a chunk (k % CROWS == 0, k > 0); otherwise as walk_pairs.
template <int W, int H, int V, class ORIG, class RED, class SW>
__device__ __forceinline__ void walk_pairs_chunked(const ORIG &orig, RED red, int x0, s2 (&prev)[4], PairAcc &acc,
                                                   SW &sw) {
  using G = Geo<W, H, V>;
  static_assert(G::CHUNKED && V == 1, "chunked pairs");
  constexpr int NBP = G::KV * G::UV / 8;  // block pairs
  auto at = [&](int k) {                  // k: wave-uniform
    if (k > 0 && k % G::CROWS == 0) {
      sw(k / G::CROWS);
      red.k0 = -k;
    }
  };
#pragma unroll 1
  for (int bp = 0; bp < NBP; bp++) {
    uint32_t dA[16], t0[16], t1[16];
    const int yb = 8 * bp;  // CU row of A's first row
    auto emit = [&](auto i_c, const s2 (&prow)[4]) {
      constexpr int i = decltype(i_c)::value;
      if constexpr (i < 4) {
        uint32_t d[4];
        residual_row<i>(prow, orig(yb + i), d);
#pragma unroll
        for (int c = 0; c < 4; c++) dA[4 * i + c] = d[c];
      } else {
        uint32_t dB[4];
        residual_row<i - 4>(prow, orig(yb + i), dB);
        if constexpr (ORIG::TR) pair_row_tr<i - 4>(dA + 4 * (i - 4), dB, t0, t1, acc);
        else pair_row<i - 4>(dA + 4 * (i - 4), dB, t0, t1, acc);
      }
    };
    if constexpr (G::UV == 1) {
      static_for<8>([&](auto i_c) {
        s2 prow[4];
        at(yb + decltype(i_c)::value);
        anchor_row<W, H>(red, yb + decltype(i_c)::value, x0, prow);
        emit(i_c, prow);
      });
    } else if constexpr (G::UV == 2) {
      const int kb = yb / 2;  // windows kb..kb+3
      static_for<4>([&](auto w_c) {
        constexpr int w = decltype(w_c)::value;
        s2 next[4], mid[4];
        at(kb + w);
        anchor_row<W, H>(red, kb + w, x0, next);
#pragma unroll
        for (int cc = 0; cc < 4; cc++) mid[cc] = avg_round(prev[cc], next[cc]);
        emit(std::integral_constant<int, 2 * w>{}, mid);
        emit(std::integral_constant<int, 2 * w + 1>{}, next);
#pragma unroll
        for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
      });
    } else {
      constexpr int NWIN = G::UV == 4 ? 2 : 1;
      static_for<NWIN>([&](auto w_c) {
        constexpr int w = decltype(w_c)::value;
        const int k = yb / G::UV + w;
        s2 next[4];
        at(k);
        anchor_row<W, H>(red, k, x0, next);
        uint32_t delta[4], num[4];
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
          delta[cc] = as_u32(next[cc]) - as_u32(prev[cc]);
          num[cc] = as_u32(pk_mad_cc<G::UV, G::UV / 2>(as_u2(prev[cc])));
        }
        static_for<G::UV>([&](auto r_c) {
          constexpr int r = decltype(r_c)::value, o = r + 1;
          s2 prow[4];
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            if constexpr (o == G::UV) {
              prow[cc] = next[cc];
            } else {
              num[cc] += delta[cc];
              prow[cc] = as_s2(as_u2(num[cc]) >> (u2){G::LV, G::LV});
            }
          }
          emit(std::integral_constant<int, w * G::UV + r>{}, prow);
        });
#pragma unroll
        for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
      });
    }
    if constexpr (ORIG::TR) {
      acc.t0 = pair_finish_tr(t0, acc.t0);
      acc.t1 = pair_finish_tr(t1, acc.t1);
    } else {
      acc.t0 = pair_finish(t0, acc.t0);
      acc.t1 = pair_finish(t1, acc.t1);
    }
  }
}

struct Ctx {
  const SearchArgs *a;
  const uint16_t *org;        // quadrant tile of original samples
  const uint16_t *ref;        // reference samples: == org (full tile) or the ALT lattice
  const uint8_t *w;           // MIP coefficients (LDS): f16 rows, then f32 accumulator rows
  const uint8_t *zero;        // zero-filled LDS (masked MFMA inputs)
  uint8_t *wave;              // wave-private LDS: CU table + scratch
  int ctu, frame;
  int fx0, fy0;               // quadrant origin in the frame
};

// floor(f) for f >= 0, 0 for f < 0: v_cvt_u32_f32 saturates out-of-range inputs.
__device__ __forceinline__ uint32_t floor_sat(float f) { return (uint32_t)f; }

// Phase A for mode pair q: reduced predictions of every CU of the task,
//   D[j][n] = C[j] + sum_k A[j][k] B[k][n]     (16x16x16 f16 MFMA, f32 accumulate, exact)
// rows j = MIP matrix outputs, columns n = (CU 8*cs + n/2, mode 2q + n%2), K = the 8 inputs
// of mode 2q (k < 8) and of mode 2q+1 (k >= 8), block-diagonal.  floor(D) clipped to
// [0, 1023] equals the reference's clamp(((offset + sum p*w) >> 6) + b0) (intra.cl:449-482;
// coefficient restatement in mip_kernels.h); phase A stores floor(D) saturated at 0 (D is
// the unclipped sample, |D| <= 8 * 1023 * 127 / 64 + 1023 < 2^16) and Red applies the upper
// clip to packed pairs on read.  Results go to scratch[pos][slot] (16-bit
// halves = modes), pos = stored position (transposed modes store output j at (j%R, j/R),
// intra.cl:402-406, 485).  CHUNKED classes produce reduced rows [4*chunk, 4*chunk + 4).
template <int W, int H, int V, bool TR>
__device__ __forceinline__ void phase_a(const Ctx &x, int lane, int ncu, int q, int chunk) {
  using G = Geo<W, H, V>;
  const int r = lane & 15, h = lane >> 4;
  const int m0 = TR ? 2 * q - G::MODES : 2 * q;
  // MIP_SIX_WAVES 3 chunks of two reduced rows: sizeId 0/1 (one 16-output block holds the
  // whole 4x4 prediction) compute it for each chunk and store that chunk's two rows (HALF);
  // transposed 8xH take the outputs of rows 2*chunk, 2*chunk + 1, all 8 columns (TR2:
  // matrix row r -> output 8 * (r >> 1) + (r & 1) + 2 * chunk, column r >> 1).
  constexpr bool HALF = G::CHUNKED && G::SID != 2;
  constexpr bool TR2 = TR && G::SID == 2 && G::CHUNKED && G::CROWS == 2;
  // A: coefficient row of mode m0 + (h >> 1), inputs 4*(h & 1)..+3
  const int jrow = TR2 ? 8 * (r >> 1) + (r & 1) : (G::SID == 2 && TR) ? 8 * (r >> 2) + (r & 3) : r;
  const uint8_t *abase = x.w + ((G::WBASE + (m0 + (h >> 1)) * G::NOUT + jrow) * 8 + 4 * (h & 1)) * 2;
  // B: column r = (slot 8*cs + r/2, mode r&1), nonzero only in the K half of its mode
  const bool bsel = (h >> 1) == (r & 1);
  const uint8_t *bbase = bsel ? x.wave + (r >> 1) * kEntryBytes + 8 * ((h & 1) ^ (TR ? 1 : 0)) : x.zero;
  // C: per output row (sizeId 1/0), a constant for sizeId 2 (mip_kernels.h)
  f4 cin;
  if constexpr (G::SID == 2) {
    cin = *reinterpret_cast<const f4 *>(reinterpret_cast<const float *>(x.w + kWeightRows * 16) + 384);
  } else {
    const float *ct = reinterpret_cast<const float *>(x.w + kWeightRows * 16) + (G::WBASE - kWeightRowOffS1);
    cin = *reinterpret_cast<const f4 *>(ct + (m0 + (r & 1)) * G::NOUT + 4 * h);
  }
  constexpr int NCS = (G::SLOTS + 7) / 8;  // column sets (8 CUs x 2 modes) of a full task
  // column sets holding CUs (scalar: the task's CU count is wave-uniform)
  const int ncs_run = __builtin_amdgcn_readfirstlane((ncu + 7) >> 3);
  constexpr int NRB = HALF ? 1 : G::CPOS / 16;  // 16-row blocks in this chunk
  // the lane's 4 results of block rb sit at stored positions pos0 + i * PSTEP
  // (padded rows: position (k, kx) at k*RP + kx + 1; outputs 4h..4h+3 share one row;
  // TR2: row i & 1, column 2h + (i >> 1) of the chunk)
  constexpr int PSTEP = TR ? G::RP : 1;
  const int pos0 = TR2 ? 2 * h : TR ? h + G::PAD : (G::PAD ? (4 * h / G::R) * G::RP + (4 * h) % G::R + 1 : 4 * h);
  uint8_t *lane_dst = x.wave + kCuTableBytes + ((r >> 1) * G::PITCH + pos0) * 4 + 2 * (r & 1);
#pragma unroll
  for (int rb = 0; rb < NRB; rb++) {
    int jofs, pofs;  // uniform: matrix row offset, stored-position offset of the block
    if constexpr (TR2) {
      jofs = 2 * chunk;
      pofs = 0;
    } else if constexpr (G::SID == 2) {
      const int rbg = G::CHUNKED ? NRB * chunk + rb : rb;  // 16-row block 0..3 of the matrix
      const int cofs = G::CHUNKED ? G::CPOS * chunk : 0;
      const int crow = G::CHUNKED ? G::CROWS * chunk * G::RP : 0;  // padded rows: the chunk's first row
      if constexpr (!TR) {
        jofs = 16 * rbg;
        pofs = G::PAD ? 2 * rbg * G::RP - crow : 16 * rbg - cofs;
      } else {  // output j = 8*(h + 4*rr) + i + 4*cc -> position (i + 4cc, h + 4rr)
        const int cc = rbg >> 1, rr = rbg & 1;
        jofs = 32 * rr + 4 * cc;
        pofs = G::PAD ? 4 * cc * G::RP + 4 * rr - crow : 32 * cc + 4 * rr - cofs;
      }
    } else {
      jofs = 0;
      pofs = HALF ? -8 * chunk : 0;  // rows 2 * chunk, 2 * chunk + 1 -> chunk rows 0, 1
    }
    const h4 av = *reinterpret_cast<const h4 *>(abase + jofs * 16);
    // classes with many column sets (one row block): all B operands read up front, so the
    // MFMAs do not each wait for an LDS read (partial tasks read unused CU-table entries)
    constexpr bool BATCH_B = NRB == 1 && NCS >= MIP_PHASEA_BATCH_NCS;
    h4 bvs[BATCH_B ? NCS : 1];
    if constexpr (BATCH_B) {
#pragma unroll
      for (int cs = 0; cs < NCS; cs++) bvs[cs] = *reinterpret_cast<const h4 *>(bbase + cs * 8 * kEntryBytes);
    }
#pragma unroll
    for (int cs = 0; cs < NCS; cs++) {
      if (cs > 0 && cs >= ncs_run) break;  // wave-uniform: partial last task
      const h4 bv = BATCH_B ? bvs[BATCH_B ? cs : 0] : *reinterpret_cast<const h4 *>(bbase + cs * 8 * kEntryBytes);
      const f4 d = __builtin_amdgcn_mfma_f32_16x16x16f16(av, bv, cin, 0, 0, 0);
      // columns of slots >= ncu hold garbage; they land in unused scratch columns unless
      // the class has fewer than 8 slots
      if ((G::SLOTS % 8 == 0 || 8 * cs + (r >> 1) < ncu) && (!HALF || TR || (h >> 1) == chunk)) {
        uint8_t *dst = lane_dst + (pofs + 8 * cs * G::PITCH) * 4;
        static_for<4>([&](auto i_c) {
          constexpr int i = decltype(i_c)::value;
          constexpr int off = TR2 ? (i & 1) * G::R + (i >> 1) : i * PSTEP;
          if (!(HALF && TR) || (i >> 1) == chunk) {
            const uint32_t v = floor_sat(d[i]);  // < 2^16; the upper clip is applied by Red
            *reinterpret_cast<uint16_t *>(dst + off * 4) = (uint16_t)v;
          }
        });
      }
    }
  }
}

// Phase A of one chunk (two reduced rows) of a 64-slot sizeId 0 / 1 task (MIP_SIX_WAVES 3:
// 4x4, 4x8).  Both modes of a pair read the same boundary vector (a pair is either untransposed
// or transposed), so the chunk's 8 outputs of both modes become the 16 matrix rows and the
// columns 16 CUs: 4 MFMAs per chunk, every result stored once (the block-diagonal layout of
// phase_a would compute all 16 outputs of 8 CUs per MFMA and keep half).  K: the 8 inputs in
// the first half, zeros in the second.
// Row r = (mode r & 1, chunk position p = ((r >> 1) >> 1) + 4 ((r >> 1) & 1)), so a lane's
// four results are both modes of positions h and h + 4 (h = lane >> 4) of CU lane & 15: the
// 16-bit stores of one instruction hit 64 distinct words of a 12-word pitch (the first
// version, rows = (mode, position), put two lanes on each word: 54 % LDS bank conflicts in the
// 4x4 class).  Chunk position p is row p >> 2 (2c + (p >> 2) of the prediction), column p & 3;
// untransposed it is output j = 8c + p, transposed (stored at (j % 4, j / 4)) output
// j = 4 (p & 3) + 2c + (p >> 2).
template <int W, int H, int V, bool TR>
__device__ __forceinline__ void phase_a_half(const Ctx &x, int lane, int q, int chunk) {
  using G = Geo<W, H, V>;
  static_assert(G::CHUNKED && G::SID != 2 && G::SLOTS == 64 && G::CROWS == 2 && !G::PAD && G::PITCH >= 8, "half chunks");
  const int r = lane & 15, h = lane >> 4;
  const int m0 = TR ? 2 * q - G::MODES : 2 * q;
  auto jout = [&](int p) { return TR ? 4 * (p & 3) + 2 * chunk + (p >> 2) : 8 * chunk + p; };
  auto pos_of_row = [](int row) { return ((row >> 1) >> 1) + 4 * ((row >> 1) & 1); };
  // A: row r, inputs 4h..4h+3 (h < 2); B: CU 16 cs + r, inputs 4h..4h+3 (h < 2)
  const uint8_t *aptr = h < 2 ? x.w + ((G::WBASE + (m0 + (r & 1)) * G::NOUT + jout(pos_of_row(r))) * 8 + 4 * h) * 2
                              : x.zero;
  const h4 av = *reinterpret_cast<const h4 *>(aptr);
  // (lanes h >= 2 read the same entries' other half: finite f16 values -- an entry holds
  // 1024 + b for every input -- times the zero A operand, so those K rows add exactly 0 to
  // the written CUs' columns; columns of slots >= ncu land in unused scratch rows)
  const uint8_t *bbase = x.wave + r * kEntryBytes + 8 * ((h & 1) ^ (TR ? 1 : 0));
  // C: rows 4h + i = (mode i & 1, position h + 4 (i >> 1))
  const float *ct = reinterpret_cast<const float *>(x.w + kWeightRows * 16) + (G::WBASE - kWeightRowOffS1);
  f4 cin;
  static_for<4>([&](auto i_c) {
    constexpr int i = decltype(i_c)::value;
    cin[i] = ct[(m0 + (i & 1)) * G::NOUT + jout(h + 4 * (i >> 1))];
  });
  h4 bvs[4];
#pragma unroll
  for (int cs = 0; cs < 4; cs++) bvs[cs] = *reinterpret_cast<const h4 *>(bbase + cs * 16 * kEntryBytes);
  uint8_t *lane_dst = x.wave + kCuTableBytes + (r * G::PITCH + h) * 4;
#pragma unroll
  for (int cs = 0; cs < 4; cs++) {
    const f4 d = __builtin_amdgcn_mfma_f32_16x16x16f16(av, bvs[cs], cin, 0, 0, 0);
    uint8_t *dst = lane_dst + 16 * cs * G::PITCH * 4;  // slots >= ncu: unused scratch rows
    static_for<4>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value;
      // (volatile LDS store: two 16-bit stores, not a v_perm-packed 32-bit one -- VALU is the bound)
      typedef __attribute__((address_space(3))) volatile uint16_t lds_u16;
      *(lds_u16 *)(dst + 16 * (i >> 1) + 2 * (i & 1)) = (uint16_t)floor_sat(d[i]);
    });
  }
}

template <int W, int H, int V>
__device__ __forceinline__ void phase_a(const Ctx &x, int lane, int ncu, int q, int chunk) {
  using G = Geo<W, H, V>;
  if constexpr (G::CHUNKED && G::SID != 2) {
    if (q >= G::MODES / 2) phase_a_half<W, H, V, true>(x, lane, q, chunk);
    else phase_a_half<W, H, V, false>(x, lane, q, chunk);
  } else {
    if (q >= Geo<W, H>::MODES / 2) phase_a<W, H, V, true>(x, lane, ncu, q, chunk);
    else phase_a<W, H, V, false>(x, lane, ncu, q, chunk);
  }
}

// Sum over aligned groups of N adjacent lanes, delivered to the last lane of each group:
// shifted adds within 16-lane rows (v_add with row_shr DPP), then row broadcasts.
template <int N>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
  if constexpr (N >= 2) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  if constexpr (N >= 4) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  if constexpr (N >= 8) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  if constexpr (N >= 16) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true); // row_shr:8
  if constexpr (N >= 32) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); // row_bcast:15
  if constexpr (N >= 64) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); // row_bcast:31
  return v;
}

// A group sum's last DPP step must run before the store branch: only the storing lane uses
// the sum, so the compiler sinks that add under the branch's exec mask, where the DPP read
// cannot fold into it (v_mov_b32_dpp + v_add_u32 instead of one v_add_u32_dpp: 4 VALU per
// mode pair in every class with more than one lane per CU).
#ifndef MIP_PIN_SUMS
#define MIP_PIN_SUMS 1  // A/B knob
#endif
__device__ __forceinline__ uint32_t pin_sum(uint32_t v) {
#if MIP_PIN_SUMS
  asm volatile("; pin" : "+v"(v));
#endif
  return v;
}

// Cost-table stores of a task: a buffer descriptor over the CTU's block (uniform per
// item), the CU's byte offset as the per-lane VGPR offset (per task) and the mode pair's
// offset as the scalar offset (per pair) -- the pair loop computes no per-lane address.
#ifndef MIP_COST_STORE_AUX
#define MIP_COST_STORE_AUX 0  // A/B: cache-policy bits of the cost-row stores
#endif
struct CtuRows {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit CtuRows(int32_t *ctu_block) {
    r = __builtin_amdgcn_make_buffer_rsrc(ctu_block, 0, MIP_COSTS_PER_CTU * 4, 0x00020000);
  }
  __device__ __forceinline__ void store(uint32_t cu_ofs, int mq, int v0, int v1) const {
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64((v2u){(unsigned)v0, (unsigned)v1}, r, (int)cu_ofs, mq * 4, MIP_COST_STORE_AUX);
  }
};

// Opaque copy of a value: keeps per-class lane arithmetic inside its switch case (hoisted
// out of the task loop it would stay live through every class and spill).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("; opaque" : "+v"(v));
  return v;
}

template <bool TR, bool LAT>
struct ViewOf {
  using type = RefTile<LAT>;
  static __device__ __forceinline__ type make(const RefTile<LAT> &r) { return r; }
};
template <bool LAT>
struct ViewOf<true, LAT> {
  using type = RefTileT<LAT>;
  static __device__ __forceinline__ type make(const RefTile<LAT> &r) { return RefTileT<LAT>{r}; }
};

// One task: CUs of class W x H (TR: the task's CUs are H x W and are searched as their
// transpose W x H -- the same MIP prediction transposed for the other orientation of each
// mode (intra.cl:417-418, 485: a transposed mode swaps the boundary halves and stores the
// output transposed), so mode pair q of the view is the CU's pair (q + MODES / 2) mod MODES;
// single-direction upsampling is the same interpolation along the other axis, and SAD / SATD
// do not change under transposition).  Wide CUs (W > H) cost up to 1.5x the VALU of their
// tall transposes (profiles/r03_shape_pmc.txt).
template <int W, int H, int V, bool LAT, bool DEC, bool TR = false>
__device__ __forceinline__ void run_task(const Ctx &x, const RefTile<LAT> &rt_tile, const WaveTask &task, int lane_in) {
  using G = Geo<W, H, V>;
  const typename ViewOf<TR, LAT>::type rt = ViewOf<TR, LAT>::make(rt_tile);
  const int lane = opaque(lane_in);
  const SearchArgs &a = *x.a;
  const int ncu = task.ncu;
  const Job *jobs = a.jobs + task.cu0;
  // lane = (slot, row part v, strip sx); lanes of one CU are adjacent
  const int slot = lane / (G::S * G::V), sub = lane % (G::S * G::V);
  const int v = sub / G::S, sx = sub % G::S, x0 = 4 * sx;
  const bool active = slot < ncu;
  const int cs = min(slot, ncu - 1);
  const Job job = jobs[cs];
  const CuPos c = cu_pos<TR>(job, x.fx0, x.fy0, rt);

  // ---- per-CU MFMA inputs of both orientations -> wave table
  if (lane < ncu) {
    const Job jb = jobs[lane];
    const CuPos cj = cu_pos<TR>(jb, x.fx0, x.fy0, rt);
    write_inputs<W, H>(cj, rt, x.wave + lane * kEntryBytes);
  }
  std::conditional_t<TR, OrigRowsT<H>, OrigRows<H>> orig;
  orig.load(x.org, c.lx + x0, c.ly);
  const size_t ctu_row = ((size_t)x.frame * a.nctus + x.ctu) * MIP_COSTS_PER_CTU;  // uniform
  const uint32_t cu_ofs = (uint32_t)job.cost * 4;                                  // < 2^19 bytes
  const CtuRows rows_cost(a.cost ? a.cost + ctu_row : nullptr), rows_sad(a.sad ? a.sad + ctu_row : nullptr),
      rows_satd(a.satd ? a.satd + ctu_row : nullptr);  // optional tables: null (never stored to)
  const uint32_t *mine = reinterpret_cast<const uint32_t *>(x.wave + kCuTableBytes) + cs * G::PITCH;
  const Red<G::R, G::RP> red{mine, 0};
  s2 top[4];  // top boundary of the strip: upsampling state above window 0
  {
    const uint2 tv = rt.top4(c.lx + x0, c.ly - 1);
    const int t4[4] = {(int)(tv.x & 0xffff), (int)(tv.x >> 16), (int)(tv.y & 0xffff), (int)(tv.y >> 16)};
#pragma unroll
    for (int cc = 0; cc < 4; cc++) top[cc] = splat(c.top ? t4[cc] : c.padT);
  }
  // padded rows in chunks: the lane's left samples stay in registers and each chunk's are
  // written to its chunk-relative rows (write_left)
  constexpr int NLV = (G::R + G::S * G::V - 1) / (G::S * G::V);
  uint32_t lvs[G::PAD && G::CHUNKED ? NLV : 1];
  uint32_t *lcol = reinterpret_cast<uint32_t *>(x.wave + kCuTableBytes) + cs * G::PITCH;
  auto write_left = [&](int chunk) {
#pragma unroll
    for (int j = 0; j < NLV; j++) {
      const int k = sub + j * G::S * G::V;
      if (active && k < G::R && k / G::CROWS == chunk) lcol[(k - chunk * G::CROWS) * G::RP] = lvs[j];
    }
  };
  if constexpr (G::PAD && G::CHUNKED) {
#pragma unroll
    for (int j = 0; j < NLV; j++) {
      const int k = sub + j * G::S * G::V;
      const uint32_t lv = k < G::R && c.left ? rt.left(c.lx - 1, c.ly + k * G::UV + G::UV - 1) : c.padL;
      lvs[j] = lv | lv << 16;
    }
    write_left(0);
  } else if constexpr (G::PAD) {
    // left boundary sample of anchor row k (CU row k*UV + UV - 1), both halves; phase A
    // never writes these positions
    for (int k = sub; k < G::R; k += G::S * G::V) {
      const uint32_t lv = c.left ? rt.left(c.lx - 1, c.ly + k * G::UV + G::UV - 1) : c.padL;
      if (active) lcol[k * G::RP] = lv | lv << 16;
    }
  }
  wave_lds_sync();

  uint32_t best = 0xffffffffu;  // DEC (decisions only): argmin over the task's pairs, cost << 5 | mode
  constexpr bool PAIRED = MIP_PAIR_BLOCKS && kPaired<W, H, V>;
#pragma unroll 1
  for (int q = task.q0; q < task.q1; q++) {
    std::conditional_t<PAIRED, PairAcc, std::conditional_t<(W * H <= 32), PackedAcc, Acc>> acc;
    s2 prev[4];
#pragma unroll
    for (int cc = 0; cc < 4; cc++) prev[cc] = top[cc];
    phase_a<W, H, V>(x, lane, ncu, q, 0);
    if constexpr (G::PAD && G::CHUNKED) {
      if (q > task.q0) write_left(0);  // the previous pair's last chunk left its rows' samples
    }
    wave_lds_sync();
    if constexpr (kSpanChunks && G::CHUNKED) {
      auto sw = [&](int c) {
        wave_lds_sync();  // every lane is done with the previous chunk
        phase_a<W, H, V>(x, lane, ncu, q, c);
        if constexpr (G::PAD) write_left(c);
        wave_lds_sync();
      };
      if constexpr (G::SID == 0) {
        walk_4x4_chunked<W, H, V>(orig, red, sw, acc);
      } else {
        static_assert(PAIRED, "chunked classes walk block pairs");
        walk_pairs_chunked<W, H, V>(orig, red, x0, prev, acc, sw);
      }
    } else if constexpr (PAIRED && G::CHUNKED) {
      walk_pairs<W, H, V>(orig, red, x0, 0, prev, acc);
      wave_lds_sync();
      phase_a<W, H, V>(x, lane, ncu, q, 1);
      wave_lds_sync();
      const Red<G::R, G::RP> red_hi{mine, -4};  // chunk 1 holds reduced rows 4..7
      walk_pairs<W, H, V>(orig, red_hi, x0, 4, prev, acc);  // prev carries anchor row 3
    } else if constexpr (PAIRED) {
      const int k0 = G::V > 1 ? v * G::KV : 0;
      if constexpr (G::V > 1) {
        if (k0 > 0) anchor_row<W, H>(red, k0 - 1, x0, prev);
      }
      walk_pairs<W, H, V>(orig, red, x0, k0, prev, acc);
    } else if constexpr (G::CHUNKED) {
      walk_strip<W, H, V>(orig, red, x0, 0, 4, prev, acc);
      wave_lds_sync();
      phase_a<W, H, V>(x, lane, ncu, q, 1);
      wave_lds_sync();
      const Red<G::R, G::RP> red_hi{mine, -4};  // chunk 1 holds reduced rows 4..7
      walk_strip<W, H, V>(orig, red_hi, x0, 4, 8, prev, acc);  // prev carries anchor row 3
    } else if constexpr (G::SID == 0) {
      walk_strip<W, H, V>(orig, red, x0, 0, 4, prev, acc);
    } else {
      // row part v: windows [v*KV, (v+1)*KV) (rows when UV == 1)
      const int k0 = G::V > 1 ? v * G::KV : 0;
      if constexpr (G::V > 1 && G::UV > 1) {
        if (k0 > 0) anchor_row<W, H>(red, k0 - 1, x0, prev);
      }
      walk_strip<W, H, V>(orig, red, x0, k0, k0 + G::KV, prev, acc);
    }
    wave_lds_sync();  // the scratch is rewritten by the next pair
    // ---- combine strips and row parts of one CU (adjacent lanes) into its last lane
    constexpr int GS = G::S * G::V;
    uint32_t sad0, sad1, satd0, satd1;
    int c0, c1;  // min(2 * SAD, SATD) of the pair's modes (intra.cl:1166)
    if constexpr (PAIRED) {
      sad0 = pin_sum(group_sum<GS>(acc.sad0));
      sad1 = pin_sum(group_sum<GS>(acc.sad1));
      satd0 = pin_sum(group_sum<GS>(acc.t0)) >> 1;
      satd1 = pin_sum(group_sum<GS>(acc.t1)) >> 1;
      c0 = min(2 * (int)sad0, (int)satd0);
      c1 = min(2 * (int)sad1, (int)satd1);
    } else if constexpr (W * H <= 32) {
      const uint32_t sp = pin_sum(group_sum<GS>(acc.sad)), tp = pin_sum(group_sum<GS>(acc.satd));
      const uint32_t cp = as_u32(__builtin_elementwise_min(as_u2(sp) << (u2){1, 1}, as_u2(tp)));
      c0 = (int)(cp & 0xffff);
      c1 = (int)(cp >> 16);
      sad0 = sp & 0xffff, sad1 = sp >> 16, satd0 = tp & 0xffff, satd1 = tp >> 16;
    } else {
      acc.flush();
      sad0 = pin_sum(group_sum<GS>(acc.sad0));
      sad1 = pin_sum(group_sum<GS>(acc.sad1));
      satd0 = pin_sum(group_sum<GS>(acc.satd0));
      satd1 = pin_sum(group_sum<GS>(acc.satd1));
      c0 = min(2 * (int)sad0, (int)satd0);
      c1 = min(2 * (int)sad1, (int)satd1);
    }
    if (active && sub == GS - 1) {
      // the CU's modes of view pair q (TR: the other orientation)
      const int mq = TR ? (2 * q < G::MODES ? 2 * q + G::MODES : 2 * q - G::MODES) : 2 * q;
      if constexpr (DEC) {
        // costs < 2^23 (256 blocks x 32736): the packed order is cost, then the lower mode
        best = min(best, min((uint32_t)c0 << 5 | (uint32_t)mq, (uint32_t)c1 << 5 | (uint32_t)(mq + 1)));
      } else {
        // every CU of a task lies inside the frame (build_work)
        rows_cost.store(cu_ofs, mq, c0, c1);
        if (a.sad) rows_sad.store(cu_ofs, mq, (int)sad0, (int)sad1);
        if (a.satd) rows_satd.store(cu_ofs, mq, (int)satd0, (int)satd1);
      }
    }
  }
  // decisions only: a task with all of a CU's pairs writes its decision; tasks that cut a
  // CU's pairs meet in one entry (atomicMin of the packed argmins, unpacked after the launch)
  if (DEC && active && sub == G::S * G::V - 1) {
    constexpr int kPairs = G::SID == 2 ? 6 : (G::SID == 1 ? 8 : 16);
    const size_t g = ((size_t)x.frame * a.nctus + x.ctu) * MIP_CUS_PER_CTU + job.cu;
    if (task.q0 == 0 && task.q1 == kPairs) {
      if (a.best_mode) a.best_mode[g] = (uint8_t)(best & 31);
      a.best_cost[g] = (int32_t)(best >> 5);
    } else {
      atomicMin((a.split_acc ? a.split_acc : reinterpret_cast<uint32_t *>(a.best_cost)) + g, best);
    }
  }
}

// Stage the quadrant window (rows -1..63, columns -4..63) of one frame into LDS, each
// sample plus its residual bias (kBiasD).  Samples are addressed like the reference does,
// by linear index fy * W + fx (intra.cl:100, 106, 236, 242, 718): columns right of the frame
// read the next row's first samples, so CUs right of the frame get the reference's
// (deterministic) costs.  Indexes past the frame's end and the columns left of a frame's
// first column read as 0 (+ bias): they only feed CUs whose costs the reference leaves
// undefined (no task) or padding branches that never select them.
// 8-byte chunk at linear index fy * width + fx (fx % 4 == 0, width % 4 == 0: a chunk lies
// entirely inside or entirely outside [0, width * height)).
__device__ __forceinline__ uint2 frame_chunk(const uint16_t *frame, int width, int height, int fx, int fy) {
  const int li = fy * width + fx;
  uint2 v = make_uint2(0, 0);
  if (fy >= 0 && fx >= 0 && li < width * height) v = *reinterpret_cast<const uint2 *>(frame + li);
  return v;
}

// Window staging by a group of P threads (P = 64: the prefetching wave; 512: the workgroup).
// Thread p takes the main chunk column 1 + (p & 15) (quadrant columns 4 (p & 15) .. +3) of
// window rows p / 16 + (P / 16) k, and the left halo chunk (columns -4..-1) of rows p + P k.
// Everything per thread but the row step is fixed per item, so a chunk costs one address
// add and the two bias adds: the loads go through a buffer descriptor over the frame, whose
// range check reads indexes past the frame's end as 0 (frame_chunk's `li < W * H`; a chunk
// lies entirely inside or outside, W % 4 == 0), the row above the frame and the columns left
// of it are forced out of range (uniform tests), and the LDS offsets are immediates.  (The
// chunk-index form, row = i / 17 per chunk, cost ~20 VALU per chunk: ~0.9 % of the kernel.)
template <int P>
struct WindowStager {
  static constexpr int RIT = P / 16;                 // window rows per main round
  static constexpr int NMAIN = (65 + RIT - 1) / RIT;  // main rounds
  static constexpr int NHALO = (65 + P - 1) / P;      // halo rounds
  static constexpr int N = NMAIN + NHALO;
  static constexpr uint32_t kOut = 0x80000000u;       // an out-of-range byte offset
  __amdgpu_buffer_rsrc_t rsrc;
  int p;                    // thread
  uint32_t vmain, vhalo, W2;  // byte offsets of its main / halo chunk in round 0 (mod 2^32), row bytes
  bool top, left;           // the window's row -1 / columns -4..-1 lie outside the frame
  uint32_t bmx, bmy, bhx, bhy;  // residual biases of its main / halo rows (kBiasD)
  __device__ __forceinline__ WindowStager(const uint16_t *frame, int width, int height, int fx0, int fy0, int thread) {
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(frame), 0, (int)((uint32_t)width * height * 2u), 0x00020000);
    p = thread;
    W2 = (uint32_t)width * 2;
    top = fy0 == 0;
    left = fx0 == 0;
    // (fy0 + 64) * width < 2^31 (mip_engine_create); the byte offsets wrap like the range
    // check's unsigned compare expects (row -1 above the frame is forced out of range anyway)
    vmain = (uint32_t)((fy0 - 1 + p / 16) * width + fx0 + 4 * (p & 15)) * 2u;
    vhalo = (uint32_t)((fy0 - 1 + p) * width + fx0 - 4) * 2u;
    const bool om = ((p / 16 - 1) & 1) != 0, oh = ((p - 1) & 1) != 0;  // row parity (RIT, P even)
    bmx = om ? bias_word(1, 0) : bias_word(0, 0);
    bmy = om ? bias_word(1, 2) : bias_word(0, 2);
    bhx = oh ? bias_word(1, 0) : bias_word(0, 0);
    bhy = oh ? bias_word(1, 2) : bias_word(0, 2);
  }
  __device__ __forceinline__ bool valid(int k) const {
    return k < NMAIN ? (k < NMAIN - 1 || p / 16 + RIT * k < 65) : p + P * (k - NMAIN) < 65;
  }
  __device__ __forceinline__ uint2 load(int k) const {
    uint32_t o;
    if (k < NMAIN) {
      o = vmain + (uint32_t)(k * RIT) * W2;
      if (k == 0 && top) o = p < 16 ? kOut : o;  // row -1 above the frame
    } else {
      o = vhalo + (uint32_t)((k - NMAIN) * P) * W2;
      if (left) o = kOut;                         // columns left of the frame
      if (k == NMAIN && top) o = p == 0 ? kOut : o;
    }
    typedef unsigned int v2u __attribute__((ext_vector_type(2)));
    const v2u v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)o, 0, 0);
    return make_uint2(v.x, v.y);
  }
  __device__ __forceinline__ void store(uint16_t *dst, int k, uint2 v) const {
    if (k < NMAIN) {
      v.x += bmx;
      v.y += bmy;
      *reinterpret_cast<uint2 *>(dst + (p / 16 + RIT * k) * kPitch + 4 + 4 * (p & 15)) = v;
    } else {
      v.x += bhx;
      v.y += bhy;
      *reinterpret_cast<uint2 *>(dst + (p + P * (k - NMAIN)) * kPitch) = v;
    }
  }
};

// (whole workgroup, NT threads: every thread's loads are issued before its first
// LDS store, so the workgroup waits for HBM once, not once per load)
// Input contract: a staged sample above 10 bits (any of bits 10..15 of the OR of the
// loaded chunks) marks the search's status word (SearchArgs::status); the costs of such a
// frame are not the reference's (the packed 16-bit / f16 arithmetic is sized for 10 bits), so
// the host reports the search as failed.  Rare path: one plain store per offending thread.
// Merged chunks (SearchArgs::frame_status): the frame's own call's status set.
#ifndef MIP_FRAME_STATUS
#define MIP_FRAME_STATUS 1  // A/B: 0 = one status set per launch (wrong statuses in merged launches)
#endif
__device__ __forceinline__ void flag_above_10_bits(uint32_t bits, const SearchArgs &a, int frame, int word) {
  if (bits & kAbove10Bits) (MIP_FRAME_STATUS && a.frame_status ? a.frame_status[frame] : a.status)[word] = 1u;
}

template <int NT>
__device__ __forceinline__ void stage_tile(uint16_t *dst, const uint16_t *frame, int width, int height,
                                           int x0, int y0, const SearchArgs &a, int fidx) {
  const WindowStager<NT> st(frame, width, height, x0, y0, (int)threadIdx.x);
  constexpr int N = WindowStager<NT>::N;
  uint2 v[N];
#pragma unroll
  for (int k = 0; k < N; k++)
    if (st.valid(k)) v[k] = st.load(k);
  uint32_t bits = 0;
#pragma unroll
  for (int k = 0; k < N; k++)
    if (st.valid(k)) {
      bits |= v[k].x | v[k].y;
      st.store(dst, k, v[k]);
    }
  flag_above_10_bits(bits, a, fidx, kStatusOrig);
}

// Item = (frame, CTU, quadrant, slice) -> quadrant origin in the frame and frame index.
struct ItemPos {
  int frame, ctu, slice, quad, ctu_x, ctu_y, fx0, fy0;
  __device__ __forceinline__ ItemPos(const SearchArgs &a, uint32_t item) {
    const int per_ctu = 4 * a.slices;
    uint32_t base = item;  // item index inside its frame
    if (a.order) {         // small launches: longest items first, all frames' in turn
      base = a.order[item / a.nframes];
      frame = item % a.nframes;
    } else {
      frame = item / (per_ctu * a.nrange);
    }
    const int gx = base % per_ctu;
    ctu = a.ctu0 + (base / per_ctu) % a.nrange;
    slice = gx % a.slices;
    quad = gx / a.slices;
    ctu_x = 128 * (ctu % a.ctu_cols);
    ctu_y = 128 * (ctu / a.ctu_cols);
    fx0 = ctu_x + 64 * (quad & 1);
    fy0 = ctu_y + 64 * (quad >> 1);
  }
};

// Stage the reference lattice (ALT): rows 4i-1 (columns -4..63), columns 4i-1 (rows -1..63),
// by linear index like the window (frame_chunk).
// check: caller-supplied references (SearchArgs::check_refs) must be 10-bit too, except frame
// columns W-2, W-1 at widths that are not multiples of 128, whose CUs the exact fixup kernel
// searches (mipgpu.cpp ctu_variants / reads_last_columns).  Samples are addressed linearly,
// so a chunk's frame column is its x modulo the width.
template <int NT>
__device__ __forceinline__ void stage_lattice(uint16_t *dst, const uint16_t *frame, int width, int height,
                                              int x0, int y0, bool check, const SearchArgs &a, int fidx) {
  // all loads first, then all LDS stores (as stage_tile)
  constexpr int kChunks = kPitch / 4, NR = 16 * kChunks, NC = 16 * 65;
  constexpr int NRL = (NR + NT - 1) / NT, NCL = (NC + NT - 1) / NT;
  uint2 rv[NRL];
  uint16_t cv[NCL];
#pragma unroll
  for (int k = 0; k < NRL; k++) {
    const int i = min((int)threadIdx.x + NT * k, NR - 1), row = i / kChunks, ch = i - row * kChunks;
    rv[k] = frame_chunk(frame, width, height, x0 - kColOff + 4 * ch, y0 + 4 * row - 1);
  }
#pragma unroll
  for (int k = 0; k < NCL; k++) {
    const int i = min((int)threadIdx.x + NT * k, NC - 1), col = i / 65, yy = i - col * 65;
    const int fy = y0 + yy - 1, fx = x0 + 4 * col - 1, li = fy * width + fx;  // linear, as frame_chunk
    cv[k] = (fy >= 0 && fx >= 0 && li < width * height) ? frame[li] : 0;
  }
  uint32_t bits = 0;
  const bool exempt_last = width % 128 != 0;  // fixup CUs exist (columns W-2, W-1)
  auto frame_col = [&](int fx) { return fx < width ? fx : fx % width; };  // fx >= 0
#pragma unroll
  for (int k = 0; k < NRL; k++) {
    const int i = min((int)threadIdx.x + NT * k, NR - 1), row = i / kChunks, ch = i - row * kChunks;
    *reinterpret_cast<uint2 *>(dst + row * kLatRowPitch + 4 * ch) = rv[k];
    if (check) {
      // .y holds the chunk's columns c+2, c+3: W-2, W-1 when c == W-4
      const int fx = x0 - kColOff + 4 * ch;
      const bool skip_y = exempt_last && fx >= 0 && frame_col(fx) == width - 4;
      bits |= rv[k].x | (skip_y ? 0u : rv[k].y);
    }
  }
  uint16_t *cols = dst + 16 * kLatRowPitch;
#pragma unroll
  for (int k = 0; k < NCL; k++) {
    const int i = min((int)threadIdx.x + NT * k, NC - 1), col = i / 65, yy = i - col * 65;
    cols[col * kLatColPitch + yy] = cv[k];
    if (check) {
      const int fx = x0 + 4 * col - 1;  // = 3 mod 4: only column W-1 can be exempt
      if (!(exempt_last && fx >= 0 && frame_col(fx) == width - 1)) bits |= cv[k];
    }
  }
  if (check) flag_above_10_bits(bits, a, fidx, kStatusRefs);
}

// Next-item prefetch (PF, non-ALT): two quadrant windows in LDS.  The first wave of an item
// to run out of tasks takes the next item from the device-wide queue and stages its window
// into the other buffer while the remaining waves finish theirs, so neither the counter's
// round trip nor the window's HBM latency stalls the whole workgroup between items (skipping
// the staging altogether measured +1.2 %).  Taking the next item early would unbalance the
// end of a launch (a reserved item waits while other workgroups run dry: 16-frame launches
// -1.4 % when every item was prefetched), so in the last two rounds of items the next one is
// taken after the current one instead; launches with fewer than MIP_PREFETCH_MIN_ITEMS items
// per workgroup do not prefetch at all (1-frame launches measured -9 % with the prefetching
// kernel).  The ALT lattice leaves no LDS for a second window.
template <bool ALT, bool PF, int NW = kSearchWaves>
constexpr int kOrgTiles = (PF || NW == kWideWaves) && !ALT ? 2 : 1;  // (16 waves: pair mode)
constexpr int kCounterWords = 12;  // [parity]: next task, finished waves, item, item taken late;
                                   // [8]: chunks this workgroup has found empty (take_item)

// The launch's items in kQueueChunks contiguous chunks (fewer if the grid is smaller), chunk
// c = [chunk_begin(c), chunk_begin(c + 1)) with its own counter a.queue[c].  Workgroup b
// takes from chunk b % K first and then from the following ones.  The hardware deals the
// workgroups round robin over the 8 XCDs, so one chunk's items -- neighbouring quadrants,
// which share the 128-byte lines of the window's left columns and of the cost rows across
// the quadrant border -- run on one XCD, close in time, and meet in its L2 (with one counter,
// neighbours ran on different XCDs: FETCH 2x the frame bytes).  Placement is only a speed
// matter: any workgroup may take any item.
__device__ __forceinline__ uint32_t queue_chunks(const SearchArgs &a) { return gridDim.x < a.chunks ? gridDim.x : a.chunks; }
__device__ __forceinline__ uint32_t chunk_begin(uint32_t nitems, uint32_t c, uint32_t k) {
  return (uint32_t)((uint64_t)nitems * c / k);
}
// One thread of the workgroup at a time (the callers are separated by barriers); *empty (LDS)
// counts the chunks this workgroup found exhausted, so each costs it one failed atomic.
__device__ __forceinline__ uint32_t take_item(const SearchArgs &a, uint32_t *empty) {
  const uint32_t k = queue_chunks(a), g = blockIdx.x % k;
  for (uint32_t j = *empty; j < k; j++) {
    const uint32_t c = g + j < k ? g + j : g + j - k;
    const uint32_t b = chunk_begin(a.nitems, c, k), n = chunk_begin(a.nitems, c + 1, k) - b;
    const uint32_t i = atomicAdd(a.queue + c, 1u);
    if (i < n) {
      *empty = j;
      return b + i;
    }
  }
  *empty = k;
  return a.nitems;  // every chunk is exhausted
}
// Are many items of the workgroup's own chunk left after `item` (the chunk's head is about
// one round of its workgroups past the item just taken)?
__device__ __forceinline__ bool far_from_end(const SearchArgs &a, uint32_t item) {
  const uint32_t k = queue_chunks(a), g = blockIdx.x % k;
  const uint32_t b = chunk_begin(a.nitems, g, k), e = chunk_begin(a.nitems, g + 1, k);
  return item >= b && item + 3 * (gridDim.x / k) < e;
}
constexpr uint32_t kTakeItem = 0xffffffffu;  // "take the next item after this one" (PF)

// CUs whose cost the reference leaves undefined (edge CTUs) of one item: MIP_COST_UNAVAILABLE,
// no search (the whole workgroup).
template <bool DEC>
__device__ __forceinline__ void fill_unavailable(const SearchArgs &a, int frame, int ctu, int vq, int slice) {
  if (DEC) {
    const size_t gbase = ((size_t)frame * a.nctus + ctu) * MIP_CUS_PER_CTU;
    const int f0 = a.dfill_begin[vq], nf = a.dfill_begin[vq + 1] - f0;
    for (int i = slice * blockDim.x + threadIdx.x; i < nf; i += a.slices * blockDim.x) {
      const size_t g = gbase + a.dfill[f0 + i];
      if (a.best_mode) a.best_mode[g] = 0xff;
      a.best_cost[g] = kUnavailable;
    }
  } else {
    const size_t cbase = ((size_t)frame * a.nctus + ctu) * (MIP_COSTS_PER_CTU / 4);
    const int f0 = a.fill_begin[vq], nf = a.fill_begin[vq + 1] - f0;
    const uint4 un = make_uint4(kUnavailable, kUnavailable, kUnavailable, kUnavailable);
    for (int i = slice * blockDim.x + threadIdx.x; i < nf; i += a.slices * blockDim.x) {
      const size_t o = cbase + a.fill[f0 + i];
      reinterpret_cast<uint4 *>(a.cost)[o] = un;
      if (a.sad) reinterpret_cast<uint4 *>(a.sad)[o] = un;
      if (a.satd) reinterpret_cast<uint4 *>(a.satd)[o] = un;
    }
  }
}

// One wave task: the size class's search over the task's CUs and mode pairs.
template <bool ALT, bool DEC>
__device__ __forceinline__ void dispatch_task(const Ctx &x, const RefTile<ALT> &rt, const WaveTask &task, int lane) {
  switch (task.cls) {
#define MIP_CASE(idx, W, H)                                                \
  case idx:                                                                \
    static_assert(kClassW[idx] == W && kClassH[idx] == H, "class table");  \
    if constexpr ((MIP_ONLY_CLASS < 0 || MIP_ONLY_CLASS == idx) && !((MIP_SKIP_CLASSES >> idx) & 1)) \
      run_task<W, H, kClassV[idx], ALT, DEC>(x, rt, task, lane);           \
    break;
    MIP_CASE(0, 64, 64) MIP_CASE(1, 32, 32) MIP_CASE(2, 32, 16) MIP_CASE(3, 16, 32)
    MIP_CASE(4, 32, 8) MIP_CASE(5, 8, 32) MIP_CASE(6, 16, 16) MIP_CASE(7, 16, 8)
    MIP_CASE(8, 8, 16) MIP_CASE(9, 32, 4) MIP_CASE(10, 4, 32) MIP_CASE(11, 16, 4)
    MIP_CASE(12, 4, 16) MIP_CASE(13, 8, 8) MIP_CASE(14, 8, 4) MIP_CASE(15, 4, 8)
    MIP_CASE(16, 4, 4)
    // row-part variants for remainder tasks (mip_kernels.h)
    MIP_CASE(17, 32, 8) MIP_CASE(18, 16, 16) MIP_CASE(19, 16, 8) MIP_CASE(20, 8, 16)
    MIP_CASE(27, 32, 16) MIP_CASE(28, 16, 32)
#undef MIP_CASE
#define MIP_CASE_TR(idx, W, H)                                                    \
  case idx:                                                                       \
    static_assert(kClassW[idx] == W && kClassH[idx] == H && kClassTR[idx], "class table"); \
    if constexpr ((MIP_ONLY_CLASS < 0 || MIP_ONLY_CLASS == idx) && !((MIP_SKIP_CLASSES >> idx) & 1)) \
      run_task<W, H, kClassV[idx], ALT, DEC, true>(x, rt, task, lane);            \
    break;
    // transposed classes: wide CUs searched as their transposes
    MIP_CASE_TR(21, 4, 32) MIP_CASE_TR(22, 4, 16) MIP_CASE_TR(23, 4, 8) MIP_CASE_TR(24, 8, 32)
    MIP_CASE_TR(25, 8, 16) MIP_CASE_TR(26, 8, 16)
#undef MIP_CASE_TR
    default: break;
  }
}

// Profiling (MIPGPU_WAVE_TIMING): item start (s_memrealtime, 100 MHz) and the workgroup's
// place (HW_ID: CU / SIMD / SE; XCC_ID) in the last three of the item's clock slots.
__device__ __forceinline__ void stamp_item_start(uint64_t *clk) {
  clk[kClockSlots - 3] = __builtin_amdgcn_s_memrealtime();
  clk[kClockSlots - 1] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                         (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32;
}

// Two items' windows staged at once (pair mode): every thread's loads of both windows are in
// flight before its first LDS store.  b = false: the second item is absent.
template <int NT>
__device__ __forceinline__ void stage_tiles2(uint16_t *dst0, const uint16_t *frame0, int x0, int y0, uint16_t *dst1,
                                             const uint16_t *frame1, int x1, int y1, bool b, int width, int height,
                                             const SearchArgs &a, int f0, int f1) {
  const WindowStager<NT> s0(frame0, width, height, x0, y0, (int)threadIdx.x);
  const WindowStager<NT> s1(frame1, width, height, x1, y1, (int)threadIdx.x);
  constexpr int N = WindowStager<NT>::N;
  uint2 v0[N], v1[N];
#pragma unroll
  for (int k = 0; k < N; k++) {
    if (s0.valid(k)) v0[k] = s0.load(k);
    if (b && s1.valid(k)) v1[k] = s1.load(k);
  }
  uint32_t bits0 = 0, bits1 = 0;
#pragma unroll
  for (int k = 0; k < N; k++) {
    if (s0.valid(k)) {
      bits0 |= v0[k].x | v0[k].y;
      s0.store(dst0, k, v0[k]);
    }
    if (b && s1.valid(k)) {
      bits1 |= v1[k].x | v1[k].y;
      s1.store(dst1, k, v1[k]);
    }
  }
  flag_above_10_bits(bits0, a, f0, kStatusOrig);
  flag_above_10_bits(bits1, a, f1, kStatusOrig);
}

// Pair mode (16-wave workgroups, one per CU; one-frame launches with original references and
// the longest-first order, launch_search): a workgroup takes two items at once -- queue
// positions p and E - 1 - p of the E items with tasks (SearchArgs::nonempty), a long one with
// a short one -- stages both windows and lets its 16 waves take the two items' tasks from one
// LDS counter (interleaved, so both lists' long tasks come first); the items without tasks
// (last in the order: bottom quadrants) are fill-only and go along with pairs p, p + P, ...
// Two items per CU run in ~150 us this way, against ~160 us one after the other.
template <bool DEC>
__device__ __forceinline__ void pair_loop(const SearchArgs &a, uint16_t *org_buf, const uint8_t *w, const uint8_t *zero,
                                          uint8_t *waves, uint32_t *counters, int wave, int lane) {
  const uint32_t ne = a.nonempty, npairs = (ne + 1) / 2;
  for (;;) {
    if (threadIdx.x == 0) {
      counters[0] = 0;
      counters[1] = atomicAdd(a.queue, 1u);  // one queue chunk (launch_search)
    }
    __syncthreads();
    const uint32_t p = counters[1];
    if (p >= npairs) break;  // workgroup-uniform
    const uint32_t i0 = p, i1 = ne - 1 - p;
    const bool two = i1 != i0;
    const ItemPos p0(a, i0), p1(a, i1);
    const int vq0 = a.ctu_var[p0.ctu] * 4 + p0.quad, vq1 = a.ctu_var[p1.ctu] * 4 + p1.quad;
    const int l0 = vq0 * a.slices + p0.slice, l1 = vq1 * a.slices + p1.slice;
    const int tb0 = a.list_begin[l0], n0 = a.list_begin[l0 + 1] - tb0;
    const int tb1 = a.list_begin[l1], n1 = two ? a.list_begin[l1 + 1] - tb1 : 0;
    fill_unavailable<DEC>(a, p0.frame, p0.ctu, vq0, p0.slice);
    if (two) fill_unavailable<DEC>(a, p1.frame, p1.ctu, vq1, p1.slice);
    for (uint32_t e = ne + p; e < a.nitems; e += npairs) {  // fill-only items
      const ItemPos pe(a, e);
      fill_unavailable<DEC>(a, pe.frame, pe.ctu, a.ctu_var[pe.ctu] * 4 + pe.quad, pe.slice);
    }
    uint16_t *org0 = org_buf, *org1 = org_buf + kTileElems;
    stage_tiles2<64 * kWideWaves>(org0, a.orig + (size_t)p0.frame * a.width * a.height, p0.fx0, p0.fy0, org1,
                                  a.orig + (size_t)p1.frame * a.width * a.height, p1.fx0, p1.fy0, two, a.width,
                                  a.height, a, p0.frame, p1.frame);
    __syncthreads();
    uint64_t *clk0 = a.wave_clock ? a.wave_clock + (size_t)i0 * kClockSlots : nullptr;
    uint64_t *clk1 = a.wave_clock && two ? a.wave_clock + (size_t)i1 * kClockSlots : nullptr;
    if (clk0 && threadIdx.x == 0) {
      stamp_item_start(clk0);
      if (clk1) stamp_item_start(clk1);
    }
    const int m = n0 < n1 ? n0 : n1;
    for (;;) {
      uint32_t tn = 0;
      if (lane == 0) tn = atomicAdd(counters, 1u);
      const int t = (int)__builtin_amdgcn_readfirstlane(tn);
      if (t >= n0 + n1) break;
      // tasks 0 .. 2m-1 alternate between the items (each list is longest first), then the
      // rest of the longer list
      const bool second = t < 2 * m ? (t & 1) != 0 : n1 > n0;
      const int k = t < 2 * m ? t >> 1 : t - m;
      const uint64_t c0 = clk0 ? __builtin_readcyclecounter() : 0;
      const WaveTask task = a.tasks[(second ? tb1 : tb0) + k];
      const Ctx x{&a, second ? org1 : org0, second ? org1 : org0, w, zero, waves + wave * kWaveStride,
                  second ? p1.ctu : p0.ctu, second ? p1.frame : p0.frame, second ? p1.fx0 : p0.fx0,
                  second ? p1.fy0 : p0.fy0};
      const RefTile<false> rt{x.ref};
      dispatch_task<false, DEC>(x, rt, task, lane);
      uint64_t *clk = second ? clk1 : clk0;
      if (clk && lane == 0) {
        if (k < kClockSlots - 3) clk[k] = __builtin_readcyclecounter() - c0;
        atomicMax(reinterpret_cast<unsigned long long *>(clk + kClockSlots - 2),
                  (unsigned long long)__builtin_amdgcn_s_memrealtime());
      }
    }
    __syncthreads();  // every wave is done with the windows and the counters
  }
}

// DEC: decisions only -- no cost table, per-CU decisions (SearchArgs::best_mode / best_cost).
// NW: waves per workgroup (kSearchWaves; kWideWaves: one workgroup per CU, small launches)
#ifndef MIP_WAVES_PER_EU
#define MIP_WAVES_PER_EU (MIP_SIX_WAVES ? 6 : 4)  // HIP-Clang: the second launch bound is the minimum waves per SIMD
#endif
// Six waves per SIMD: the MIP tables are read from global memory (L1 / L2) instead of LDS
// and the search never prefetches the next window (no LDS for a second one).
#ifndef MIP_TABLES_GLOBAL
#define MIP_TABLES_GLOBAL 0  // A/B: the MIP tables from global memory at four waves per SIMD too
#endif
constexpr bool kTablesInLds = (!MIP_SIX_WAVES || MIP_SIX_WAVES == 3) && !MIP_TABLES_GLOBAL;
// (MIP_SIX_WAVES 3: two windows, the tables and 12 x 4 KB of wave areas fill 81 648 of the
// 81 920 bytes a workgroup may take with two per CU)
#ifndef MIP_S6_PF
#define MIP_S6_PF 1  // A/B: next-item prefetch in the MIP_SIX_WAVES 3 build
#endif
#define MIP_PF_KERNEL (!MIP_SIX_WAVES || (MIP_SIX_WAVES == 3 && MIP_S6_PF))
constexpr bool kPrefetchKernel = MIP_PF_KERNEL;
template <bool ALT, bool DEC, bool PF_, int NW>
__global__ __launch_bounds__(64 * NW, NW == kWideWaves ? 4 : MIP_WAVES_PER_EU) void mip_search_kernel(SearchArgs a) {
  constexpr bool PF = PF_ && !ALT && NW == kSearchWaves && kPrefetchKernel;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint16_t *org_buf = reinterpret_cast<uint16_t *>(smem);  // kOrgTiles windows
  uint16_t *lattice = org_buf + kOrgTiles<ALT, PF, NW> * kTileElems;
  uint8_t *tab = smem + (kOrgTiles<ALT, PF, NW> * kTileElems + (ALT ? kLatElems : 0)) * 2;
  uint8_t *zero = tab + (kTablesInLds ? kTableBytes : 0);
  uint8_t *waves = zero + kZeroBytes;
  uint32_t *counters = reinterpret_cast<uint32_t *>(waves + NW * kWaveStride);
  const uint8_t *w = kTablesInLds ? tab : reinterpret_cast<const uint8_t *>(a.tables);

  if constexpr (kTablesInLds)
    for (int i = threadIdx.x; i < kTableBytes / 16; i += blockDim.x)
      reinterpret_cast<uint4 *>(tab)[i] = a.tables[i];
  for (int i = threadIdx.x; i < kZeroBytes / 16; i += blockDim.x)
    reinterpret_cast<uint4 *>(zero)[i] = make_uint4(0, 0, 0, 0);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;

  if (NW == kWideWaves && !ALT && !PF && a.nonempty > 0) {  // uniform: pair mode
    pair_loop<DEC>(a, org_buf, w, zero, waves, counters, wave, lane);
  } else {
  // Persistent workgroups (as many as are resident) take items = (frame, CTU, quadrant,
  // slice) from a device-wide queue (take_item), in order: the hardware's static round-robin of
  // workgroups over XCDs and CUs cannot balance items of unequal cost (edge CTUs).
  // (PF: the first item is taken like a late one, by the loop)
  if (threadIdx.x < kCounterWords) counters[threadIdx.x] = threadIdx.x == 2 && PF ? kTakeItem : 0u;
  __syncthreads();
  if (!PF) {
    if (threadIdx.x == 0) counters[2] = take_item(a, counters + 8);
    __syncthreads();
  }
  int par = 0;          // workgroup-uniform: parity of the item (window buffer, counter set)
  for (;;) {
    uint32_t *next_task = counters + 4 * par, *finished = next_task + 1;
    uint32_t item = next_task[2];
    bool staged = PF;  // workgroup-uniform: the window of the item is in LDS
    if (PF && item == kTakeItem) {  // near the end of the launch: take the item now
      if (threadIdx.x == 0) next_task[3] = take_item(a, counters + 8);
      __syncthreads();
      item = next_task[3];
      staged = false;
    }
    if (item >= a.nitems) break;  // workgroup-uniform
    const ItemPos ip(a, item);
    const int ctu = ip.ctu, frame = ip.frame, slice = ip.slice, quad = ip.quad, fx0 = ip.fx0, fy0 = ip.fy0;
    const size_t fofs = (size_t)frame * a.width * a.height;
    const int var = a.ctu_var[ctu];  // work / fill lists of the CTU's variant (mipgpu.cpp ctu_variants)
    const int vq = var * 4 + quad, list = vq * a.slices + slice;
    const int tbase = a.list_begin[list], ntasks = a.list_begin[list + 1] - tbase;
    uint16_t *org = org_buf + (PF ? par * kTileElems : 0);
    uint16_t *ref = ALT ? lattice : org;

    fill_unavailable<DEC>(a, frame, ctu, vq, slice);
    if (ntasks > 0) {  // workgroup-uniform
      if (!PF || !staged) {
        stage_tile<64 * NW>(org, a.orig + fofs, a.width, a.height, fx0, fy0, a, frame);
        if (ALT) stage_lattice<64 * NW>(ref, a.refs + fofs, a.width, a.height, fx0, fy0, a.check_refs != 0, a, frame);
        __syncthreads();
      }

      const Ctx x{&a, org, ref, w, zero, waves + wave * kWaveStride, ctu, frame, fx0, fy0};
      const RefTile<ALT> rt{ref};
      // Waves take the item's tasks (longest first) from an LDS counter, so early
      // finishers pick up the slack of waves the SIMD arbiter serves later.
      uint64_t *clk = a.wave_clock ? a.wave_clock + (size_t)item * kClockSlots : nullptr;
      if (clk && threadIdx.x == 0) stamp_item_start(clk);
      for (;;) {
        uint32_t tn = 0;
        if (lane == 0) tn = atomicAdd(next_task, 1u);
        const int t = (int)__builtin_amdgcn_readfirstlane(tn);
        if (t >= ntasks) break;
#if MIP_PRIO_BALANCE
        // Two workgroups share a CU, and the SIMD arbiter serves the older waves first: in a
        // small launch the first workgroup of a CU finished its item in 98 us while the
        // second, starved, took 170 us (profiles/r04_item_timeline_1frame.csv).  A wave's
        // priority follows the share of its item still to do, so the workgroup that is
        // behind is served first and the two finish together.
        {
          const int rem4 = 4 * (ntasks - t);  // uniform
          if (rem4 > 3 * ntasks) __builtin_amdgcn_s_setprio(3);
          else if (rem4 > 2 * ntasks) __builtin_amdgcn_s_setprio(2);
          else if (rem4 > ntasks) __builtin_amdgcn_s_setprio(1);
          else __builtin_amdgcn_s_setprio(0);
        }
#endif
        const uint64_t c0 = clk ? __builtin_readcyclecounter() : 0;
        const WaveTask task = a.tasks[tbase + t];
        dispatch_task<ALT, DEC>(x, rt, task, lane);
        if (clk && lane == 0 && t < kClockSlots - 3) clk[t] = __builtin_readcyclecounter() - c0;
      }
      if (clk && lane == 0) atomicMax(reinterpret_cast<unsigned long long *>(clk + kClockSlots - 2),
                                      (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    // ---- next item: its index (and, PF, its window) go to the other parity's slots, which
    // no wave reads during this item
    if (PF) {
      uint32_t *nxt = counters + 4 * (par ^ 1);
      uint32_t r = 0;
      if (lane == 0) r = atomicAdd(finished, 1u);
      if (__builtin_amdgcn_readfirstlane(r) == 0) {  // wave-uniform: the first idle wave
        // Taking the next item before this one is done is worth it only while many items
        // are left: in the last rounds a reserved item would wait for this workgroup while
        // others run dry, so there the next item is taken after the item (kTakeItem).
        // (far_from_end: in the workgroup's own chunk, more than three rounds of its
        // workgroups left)
        uint32_t n = kTakeItem;
        if (lane == 0 && far_from_end(a, item)) n = take_item(a, counters + 8);
        const uint32_t nitem = __builtin_amdgcn_readfirstlane(n);
        if (nitem < a.nitems) {  // (kTakeItem >= nitems)
          const ItemPos np(a, nitem);
          const uint16_t *nframe = a.orig + (size_t)np.frame * a.width * a.height;
          uint16_t *dst = org_buf + (par ^ 1) * kTileElems;
          // loads in flight MIP_PF_BATCH at a time, then their stores
          const WindowStager<64> st(nframe, a.width, a.height, np.fx0, np.fy0, lane);
          constexpr int NL = WindowStager<64>::N, NB = MIP_PF_BATCH;
          uint32_t bits = 0;
#pragma unroll
          for (int k0 = 0; k0 < NL; k0 += NB) {
            uint2 v[NB];
#pragma unroll
            for (int k = 0; k < NB; k++)
              if (k0 + k < NL && st.valid(k0 + k)) v[k] = st.load(k0 + k);
#pragma unroll
            for (int k = 0; k < NB; k++)
              if (k0 + k < NL && st.valid(k0 + k)) {
                bits |= v[k].x | v[k].y;
                st.store(dst, k0 + k, v[k]);
              }
          }
          flag_above_10_bits(bits, a, np.frame, kStatusOrig);
        }
        if (lane == 0) {
          nxt[0] = 0;
          nxt[1] = 0;
          nxt[2] = nitem;
        }
      }
      __syncthreads();  // the window and the counters of the next item are in place
    } else {
      __syncthreads();  // every wave is done with the window and the item's counters
      if (threadIdx.x == 0) {
        next_task[0] = 0;
        next_task[2] = take_item(a, counters + 8);
      }
      __syncthreads();  // the next item is in place
    }
    if (PF) par ^= 1;  // (a loop-carried parity costs the ALT kernel ~30 VGPRs)
  }
  }
  // The last workgroup to leave resets the queue's counters for the next launch that uses it
  // (the host never runs two launches on one pair at the same time).
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(a.queue + kQueueChunks, 1u) == gridDim.x - 1) {
      for (int c = 0; c < kQueueChunks; c++) atomicExch(a.queue + c, 0u);
      atomicExch(a.queue + kQueueChunks, 0u);
    }
  }
}

// Decision list of one CU: the k lowest-cost of its M modes (ties to the lower mode), by
// repeated selection over the row held in registers; 0xff / kUnavailable past the M modes
// and for unavailable CUs (every entry of such a row is kUnavailable).
template <int M>
__device__ __forceinline__ void topk_row(const int32_t *row, int k, uint8_t *mo, int32_t *co) {
  int v[M];
#pragma unroll
  for (int m = 0; m < M; m += 4) {  // rows start 16-byte aligned (12, 16 or 32 entries per CU)
    const int4 q = *reinterpret_cast<const int4 *>(row + m);
    v[m] = q.x, v[m + 1] = q.y, v[m + 2] = q.z, v[m + 3] = q.w;
  }
  const bool unavailable = v[0] == kUnavailable;
  uint32_t used = 0;
  for (int r = 0; r < k; r++) {
    int best = 0, bc = 0;
    bool found = false;
#pragma unroll
    for (int m = 0; m < M; m++)
      if (!((used >> m) & 1) && (!found || v[m] < bc)) best = m, bc = v[m], found = true;
    const bool ok = found && !unavailable;
    if (ok) used |= 1u << best;
    if (mo) mo[r] = ok ? (uint8_t)best : 0xff;
    if (co) co[r] = ok ? bc : kUnavailable;
  }
}

// Per-CU decision lists (k = 1: the argmin).
#if !MIP_FOUR_WAVE_TWIN
__global__ __launch_bounds__(256) void best_mode_kernel(BestArgs a) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.total_cus) return;
  const int ctu = g / MIP_CUS_PER_CTU;
  int r = g - ctu * MIP_CUS_PER_CTU, s = 0;
#pragma unroll
  for (int step = 32; step; step >>= 1)  // last shape whose first CU is <= r
    if (s + step < MIP_NUM_SHAPES && c_shape_start.v[s + step] <= r) s += step;
  r -= c_shape_start.v[s];
  const mip_shape_desc sd = c_shapes[s];
  const int32_t *row = a.cost + (size_t)ctu * MIP_COSTS_PER_CTU + sd.cost_offset + (size_t)r * 2 * sd.modes;
  uint8_t *mo = a.best_mode ? a.best_mode + (size_t)g * a.k : nullptr;
  int32_t *co = a.best_cost ? a.best_cost + (size_t)g * a.k : nullptr;
  switch (sd.modes) {
    case 6: topk_row<12>(row, a.k, mo, co); break;
    case 8: topk_row<16>(row, a.k, mo, co); break;
    default: topk_row<32>(row, a.k, mo, co); break;
  }
}

// Split CUs of decisions-only searches: all ones before the search (init), packed argmin ->
// decision list of length 1 after it (the layout of best_mode_kernel with k = 1).
template <bool INIT>
__global__ __launch_bounds__(256) void dec_split_kernel(SplitArgs a, int total) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int j = t % a.max_split, r = t / a.max_split, ctu = a.ctu0 + r % a.nrange, frame = r / a.nrange;
  const int v = a.ctu_var[ctu], b = a.split_begin[v];
  if (j >= a.split_begin[v + 1] - b) return;
  const size_t g = ((size_t)frame * a.nctus + ctu) * MIP_CUS_PER_CTU + a.split[b + j];
  if (INIT) {
    if (a.acc) a.acc[g] = ~0u;
    else a.best_cost[g] = -1;
  } else {
    uint32_t p;
    if (a.acc) {
      p = a.acc[g];
      a.acc[g] = ~0u;  // initialised for the next launch
    } else {
      p = (uint32_t)a.best_cost[g];
    }
    const bool ok = p != 0xffffffffu;
    if (a.best_mode) a.best_mode[g] = ok ? (uint8_t)(p & 31) : (uint8_t)0xff;
    a.best_cost[g] = ok ? (int32_t)(p >> 5) : kUnavailable;
  }
}

#endif  // !MIP_FOUR_WAVE_TWIN
}  // namespace

static constexpr size_t search_lds_bytes_c(bool alt, bool pf, int waves) {  // (internal: differs per compilation)
  return (size_t)(((pf || waves == kWideWaves) && !alt ? 2 : 1) * kTileElems + (alt ? kLatElems : 0)) * 2 +
         (kTablesInLds ? kTableBytes : 0) + kZeroBytes + (size_t)waves * kWaveStride + kCounterWords * 4;
}
size_t search_lds_bytes(bool alt, bool pf, int waves) {
  const bool two = (pf || waves == kWideWaves) && !alt;  // kOrgTiles
  return (size_t)((two ? 2 : 1) * kTileElems + (alt ? kLatElems : 0)) * 2 + (kTablesInLds ? kTableBytes : 0) + kZeroBytes +
         (size_t)waves * kWaveStride + kCounterWords * 4;
}

static_assert(!MIP_SIX_WAVES || MIP_SIX_WAVES == 2 ||
                  search_lds_bytes_c(false, MIP_PF_KERNEL, kSearchWaves) * 2 <= 160 * 1024, "two workgroups per CU");

template <bool ALT, bool DEC, bool PF, int NW>
static int resident_per_cu() {
  int per_cu = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, mip_search_kernel<ALT, DEC, PF, NW>, 64 * NW,
                                                      search_lds_bytes(ALT, PF, NW)) == hipSuccess ? per_cu : 0;
}

int search_resident_groups(bool alt, bool wide) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  // every variant of a width shares the grid size
  constexpr int S = kSearchWaves, L = kWideWaves;
  int per_cu;
  if (wide && MIP_FOUR_WAVE_TWIN) return 0;
  if (wide && !MIP_FOUR_WAVE_TWIN)
    per_cu = alt ? std::min(resident_per_cu<true, false, false, L>(), resident_per_cu<true, true, false, L>())
                 : std::min(resident_per_cu<false, false, false, L>(), resident_per_cu<false, true, false, L>());
  else
    per_cu = alt ? std::min(resident_per_cu<true, false, false, S>(), resident_per_cu<true, true, false, S>())
                 : std::min({resident_per_cu<false, false, false, S>(), resident_per_cu<false, true, false, S>(),
#if MIP_PREFETCH_MIN_ITEMS < 1000000 && MIP_PF_KERNEL  // (builds that never prefetch: the others' grid)
                             resident_per_cu<false, false, true, S>(), resident_per_cu<false, true, true, S>()
#endif
                             });
  return per_cu >= 1 ? cus * per_cu : 0;
}

hipError_t launch_search(const SearchArgs &args, int nframes, bool alt_refs, int resident, bool wide, hipStream_t s,
                         hipEvent_t done) {
  if (args.slices < 1 || !args.queue || !args.status || resident < 1) return hipErrorInvalidValue;
  SearchArgs a = args;
  if (a.ctu0 < 0 || a.nrange < 1 || a.ctu0 + a.nrange > a.nctus) return hipErrorInvalidValue;
  const long long nitems = (long long)(4 * a.slices) * a.nrange * nframes;
  if (nitems >= 0xffffffffLL) return hipErrorInvalidValue;
  a.nitems = (uint32_t)nitems;
  // XCD chunks of the item queue: only launches with many items per workgroup gain from the
  // locality; in short launches (1-2 1080p frames: ~2 items per workgroup) the chunks' uneven
  // ends cost 3-6 % (one counter: 1 frame 0.198 vs 0.204 ms, 2 frames 0.325 vs 0.343 ms)
  const char *qc = getenv("MIPGPU_QUEUE_CHUNKS");  // tuning knob
  a.chunks = qc && atoi(qc) >= 1 && atoi(qc) <= kQueueChunks
                 ? (uint32_t)atoi(qc)
                 : (a.nitems >= (uint32_t)MIP_PREFETCH_MIN_ITEMS * (uint32_t)resident ? (uint32_t)kQueueChunks : 1u);
  a.nframes = (uint32_t)nframes;
  if (a.chunks > 1 || a.ctu0 != 0 || a.nrange != a.nctus) a.order = nullptr;  // large or range launches
  if (!wide || alt_refs || !a.order || a.chunks != 1 || a.nonempty > a.nitems) a.nonempty = 0;  // pair mode
  const char *env = getenv("MIPGPU_GROUPS");  // tuning knob: persistent grid size
  const int groups = std::min<long long>(env && atoi(env) > 0 ? atoi(env) : resident, a.nitems);
  const bool dec = a.cost == nullptr;
  if (dec && (!a.best_cost || !a.dfill_begin)) return hipErrorInvalidValue;
  const bool pf = kPrefetchKernel && !alt_refs && !wide && a.nitems >= (uint32_t)MIP_PREFETCH_MIN_ITEMS * (uint32_t)groups;
  const size_t lds = search_lds_bytes(alt_refs, pf, wide ? kWideWaves : kSearchWaves);
  const dim3 grid(groups);
  constexpr int S = kSearchWaves, L = kWideWaves;
  (void)L;
  auto go = [&](auto kern, const dim3 &block) {  // with `done`: the dispatch itself records it (no marker packet)
    if (done) hipExtLaunchKernelGGL(kern, grid, block, (uint32_t)lds, s, nullptr, done, 0u, a);
    else hipLaunchKernelGGL(kern, grid, block, lds, s, a);
  };
  if (wide) {
#if MIP_FOUR_WAVE_TWIN
    return hipErrorInvalidValue;  // (the twin serves batched-width launches only)
#else
    const dim3 block(64 * L);
    if (alt_refs) {
      if (dec) go(mip_search_kernel<true, true, false, L>, block);
      else go(mip_search_kernel<true, false, false, L>, block);
    } else {
      if (dec) go(mip_search_kernel<false, true, false, L>, block);
      else go(mip_search_kernel<false, false, false, L>, block);
    }
    return hipGetLastError();
#endif
  }
  const dim3 block(64 * S);
  if (alt_refs) {
    if (dec) go(mip_search_kernel<true, true, false, S>, block);
    else go(mip_search_kernel<true, false, false, S>, block);
  } else if (pf) {
    if (dec) go(mip_search_kernel<false, true, true, S>, block);
    else go(mip_search_kernel<false, false, true, S>, block);
  } else {
    if (dec) go(mip_search_kernel<false, true, false, S>, block);
    else go(mip_search_kernel<false, false, false, S>, block);
  }
  return hipGetLastError();
}

#if !MIP_FOUR_WAVE_TWIN
hipError_t launch_dec_split(const SplitArgs &a, int nframes, bool init, hipStream_t s) {
  if (a.max_split < 1) return hipSuccess;  // no split CUs
  const long long total = (long long)nframes * a.nrange * a.max_split;
  if (!a.best_cost || !a.split || total >= (1LL << 31)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (init) hipLaunchKernelGGL(dec_split_kernel<true>, grid, dim3(256), 0, s, a, (int)total);
  else hipLaunchKernelGGL(dec_split_kernel<false>, grid, dim3(256), 0, s, a, (int)total);
  return hipGetLastError();
}

hipError_t launch_best_modes(const BestArgs &a, hipStream_t s) {
  if (a.k < 1 || a.k > kMaxBestK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(best_mode_kernel, dim3((a.total_cus + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}
#endif  // !MIP_FOUR_WAVE_TWIN

}  // namespace mipgpu
