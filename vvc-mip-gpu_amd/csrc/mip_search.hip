// mip_search.hip -- fused MIP mode search for gfx950 (MI355X).
//
// One kernel does what the reference splits over initBoundaries, MIP_ReducedPred and
// three upsampleDistortion builds (intra.cl:17-1171): boundary downsampling, the MIP
// matrix-vector products, linear upsampling, SAD and 4x4-Hadamard SATD and the
// min(2*SAD, SATD) cost -- without any intermediate in HBM (the reference round-trips
// ~1.2 GB of reduced predictions per 1080p frame, main.cpp:443-444).
//
// Work decomposition
//   workgroup = (CTU quadrant, slice), kWaves waves.  No CU of the 47 shapes straddles a
//               64x64 quadrant, so a workgroup stages only its quadrant (+1 row above,
//               +4 columns left: the reference samples) in LDS, 8.8 KB.
//   wave      = one WaveTask: up to 64/S jobs (CU, mode pair) of ONE shape, so every
//               loop bound and branch is wave-uniform.
//   lane      = (job, 4-column strip).  The two modes of a pair travel in the two 16-bit
//               halves of each VGPR: upsampling, SAD and the Hadamard are packed int16
//               VALU ops (v_pk_*); all intermediates provably fit 16 bits (bounds inline).
//   Phase A   (shapes whose strips share reduced-prediction values, W > R): the wave
//               computes each job's reduced prediction once (v_dot2_i32_i16) into a
//               wave-private LDS scratch in the reference's stored order.
//   Phase B   every lane walks its strip 4x4 block by 4x4 block: anchors (horizontal
//               pass), vertical interpolation, SAD and SATD; strips of one job are adjacent
//               lanes and are combined with xor shuffles.  Shapes with W == R (no sharing)
//               compute their matrix products directly in phase B.
//
// Bit-exactness: every step restates the reference integer semantics (citations inline);
// tests/test_gpu_parity.py checks the tables bit for bit against the C oracle, which is
// pinned to the reference kernels' own outputs (tests/golden/).
#include "mip_kernels.h"
#include "mip_tables.h"

namespace mipgpu {
namespace {

typedef short __attribute__((ext_vector_type(2))) s2;
typedef unsigned short __attribute__((ext_vector_type(2))) u2;

__constant__ mip_shape_desc c_shapes[MIP_NUM_SHAPES] = MIP_SHAPE_TABLE;
// Size class of each shape (index into the run_task<W, H> instantiations).
__constant__ uint8_t c_shape_class[MIP_NUM_SHAPES] = {
    0, 1, 2, 3, 4, 5, 6, 7, 8,                                  // aligned SizeId 2
    2, 3, 4, 4, 5, 5, 6, 6, 6, 7, 7, 7, 7, 7, 8, 8, 8, 8, 8,    // NA SizeId 2
    9, 10, 11, 12, 13, 14, 14, 15, 15,                          // aligned SizeId 1
    11, 12, 13, 13, 13, 13, 13, 14, 15,                         // NA SizeId 1
    16};                                                        // 4x4

constexpr int kWaves = 8;        // waves per workgroup
constexpr int kPitch = 68;       // LDS row pitch in samples (34 dwords: conflict-free rows)
constexpr int kColOff = 4;       // LDS column of quadrant column 0 (-4..-1: left halo)
constexpr int kTileElems = (65 * kPitch + 7) / 8 * 8;  // quadrant rows -1..63
constexpr int kJobWords = 8;     // job-table entry (dwords)
constexpr int kScratchWords = 16 * 65;                  // 16 jobs x (64 + 1) packed pairs
constexpr int kWaveWords = 64 * kJobWords + kScratchWords;
constexpr int kUnavailable = 0x7fffffff;

__device__ __forceinline__ int tidx(int x, int y) { return (y + 1) * kPitch + x + kColOff; }
__device__ __forceinline__ s2 as_s2(uint32_t v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ u2 as_u2(s2 v) { return __builtin_bit_cast(u2, v); }
__device__ __forceinline__ s2 as_s2(u2 v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ uint32_t as_u32(s2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ s2 splat(int v) { return s2{(short)v, (short)v}; }
__device__ __forceinline__ s2 smax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ s2 smin(s2 a, s2 b) { return __builtin_elementwise_min(a, b); }

constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v / 2); }

// LDS fence for data handed between lanes of ONE wave (wave-private scratch).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Compile-time geometry of a CU shape (W x H).
template <int W, int H>
struct Geo {
  static constexpr int SID = (W == 4 && H == 4) ? 0 : ((W == 4 || H == 4 || (W == 8 && H == 8)) ? 1 : 2);
  static constexpr int R = SID == 2 ? 8 : 4;          // reduced prediction side
  static constexpr int RBS = SID == 0 ? 2 : 4;        // reduced boundary length per side
  static constexpr int NOUT = R * R;
  static constexpr int UH = W / R, UV = H / R;        // upsampling factors
  static constexpr int LH = ilog2c(UH), LV = ilog2c(UV);
  static constexpr int S = W / 4;                     // strips per CU
  static constexpr bool DIRECT = UH == 1;             // no reduced value shared by strips
};

// Matrix-vector product of one mode for output j, intra.cl:449-482: ((offset + p.w) >> 6)
// + b0, clipped to 10 bits.  All operands are small integers, v_dot2_i32_i16 is exact.
template <int SID>
__device__ __forceinline__ int gemv(const s2 (&p)[4], const int16_t *wrow, int offset, int b0) {
  int acc = offset;
  if (SID == 0) {
    const uint2 w = *reinterpret_cast<const uint2 *>(wrow);
    acc = __builtin_amdgcn_sdot2(p[0], as_s2(w.x), acc, false);
    acc = __builtin_amdgcn_sdot2(p[1], as_s2(w.y), acc, false);
  } else {
    const uint4 w = *reinterpret_cast<const uint4 *>(wrow);
    acc = __builtin_amdgcn_sdot2(p[0], as_s2(w.x), acc, false);
    acc = __builtin_amdgcn_sdot2(p[1], as_s2(w.y), acc, false);
    acc = __builtin_amdgcn_sdot2(p[2], as_s2(w.z), acc, false);
    acc = __builtin_amdgcn_sdot2(p[3], as_s2(w.w), acc, false);
  }
  return min(max((acc >> 6) + b0, 0), 1023);
}

// MIP inputs of one job: packed p vector, offset, b0, weight rows of its two modes.
struct MipIn {
  s2 p[4];
  int offset, b0;
  int wrow;        // first weight row (16-B rows) of mode 2q mod modes (Job::wrow)
  bool transposed;
};

// Per-CU geometry + boundary padding, quadrant-relative.
struct CuPos {
  int lx, ly;      // CU origin inside the quadrant
  bool top, left;  // reference row above / column left lies inside the frame
  int padT, padL;  // padding values, intra.cl:102-106, 238-242
};

__device__ __forceinline__ uint2 lds_row4(const uint16_t *tile, int x, int y) {
  return *reinterpret_cast<const uint2 *>(tile + tidx(x, y));
}

__device__ __forceinline__ CuPos cu_pos(const Job &j, int ctu_x, int ctu_y, int qx, int qy, const uint16_t *rt) {
  CuPos c;
  c.lx = j.lx;
  c.ly = j.ly;
  c.top = ctu_y + qy + c.ly > 0;
  c.left = ctu_x + qx + c.lx > 0;
  c.padT = c.left ? rt[tidx(c.lx - 1, c.ly)] : 512;   // top edge: sample (x-1, 0)
  c.padL = c.top ? rt[tidx(c.lx, c.ly - 1)] : 512;    // left edge: sample (0, y-1)
  return c;
}

// Reduced boundaries and MIP input vector of one job, intra.cl:71-73, 127-141, 202-204,
// 259-279 (box downsampling; a factor of 1 is a copy) and intra.cl:415-454.
template <int W, int H>
__device__ __forceinline__ MipIn mip_inputs(const CuPos &c, uint32_t wrow, const uint16_t *rt) {
  using G = Geo<W, H>;
  constexpr int dfT = W / G::RBS, l2T = ilog2c(dfT), rndT = dfT > 1 ? dfT / 2 : 0;
  constexpr int dfL = H / G::RBS, l2L = ilog2c(dfL), rndL = dfL > 1 ? dfL / 2 : 0;
  int redT[G::RBS], redL[G::RBS];
#pragma unroll
  for (int i = 0; i < G::RBS; i++) {
    int s = 0;
    if constexpr (dfT >= 4) {
#pragma unroll
      for (int t = 0; t < dfT; t += 4) {
        const uint2 v = lds_row4(rt, c.lx + i * dfT + t, c.ly - 1);
        s += (v.x & 0xffff) + (v.x >> 16) + (v.y & 0xffff) + (v.y >> 16);
      }
    } else {
#pragma unroll
      for (int t = 0; t < dfT; t++) s += rt[tidx(c.lx + i * dfT + t, c.ly - 1)];
    }
    redT[i] = c.top ? (s + rndT) >> l2T : c.padT;
    int l = 0;
#pragma unroll
    for (int t = 0; t < dfL; t++) l += rt[tidx(c.lx - 1, c.ly + i * dfL + t)];
    redL[i] = c.left ? (l + rndL) >> l2L : c.padL;
  }
  MipIn m;
  m.transposed = (wrow & kJobTransposed) != 0;
  m.wrow = wrow & ~(uint32_t)kJobTransposed;
  int b[8];
#pragma unroll
  for (int i = 0; i < G::RBS; i++) {
    b[i] = m.transposed ? redL[i] : redT[i];
    b[G::RBS + i] = m.transposed ? redT[i] : redL[i];
  }
#pragma unroll
  for (int i = 2 * G::RBS; i < 8; i++) b[i] = b[0];
  m.b0 = b[0];
  int pv[8], psum = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) pv[i] = b[i] - m.b0;
  pv[0] = G::SID == 2 ? 0 : 512 - m.b0;  // intra.cl:446
#pragma unroll
  for (int i = 0; i < 2 * G::RBS; i++) psum += pv[i];
  m.offset = 32 - 32 * psum;             // intra.cl:449-454
#pragma unroll
  for (int i = 0; i < 4; i++) m.p[i] = s2{(short)pv[2 * i], (short)pv[2 * i + 1]};
  return m;
}

// Both modes of a pair at stored reduced position (k, kx); transposed modes store output
// j at (j % R, j / R), intra.cl:402-406, 485.
template <int W, int H>
__device__ __forceinline__ s2 red_direct(const MipIn &m, const int16_t *w, int k, int kx) {
  using G = Geo<W, H>;
  const int j = m.transposed ? kx * G::R + k : k * G::R + kx;
  const int a = gemv<G::SID>(m.p, w + (m.wrow + j) * 8, m.offset, m.b0);
  const int b = gemv<G::SID>(m.p, w + (m.wrow + G::NOUT + j) * 8, m.offset, m.b0);
  return s2{(short)a, (short)b};
}

struct BlockAcc {
  s2 t[16];  // row-transformed residual
  s2 pos;    // sum of max(d, 0)
};

// One residual row of a 4x4 block: d = orig - pred, positive-part sum, row butterflies.
__device__ __forceinline__ void block_row(BlockAcc &b, int i, const s2 (&prow)[4], uint2 orow) {
  const s2 o01 = as_s2(orow.x), o23 = as_s2(orow.y);
  const s2 d0 = s2{o01.x, o01.x} - prow[0], d1 = s2{o01.y, o01.y} - prow[1];
  const s2 d2 = s2{o23.x, o23.x} - prow[2], d3 = s2{o23.y, o23.y} - prow[3];
  const s2 p = smax(d0, splat(0)) + smax(d1, splat(0)) + smax(d2, splat(0)) + smax(d3, splat(0));
  b.pos = i == 0 ? p : b.pos + p;
  const s2 s0 = d0 + d1, s1 = d0 - d1, s2_ = d2 + d3, s3 = d2 - d3;
  b.t[4 * i + 0] = s0 + s2_;
  b.t[4 * i + 1] = s1 + s3;
  b.t[4 * i + 2] = s0 - s2_;
  b.t[4 * i + 3] = s1 - s3;
}

// SAD and SATD of the block for both modes (packed 16-bit).
// d = orig - pred in [-1023, 1023].  Hadamard intermediates: rows <= 4092, column sums
// <= 8184, DC <= 16368 -- all int16.  SATD per block (kernel_aux_functions.cl:142-249):
//   (sum_k |c_k| - |c_0| + (|c_0| >> 2) + 1) >> 1.
// The last butterfly is folded with |a+b| + |a-b| = 2 max(|a|, |b|), so with T = sum of
// the seven non-DC pair maxima and U = |AC0| + (|DC| >> 2):  satd = T + ((U + 1) >> 1).
// By Parseval (||c||_2 = 4 ||d||_2) satd <= 32736 and T <= satd, so u16 holds both.
// SAD = sum |d| = 2 * sum max(d, 0) - DC <= 16368, exact in 16 bits for the same reason.
__device__ __forceinline__ void block_finish(const BlockAcc &b, u2 &sad, u2 &satd) {
  s2 T = splat(0), dc = splat(0), ac = splat(0);
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const s2 u0 = b.t[c] + b.t[4 + c], u1 = b.t[c] - b.t[4 + c];
    const s2 u2_ = b.t[8 + c] + b.t[12 + c], u3 = b.t[8 + c] - b.t[12 + c];
    if (c == 0) {
      dc = u0 + u2_;
      ac = u0 - u2_;
    } else {
      T += smax(smax(u0, u2_), splat(0) - smin(u0, u2_));
    }
    T += smax(smax(u1, u3), splat(0) - smin(u1, u3));
  }
  const s2 adc = smax(dc, splat(0) - dc), aac = smax(ac, splat(0) - ac);
  const u2 U = as_u2(aac) + (as_u2(adc) >> (u2){2, 2});
  satd = as_u2(T) + ((U + (u2){1, 1}) >> (u2){1, 1});
  sad = as_u2(b.pos + b.pos - dc);
}

// Packed block results -> 32-bit per-mode accumulators.
struct Acc {
  uint32_t sad0 = 0, sad1 = 0, satd0 = 0, satd1 = 0;
  __device__ __forceinline__ void add(u2 sad, u2 satd) {
    sad0 = __builtin_amdgcn_udot2(sad, (u2){1, 0}, sad0, false);
    sad1 = __builtin_amdgcn_udot2(sad, (u2){0, 1}, sad1, false);
    satd0 = __builtin_amdgcn_udot2(satd, (u2){1, 0}, satd0, false);
    satd1 = __builtin_amdgcn_udot2(satd, (u2){0, 1}, satd1, false);
  }
};

struct Ctx {
  const SearchArgs *a;
  const uint16_t *org, *ref;  // quadrant tiles (distortion / reference samples)
  const int16_t *w;           // expanded weights (LDS)
  uint32_t *wave;             // wave-private LDS: job table + reduced-prediction scratch
  int ctu, frame, ctu_x, ctu_y, qx, qy;  // qx, qy: quadrant origin inside the CTU
};

// Horizontal pass of anchor row k (CU row k*UV + UV-1) at strip columns x0..x0+3,
// intra.cl:816-843; the first UH columns interpolate from the left boundary sample.
// ((UH-o)*before + o*after + UH/2) >> LH == (base + o*delta) >> LH with
// base = (before << LH) + UH/2; the sum equals the reference numerator, in [0, 8188].
template <int W, int H, class RED>
__device__ __forceinline__ void anchor_row(const RED &red, int k, int x0, int left_k, s2 (&a)[4]) {
  using G = Geo<W, H>;
  if constexpr (G::UH == 1) {
#pragma unroll
    for (int c = 0; c < 4; c++) a[c] = red(k, x0 + c);
  } else if constexpr (G::UH == 2) {
    const int kx = x0 >> 1;  // covers kx, kx+1
    const s2 r0 = red(k, kx), r1 = red(k, kx + 1);
    const s2 before = kx == 0 ? splat(left_k) : red(k, max(kx - 1, 0));
    a[0] = (before + r0 + splat(1)) >> splat(1);
    a[1] = r0;
    a[2] = (r0 + r1 + splat(1)) >> splat(1);
    a[3] = r1;
  } else {
    const int kx = x0 >> G::LH;
    const s2 after = red(k, kx);
    const s2 before = kx == 0 ? splat(left_k) : red(k, max(kx - 1, 0));
    const s2 delta = after - before;
    const s2 base = (before << splat(G::LH)) + splat(G::UH / 2);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int o = ((x0 + c) & (G::UH - 1)) + 1;
      a[c] = (splat(o) * delta + base) >> splat(G::LH);
    }
  }
}

// Walk one strip of one job: prediction rows (upsampling, intra.cl:815-912) streamed
// through the block transform.  The loops follow the upsampling windows, so every
// interpolation weight is a compile-time constant (or a wave-uniform loop index).
template <int W, int H, class RED>
__device__ __forceinline__ void walk_strip(const Ctx &x, const CuPos &c, const RED &red, int x0, Acc &acc) {
  using G = Geo<W, H>;
  const uint16_t *rt = x.ref, *ot = x.org;
  auto left_at = [&](int y) { return c.left ? (int)rt[tidx(c.lx - 1, c.ly + y)] : c.padL; };
  auto orow = [&](int y) { return lds_row4(ot, c.lx + x0, c.ly + y); };
  if constexpr (G::SID == 0) {
    // 4x4 CU: the reduced prediction is the prediction (intra.cl:934-936, 995).
    BlockAcc b;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      s2 prow[4];
#pragma unroll
      for (int cc = 0; cc < 4; cc++) prow[cc] = red(i, cc);
      block_row(b, i, prow, orow(i));
    }
    u2 sad, satd;
    block_finish(b, sad, satd);
    acc.add(sad, satd);
  } else if constexpr (G::UV == 1) {
    // every row is an anchor row (horizontal pass only)
#pragma unroll 1
    for (int by = 0; by < H / 4; by++) {
      BlockAcc b;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        s2 prow[4];
        anchor_row<W, H>(red, 4 * by + i, x0, left_at(4 * by + i), prow);
        block_row(b, i, prow, orow(4 * by + i));
      }
      u2 sad, satd;
      block_finish(b, sad, satd);
      acc.add(sad, satd);
    }
  } else {
    // Vertical pass (intra.cl:867-893): row o (1..UV) of window k interpolates between
    // anchor k-1 (or the top boundary) and anchor k: (base + o*delta) >> LV with
    // base = (prev << LV) + UV/2, the reference numerator, in [0, 8188]; o = UV gives the
    // anchor itself.  16-bit wrap-around in o*delta cancels in the in-range sum.
    s2 prev[4];
    {
      const uint2 tv = lds_row4(rt, c.lx + x0, c.ly - 1);
      const int t4[4] = {(int)(tv.x & 0xffff), (int)(tv.x >> 16), (int)(tv.y & 0xffff), (int)(tv.y >> 16)};
#pragma unroll
      for (int cc = 0; cc < 4; cc++) prev[cc] = splat(c.top ? t4[cc] : c.padT);
    }
    if constexpr (G::UV == 2) {
      // two windows per 4x4 block
#pragma unroll 1
      for (int by = 0; by < H / 4; by++) {
        BlockAcc b;
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const int k = 2 * by + h;
          s2 next[4], mid[4];
          anchor_row<W, H>(red, k, x0, left_at(2 * k + 1), next);
#pragma unroll
          for (int cc = 0; cc < 4; cc++) mid[cc] = as_s2((as_u2(prev[cc]) + as_u2(next[cc]) + (u2){1, 1}) >> (u2){1, 1});
          block_row(b, 2 * h, mid, orow(2 * k));
          block_row(b, 2 * h + 1, next, orow(2 * k + 1));
#pragma unroll
          for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
        }
        u2 sad, satd;
        block_finish(b, sad, satd);
        acc.add(sad, satd);
      }
    } else {
      constexpr int NB = G::UV / 4;  // blocks per window
#pragma unroll 1
      for (int k = 0; k < G::R; k++) {
        s2 next[4];
        anchor_row<W, H>(red, k, x0, left_at(k * G::UV + G::UV - 1), next);
        u2 delta[4], base[4];
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
          delta[cc] = as_u2(next[cc]) - as_u2(prev[cc]);
          base[cc] = (as_u2(prev[cc]) << (u2){G::LV, G::LV}) + (u2){G::UV / 2, G::UV / 2};
        }
#pragma unroll 2
        for (int bi = 0; bi < NB; bi++) {
          BlockAcc b;
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const unsigned short o = (unsigned short)(4 * bi + i + 1);
            s2 prow[4];
#pragma unroll
            for (int cc = 0; cc < 4; cc++) prow[cc] = as_s2(((u2){o, o} * delta[cc] + base[cc]) >> (u2){G::LV, G::LV});
            block_row(b, i, prow, orow(k * G::UV + 4 * bi + i));
          }
          u2 sad, satd;
          block_finish(b, sad, satd);
          acc.add(sad, satd);
        }
#pragma unroll
        for (int cc = 0; cc < 4; cc++) prev[cc] = next[cc];
      }
    }
  }
}

template <int W, int H>
__device__ __forceinline__ void run_task(const Ctx &x, const WaveTask &task, int lane) {
  using G = Geo<W, H>;
  const SearchArgs &a = *x.a;
  const int nj = task.njobs;
  const Job *jobs = a.jobs + task.job0;
  const int jl = lane / G::S, sx = lane - jl * G::S, x0 = 4 * sx;
  const bool active = jl < nj;
  const Job job = jobs[min(jl, nj - 1)];
  const CuPos c = cu_pos(job, x.ctu_x, x.ctu_y, x.qx, x.qy, x.ref);
  Acc acc;

  if constexpr (G::DIRECT) {
    const MipIn m = mip_inputs<W, H>(c, job.wrow, x.ref);
    auto red = [&](int k, int kx) { return red_direct<W, H>(m, x.w, k, kx); };
    walk_strip<W, H>(x, c, red, x0, acc);
  } else {
    // ---- phase A: each job's reduced prediction once, into the wave's scratch
    uint32_t *table = x.wave;
    uint32_t *scr = x.wave + 64 * kJobWords;
    constexpr int kStride = G::NOUT + 1;  // +1 dword: different jobs hit different banks
    if (lane < nj) {
      const Job jb = jobs[lane];
      const CuPos cj = cu_pos(jb, x.ctu_x, x.ctu_y, x.qx, x.qy, x.ref);
      const MipIn m = mip_inputs<W, H>(cj, jb.wrow, x.ref);
      uint4 *e = reinterpret_cast<uint4 *>(table + lane * kJobWords);
      e[0] = make_uint4(as_u32(m.p[0]), as_u32(m.p[1]), as_u32(m.p[2]), as_u32(m.p[3]));
      e[1] = make_uint4((uint32_t)m.offset, (uint32_t)m.b0, (uint32_t)m.wrow, (uint32_t)m.transposed);
    }
    wave_lds_sync();
    const int total = nj * G::NOUT;
#pragma unroll 1
    for (int o = lane; o < ((total + 63) & ~63); o += 64) {
      const int jb = min(o / G::NOUT, nj - 1), j = o % G::NOUT;
      const uint4 *e = reinterpret_cast<const uint4 *>(table + jb * kJobWords);
      const uint4 e0 = e[0], e1 = e[1];
      const s2 p[4] = {as_s2(e0.x), as_s2(e0.y), as_s2(e0.z), as_s2(e0.w)};
      const int off = (int)e1.x, b0 = (int)e1.y, wrow = (int)e1.z;
      const int v0 = gemv<G::SID>(p, x.w + (wrow + j) * 8, off, b0);
      const int v1 = gemv<G::SID>(p, x.w + (wrow + G::NOUT + j) * 8, off, b0);
      const int pos = e1.w ? (j % G::R) * G::R + j / G::R : j;
      if (o < total) scr[jb * kStride + pos] = (uint32_t)v0 | ((uint32_t)v1 << 16);
    }
    wave_lds_sync();
    // ---- phase B
    const uint32_t *mine = scr + min(jl, nj - 1) * kStride;
    auto red = [&](int k, int kx) { return as_s2(mine[k * G::R + kx]); };
    walk_strip<W, H>(x, c, red, x0, acc);
    wave_lds_sync();  // scratch and table are reused by the next task
  }

  // ---- combine the strips of one job: adjacent lanes, xor butterfly
#pragma unroll
  for (int off = 1; off < G::S; off <<= 1) {
    acc.sad0 += __shfl_xor(acc.sad0, off);
    acc.sad1 += __shfl_xor(acc.sad1, off);
    acc.satd0 += __shfl_xor(acc.satd0, off);
    acc.satd1 += __shfl_xor(acc.satd1, off);
  }
  if (active && sx == 0) {
    const int fx = x.ctu_x + x.qx + c.lx, fy = x.ctu_y + x.qy + c.ly;
    const bool avail = fx + W <= a.width && fy + H <= a.height;
    const size_t idx = ((size_t)x.frame * a.nctus + x.ctu) * MIP_COSTS_PER_CTU + job.cost;
    const int c0 = avail ? min(2 * (int)acc.sad0, (int)acc.satd0) : kUnavailable;  // intra.cl:1166
    const int c1 = avail ? min(2 * (int)acc.sad1, (int)acc.satd1) : kUnavailable;
    *reinterpret_cast<int2 *>(a.cost + idx) = make_int2(c0, c1);
    if (a.sad)
      *reinterpret_cast<int2 *>(a.sad + idx) = avail ? make_int2(acc.sad0, acc.sad1) : make_int2(kUnavailable, kUnavailable);
    if (a.satd)
      *reinterpret_cast<int2 *>(a.satd + idx) = avail ? make_int2(acc.satd0, acc.satd1) : make_int2(kUnavailable, kUnavailable);
  }
}

// Stage the quadrant window (rows -1..63, columns -4..63) of one frame into LDS.  Samples
// outside the frame read as 0; they only feed CUs whose results are discarded or padding
// branches that never select them.
__device__ __forceinline__ void stage_tile(uint16_t *dst, const uint16_t *frame, int width, int height,
                                           int x0, int y0) {
  constexpr int kChunks = kPitch / 4;  // 17 chunks of 4 samples per row
  for (int i = threadIdx.x; i < 65 * kChunks; i += blockDim.x) {
    const int row = i / kChunks, ch = i - row * kChunks;
    const int fy = y0 - 1 + row, fx = x0 - kColOff + 4 * ch;
    uint2 v = make_uint2(0, 0);
    if (fy >= 0 && fy < height && fx >= 0 && fx + 4 <= width)
      v = *reinterpret_cast<const uint2 *>(frame + (size_t)fy * width + fx);
    *reinterpret_cast<uint2 *>(dst + row * kPitch + 4 * ch) = v;
  }
}

template <bool ALT>
__global__ __launch_bounds__(64 * kWaves, 4) void mip_search_kernel(SearchArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t *org = smem;
  uint16_t *ref = ALT ? smem + kTileElems : smem;
  int16_t *w = reinterpret_cast<int16_t *>(smem + (ALT ? 2 : 1) * kTileElems);
  uint32_t *waves = reinterpret_cast<uint32_t *>(w + kWeightWords);

  const int slice = blockIdx.x % a.slices, quad = blockIdx.x / a.slices;
  const int ctu = blockIdx.y, frame = blockIdx.z;
  const int ctu_x = 128 * (ctu % a.ctu_cols), ctu_y = 128 * (ctu / a.ctu_cols);
  const int qx = 64 * (quad & 1), qy = 64 * (quad >> 1);
  const size_t fofs = (size_t)frame * a.width * a.height;

  stage_tile(org, a.orig + fofs, a.width, a.height, ctu_x + qx, ctu_y + qy);
  if (ALT) stage_tile(ref, a.refs + fofs, a.width, a.height, ctu_x + qx, ctu_y + qy);
  for (int i = threadIdx.x; i < kWeightWords / 8; i += blockDim.x)
    reinterpret_cast<uint4 *>(w)[i] = reinterpret_cast<const uint4 *>(a.weights)[i];
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const Ctx x{&a, org, ref, w, waves + wave * kWaveWords, ctu, frame, ctu_x, ctu_y, qx, qy};
  const int t0 = a.task_begin[quad], t1 = a.task_begin[quad + 1];
  for (int t = t0 + slice * kWaves + wave; t < t1; t += kWaves * a.slices) {
    const WaveTask task = a.tasks[t];
    switch (c_shape_class[task.shape]) {
#define MIP_CASE(idx, W, H) \
  case idx: run_task<W, H>(x, task, lane); break;
      MIP_CASE(0, 64, 64) MIP_CASE(1, 32, 32) MIP_CASE(2, 32, 16) MIP_CASE(3, 16, 32)
      MIP_CASE(4, 32, 8) MIP_CASE(5, 8, 32) MIP_CASE(6, 16, 16) MIP_CASE(7, 16, 8)
      MIP_CASE(8, 8, 16) MIP_CASE(9, 32, 4) MIP_CASE(10, 4, 32) MIP_CASE(11, 16, 4)
      MIP_CASE(12, 4, 16) MIP_CASE(13, 8, 8) MIP_CASE(14, 8, 4) MIP_CASE(15, 4, 8)
      MIP_CASE(16, 4, 4)
#undef MIP_CASE
      default: break;
    }
  }
}

// Per-CU argmin over the cost row (lowest mode wins ties); 0xff for unavailable CUs.
__global__ __launch_bounds__(256) void best_mode_kernel(BestArgs a) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.total_cus) return;
  const int ctu = g / MIP_CUS_PER_CTU;
  int r = g - ctu * MIP_CUS_PER_CTU, s = 0;
  while (r >= c_shapes[s].ncu) r -= c_shapes[s++].ncu;
  const mip_shape_desc sd = c_shapes[s];
  const int32_t *row = a.cost + (size_t)ctu * MIP_COSTS_PER_CTU + sd.cost_offset + (size_t)r * 2 * sd.modes;
  int best = 0, bc = row[0];
  for (int m = 1; m < 2 * sd.modes; m++)
    if (row[m] < bc) bc = row[m], best = m;
  if (a.best_mode) a.best_mode[g] = bc == kUnavailable ? 0xff : (uint8_t)best;
  if (a.best_cost) a.best_cost[g] = bc;
}

}  // namespace

size_t search_lds_bytes(bool alt) {
  return ((alt ? 2 : 1) * kTileElems + kWeightWords) * 2 + (size_t)kWaves * kWaveWords * 4;
}

hipError_t launch_search(const SearchArgs &a, int nframes, bool alt_refs, hipStream_t s) {
  if (a.slices < 1) return hipErrorInvalidValue;
  const dim3 grid(4 * a.slices, a.nctus, nframes);
  const size_t lds = search_lds_bytes(alt_refs);
  if (alt_refs)
    hipLaunchKernelGGL(mip_search_kernel<true>, grid, dim3(64 * kWaves), lds, s, a);
  else
    hipLaunchKernelGGL(mip_search_kernel<false>, grid, dim3(64 * kWaves), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_best_modes(const BestArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(best_mode_kernel, dim3((a.total_cus + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace mipgpu
