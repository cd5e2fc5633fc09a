// mip_search.hip -- fused MIP mode search for gfx950 (MI355X).
//
// One kernel does what the reference splits over initBoundaries, MIP_ReducedPred and
// three upsampleDistortion builds (intra.cl:17-1171): boundary downsampling, the MIP
// matrix-vector products, linear upsampling, SAD and 4x4-Hadamard SATD, and the
// min(2*SAD, SATD) cost, without writing any intermediate to HBM (the reference
// round-trips ~1.2 GB of reduced predictions per 1080p frame, main.cpp:443-444).
//
// Work decomposition
//   workgroup = (CTU, slice), 256 threads.  The CTU's samples (+1 row above, +4 columns
//   left) are staged once in LDS; so are the expanded MIP weights.
//   wave      = one WaveTask: 64 lanes of a single CU shape (so every loop bound and
//               branch is wave-uniform).
//   lane      = (CU, mode pair, 4-column strip).  The two modes of a pair travel in the
//               two 16-bit halves of every VGPR, so upsampling, SAD and the Hadamard run
//               as packed int16 VALU ops (v_pk_*) - all intermediates provably fit in
//               16 bits (see the bounds noted at each step).
//   The strip lanes of one (CU, pair) are adjacent; their partial SAD/SATD are reduced
//   with cross-lane shuffles at the end.
//
// Bit-exactness: every arithmetic step restates the reference integer semantics
// (citations inline); tests/test_gpu_parity.py checks the tables bit for bit against the
// C oracle, which is itself pinned to the reference kernels' outputs (tests/golden/).
#include "mip_kernels.h"
#include "mip_tables.h"

namespace mipgpu {
namespace {

typedef short __attribute__((ext_vector_type(2))) s2;
typedef unsigned short __attribute__((ext_vector_type(2))) u2;

__constant__ mip_shape_desc c_shapes[MIP_NUM_SHAPES] = MIP_SHAPE_TABLE;
// Size class of each shape (index into the run_task<W, H> instantiations below).
__constant__ uint8_t c_shape_class[MIP_NUM_SHAPES] = {
    0, 1, 2, 3, 4, 5, 6, 7, 8,                                  // aligned SizeId 2
    2, 3, 4, 4, 5, 5, 6, 6, 6, 7, 7, 7, 7, 7, 8, 8, 8, 8, 8,    // NA SizeId 2
    9, 10, 11, 12, 13, 14, 14, 15, 15,                          // aligned SizeId 1
    11, 12, 13, 13, 13, 13, 13, 14, 15,                         // NA SizeId 1
    16};                                                        // 4x4

constexpr int kPitch = 132;   // LDS row pitch in samples: 66 dwords, rows rotate banks by 2
constexpr int kColOff = 4;    // LDS column of CTU column 0 (columns -4..-1 hold the left halo)
constexpr int kTileElems = (129 * kPitch + 7) / 8 * 8;  // CTU rows -1..127, 16-B multiple
constexpr int kUnavailable = 0x7fffffff;

__device__ __forceinline__ int tidx(int x, int y) { return (y + 1) * kPitch + x + kColOff; }
__device__ __forceinline__ s2 as_s2(uint32_t v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ u2 as_u2(s2 v) { return __builtin_bit_cast(u2, v); }
__device__ __forceinline__ s2 splat(int v) { return s2{(short)v, (short)v}; }
__device__ __forceinline__ s2 smax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ s2 smin(s2 a, s2 b) { return __builtin_elementwise_min(a, b); }

constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v / 2); }

__device__ __forceinline__ int axis_pos(int base, int step, int dual, int i) {
  return dual ? base + (i >> 1) * step + (i & 1) * dual : base + i * step;
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
  static constexpr int WROW = SID == 2 ? 0 : (SID == 1 ? kWeightRowOffS1 : kWeightRowOffS0);
};

struct Tile {
  const uint16_t *org;  // distortion samples
  const uint16_t *ref;  // reference samples (== org unless alternative references)
  const int16_t *w;     // expanded weights
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
  const int v = (acc >> 6) + b0;
  return min(max(v, 0), 1023);
}

// Per-lane state of one (CU, mode pair, strip) evaluation.
template <int W, int H>
struct Lane {
  using G = Geo<W, H>;
  s2 p[4];
  int offset, b0;
  const int16_t *w0, *w1;  // weight rows of the two modes
  bool transposed;

  // Reduced-prediction value of both modes at stored position (k, kx); transposed modes
  // store output j at (j % R, j / R), intra.cl:402-406, 485.
  __device__ __forceinline__ s2 red(int k, int kx) const {
    const int j = transposed ? kx * G::R + k : k * G::R + kx;
    const int a = gemv<G::SID>(p, w0 + j * 8, offset, b0);
    const int b = gemv<G::SID>(p, w1 + j * 8, offset, b0);
    return s2{(short)a, (short)b};
  }
};

// Horizontally upsampled anchor row k (CU row k*UV + UV-1) at the 4 strip columns
// x0..x0+3, intra.cl:816-843: the first UH columns interpolate from the left boundary.
// Values stay in [0, 1023]; (UH-o)*before + o*after + UH/2 <= 8188 fits int16.
template <int W, int H>
__device__ __forceinline__ void anchor_row(const Lane<W, H> &L, int k, int x0, int left_k, s2 (&a)[4]) {
  using G = Geo<W, H>;
  if constexpr (G::UH == 1) {
#pragma unroll
    for (int c = 0; c < 4; c++) a[c] = L.red(k, x0 + c);
  } else if constexpr (G::UH == 2) {
    const int kx = x0 >> 1;  // covers kx, kx+1
    const s2 r0 = L.red(k, kx), r1 = L.red(k, kx + 1);
    const s2 before = kx == 0 ? splat(left_k) : L.red(k, max(kx - 1, 0));
    a[0] = (before + r0 + splat(1)) >> splat(1);
    a[1] = r0;
    a[2] = (r0 + r1 + splat(1)) >> splat(1);
    a[3] = r1;
  } else {
    const int kx = x0 >> G::LH;
    const s2 after = L.red(k, kx);
    const s2 before = kx == 0 ? splat(left_k) : L.red(k, max(kx - 1, 0));
    const s2 delta = after - before;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const int o = ((x0 + c) & (G::UH - 1)) + 1;
      a[c] = before + ((splat(o) * delta + splat(G::UH / 2)) >> splat(G::LH));
    }
  }
}

// SAD and SATD of one 4x4 block for both modes (packed), added to 32-bit accumulators.
// d = orig - pred in [-1023, 1023].  Hadamard intermediates: rows <= 4092, column sums
// <= 8184, DC <= 16368 -- all int16.  SATD per block (kernel_aux_functions.cl:142-249):
//   (sum_k |c_k| - |c_0| + (|c_0| >> 2) + 1) >> 1.
// The last butterfly is folded with |a+b| + |a-b| = 2 max(|a|, |b|), so with T = sum of
// the seven non-DC pair maxima and U = |AC0| + (|DC| >> 2):  satd = T + ((U + 1) >> 1).
// By Parseval (||c||_2 = 4 ||d||_2) satd <= 32736 and T <= satd, so u16 holds both.
// SAD = sum |d| = 2 * sum max(d, 0) - DC, exact in 16 bits for the same reason.
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

// Column butterflies, SATD and SAD of the block, added to the 32-bit accumulators.
__device__ __forceinline__ void block_finish(const BlockAcc &b, uint32_t &sad0, uint32_t &sad1,
                                             uint32_t &satd0, uint32_t &satd1) {
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
  const u2 satd = as_u2(T) + ((U + (u2){1, 1}) >> (u2){1, 1});
  const u2 sad = as_u2(b.pos + b.pos - dc);
  sad0 = __builtin_amdgcn_udot2(sad, (u2){1, 0}, sad0, false);
  sad1 = __builtin_amdgcn_udot2(sad, (u2){0, 1}, sad1, false);
  satd0 = __builtin_amdgcn_udot2(satd, (u2){1, 0}, satd0, false);
  satd1 = __builtin_amdgcn_udot2(satd, (u2){0, 1}, satd1, false);
}

__device__ __forceinline__ uint2 lds_row4(const uint16_t *tile, int x, int y) {
  return *reinterpret_cast<const uint2 *>(tile + tidx(x, y));
}

// Evaluate one WaveTask for a CU shape of size W x H.
template <int W, int H>
__device__ __forceinline__ void run_task(const SearchArgs &a, const Tile &tile, int shape, int job0, int lane,
                         int ctu, int frame, int ctu_x, int ctu_y) {
  using G = Geo<W, H>;
  const mip_shape_desc sd = c_shapes[shape];
  const int modes = sd.modes;             // pairs per CU == modes (2*modes entries)
  const int njobs = sd.ncu * modes;
  int job = job0 + lane / G::S;
  const int sx = lane % G::S, x0 = 4 * sx;
  const bool active = job < njobs;
  if (!active) job = njobs - 1;
  // q-major job order (job = q * ncu + cu): the lanes of a wave share the mode pair, so the
  // weight-row reads of the matrix products broadcast instead of bank-conflicting.
  const int q = job / sd.ncu, cu = job - q * sd.ncu;
  const int cx = axis_pos(sd.xb, sd.xs, sd.xd, cu % sd.ncols);
  const int cy = axis_pos(sd.yb, sd.ys, sd.yd, cu / sd.ncols);
  const int fx = ctu_x + cx, fy = ctu_y + cy;
  const bool avail = fx + W <= a.width && fy + H <= a.height;

  // ---- boundaries, intra.cl:96-107 / 232-243 padding, 71-73 / 127-141 downsampling
  const uint16_t *rt = tile.ref;
  const int padT = fx > 0 ? rt[tidx(cx - 1, cy)] : 512;      // top edge: sample (x-1, 0)
  const int padL = fy > 0 ? rt[tidx(cx, cy - 1)] : 512;      // left edge: sample (0, y-1)
  int redT[G::RBS], redL[G::RBS];
  {
    constexpr int dfT = W / G::RBS, l2T = ilog2c(dfT), rndT = dfT > 1 ? dfT / 2 : 0;
    constexpr int dfL = H / G::RBS, l2L = ilog2c(dfL), rndL = dfL > 1 ? dfL / 2 : 0;
#pragma unroll
    for (int i = 0; i < G::RBS; i++) {
      int s = 0;
      if (dfT >= 4) {
#pragma unroll
        for (int t = 0; t < dfT; t += 4) {
          const uint2 v = lds_row4(rt, cx + i * dfT + t, cy - 1);
          s += (v.x & 0xffff) + (v.x >> 16) + (v.y & 0xffff) + (v.y >> 16);
        }
      } else {
#pragma unroll
        for (int t = 0; t < dfT; t++) s += rt[tidx(cx + i * dfT + t, cy - 1)];
      }
      redT[i] = fy > 0 ? (s + rndT) >> l2T : padT;
      int l = 0;
#pragma unroll
      for (int t = 0; t < dfL; t++) l += rt[tidx(cx - 1, cy + i * dfL + t)];
      redL[i] = fx > 0 ? (l + rndL) >> l2L : padL;
    }
  }

  // ---- MIP input vector, intra.cl:415-454 (pair q: modes 2q, 2q+1; transposed if >= modes)
  Lane<W, H> L;
  const int m0 = 2 * q;
  L.transposed = m0 >= modes;
  const int mw = L.transposed ? m0 - modes : m0;
  {
    int b[8];
#pragma unroll
    for (int i = 0; i < G::RBS; i++) {
      b[i] = L.transposed ? redL[i] : redT[i];
      b[G::RBS + i] = L.transposed ? redT[i] : redL[i];
    }
#pragma unroll
    for (int i = 2 * G::RBS; i < 8; i++) b[i] = b[0];
    L.b0 = b[0];
    int pv[8], psum = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) pv[i] = b[i] - L.b0;
    pv[0] = G::SID == 2 ? 0 : 512 - L.b0;
#pragma unroll
    for (int i = 0; i < 2 * G::RBS; i++) psum += pv[i];
    L.offset = 32 - 32 * psum;
#pragma unroll
    for (int i = 0; i < 4; i++) L.p[i] = s2{(short)pv[2 * i], (short)pv[2 * i + 1]};
  }
  L.w0 = tile.w + (G::WROW + mw * G::NOUT) * 8;
  L.w1 = L.w0 + G::NOUT * 8;

  uint32_t sad0 = 0, sad1 = 0, satd0 = 0, satd1 = 0;
  const uint16_t *ot = tile.org;

  if constexpr (G::SID == 0) {
    // 4x4 CU: the reduced prediction is the prediction (intra.cl:934-936, 995).
    BlockAcc acc;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      s2 prow[4];
#pragma unroll
      for (int c = 0; c < 4; c++) prow[c] = L.red(i, c);
      block_row(acc, i, prow, lds_row4(ot, cx, cy + i));
      __builtin_amdgcn_sched_barrier(0);
    }
    block_finish(acc, sad0, sad1, satd0, satd1);
  } else {
    // ---- walk the strip downwards, 4x4 block by 4x4 block (intra.cl:815-1117)
    s2 prev[4], next[4];
    {
      const uint2 tv = fy > 0 ? lds_row4(rt, cx + x0, cy - 1) : make_uint2(0, 0);
      const int t4[4] = {(int)(tv.x & 0xffff), (int)(tv.x >> 16), (int)(tv.y & 0xffff), (int)(tv.y >> 16)};
#pragma unroll
      for (int c = 0; c < 4; c++) prev[c] = splat(fy > 0 ? t4[c] : padT);  // refT (vertical "before")
    }
    int kcur = -1;
#pragma unroll 1
    for (int by = 0; by < H / 4; by++) {
      BlockAcc acc;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int y = 4 * by + i;
        s2 prow[4];
        if constexpr (G::UV == 1) {
          const int leftv = fx > 0 ? rt[tidx(cx - 1, cy + y)] : padL;
          anchor_row<W, H>(L, y, x0, leftv, prow);
        } else {
          const int k = y >> G::LV;
          if (k != kcur) {  // wave-uniform
            if (kcur >= 0) {
#pragma unroll
              for (int c = 0; c < 4; c++) prev[c] = next[c];
            }
            const int ya = k * G::UV + G::UV - 1;
            const int leftv = fx > 0 ? rt[tidx(cx - 1, cy + ya)] : padL;
            anchor_row<W, H>(L, k, x0, leftv, next);
            kcur = k;
          }
          const int o = (y & (G::UV - 1)) + 1;  // intra.cl:876-891
#pragma unroll
          for (int c = 0; c < 4; c++)
            prow[c] = o == G::UV ? next[c]
                                 : prev[c] + ((splat(o) * (next[c] - prev[c]) + splat(G::UV / 2)) >> splat(G::LV));
        }
        block_row(acc, i, prow, lds_row4(ot, cx + x0, cy + y));
        __builtin_amdgcn_sched_barrier(0);
      }
      block_finish(acc, sad0, sad1, satd0, satd1);
    }
  }

  // ---- combine the strips of one (CU, pair): adjacent lanes, xor-butterfly
#pragma unroll
  for (int off = 1; off < G::S; off <<= 1) {
    sad0 += __shfl_xor(sad0, off);
    sad1 += __shfl_xor(sad1, off);
    satd0 += __shfl_xor(satd0, off);
    satd1 += __shfl_xor(satd1, off);
  }
  if (active && sx == 0) {
    const size_t base = ((size_t)frame * a.nctus + ctu) * MIP_COSTS_PER_CTU + sd.cost_offset +
                        (size_t)cu * 2 * modes + m0;
    const int c0 = avail ? min(2 * (int)sad0, (int)satd0) : kUnavailable;  // intra.cl:1166
    const int c1 = avail ? min(2 * (int)sad1, (int)satd1) : kUnavailable;
    *reinterpret_cast<int2 *>(a.cost + base) = make_int2(c0, c1);
    if (a.sad) *reinterpret_cast<int2 *>(a.sad + base) = avail ? make_int2(sad0, sad1) : make_int2(kUnavailable, kUnavailable);
    if (a.satd) *reinterpret_cast<int2 *>(a.satd + base) = avail ? make_int2(satd0, satd1) : make_int2(kUnavailable, kUnavailable);
  }
}

// Stage a 129 x 132 window (CTU rows -1..127, columns -4..127) of one frame into LDS.
// Samples outside the frame read as 0; they only feed CUs whose results are discarded
// or padding branches that never select them.
__device__ __forceinline__ void stage_tile(uint16_t *dst, const uint16_t *frame, int width, int height,
                                           int ctu_x, int ctu_y) {
  constexpr int kChunks = kPitch / 4;  // 33 chunks of 4 samples per row
  for (int i = threadIdx.x; i < 129 * kChunks; i += blockDim.x) {
    const int row = i / kChunks, ch = i - row * kChunks;
    const int fy = ctu_y - 1 + row, fx = ctu_x - kColOff + 4 * ch;
    uint2 v = make_uint2(0, 0);
    if (fy >= 0 && fy < height && fx >= 0 && fx + 4 <= width)
      v = *reinterpret_cast<const uint2 *>(frame + (size_t)fy * width + fx);
    *reinterpret_cast<uint2 *>(dst + row * kPitch + 4 * ch) = v;
  }
}

template <bool ALT>
__global__ __launch_bounds__(256, 3) void mip_search_kernel(SearchArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t *org = smem;
  uint16_t *ref = ALT ? smem + kTileElems : smem;
  int16_t *w = reinterpret_cast<int16_t *>(smem + (ALT ? 2 : 1) * kTileElems);

  const int slice = blockIdx.x, ctu = blockIdx.y, frame = blockIdx.z;
  const int ctu_x = 128 * (ctu % a.ctu_cols), ctu_y = 128 * (ctu / a.ctu_cols);
  const size_t fofs = (size_t)frame * a.width * a.height;

  stage_tile(org, a.orig + fofs, a.width, a.height, ctu_x, ctu_y);
  if (ALT) stage_tile(ref, a.refs + fofs, a.width, a.height, ctu_x, ctu_y);
  for (int i = threadIdx.x; i < kWeightWords / 8; i += blockDim.x)
    reinterpret_cast<uint4 *>(w)[i] = reinterpret_cast<const uint4 *>(a.weights)[i];
  __syncthreads();

  const Tile tile{org, ref, w};
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int stride = 4 * a.slices;
  for (int t = slice * 4 + wave; t < a.ntasks; t += stride) {
    const WaveTask task = a.tasks[t];
    const int s = task.shape, j0 = task.job0;
    // Shapes share code by size class (17 distinct W x H among the 47 shapes).
    switch (c_shape_class[s]) {
#define MIP_CASE(idx, W, H) \
  case idx: run_task<W, H>(a, tile, s, j0, lane, ctu, frame, ctu_x, ctu_y); break;
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

size_t search_lds_bytes(bool alt) { return ((alt ? 2 : 1) * kTileElems + kWeightWords) * 2; }

hipError_t launch_search(const SearchArgs &a, int nframes, bool alt_refs, hipStream_t s) {
  const dim3 grid(a.slices, a.nctus, nframes);
  const size_t lds = search_lds_bytes(alt_refs);
  if (alt_refs)
    hipLaunchKernelGGL(mip_search_kernel<true>, grid, dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL(mip_search_kernel<false>, grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_best_modes(const BestArgs &a, hipStream_t s) {
  hipLaunchKernelGGL(best_mode_kernel, dim3((a.total_cus + 255) / 256), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace mipgpu
