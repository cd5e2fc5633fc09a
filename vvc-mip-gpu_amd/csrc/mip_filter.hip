// mip_filter.hip -- LDS-tiled low-pass filters of the reference samples (gfx950).
//
// All eight reference filters work per 128x32 quarter-CTU tile plus a 1- or 2-sample halo,
// because the reference's halo gates are defined per tile; so does this kernel (one
// 128-thread workgroup per tile; HBM-bound: one read and one write of the frame).
//  * 2-D (filterFrame_2d_{int,float}[_5x5]_quarterCtu, intra.cl:2856, 1639, 3042, 2311):
//    a halo cell is loaded when the reference would load it (tap_valid) and marked invalid
//    (-1) otherwise; each output is the normalised convolution over its valid taps.
//  * separable (filterFrame_1d_{int,float}[_5x5], intra.cl:3267, 1828, 3508, 2539): row 0
//    of the 2-D kernel applied horizontally (halo rows included) and then vertically, with
//    the reference's fetch conditions (sep_fetch) and its position-class scales
//    (oracle/mip_oracle.c filter_1d_tile3/5 documents the rules).
//
// One computation serves both: every kernel of the library is t (x) t + d * delta, with t =
// row 0 of the 2-D kernel and d the centre excess (tests/test_tables.py checks this), so
//    numerator = sum_i t_i * sum_j t_j * max(v_ij, 0)  (+ d * centre for the 2-D filters)
// is a horizontal pass in packed 16-bit lanes (4 columns per thread, v_pk_mad_u16; sums <=
// 9 * 1023) followed by a vertical v_dot2 pass.  The 2-D scale is the full kernel sum
// minus the same separable pass over the invalid-cell indicator (only in tiles that have
// an invalid cell: frame borders and the reference's stricter halo gates); the separable
// scale is the reference's closed-form position class.
// Rounding: int (sum + scale/2) / scale (exact multiply-high for the uniform scale);
// float round(sum * R(scale)) where R(s) = ldexp(rcp(frexp_mant(s)), -frexp_exp(s)) --
// exactly the reference's own fp32 division sequence (frexp, v_rcp_f32, v_mul, v_ldexp:
// the AMD OpenCL lowering of '/', read from the reference's code objects), since scaling
// by a power of two commutes with the multiply's rounding.
#include <algorithm>

#include "mip_kernels.h"
#include "mip_tables.h"

namespace mipgpu {
namespace {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef unsigned short u2 __attribute__((ext_vector_type(2)));

// Threads per tile: thread t owns columns 4(t&31).. +3 and 1024/NT rows from (1024/NT)(t>>5).
// Separable filters: 64 (one wave, 16 rows per thread: each thread's horizontal passes of
// the 2 RAD halo rows serve 16 output rows instead of 8); 2-D filters: 128 (384 x 1080p, one
// box, two reps: separable 3 taps 0.679 -> 0.638 ms, 5 taps 0.680-0.707 -> 0.640-0.657 ms,
// 2-D unchanged; 256 threads slower throughout; profiles/r06_filter_threads.txt).
// MIP_FILTER_THREADS (A/B): one count for all eight.
#ifndef MIP_FILTER_THREADS
#define MIP_FILTER_THREADS 0
#endif
template <bool SEP>
constexpr int kThreadsOf = MIP_FILTER_THREADS ? MIP_FILTER_THREADS : (SEP ? 64 : 128);
#ifndef MIP_FILTER_TPW
#define MIP_FILTER_TPW 1
#endif
constexpr int kTPW = MIP_FILTER_TPW;  // tiles per workgroup (128 threads each); 2 and 4 measured slower
#ifndef MIP_FILTER_NT
#define MIP_FILTER_NT 1  // filtered samples stored non-temporally (streamed out, -3 % time)
#endif
constexpr int kCO = 8;         // LDS column of tile column 0 (interior rows 16-byte aligned)
constexpr int kTWP = 144;      // LDS row pitch in samples

__constant__ uint16_t c_taps3[5 * 9] = MIP_TAPS_3x3;
__constant__ uint16_t c_taps5[3 * 25] = MIP_TAPS_5x5;

// The reference's fp32 division v / s as a multiplication (see the header).
__device__ __forceinline__ float ref_recip(float s) {
  return __builtin_amdgcn_ldexpf(__builtin_amdgcn_rcpf(__builtin_amdgcn_frexp_mantf(s)),
                                 -__builtin_amdgcn_frexp_expf(s));
}

// round(x) for x >= 0 (round half up == round half away from zero): v_cvt_rpi_i32_f32
// computes floor(x + 0.5) without rounding the sum.
__device__ __forceinline__ uint32_t round_pos(float x) {
  int r;
  asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
  return (uint32_t)r;
}

// Validity of tile cell (ty, tc) of the tile at (qx, qy): 3x3 gates intra.cl:2903-2966,
// 5x5 gates intra.cl:3096-3189.  Interior cells: inside the frame.
__device__ __forceinline__ bool tap_valid(int rad, int qx, int qy, int ty, int tc, int W, int H) {
  const int WH = W * H;                            // < 2^31 (launch_filter)
  const int g = __mul24(qy + ty, W) + qx + tc;     // linear index, as the reference computes it
  const bool top = ty < 0, bot = ty >= 32, lft = tc < 0, rgt = tc >= 128;
  if (!top && !bot && !lft && !rgt) return qy + ty < H && qx + tc < W;
  if ((top || bot) && (lft || rgt)) {
    const bool vy = top ? qy > 0 : qy + ty < H - 1;
    const bool vx = lft ? qx > 0 : qx + tc < W - 1;
    return vy && vx;
  }
  if (top || bot) {
    if (!(g > 0 && g < WH)) return false;
    if (rad == 1) return true;
    return top ? qy > 0 : qy + ty + 2 < H - 1;
  }
  return g > 0 && g < WH && qx + tc > 0 && qx + tc < W - 1;
}

// Separable filters: is halo cell (ty, tc) fetched from the frame (intra.cl:3296-3345 for
// 3 taps, 3566-3640 for 5 taps)?
template <int RAD>
__device__ __forceinline__ bool sep_fetch(int qx, int qy, int ty, int tc, int W, int H) {
  const int WH = W * H;
  const int g = __mul24(qy + ty, W) + qx + tc;
  const bool top = ty < 0, bot = ty >= 32, lft = tc < 0, rgt = tc >= 128;
  if (RAD == 1) {
    if ((top || bot) && (lft || rgt)) {
      const int b = __mul24(qy, W) + qx;
      if (top && lft) return b - W - 1 > 0 && qx > 0 && qy > 0;
      if (top) return b - W + 128 > 0 && qx + 128 < W - 1 && qy > 0;
      if (lft) return b + 32 * W - 1 < WH && qx > 0 && qy + 32 < H - 1;
      return b + 32 * W + 128 < WH && qx + 128 < W - 1 && qy + 32 < H - 1;
    }
    if (top || bot) return g > 0 && g < WH;
    return g > 0 && g < WH && (lft ? qx > 0 : qx + 129 < W - 1);
  }
  if ((top || bot) && (lft || rgt)) {
    const bool vy = top ? qy > 0 : qy + ty < H - 1;   // rows Y+32 / Y+33
    const bool vx = lft ? qx > 0 : qx + tc < W - 1;   // columns X+128 / X+129
    return vy && vx;
  }
  if (top) return g > 0 && g < WH && qy > 0;
  if (bot) return g > 0 && g < WH && qy + ty + 2 < H - 1;
  return g > 0 && g < WH && qx + tc > 0 && qx + tc < W - 1;
}

// Tile cell inside the 128x32 tile, read like the reference: by linear index y * W + x, so
// columns right of the frame are the next row's first samples (intra.cl:2905, 3098, 3331,
// 3597).  Rows below the frame: 2-D and separable 5 taps -1 (invalid), separable 3 taps read
// them unguarded (intra.cl:3330-3332, past the frame's end).  Reads past the frame's end give
// outputs the reference leaves undefined (they depend on the next frame slot); they read 0
// here.
template <int RAD, bool SEP>
__device__ __forceinline__ short inner_value(const uint16_t *in, int x, int y, int W, int H) {
  if (y < H) {
    const int li = y * W + x;
    return li < W * H ? (short)in[li] : 0;
  }
  return (SEP && RAD == 1) ? 0 : -1;
}

// Stage the tile (+halo) in LDS: interior rows with 16-byte loads when the rows are
// 16-byte aligned (W % 8 == 0), halo cells one by one with the reference's gates.  Every
// phase issues all of a thread's loads before its first LDS store, so a workgroup waits for
// HBM once per phase, not once per load (a load -> store loop waits for every load).
// Returns whether this thread stored an invalid (-1) cell.
template <int RAD, bool SEP>
__device__ __forceinline__ bool stage(short *tile, const uint16_t *in, int qx, int qy, int W, int H) {
  constexpr int kThreads = kThreadsOf<SEP>;
  constexpr int TW = 128 + 2 * RAD;
  const int t = threadIdx.x % kThreads;
  bool invalid = false;
  // Interior tile: with a margin of one tile / 16 samples to every frame border, every
  // gate of every filter (tap_valid / sep_fetch / inner_value) admits every cell, so the
  // tile and its halo are plain samples: rows -RAD..31+RAD, columns -8..135 as 16-byte
  // loads (the LDS row pitch is exactly those 144 columns).
  if ((W & 7) == 0 && qx >= 128 && qy >= 32 && qx + 144 <= W - 2 && qy + 40 <= H - 2) {
    constexpr int NV = (32 + 2 * RAD) * (kTWP / 8), NPT = (NV + kThreads - 1) / kThreads;
    uint4 v[NPT];
#pragma unroll
    for (int p = 0; p < NPT; p++) {
      // the last round's spare threads repeat chunk NV - 1 (same value, same LDS slot)
      const int i = min(t + p * kThreads, NV - 1), r = i / (kTWP / 8), k = i - r * (kTWP / 8);
      v[p] = *reinterpret_cast<const uint4 *>(in + (size_t)(qy - RAD + r) * W + qx - 8 + 8 * k);
    }
#pragma unroll
    for (int p = 0; p < NPT; p++) {
      const int i = min(t + p * kThreads, NV - 1), r = i / (kTWP / 8), k = i - r * (kTWP / 8);
      *reinterpret_cast<uint4 *>(tile + r * kTWP + 8 * k) = v[p];
    }
    return false;
  }
  // Halo: RAD rows above and below (corners included), RAD columns left and right --
  // gathered first, so its loads are in flight with the tile's; stored last.
  constexpr int NROW = 2 * RAD * TW, NHALO = NROW + 2 * RAD * 32, NPH = (NHALO + kThreads - 1) / kThreads;
  short hv[NPH];
  int hidx[NPH];
#pragma unroll
  for (int p = 0; p < NPH; p++) {
    const int i = min(t + p * kThreads, NHALO - 1);  // spare threads repeat the last cell
    int ty, tc;
    if (i < NROW) {
      const int r = i / TW;
      tc = i - r * TW - RAD;
      ty = r < RAD ? r - RAD : 32 + r - RAD;
    } else {
      const int j = i - NROW, r = j / (2 * RAD), q = j - r * 2 * RAD;
      ty = r;
      tc = q < RAD ? q - RAD : 128 + q - RAD;
    }
    const bool fetch = SEP ? sep_fetch<RAD>(qx, qy, ty, tc, W, H) : tap_valid(RAD, qx, qy, ty, tc, W, H);
    hv[p] = fetch ? (short)in[(long long)(qy + ty) * W + qx + tc] : (SEP && RAD == 1 ? 0 : -1);
    hidx[p] = (ty + RAD) * kTWP + kCO + tc;
  }
  if ((W & 7) == 0) {
    // W % 8 == 0: a chunk of 8 columns lies entirely inside or entirely outside the frame's
    // linear extent; rows below the frame and indexes past its end read inner_value's fill
    constexpr int NC = 512 / kThreads;  // 16-byte chunks of the 32 x 128 tile per thread
    uint4 v[NC];
#pragma unroll
    for (int p = 0; p < NC; p++) {
      const int i = p * kThreads + t, r = i >> 4, k = i & 15;
      const int y = qy + r, x = qx + 8 * k;
      if (y < H && y * W + x + 8 <= W * H) {
        v[p] = *reinterpret_cast<const uint4 *>(in + y * W + x);
      } else {
        const short fv = (y < H || (SEP && RAD == 1)) ? 0 : -1;
        invalid |= fv < 0;
        const uint32_t f2 = (uint32_t)(uint16_t)fv * 0x10001u;
        v[p] = make_uint4(f2, f2, f2, f2);
      }
    }
#pragma unroll
    for (int p = 0; p < NC; p++) {
      const int i = p * kThreads + t, r = i >> 4, k = i & 15;
      *reinterpret_cast<uint4 *>(tile + (r + RAD) * kTWP + kCO + 8 * k) = v[p];
    }
  } else {
    for (int i0 = t; i0 < 32 * 128; i0 += 8 * kThreads) {
      short v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int i = i0 + u * kThreads, r = i >> 7, c = i & 127;
        v[u] = inner_value<RAD, SEP>(in, qx + c, qy + r, W, H);
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int i = i0 + u * kThreads, r = i >> 7, c = i & 127;
        invalid |= v[u] < 0;
        tile[(r + RAD) * kTWP + kCO + c] = v[u];
      }
    }
  }
#pragma unroll
  for (int p = 0; p < NPH; p++) {
    invalid |= hv[p] < 0;
    tile[hidx[p]] = hv[p];
  }
  return invalid;
}

__device__ __forceinline__ u2 as_u2(uint32_t v) { return __builtin_bit_cast(u2, v); }
__device__ __forceinline__ uint32_t as_u32(u2 v) { return __builtin_bit_cast(uint32_t, v); }

// Horizontal pass of one LDS row at the thread's columns c0..c0+3 (`row` points at column
// c0-2): packed sums sum_j t_j * f(v[c + j - RAD]) for columns (c0, c0+1) and (c0+2, c0+3);
// f(v) = max(v, 0) (numerator) or [v < 0] (invalid indicator).
template <int RAD, bool IND>
__device__ __forceinline__ void hpass(const short *row, const u2 (&tt)[5], u2 &p01, u2 &p23) {
  const uint32_t *row32 = reinterpret_cast<const uint32_t *>(row);  // 4-byte aligned
  uint32_t m[4] = {row32[0], row32[1], row32[2], row32[3]};        // columns c0-2 .. c0+5
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (IND) m[k] = as_u32(as_u2(m[k]) >> (u2){15, 15});
    else m[k] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(s2, m[k]), (s2){0, 0}));
  }
  const u2 M0 = as_u2(m[0]), M1 = as_u2(m[1]), M2 = as_u2(m[2]), M3 = as_u2(m[3]);
  const u2 S0 = as_u2(__builtin_amdgcn_alignbit(m[1], m[0], 16));  // columns c0-1, c0
  const u2 S1 = as_u2(__builtin_amdgcn_alignbit(m[2], m[1], 16));  // c0+1, c0+2
  const u2 S2 = as_u2(__builtin_amdgcn_alignbit(m[3], m[2], 16));  // c0+3, c0+4
  if (RAD == 1) {
    p01 = tt[0] * S0 + tt[1] * M1 + tt[2] * S1;
    p23 = tt[0] * S1 + tt[1] * M2 + tt[2] * S2;
  } else {
    p01 = tt[0] * M0 + tt[1] * S0 + tt[2] * M1 + tt[3] * S1 + tt[4] * M2;
    p23 = tt[0] * M1 + tt[1] * S1 + tt[2] * M2 + tt[3] * S2 + tt[4] * M3;
  }
}

// Vertical pass: sum_i t_i * hp[i], low and high column.
template <int KS>
__device__ __forceinline__ void vpass(const u2 *hp, const int (&t)[5], uint32_t &lo, uint32_t &hi) {
  lo = hi = 0;
#pragma unroll
  for (int i = 0; i < KS; i++) {
    lo = __builtin_amdgcn_udot2(hp[i], (u2){(unsigned short)t[i], 0}, lo, false);
    hi = __builtin_amdgcn_udot2(hp[i], (u2){0, (unsigned short)t[i]}, hi, false);
  }
}

// Exact (x + s/2) / s for x + s/2 < 2^24, s >= 1 (float estimate, one correction step).
__device__ __forceinline__ uint32_t div_round(int x, int s) {
  const int n = x + (s >> 1);
  int q = (int)((float)n * __builtin_amdgcn_rcpf((float)s));
  const int r = n - q * s;
  q += (r >= s) - (r < 0);
  return (uint32_t)q;
}

// Separable position-class scale of pixel (x, y) (intra.cl:3281-3285, 3523-3557).
template <int RAD>
__device__ __forceinline__ int sep_scale(int x, int y, int W, int H, int full, const int (&cls)[7]) {
  if (RAD == 1) {
    const int nb = (y == 0) + (y == H - 1) + (x == 0) + (x == W - 1);
    return nb >= 2 ? cls[0] : (nb ? cls[1] : full);
  }
  const bool otb = y == 0 || y == H - 1, itb = y == 1 || y == H - 2;
  const bool olr = x == 0 || x == W - 1, ilr = x == 1 || x == W - 2;
  const bool o_corner = otb && olr, i_corner = itb && ilr;
  const bool iface = (olr && itb) || (ilr && otb);
  int sc = full;
  if (o_corner) sc = cls[2];
  if (i_corner) sc = cls[3];
  if (!o_corner && !iface && (otb || olr)) sc = cls[5];
  if (!i_corner && !iface && (itb || ilr)) sc = cls[6];
  if (iface) sc = cls[4];
  return sc;
}

template <int RAD, bool FLOAT, bool SEP>
__global__ __launch_bounds__(kThreadsOf<SEP> * kTPW) void filter_kernel(FilterArgs a) {
  constexpr int kThreads = kThreadsOf<SEP>, kRows = 32 * 32 / kThreads;
  static_assert(kThreads == 64 || kThreads == 128 || kThreads == 256, "threads per tile");
  constexpr int KS = 2 * RAD + 1, TH = 32 + 2 * RAD, NR = kRows + 2 * RAD;
  __shared__ __attribute__((aligned(16))) short tiles[kTPW][TH * kTWP];
  const int W = a.width, H = a.height;
  const int sub = kTPW > 1 ? (int)threadIdx.x / kThreads : 0;  // tile of this thread's 128-thread group
  short *tile = tiles[sub];
  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs, so workgroup b
  // takes tile (b % 8) * per + b / 8 -- each XCD walks a contiguous band of tiles and the
  // halo rows / columns it shares with its neighbours are fetched into its own L2.
  const int tiles_x = (W + 127) / 128, tiles_y = (H + 31) / 32, per_frame = tiles_x * tiles_y;
  const int total = per_frame * a.nframes, units = (total + kTPW - 1) / kTPW, per = (units + 7) / 8;
  const int tid = ((int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3)) * kTPW + sub;
  if (tid >= total) return;  // whole waves leave (a barrier does not wait for ended waves)
  const int f = tid / per_frame, tr = tid - f * per_frame, ty = tr / tiles_x;
  const int qx = 128 * (tr - ty * tiles_x), qy = 32 * ty;
  const uint16_t *in = a.in + (size_t)f * W * H;
  const bool inv_local = stage<RAD, SEP>(tile, in, qx, qy, W, H);
  const bool irregular = __syncthreads_or(inv_local);  // some cell of the window is invalid

  const uint16_t *k2 = RAD == 1 ? c_taps3 + 9 * a.kernel_idx : c_taps5 + 25 * a.kernel_idx;
  int t[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < KS; i++) t[i] = k2[i];
  u2 tt[5];
#pragma unroll
  for (int i = 0; i < 5; i++) tt[i] = (u2){(unsigned short)t[i], (unsigned short)t[i]};
  int tsum = 0;
#pragma unroll
  for (int i = 0; i < KS; i++) tsum += t[i];
  const int d = SEP ? 0 : (int)k2[RAD * KS + RAD] - t[RAD] * t[RAD];  // centre excess
  int full = tsum * tsum + d;

  // Separable class scales: 3 taps {corner, edge}; 5 taps {-, -, outer corner, inner
  // corner, interface, outer edge, inner edge} (oracle filter_1d_tile3/5).
  int cls[7] = {0, 0, 0, 0, 0, 0, 0};
  if (SEP) {
    if (RAD == 1) {
      full = 4 * t[0] + 4 * t[1] + t[1] * t[1];
      cls[0] = t[0] + 2 * t[1] + t[1] * t[1];
      cls[1] = 2 * t[0] + 3 * t[1] + t[1] * t[1];
    } else {
      full = 0;
#pragma unroll
      for (int i = 0; i < 5; i++)
#pragma unroll
        for (int j = 0; j < 5; j++) {
          const int v = k2[i * 5 + j];
          full += v;
          if (i >= 2 && j >= 2) cls[2] += v;
          if (i >= 1 && j >= 1) cls[3] += v;
          if (i >= 1 && j >= 2) cls[4] += v;
          if (j >= 2) cls[5] += v;
          if (j >= 1) cls[6] += v;
        }
    }
  }

  const int c0 = 4 * (threadIdx.x & 31), r0 = kRows * ((threadIdx.x % kThreads) >> 5);
  const short *rowp = tile + r0 * kTWP + kCO - 2 + c0;
  // Horizontal sums are produced one row ahead of the vertical pass that consumes them
  // (a sliding window of KS rows stays live, not all NR: fewer VGPRs, higher occupancy).
  u2 h01[NR], h23[NR];
#pragma unroll
  for (int r = 0; r < KS - 1; r++) hpass<RAD, false>(rowp + r * kTWP, tt, h01[r], h23[r]);

  // Uniform scale: every window fully valid (2-D) / no frame-border class (separable).
  const bool uniform = SEP ? (qx >= 2 && qx + 128 <= W - 2 && qy >= 2 && qy + 32 <= H - 2) : !irregular;
  u2 n01[NR], n23[NR];
  if (!SEP && !uniform) {
#pragma unroll
    for (int r = 0; r < KS - 1; r++) hpass<RAD, true>(rowp + r * kTWP, tt, n01[r], n23[r]);
  }
  const bool narrow = tsum * tsum * 1023 < 65536;  // separable part of the sum fits 16 bits
  const float rf = ref_recip((float)full);
  const uint32_t magic = (uint32_t)(0x100000000ull / (unsigned)full) + ((0x100000000ull % (unsigned)full) != 0);

  uint16_t *out = a.out + (size_t)f * W * H;
#pragma unroll
  for (int r = 0; r < kRows; r++) {
    const int y = qy + r0 + r;
    hpass<RAD, false>(rowp + (r + KS - 1) * kTWP, tt, h01[r + KS - 1], h23[r + KS - 1]);
    uint32_t num[4];
    if (narrow) {  // sums < 2^16: packed vertical pass
      u2 v01 = tt[0] * h01[r], v23 = tt[0] * h23[r];
#pragma unroll
      for (int i = 1; i < KS; i++) {
        v01 += tt[i] * h01[r + i];
        v23 += tt[i] * h23[r + i];
      }
      num[0] = as_u32(v01) & 0xffff;
      num[1] = as_u32(v01) >> 16;
      num[2] = as_u32(v23) & 0xffff;
      num[3] = as_u32(v23) >> 16;
    } else {
      vpass<KS>(h01 + r, t, num[0], num[1]);
      vpass<KS>(h23 + r, t, num[2], num[3]);
    }
    if (!SEP && d != 0) {
      const uint32_t *cp = reinterpret_cast<const uint32_t *>(rowp + (r + RAD) * kTWP + 2);  // centres c0..c0+3
      const uint32_t cv0 = cp[0], cv1 = cp[1];
      num[0] += d * (int)(cv0 & 0xffff);
      num[1] += d * (int)(cv0 >> 16);
      num[2] += d * (int)(cv1 & 0xffff);
      num[3] += d * (int)(cv1 >> 16);
    }
    uint32_t res[4];
    if (uniform) {
#pragma unroll
      for (int c = 0; c < 4; c++) {
        if (FLOAT) res[c] = round_pos((float)num[c] * rf);
        else res[c] = __umulhi(num[c] + (uint32_t)(full >> 1), magic);
      }
    } else {
      uint32_t def[4] = {0, 0, 0, 0};
      if (!SEP) {
        hpass<RAD, true>(rowp + (r + KS - 1) * kTWP, tt, n01[r + KS - 1], n23[r + KS - 1]);
        vpass<KS>(n01 + r, t, def[0], def[1]);
        vpass<KS>(n23 + r, t, def[2], def[3]);
      }
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int s = SEP ? sep_scale<RAD>(qx + c0 + c, y, W, H, full, cls) : full - (int)def[c];
        if (FLOAT) res[c] = round_pos((float)num[c] * ref_recip((float)s));
        else res[c] = div_round((int)num[c], s);
      }
    }
    const int x = qx + c0;
    if (y >= H || x >= W) continue;
    uint16_t *o = out + (size_t)y * W + x;
    if ((W & 3) == 0 && x + 4 <= W) {
#if MIP_FILTER_NT
      typedef unsigned int v2u __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store((v2u){res[0] | (res[1] << 16), res[2] | (res[3] << 16)}, reinterpret_cast<v2u *>(o));
#else
      *reinterpret_cast<uint2 *>(o) = make_uint2(res[0] | (res[1] << 16), res[2] | (res[3] << 16));
#endif
    } else {
#pragma unroll
      for (int c = 0; c < 4; c++)
        if (x + c < W) o[c] = (uint16_t)res[c];
    }
  }
}

// Streaming copy (bench.py's calibration of the filter's HBM roofline, mip_copy_device): 16
// bytes per lane, four loads in flight per lane before their stores, grid-stride over the
// buffer -- the guide's measured achievable copy is this form (MI355X_MICROARCH.md: float4
// copy 6.29 TB/s).
__global__ __launch_bounds__(256) void copy_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * 1024;
  size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x;
  for (; i + 768 < n16; i += stride) {
    const uint4 v0 = src[i], v1 = src[i + 256], v2 = src[i + 512], v3 = src[i + 768];
    dst[i] = v0;
    dst[i + 256] = v1;
    dst[i + 512] = v2;
    dst[i + 768] = v3;
  }
  for (; i < n16; i += 256) dst[i] = src[i];
}

}  // namespace

// One workgroup row per piece (blockIdx.y); 16-byte words where both ends are 16-byte aligned,
// then the tail bytes.
__global__ __launch_bounds__(256) void gather_copy_kernel(CopyPieces a) {
  if ((int)blockIdx.y >= a.n) return;
  const CopyPiece c = a.p[blockIdx.y];
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x, t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t n16 = (((uintptr_t)c.src | (uintptr_t)c.dst) & 15) == 0 ? c.bytes / 16 : 0;
  for (uint64_t i = t0; i < n16; i += step) reinterpret_cast<uint4 *>(c.dst)[i] = reinterpret_cast<const uint4 *>(c.src)[i];
  for (uint64_t i = n16 * 16 + t0; i < c.bytes; i += step) c.dst[i] = c.src[i];
}

hipError_t launch_gather_copy(const CopyPieces &a, hipStream_t s) {
  if (a.n < 1) return hipSuccess;
  if (a.n > kMaxCopyPieces) return hipErrorInvalidValue;
  uint64_t most = 0;
  for (int i = 0; i < a.n; i++) most = std::max<uint64_t>(most, a.p[i].bytes);
  const unsigned bx = (unsigned)std::min<uint64_t>(64, std::max<uint64_t>(1, (most / 16 + 255) / 256));
  hipLaunchKernelGGL(gather_copy_kernel, dim3(bx, (unsigned)a.n), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_copy(const void *src, void *dst, size_t bytes, hipStream_t s) {
  if (bytes % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16) return hipErrorInvalidValue;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return hipErrorInvalidValue;
  const size_t n16 = bytes / 16, blocks = std::min<size_t>((size_t)cus * 8, (n16 + 1023) / 1024);
  hipLaunchKernelGGL(copy_kernel, dim3((unsigned)std::max<size_t>(1, blocks)), dim3(256), 0, s,
                     (const uint4 *)src, (uint4 *)dst, n16);
  return hipGetLastError();
}

hipError_t launch_filter(const FilterArgs &a, hipStream_t s) {
  const long long total = (long long)((a.width + 127) / 128) * ((a.height + 31) / 32) * a.nframes;
  if (total > (1LL << 30) || (long long)(a.width + 256) * (a.height + 64) >= (1LL << 31) || a.width >= (1 << 22) ||
      a.height >= (1 << 22))
    return hipErrorInvalidValue;  // 32-bit / 24-bit index arithmetic in the gates
  const long long units = (total + kTPW - 1) / kTPW;
  const dim3 grid((unsigned)((units + 7) / 8 * 8));
  const dim3 sep_block(kThreadsOf<true> * kTPW), block(kThreadsOf<false> * kTPW);
  switch (a.filter) {
    case 0: hipLaunchKernelGGL((filter_kernel<1, false, true>), grid, sep_block, 0, s, a); break;
    case 1: hipLaunchKernelGGL((filter_kernel<1, true, true>), grid, sep_block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((filter_kernel<1, false, false>), grid, block, 0, s, a); break;
    case 3: hipLaunchKernelGGL((filter_kernel<1, true, false>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((filter_kernel<2, false, true>), grid, sep_block, 0, s, a); break;
    case 5: hipLaunchKernelGGL((filter_kernel<2, true, true>), grid, sep_block, 0, s, a); break;
    case 6: hipLaunchKernelGGL((filter_kernel<2, false, false>), grid, block, 0, s, a); break;
    case 7: hipLaunchKernelGGL((filter_kernel<2, true, false>), grid, block, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mipgpu
