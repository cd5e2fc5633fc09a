// mip_filter.hip -- LDS-tiled low-pass filters of the reference samples (gfx950).
//
// All eight reference filters work per 128x32 quarter-CTU tile plus a 1- or 2-sample
// halo, because the reference's halo gates are defined per tile; so do these kernels
// (one workgroup per tile, HBM-bound: one read and one write of the frame).
//  * 2-D (filterFrame_2d_{int,float}[_5x5]_quarterCtu, intra.cl:2856, 1639, 3042, 2311):
//    a halo cell is loaded when the reference would load it (restated in tap_valid) and
//    marked invalid (-1) otherwise; each output is the normalised convolution over its
//    valid taps.
//  * separable (filterFrame_1d_{int,float}[_5x5], intra.cl:3267, 1828, 3508, 2539): row 0
//    of the 2-D kernel applied horizontally (halo rows included) and then vertically,
//    with the reference's fetch conditions (sep_fetch) and its position-class scales
//    (oracle/mip_oracle.c filter_1d_tile3/5 documents the rules).
// Rounding: int (sum + scale/2) / scale; float round(ref_fdiv(sum, scale)) where
// ref_fdiv is the reference's own fp32 division sequence (frexp, v_rcp_f32, v_mul,
// v_ldexp: the AMD OpenCL lowering of '/', read from the reference's code objects),
// which differs from IEEE division at exact ties for scales like 12 or 24.
#include "mip_kernels.h"
#include "mip_tables.h"

namespace mipgpu {
namespace {

__device__ __forceinline__ float ref_fdiv(float v, float s) {
  const float ms = __builtin_amdgcn_frexp_mantf(s);
  const int es = __builtin_amdgcn_frexp_expf(s);
  const float mv = __builtin_amdgcn_frexp_mantf(v);
  const int ev = __builtin_amdgcn_frexp_expf(v);
  return __builtin_amdgcn_ldexpf(mv * __builtin_amdgcn_rcpf(ms), ev - es);
}

__constant__ uint16_t c_taps3[5 * 9] = MIP_TAPS_3x3;
__constant__ uint16_t c_taps5[3 * 25] = MIP_TAPS_5x5;

// Validity of tile cell (ty, tc) of the tile at (qx, qy): 3x3 gates intra.cl:2903-2966,
// 5x5 gates intra.cl:3096-3189.  Interior cells: inside the frame.
__device__ __forceinline__ bool tap_valid(int rad, int qx, int qy, int ty, int tc, int W, int H) {
  const long long WH = (long long)W * H;
  const long long g = (long long)(qy + ty) * W + qx + tc;
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

template <int RAD, bool FLOAT>
__global__ __launch_bounds__(256) void filter2d_kernel(FilterArgs a) {
  constexpr int KS = 2 * RAD + 1;
  constexpr int TW = 128 + 2 * RAD, TH = 32 + 2 * RAD;
  constexpr int PITCH = TW + 1;
  __shared__ short tile[TH * PITCH];
  const int qx = 128 * blockIdx.x, qy = 32 * blockIdx.y, f = blockIdx.z;
  const int W = a.width, H = a.height;
  const uint16_t *in = a.in + (size_t)f * W * H;
  for (int i = threadIdx.x; i < TH * TW; i += blockDim.x) {
    const int r = i / TW, c = i - r * TW;
    const int ty = r - RAD, tc = c - RAD;
    short v = -1;
    if (tap_valid(RAD, qx, qy, ty, tc, W, H)) v = (short)in[(size_t)(qy + ty) * W + qx + tc];
    tile[r * PITCH + c] = v;
  }
  __syncthreads();
  const uint16_t *taps = RAD == 1 ? c_taps3 + 9 * a.kernel_idx : c_taps5 + 25 * a.kernel_idx;
  int k[KS * KS];
#pragma unroll
  for (int i = 0; i < KS * KS; i++) k[i] = taps[i];
  uint16_t *out = a.out + (size_t)f * W * H;
  for (int i = threadIdx.x; i < 128 * 32; i += blockDim.x) {
    const int ty = i >> 7, tc = i & 127;
    if (qy + ty >= H || qx + tc >= W) continue;
    int sum = 0, scale = 0;
#pragma unroll
    for (int dy = 0; dy < KS; dy++)
#pragma unroll
      for (int dx = 0; dx < KS; dx++) {
        const int v = tile[(ty + dy) * PITCH + tc + dx];
        const int c = v >= 0 ? k[dy * KS + dx] : 0;
        sum += c * max(v, 0);
        scale += c;
      }
    int r;
    if (FLOAT) r = (int)roundf(ref_fdiv((float)sum, (float)scale));
    else r = (sum + scale / 2) / scale;
    out[(size_t)(qy + ty) * W + qx + tc] = (uint16_t)r;
  }
}

// Separable filters: is tile cell (ty, tc) fetched from the frame (intra.cl:3296-3345
// for 3 taps, 3566-3640 for 5 taps)?  Cells inside the tile are always fetched by the
// 3-tap kernels (no bound check; samples below / right of the frame read 0 here) and
// for rows inside the frame by the 5-tap kernels.
template <int RAD>
__device__ __forceinline__ bool sep_fetch(int qx, int qy, int ty, int tc, int W, int H) {
  const long long WH = (long long)W * H;
  const long long g = (long long)(qy + ty) * W + qx + tc;
  const bool top = ty < 0, bot = ty >= 32, lft = tc < 0, rgt = tc >= 128;
  if (!top && !bot && !lft && !rgt) return RAD == 1 || qy + ty < H;
  if (RAD == 1) {
    if ((top || bot) && (lft || rgt)) {
      const long long b = (long long)qy * W + qx;
      if (top && lft) return b - W - 1 > 0 && qx > 0 && qy > 0;
      if (top) return b - W + 128 > 0 && qx + 128 < W - 1 && qy > 0;
      if (lft) return b + 32LL * W - 1 < WH && qx > 0 && qy + 32 < H - 1;
      return b + 32LL * W + 128 < WH && qx + 128 < W - 1 && qy + 32 < H - 1;
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

template <int RAD, bool FLOAT>
__global__ __launch_bounds__(256) void filter1d_kernel(FilterArgs a) {
  constexpr int KS = 2 * RAD + 1;
  constexpr int TW = 128 + 2 * RAD, TH = 32 + 2 * RAD;
  __shared__ short tile[TH * TW];
  __shared__ int hsum[TH * 128];  // horizontal pass; -1: tile row outside the frame (5 taps)
  const int qx = 128 * blockIdx.x, qy = 32 * blockIdx.y, f = blockIdx.z;
  const int W = a.width, H = a.height;
  const uint16_t *in = a.in + (size_t)f * W * H;
  for (int i = threadIdx.x; i < TH * TW; i += blockDim.x) {
    const int r = i / TW, c = i - r * TW;
    const int ty = r - RAD, tc = c - RAD, y = qy + ty, x = qx + tc;
    short v = RAD == 1 ? 0 : -1;  // not fetched: 0 (3 taps) / dropped (5 taps)
    // Fetched halo cells read the reference's linear index (in range by sep_fetch; it
    // wraps into the neighbouring row only when W % 128 != 0); interior cells outside
    // the frame read 0.
    const bool inner = ty >= 0 && ty < 32 && tc >= 0 && tc < 128;
    if (sep_fetch<RAD>(qx, qy, ty, tc, W, H))
      v = !inner ? (short)in[(long long)y * W + x] : (y < H && x < W) ? (short)in[(size_t)y * W + x] : 0;
    tile[i] = v;
  }
  const uint16_t *k2 = RAD == 1 ? c_taps3 + 9 * a.kernel_idx : c_taps5 + 25 * a.kernel_idx;
  int t[KS];
#pragma unroll
  for (int i = 0; i < KS; i++) t[i] = k2[i];  // row 0 of the 2-D kernel
  __syncthreads();
  for (int i = threadIdx.x; i < TH * 128; i += blockDim.x) {
    const int r = i >> 7, c = i & 127;
    int acc = 0;
#pragma unroll
    for (int d = 0; d < KS; d++) acc += max((int)tile[r * TW + c + d], 0) * t[d];
    const bool row_ok = RAD == 1 || (qy + r - RAD >= 0 && qy + r - RAD < H);
    hsum[i] = row_ok ? acc : -1;
  }
  __syncthreads();
  int full, s_corner = 0, s_edge = 0, oc = 0, ic = 0, itf = 0, oe = 0, ie = 0;
  if (RAD == 1) {
    full = 4 * t[0] + 4 * t[1] + t[1] * t[1];
    s_corner = t[0] + 2 * t[1] + t[1] * t[1];
    s_edge = 2 * t[0] + 3 * t[1] + t[1] * t[1];
  } else {
    full = 0;
    for (int i = 0; i < 5; i++)
      for (int j = 0; j < 5; j++) {
        const int v = k2[i * 5 + j];
        full += v;
        if (i >= 2 && j >= 2) oc += v;
        if (i >= 1 && j >= 1) ic += v;
        if (i >= 1 && j >= 2) itf += v;
        if (j >= 2) oe += v;
        if (j >= 1) ie += v;
      }
  }
  uint16_t *out = a.out + (size_t)f * W * H;
  for (int i = threadIdx.x; i < 128 * 32; i += blockDim.x) {
    const int ty = i >> 7, tc = i & 127, y = qy + ty, x = qx + tc;
    if (y >= H || x >= W) continue;
    int v = 0, sc = full;
#pragma unroll
    for (int d = 0; d < KS; d++) {
      const int h = hsum[(ty + d) * 128 + tc];
      if (h < 0) sc -= t[d];
      else v += h * t[d];
    }
    if (RAD == 1) {
      const int nb = (y == 0) + (y == H - 1) + (x == 0) + (x == W - 1);
      sc = nb >= 2 ? s_corner : (nb ? s_edge : full);
    } else {
      const bool otb = y == 0 || y == H - 1, itb = y == 1 || y == H - 2;
      const bool olr = x == 0 || x == W - 1, ilr = x == 1 || x == W - 2;
      const bool o_corner = otb && olr, i_corner = itb && ilr;
      const bool iface = (olr && itb) || (ilr && otb);
      if (o_corner) sc = oc;
      if (i_corner) sc = ic;
      if (!o_corner && !iface && (otb || olr)) sc = oe;
      if (!i_corner && !iface && (itb || ilr)) sc = ie;
      if (iface) sc = itf;
    }
    int r;
    if (FLOAT) r = (int)roundf(ref_fdiv((float)v, (float)sc));
    else r = (v + sc / 2) / sc;
    out[(size_t)y * W + x] = (uint16_t)r;
  }
}

}  // namespace

hipError_t launch_filter(const FilterArgs &a, hipStream_t s) {
  const dim3 grid((a.width + 127) / 128, (a.height + 31) / 32, a.nframes);
  switch (a.filter) {
    case 0: hipLaunchKernelGGL((filter1d_kernel<1, false>), grid, dim3(256), 0, s, a); break;
    case 1: hipLaunchKernelGGL((filter1d_kernel<1, true>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((filter2d_kernel<1, false>), grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((filter2d_kernel<1, true>), grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((filter1d_kernel<2, false>), grid, dim3(256), 0, s, a); break;
    case 5: hipLaunchKernelGGL((filter1d_kernel<2, true>), grid, dim3(256), 0, s, a); break;
    case 6: hipLaunchKernelGGL((filter2d_kernel<2, false>), grid, dim3(256), 0, s, a); break;
    case 7: hipLaunchKernelGGL((filter2d_kernel<2, true>), grid, dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mipgpu
