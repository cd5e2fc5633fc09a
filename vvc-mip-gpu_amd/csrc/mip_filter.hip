// mip_filter.hip -- LDS-tiled low-pass filters of the reference samples (gfx950).
//
// 2-D kernels (filterFrame_2d_{int,float}[_5x5]_quarterCtu, intra.cl:2856, 1639, 3042,
// 2311): one workgroup per 128x32 quarter-CTU tile plus a 1- or 2-sample halo, as in the
// reference, because the reference's halo gates are defined per tile.  A halo cell is
// loaded when the reference would load it (restated below) and marked invalid (-1)
// otherwise; each output is the normalised convolution over its valid taps,
//     int:   (sum + scale/2) / scale         (intra.cl:3011, 3235)
//     float: roundf(float(sum) / float(scale)) with IEEE division (intra.cl:1794, 2507)
// The float twins are computed in fp32 as the reference does; for non-negative inputs
// they equal the integer form whenever division is correctly rounded (HIP default).
#include "mip_kernels.h"
#include "mip_tables.h"

namespace mipgpu {
namespace {

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
    if (FLOAT) r = (int)roundf((float)sum / (float)scale);
    else r = (sum + scale / 2) / scale;
    out[(size_t)(qy + ty) * W + qx + tc] = (uint16_t)r;
  }
}

}  // namespace

hipError_t launch_filter(const FilterArgs &a, hipStream_t s) {
  const dim3 grid((a.width + 127) / 128, (a.height + 31) / 32, a.nframes);
  switch (a.filter) {
    case 2: hipLaunchKernelGGL((filter2d_kernel<1, false>), grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((filter2d_kernel<1, true>), grid, dim3(256), 0, s, a); break;
    case 6: hipLaunchKernelGGL((filter2d_kernel<2, false>), grid, dim3(256), 0, s, a); break;
    case 7: hipLaunchKernelGGL((filter2d_kernel<2, true>), grid, dim3(256), 0, s, a); break;
    default: return hipErrorInvalidValue;  // separable variants: not yet on the HIP path
  }
  return hipGetLastError();
}

}  // namespace mipgpu
