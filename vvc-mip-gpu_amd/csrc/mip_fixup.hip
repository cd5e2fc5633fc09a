// mip_fixup.hip -- exact per-CU MIP search for the few CUs whose reference samples may
// exceed 10 bits (gfx950).
//
// The search kernel (mip_search.hip) packs two modes into 16-bit halves and feeds the MFMA
// with f16 samples: both are exact for 10-bit reference samples only.  At frame widths that
// are not multiples of 128 the reference's separable filters give the last one or two frame
// columns values up to ~1.7 x 1023 (mipgpu.cpp reads_last_columns), so with alternative
// references the CUs that read those columns are left out of the search kernel's work lists
// and searched here, one 64-thread workgroup per (frame, CU), in plain 32-bit integer
// arithmetic -- the reference's own semantics:
//   boundaries   intra.cl:96-107, 232-243 (linear indexes, padding), 127-141, 259-279
//   GEMV         intra.cl:415-485 (p_0, offset, shift 6, clip to 10 bits, transposition)
//   upsampling   intra.cl:815-912 (horizontal on the anchor rows, then vertical)
//   distortion   intra.cl:922-1166, kernel_aux_functions.cl:142-249 (min(2 SAD, SATD))
// A few hundred CUs per frame at most; the launch is a small fraction of the search.
#include "mip_kernels.h"
#include "mip_tables.h"

namespace mipgpu {
namespace {

__constant__ mip_shape_desc f_shapes[MIP_NUM_SHAPES] = MIP_SHAPE_TABLE;
__constant__ uint8_t f_w0[16 * 16 * 4] = MIP_WEIGHTS_S0;
__constant__ uint8_t f_w1[8 * 16 * 8] = MIP_WEIGHTS_S1;
__constant__ uint8_t f_w2[6 * 64 * 7] = MIP_WEIGHTS_S2;

__device__ __forceinline__ int ilog2i(int v) { return 31 - __clz(v); }

__device__ __forceinline__ int axis(int base, int step, int dual, int i) {
  return dual ? base + (i / 2) * step + (i % 2) * dual : base + i * step;
}

// kernel_aux_functions.cl:142-249 (VTM xCalcHADs4x4, DC term scaled, (satd + 1) >> 1)
__device__ int satd4x4(const int *d) {
  int m[16], e[16];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    m[i] = d[i] + d[12 + i];
    m[4 + i] = d[4 + i] + d[8 + i];
    m[8 + i] = d[4 + i] - d[8 + i];
    m[12 + i] = d[i] - d[12 + i];
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    e[i] = m[i] + m[4 + i];
    e[4 + i] = m[8 + i] + m[12 + i];
    e[8 + i] = m[i] - m[4 + i];
    e[12 + i] = m[12 + i] - m[8 + i];
  }
  int s = 0, dc = 0;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int *q = e + 4 * r;
    const int t0 = q[0] + q[3], t1 = q[1] + q[2], t2 = q[1] - q[2], t3 = q[0] - q[3];
    if (r == 0) dc = abs(t0 + t1);
    s += abs(t0 + t1) + abs(t0 - t1) + abs(t2 + t3) + abs(t3 - t2);
  }
  s = s - dc + (dc >> 2);
  return (s + 1) >> 1;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(64) void fixup_kernel(SearchArgs a, const FixupCu *cus, int n) {
  __shared__ int top[64], left[64], red[8], rpred[64];
  __shared__ int pred[64 * 64];
  const int item = blockIdx.x % n, frame = blockIdx.x / n, t = threadIdx.x;
  const FixupCu c = cus[item];
  if ((int)c.ctu < a.ctu0 || (int)c.ctu >= a.ctu0 + a.nrange) return;  // workgroup-uniform
  const mip_shape_desc sd = f_shapes[c.shape];
  int cu = c.cu;
  for (int s = 0; s < c.shape; s++) cu -= f_shapes[s].ncu;
  const int W = a.width, H = a.height, w = sd.w, h = sd.h;
  const int x = 128 * ((int)c.ctu % a.ctu_cols) + axis(sd.xb, sd.xs, sd.xd, cu % sd.ncols);
  const int y = 128 * ((int)c.ctu / a.ctu_cols) + axis(sd.yb, sd.ys, sd.yd, cu / sd.ncols);
  const uint16_t *S = a.orig + (size_t)frame * W * H, *F = a.refs + (size_t)frame * W * H;
  // complete boundaries (linear indexes, intra.cl:100, 106, 236, 242)
  if (t < w) top[t] = y > 0 ? F[(y - 1) * W + x + t] : (x == 0 ? 512 : F[x - 1]);
  if (t < h) left[t] = x > 0 ? F[(y + t) * W + x - 1] : (y == 0 ? 512 : F[(y - 1) * W]);
  __syncthreads();
  const int rbs = (w == 4 && h == 4) ? 2 : 4;
  if (t < 2 * rbs) {  // reduced boundaries: box averages; a factor of 1 is a copy
    const int side = t / rbs, i = t % rbs, len = side ? h : w, df = len / rbs, l2 = ilog2i(df);
    const int rnd = df > 1 ? 1 << (l2 - 1) : 0;
    const int *src = side ? left : top;
    int s = 0;
    for (int k = 0; k < df; k++) s += src[i * df + k];
    red[side * 4 + i] = (s + rnd) >> l2;
  }
  __syncthreads();
  const int sid = sd.size_id, r = sid == 2 ? 8 : 4, nin = 2 * rbs, modes = sd.modes, M = 2 * modes;
  const int uh = w / r, uv = h / r, lh = ilog2i(uh), lv = ilog2i(uv);
  const size_t cbase = ((size_t)frame * a.nctus + c.ctu) * MIP_COSTS_PER_CTU + sd.cost_offset + (size_t)cu * M;
  uint32_t best = 0xffffffffu;
  for (int m = 0; m < M; m++) {
    const int mode = m % modes;
    const bool tr = m >= modes;
    if (t < r * r) {  // reduced prediction (intra.cl:415-485)
      int b[8];
      for (int i = 0; i < rbs; i++) {
        b[i] = tr ? red[4 + i] : red[i];
        b[rbs + i] = tr ? red[i] : red[4 + i];
      }
      const int b0 = b[0];
      int p[8], psum = 0;
      for (int i = 0; i < nin; i++) p[i] = b[i] - b0;
      p[0] = sid == 2 ? 0 : 512 - b0;
      for (int i = 0; i < nin; i++) psum += p[i];
      int acc = 32 - 32 * psum;
      for (int i = 0; i < nin; i++) {
        int wt;
        if (sid == 2) wt = i == 0 ? 0 : f_w2[(mode * 64 + t) * 7 + i - 1];
        else if (sid == 1) wt = f_w1[(mode * 16 + t) * 8 + i];
        else wt = f_w0[(mode * 16 + t) * 4 + i];
        acc += p[i] * wt;
      }
      const int v = min(max((acc >> 6) + b0, 0), 1023);
      rpred[tr ? (t % r) * r + t / r : t] = v;
    }
    __syncthreads();
    if (sid == 0) {
      if (t < 16) pred[t] = rpred[t];
    } else {
      for (int i = t; i < r * w; i += 64) {  // horizontal pass on the anchor rows
        const int k = i / w, xx = i % w, ya = k * uv + uv - 1;
        int v;
        if (uh == 1) {
          v = rpred[k * r + xx];
        } else {
          const int o = xx % uh + 1;
          const int before = xx < uh ? left[ya] : rpred[k * r + (xx >> lh) - 1];
          v = ((uh - o) * before + o * rpred[k * r + (xx >> lh)] + (1 << (lh - 1))) >> lh;
        }
        pred[ya * w + xx] = v;
      }
      __syncthreads();
      if (uv > 1)
        for (int i = t; i < h * w; i += 64) {  // vertical pass (anchor rows keep their values)
          const int yy = i / w, xx = i % w;
          if (yy % uv == uv - 1) continue;
          const int o = yy % uv + 1, kk = yy >> lv;
          const int before = yy < uv ? top[xx] : pred[(kk * uv - 1) * w + xx];
          pred[i] = ((uv - o) * before + o * pred[(kk * uv + uv - 1) * w + xx] + (1 << (lv - 1))) >> lv;
        }
    }
    __syncthreads();
    int sad = 0, satd = 0;
    for (int i = t; i < h * w; i += 64) sad += abs((int)S[(y + i / w) * W + x + i % w] - pred[i]);
    const int bw = w / 4, nb = bw * (h / 4);
    for (int bi = t; bi < nb; bi += 64) {
      const int bx = 4 * (bi % bw), by = 4 * (bi / bw);
      int d[16];
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const int yy = by + k / 4, xx = bx + k % 4;
        d[k] = (int)S[(y + yy) * W + x + xx] - pred[yy * w + xx];
      }
      satd += satd4x4(d);
    }
    sad = wave_sum(sad);
    satd = wave_sum(satd);
    const int cost = min(2 * sad, satd);
    if (t == 0) {
      if (a.cost) {
        a.cost[cbase + m] = cost;
        if (a.sad) a.sad[cbase + m] = sad;
        if (a.satd) a.satd[cbase + m] = satd;
      }
      best = min(best, ((uint32_t)cost << 5) | (uint32_t)m);  // ties to the lower mode
    }
    __syncthreads();  // rpred / pred are rewritten by the next mode
  }
  if (!a.cost && t == 0) {  // decisions only: fixup CUs are never split
    const size_t g = ((size_t)frame * a.nctus + c.ctu) * MIP_CUS_PER_CTU + c.cu;
    if (a.best_mode) a.best_mode[g] = (uint8_t)(best & 31);
    a.best_cost[g] = (int32_t)(best >> 5);
  }
}

}  // namespace

hipError_t launch_fixup(const SearchArgs &a, const FixupCu *cus, int n, int nframes, hipStream_t s) {
  if (n < 1 || nframes < 1) return hipSuccess;
  const long long groups = (long long)n * nframes;
  if (groups >= (1LL << 31) || !cus || (!a.cost && !a.best_cost)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fixup_kernel, dim3((unsigned)groups), dim3(64), 0, s, a, cus, n);
  return hipGetLastError();
}

}  // namespace mipgpu
