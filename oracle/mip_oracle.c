/* mip_oracle.c -- TEST INFRASTRUCTURE ONLY (see mip_oracle.h).
 *
 * A deliberately plain, scalar restatement of the reference algorithm, one CU and one
 * mode at a time, in frame coordinates.  No tiling, no vectorisation: readability is
 * the point; it is the checker for the HIP path, never part of it.
 *
 * Reference anchors (iagostorch/VVC-MIP-GPU @ /root/reference):
 *   boundaries          intra.cl:17-344   (initBoundaries)
 *   reduced prediction  intra.cl:349-543  (MIP_ReducedPred), weights mip_matrix.cl
 *   upsampling          intra.cl:815-912  (upsampleDistortion, horizontal then vertical)
 *   SAD / SATD / cost   intra.cl:922-1166, kernel_aux_functions.cl:142-249 (satd_4x4)
 *   2-D filters         intra.cl:2856-3040, 1639-1826, 3042-3265, 2311-2537
 *   separable filters   intra.cl:3267-3506, 1828-2087, 3508-3823, 2539-2854
 *   cost layout         constants.h:1558-1631 (ALL_stridedDistortionsPerCtu)
 */
#include "mip_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../vvc-mip-gpu_amd/csrc/mip_tables.h"

static const mip_shape_desc SHAPES[MIP_NUM_SHAPES] = MIP_SHAPE_TABLE;
static const uint8_t W_S0[16 * 16 * 4] = MIP_WEIGHTS_S0;
static const uint8_t W_S1[8 * 16 * 8] = MIP_WEIGHTS_S1;
static const uint8_t W_S2[6 * 64 * 7] = MIP_WEIGHTS_S2;
static const uint16_t TAPS3[5 * 9] = MIP_TAPS_3x3;
static const uint16_t TAPS5[3 * 25] = MIP_TAPS_5x5;

static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) l++;
  return l;
}

static int axis_pos(int base, int step, int dual, int i) {
  return dual ? base + (i / 2) * step + (i % 2) * dual : base + i * step;
}

int mipo_num_ctus(int width, int height) {
  return ((width + 127) / 128) * ((height + 127) / 128); /* intra.cl:31-33 */
}

int64_t mipo_costs_per_frame(int width, int height) {
  return (int64_t)mipo_num_ctus(width, height) * MIP_COSTS_PER_CTU;
}

/* ---------------------------------------------------------------- boundaries --- */

/* Complete and reduced boundaries of the CU at frame position (x, y).
 * Padding rules intra.cl:96-107 (top) and 232-243 (left); box downsampling with
 * (sum + 2^(log2 df - 1)) >> log2 df, intra.cl:71-73, 127-141, 202-204, 259-279.
 * A downsampling factor of 1 is a plain copy (the OpenCL `1 << -1` rounding term
 * truncates to 0 in a short, intra.cl:73). */
void mipo_cu_boundaries(const uint16_t *refs, int width, int height, int x, int y, int w,
                        int h, int16_t *top, int16_t *left, int16_t *red_top,
                        int16_t *red_left) {
  (void)height;
  for (int i = 0; i < w; i++) {
    int v;
    if (y > 0) v = refs[(size_t)(y - 1) * width + x + i];
    else if (x == 0) v = 512;
    else v = refs[x - 1];
    top[i] = (int16_t)v;
  }
  for (int i = 0; i < h; i++) {
    int v;
    if (x > 0) v = refs[(size_t)(y + i) * width + x - 1];
    else if (y == 0) v = 512;
    else v = refs[(size_t)(y - 1) * width];
    left[i] = (int16_t)v;
  }
  const int rbs = (w == 4 && h == 4) ? 2 : 4;
  for (int side = 0; side < 2; side++) {
    const int n = side ? h : w;
    const int16_t *src = side ? left : top;
    int16_t *dst = side ? red_left : red_top;
    const int df = n / rbs, l2 = ilog2(df), rnd = df > 1 ? 1 << (l2 - 1) : 0;
    for (int i = 0; i < rbs; i++) {
      int s = 0;
      for (int t = 0; t < df; t++) s += src[i * df + t];
      dst[i] = (int16_t)((s + rnd) >> l2);
    }
  }
}

/* --------------------------------------------------------- reduced prediction --- */

/* Clip events of the reduced prediction ([0]: below 0, [1]: above 1023), for tests that
 * need inputs exercising both clips (mipo_clip_counts). */
static long long mipo_clips[2];

void mipo_clip_counts(long long *out, int reset) {
  out[0] = __atomic_load_n(&mipo_clips[0], __ATOMIC_RELAXED);
  out[1] = __atomic_load_n(&mipo_clips[1], __ATOMIC_RELAXED);
  if (reset) mipo_clips[0] = mipo_clips[1] = 0;
}

/* Matrix-vector product of one mode, intra.cl:415-487.  Output stored at the
 * transposed position for transposed modes (intra.cl:402-406, 485). */
void mipo_reduced_pred(int size_id, int mode, int transposed, const int16_t *red_top,
                       const int16_t *red_left, int16_t *pred) {
  const int rbs = size_id == 0 ? 2 : 4;
  const int r = size_id == 2 ? 8 : 4;
  const int nin = 2 * rbs;
  int b[8];
  for (int i = 0; i < rbs; i++) {
    b[i] = transposed ? red_left[i] : red_top[i];
    b[rbs + i] = transposed ? red_top[i] : red_left[i];
  }
  const int b0 = b[0];
  int p[8];
  for (int i = 0; i < nin; i++) p[i] = b[i] - b0;
  p[0] = size_id == 2 ? 0 : (1 << 9) - b0; /* intra.cl:446 */
  int psum = 0;
  for (int i = 0; i < nin; i++) psum += p[i];
  const int offset = 32 - 32 * psum; /* intra.cl:449-454 */
  for (int j = 0; j < r * r; j++) {
    int acc = offset;
    for (int i = 0; i < nin; i++) {
      int w;
      if (size_id == 2) w = i == 0 ? 0 : W_S2[(mode * 64 + j) * 7 + i - 1]; /* 459-463 */
      else if (size_id == 1) w = W_S1[(mode * 16 + j) * 8 + i];
      else w = W_S0[(mode * 16 + j) * 4 + i];
      acc += p[i] * w;
    }
    int v = (acc >> 6) + b0;
    if (v < 0 || v > 1023) __atomic_fetch_add(&mipo_clips[v > 1023], 1, __ATOMIC_RELAXED);
    v = v < 0 ? 0 : (v > 1023 ? 1023 : v);
    const int pos = transposed ? (j % r) * r + j / r : j;
    pred[pos] = (int16_t)v;
  }
}

/* ------------------------------------------------------------------ upsampling --- */

/* intra.cl:815-912: horizontal pass on rows k*upV + upV-1 (left boundary as the
 * "before" sample of the first window), then vertical pass on every row (top
 * boundary as "before").  Factor 1 = copy. */
static void upsample(const int16_t *red, int r, int w, int h, const int16_t *top,
                     const int16_t *left, int16_t *out) {
  const int uh = w / r, uv = h / r, lh = ilog2(uh), lv = ilog2(uv);
  for (int k = 0; k < r; k++) {
    const int ya = k * uv + uv - 1;
    for (int x = 0; x < w; x++) {
      int v;
      if (uh == 1) {
        v = red[k * r + x];
      } else {
        const int o = x % uh + 1;
        const int before = x < uh ? left[ya] : red[k * r + (x >> lh) - 1];
        const int after = red[k * r + (x >> lh)];
        v = ((uh - o) * before + o * after + (1 << (lh - 1))) >> lh;
      }
      out[ya * w + x] = (int16_t)v;
    }
  }
  if (uv == 1) return;
  for (int y = 0; y < h; y++) {
    if (y % uv == uv - 1) continue; /* anchor rows keep their value */
    const int o = y % uv + 1, kk = y >> lv;
    for (int x = 0; x < w; x++) {
      const int before = y < uv ? top[x] : out[(kk * uv - 1) * w + x];
      const int after = out[(kk * uv + uv - 1) * w + x];
      out[y * w + x] = (int16_t)(((uv - o) * before + o * after + (1 << (lv - 1))) >> lv);
    }
  }
}

/* ------------------------------------------------------------------ distortion --- */

static int iabs(int v) { return v < 0 ? -v : v; }

/* 4x4 Hadamard SATD as in kernel_aux_functions.cl:142-249 (VTM xCalcHADs4x4 with the
 * JVET_R0164 DC scaling and final (satd+1)>>1). */
static int satd4x4(const int *d) {
  int m[16], e[16];
  for (int i = 0; i < 4; i++) {
    m[i] = d[i] + d[12 + i];
    m[4 + i] = d[4 + i] + d[8 + i];
    m[8 + i] = d[4 + i] - d[8 + i];
    m[12 + i] = d[i] - d[12 + i];
  }
  for (int i = 0; i < 4; i++) {
    e[i] = m[i] + m[4 + i];
    e[4 + i] = m[8 + i] + m[12 + i];
    e[8 + i] = m[i] - m[4 + i];
    e[12 + i] = m[12 + i] - m[8 + i];
  }
  for (int row = 0; row < 4; row++) {
    const int *s = e + 4 * row;
    int t0 = s[0] + s[3], t1 = s[1] + s[2], t2 = s[1] - s[2], t3 = s[0] - s[3];
    m[4 * row + 0] = t0 + t1;
    m[4 * row + 1] = t0 - t1;
    m[4 * row + 2] = t2 + t3;
    m[4 * row + 3] = t3 - t2;
  }
  int satd = 0;
  for (int k = 0; k < 16; k++) satd += iabs(m[k]);
  satd -= iabs(m[0]);
  satd += iabs(m[0]) >> 2;
  return (satd + 1) >> 1;
}

static void cu_distortion(const uint16_t *orig, int width, int x, int y, int w, int h,
                          const int16_t *pred, int *sad_out, int *satd_out) {
  int sad = 0, satd = 0;
  for (int yy = 0; yy < h; yy++)
    for (int xx = 0; xx < w; xx++)
      sad += iabs((int)orig[(size_t)(y + yy) * width + x + xx] - pred[yy * w + xx]);
  for (int by = 0; by < h; by += 4)
    for (int bx = 0; bx < w; bx += 4) {
      int d[16];
      for (int i = 0; i < 16; i++) {
        const int yy = by + i / 4, xx = bx + i % 4;
        d[i] = (int)orig[(size_t)(y + yy) * width + x + xx] - pred[yy * w + xx];
      }
      satd += satd4x4(d);
    }
  *sad_out = sad;
  *satd_out = satd;
}

/* ---------------------------------------------------------------------- search --- */

/* Is the reference's cost of the CU at frame position (x, y) defined?  The reference reads
 * samples by linear index y' * W + x' (intra.cl:100, 106, 236, 242, 718), so a CU right of
 * the frame reads the next row's samples -- deterministic -- as long as every index stays
 * below W * H.  The largest index a CU reads is its bottom-right original sample,
 * (y + h - 1) * W + x + w - 1 (its reference row / column indexes are smaller).  CUs with
 * y + h > H are skipped by initBoundaries (intra.cl:96-98, 232-234): stale LDS. */
int mipo_cu_defined(int width, int height, int x, int y, int w, int h) {
  return y + h <= height && (long long)(y + h - 1) * width + x + w - 1 < (long long)width * height;
}

static void search_ctu(const uint16_t *orig, const uint16_t *refs, int width, int height,
                       int ctu, int32_t *cost, int32_t *sad, int32_t *satd) {
  const int ctu_cols = (width + 127) / 128;
  const int cx = 128 * (ctu % ctu_cols), cy = 128 * (ctu / ctu_cols);
  int16_t top[64], left[64], rt[4], rl[4], red[64], pred[64 * 64];
  for (int s = 0; s < MIP_NUM_SHAPES; s++) {
    const mip_shape_desc *sd = &SHAPES[s];
    const int w = sd->w, h = sd->h, nm = 2 * sd->modes, r = sd->size_id == 2 ? 8 : 4;
    for (int cu = 0; cu < sd->ncu; cu++) {
      const int x = cx + axis_pos(sd->xb, sd->xs, sd->xd, cu % sd->ncols);
      const int y = cy + axis_pos(sd->yb, sd->ys, sd->yd, cu / sd->ncols);
      const size_t base = (size_t)ctu * MIP_COSTS_PER_CTU + sd->cost_offset + (size_t)cu * nm;
      if (!mipo_cu_defined(width, height, x, y, w, h)) {
        for (int m = 0; m < nm; m++) {
          cost[base + m] = MIPO_UNAVAILABLE;
          if (sad) sad[base + m] = MIPO_UNAVAILABLE;
          if (satd) satd[base + m] = MIPO_UNAVAILABLE;
        }
        continue;
      }
      mipo_cu_boundaries(refs, width, height, x, y, w, h, top, left, rt, rl);
      for (int m = 0; m < nm; m++) {
        mipo_reduced_pred(sd->size_id, m % sd->modes, m >= sd->modes, rt, rl, red);
        const int16_t *p = red;
        if (sd->size_id > 0) {
          upsample(red, r, w, h, top, left, pred);
          p = pred;
        }
        int a, b;
        cu_distortion(orig, width, x, y, w, h, p, &a, &b);
        cost[base + m] = 2 * a < b ? 2 * a : b; /* intra.cl:1166 */
        if (sad) sad[base + m] = a;
        if (satd) satd[base + m] = b;
      }
    }
  }
}

void mipo_search_ctus(const uint16_t *orig, const uint16_t *refs, int width, int height,
                      int ctu0, int ctu1, int32_t *cost, int32_t *sad, int32_t *satd,
                      int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
  for (int c = ctu0; c < ctu1; c++) search_ctu(orig, refs, width, height, c, cost, sad, satd);
  (void)nthreads;
}

void mipo_search_frame(const uint16_t *orig, const uint16_t *refs, int width, int height,
                       int32_t *cost, int32_t *sad, int32_t *satd, int nthreads) {
  mipo_search_ctus(orig, refs, width, height, 0, mipo_num_ctus(width, height), cost, sad,
                   satd, nthreads);
}

void mipo_best_modes(const int32_t *cost, int nctus, uint8_t *best_mode, int32_t *best_cost) {
  size_t cu_out = 0;
  for (int c = 0; c < nctus; c++)
    for (int s = 0; s < MIP_NUM_SHAPES; s++) {
      const mip_shape_desc *sd = &SHAPES[s];
      const int nm = 2 * sd->modes;
      for (int cu = 0; cu < sd->ncu; cu++, cu_out++) {
        const int32_t *row = cost + (size_t)c * MIP_COSTS_PER_CTU + sd->cost_offset + (size_t)cu * nm;
        int best = 0;
        for (int m = 1; m < nm; m++)
          if (row[m] < row[best]) best = m;
        best_mode[cu_out] = row[best] == MIPO_UNAVAILABLE ? 0xff : (uint8_t)best;
        if (best_cost) best_cost[cu_out] = row[best];
      }
    }
}

/* --------------------------------------------------------------------- filters --- */

#include "rcp_table.h"

/* The reference's float division v / s as compiled by the AMD OpenCL compiler for gfx950
 * (disassembly of oracle/_ref): v = mv * 2^ev, s = ms * 2^es (frexp), q = mv * rcp(ms)
 * with the hardware v_rcp_f32 (1 ulp; e.g. rcp(0.75) = 0x3faaaaaa), result ldexp(q, ev-es).
 * rcp values: rcp_table.h, captured on an MI355X by tools/rcp_table.hip.  The scales of
 * the filters are integers 1..1024. */
static float ref_fdiv(float v, int s) {
  int es, ev;
  (void)frexpf((float)s, &es);
  float rcp;
  const unsigned bits = MIPO_RCP_TABLE[s - 1];
  memcpy(&rcp, &bits, 4);
  const float mv = frexpf(v, &ev);
  const volatile float q = mv * rcp; /* one fp32 rounding, as v_mul_f32 */
  return ldexpf(q, ev - es);
}

/* ---------------------------------------------------------- filter tiles ---
 * Every filter kernel of the reference works on 128x32 quarter-CTU tiles, one work-group per
 * tile (wg = ty * tiles_x + tx, intra.cl:2873-2879), and addresses the frame by LINEAR index
 * (qy + r) * W + qx + c.  The oracle restates one tile at a time: tile_2d / tile_sep3 /
 * tile_sep5 fill the tile's LDS the way the reference does and compute its 128 x rows
 * outputs, each with a POISON flag = "depends on memory outside this frame" (a read at a
 * linear index >= W * H: the next frame slot or the buffer's padding, never written for this
 * frame).  A poisoned cell reads 0 (as the HIP kernel does), so poisoned outputs still get
 * a value -- one the reference does not define.  filter_run then writes them like the
 * reference (see there).
 *
 * LDS cell: value, or -1 for a cell the reference marks invalid, and the poison flag. */
typedef struct {
  int16_t v;
  uint8_t p;
} cell_t;

/* Interior cell (ty, tc) of the tile at (qx, qy), read by linear index: right of the frame
 * the index wraps into the next row (intra.cl:2905, 3098, 3331, 3597); past the frame end it
 * is poison. */
static cell_t interior_cell(const uint16_t *in, int W, int H, int qx, int qy, int ty, int tc) {
  const long long idx = (long long)(qy + ty) * W + qx + tc;
  cell_t c = {0, 0};
  (void)H;
  if (idx < (long long)W * H) c.v = (int16_t)in[idx];
  else c.p = 1;
  return c;
}

/* Halo gates of the 2-D quarter-CTU kernels: 3x3 intra.cl:2913-2966 (float twin 1696-1749),
 * 5x5 intra.cl:3103-3189 (float twin 2372-2461).  (ty, tc) outside the 128x32 interior. */
static int halo_valid_2d(int ksz, int qx, int qy, int ty, int tc, int W, int H) {
  const long long WH = (long long)W * H;
  const long long g = (long long)(qy + ty) * W + qx + tc;
  const int top = ty < 0, bot = ty >= 32, lft = tc < 0, rgt = tc >= 128;
  if ((top || bot) && (lft || rgt)) { /* corners */
    const int vy = top ? qy > 0 : qy + ty < H - 1;
    const int vx = lft ? qx > 0 : qx + tc < W - 1;
    return vy && vx;
  }
  if (top || bot) {
    if (!(g > 0 && g < WH)) return 0;
    if (ksz == 3) return 1;
    return top ? qy > 0 : qy + ty + 2 < H - 1;
  }
  return g > 0 && g < WH && qx + tc > 0 && qx + tc < W - 1;
}

static int round_div(int sum, int scale, int is_float) {
  if (is_float) return (int)roundf(ref_fdiv((float)sum, scale)); /* intra.cl:1794, 2507 */
  return (sum + scale / 2) / scale;                              /* intra.cl:3011, 3235 */
}

/* 2-D quarter-CTU kernels (intra.cl:2856, 1639, 3042, 2311): interior rows inside the frame
 * are read (linear index), other interior rows are -1 (2904-2909); halo cells per the gates.
 * Output = sum of c * v over the valid (>= 0) cells / sum of their c (2993-3011). */
static void tile_2d(const uint16_t *in, int W, int H, int qx, int qy, const uint16_t *taps, int ksz,
                    int is_float, int rows, int16_t *ov, uint8_t *op) {
  enum { P = 132 };
  static cell_t t[36 * P];
  const int R = ksz / 2;
  for (int ty = -R; ty < 32 + R; ty++)
    for (int tc = -R; tc < 128 + R; tc++) {
      cell_t c = {-1, 0};
      if (ty >= 0 && ty < 32 && tc >= 0 && tc < 128) {
        if (qy + ty < H) c = interior_cell(in, W, H, qx, qy, ty, tc);
      } else if (halo_valid_2d(ksz, qx, qy, ty, tc, W, H)) {
        c.v = (int16_t)in[(long long)(qy + ty) * W + qx + tc];
      }
      t[(ty + R) * P + tc + R] = c;
    }
  for (int r = 0; r < rows; r++)
    for (int c = 0; c < 128; c++) {
      int sum = 0, scale = 0, poison = 0;
      for (int dy = -R; dy <= R; dy++)
        for (int dx = -R; dx <= R; dx++) {
          const cell_t e = t[(r + dy + R) * P + c + dx + R];
          const int k = taps[(dy + R) * ksz + dx + R];
          poison |= e.p;
          if (e.v < 0) continue;
          sum += k * e.v;
          scale += k;
        }
      ov[r * 128 + c] = (int16_t)round_div(sum, scale, is_float);
      op[r * 128 + c] = (uint8_t)poison;
    }
}

/* Separable 3-tap kernels filterFrame_1d_{int,float} (intra.cl:3267, 1828):
 *  - taps t = row 0 of the 2-D kernel, applied horizontally and then vertically;
 *  - LDS zeroed (3311-3320), interior fetched UNGUARDED (3330-3332: rows below the frame
 *    read past its end -> poison), halo rows / columns / corners with the gates 3336-3366
 *    (unfetched halo cells stay 0);
 *  - horizontal pass over all 34 rows (3377-3405), vertical pass (3418-3478) with the
 *    closed-form scales: (2+t1)^2 inside, (1+t1)(2+t1) on a frame edge row / column,
 *    (1+t1)^2 in a corner (t0 = t2 = 1 for every kernel of the library) (3281-3285);
 *  - rounding: int (v + s/2)/s, float round(v/s) on float operands. */
static void tile_sep3(const uint16_t *in, int W, int H, int X, int Y, const uint16_t *taps, int is_float,
                      int rows, int16_t *ov, uint8_t *op) {
  enum { P = 130, R = 34 };
  static cell_t tile[R * P];
  static double hp[R * P];
  static uint8_t hpp[R * P];
  const int t0 = taps[0], t1 = taps[1], t2 = taps[2];
  memset(tile, 0, sizeof tile);
  for (int r = 0; r < 32; r++)
    for (int c = 0; c < 128; c++) tile[(r + 1) * P + c + 1] = interior_cell(in, W, H, X, Y, r, c);
  const long long WH = (long long)W * H;
  for (int side = 0; side < 2; side++)  /* top (row Y-1) and bottom (row Y+32) halo rows */
    for (int c = 0; c < 128; c++) {
      const long long idx = (long long)(Y - 1 + 33 * side) * W + X + c;
      if (idx > 0 && idx < WH) tile[(33 * side) * P + 1 + c].v = (int16_t)in[idx];
    }
  for (int r = 1; r <= 32; r++)       /* left (X-1) and right (X+128) halo columns */
    for (int side = 0; side < 2; side++) {
      const long long idx = (long long)(Y + r - 1) * W + X - 1 + 129 * side;
      if (idx > 0 && idx < WH && X + side > 0 && X + 129 * side < W - 1) tile[r * P + 129 * side].v = (int16_t)in[idx];
    }
  const long long b = (long long)Y * W + X;
  if (b - W - 1 > 0 && X > 0 && Y > 0) tile[0].v = (int16_t)in[b - W - 1];
  if (b - W + 128 > 0 && X + 128 < W - 1 && Y > 0) tile[129].v = (int16_t)in[b - W + 128];
  if (b + 32LL * W - 1 < WH && X > 0 && Y + 32 < H - 1) tile[33 * P].v = (int16_t)in[b + 32LL * W - 1];
  if (b + 32LL * W + 128 < WH && X + 128 < W - 1 && Y + 32 < H - 1) tile[33 * P + 129].v = (int16_t)in[b + 32LL * W + 128];
  for (int r = 0; r < R; r++)         /* horizontal pass (halo rows included) */
    for (int c = 1; c <= 128; c++) {
      const cell_t *e = tile + r * P + c;
      hp[r * P + c] = (double)e[-1].v * t0 + (double)e[0].v * t1 + (double)e[1].v * t2;
      hpp[r * P + c] = e[-1].p | e[0].p | e[1].p;
    }
  const int full = 4 * t0 + 4 * t1 + t1 * t1, corner = t0 + 2 * t1 + t1 * t1, edge = 2 * t0 + 3 * t1 + t1 * t1;
  for (int r = 0; r < rows; r++)
    for (int c = 0; c < 128; c++) {
      const int y = Y + r, x = X + c;
      const int nb = (y == 0) + (y == H - 1) + (x == 0) + (x == W - 1);
      const int sc = nb >= 2 ? corner : (nb ? edge : full);
      const int k = (r + 1) * P + c + 1;
      const double v = hp[k - P] * t0 + hp[k] * t1 + hp[k + P] * t2;
      const int poison = hpp[k - P] | hpp[k] | hpp[k + P];
      int res;
      if (is_float) res = (int)roundf(ref_fdiv((float)v, sc));
      else res = ((int)v + sc / 2) / sc;
      ov[r * 128 + c] = (int16_t)res;
      op[r * 128 + c] = (uint8_t)poison;
    }
}

/* Separable 5-tap kernels filterFrame_1d_{int,float}_5x5 (intra.cl:3508, 2539):
 *  - LDS filled with -1 (3576-3585), interior rows inside the frame fetched (3595-3598),
 *    halo per the gates 3606-3688;
 *  - horizontal pass only for tile rows that are frame rows (3705-3726), -1 cells count 0;
 *  - vertical pass: each row without a horizontal pass drops its tap weight from the 2-D full
 *    scale, then the position classes (outer / inner edge rows and columns, corners,
 *    "interface") select 2-D sub-sums of the 5x5 kernel as the scale (3523-3557, 3749-3788). */
static void tile_sep5(const uint16_t *in, int W, int H, int X, int Y, const uint16_t *k2d, int is_float,
                      int rows, int16_t *ov, uint8_t *op) {
  enum { P = 132, R = 36 };
  static cell_t tile[R * P];
  static double hp[R * P];
  static uint8_t hpp[R * P];
  static int hv[R];
  const uint16_t *t = k2d; /* row 0 */
  int full = 0, oc = 0, ic = 0, itf = 0, oe = 0, ie = 0;
  for (int i = 0; i < 5; i++)
    for (int j = 0; j < 5; j++) {
      const int v = k2d[i * 5 + j];
      full += v;
      if (i >= 2 && j >= 2) oc += v;
      if (i >= 1 && j >= 1) ic += v;
      if (i >= 1 && j >= 2) itf += v;
      if (j >= 2) oe += v;
      if (j >= 1) ie += v;
    }
  for (int i = 0; i < R * P; i++) tile[i] = (cell_t){-1, 0};
  const long long WH = (long long)W * H, b = (long long)Y * W + X;
  for (int r = 0; r < 32; r++)
    if (Y + r < H)
      for (int c = 0; c < 128; c++) tile[(r + 2) * P + c + 2] = interior_cell(in, W, H, X, Y, r, c);
  for (int r = 0; r < 2; r++)         /* top halo rows Y-2, Y-1 */
    for (int c = 0; c < 128; c++) {
      const long long idx = b - 2LL * W + (long long)r * W + c;
      if (idx > 0 && idx < WH && Y > 0) tile[r * P + 2 + c].v = (int16_t)in[idx];
    }
  for (int r = 34; r < 36; r++)       /* bottom halo rows Y+32, Y+33: need Y + r < H - 1 */
    for (int c = 0; c < 128; c++) {
      const long long idx = b - 2LL * W + (long long)r * W + c;
      if (idx > 0 && idx < WH && Y + r < H - 1) tile[r * P + 2 + c].v = (int16_t)in[idx];
    }
  for (int r = 0; r < 32; r++)        /* side halo columns X-2, X-1, X+128, X+129 */
    for (int q = 0; q < 4; q++) {
      const int c = q < 2 ? q : q + 128;
      const long long idx = b - 2 + (long long)r * W + c;
      if (idx > 0 && idx < WH && X - 2 + c > 0 && X - 2 + c < W - 1) tile[(2 + r) * P + c].v = (int16_t)in[idx];
    }
  if (X > 0 && Y > 0) {
    tile[0].v = (int16_t)in[b - 2 * W - 2];
    tile[1].v = (int16_t)in[b - 2 * W - 1];
    tile[P].v = (int16_t)in[b - W - 2];
    tile[P + 1].v = (int16_t)in[b - W - 1];
  }
  if (Y > 0) {
    if (X + 128 < W - 1) {
      tile[P - 2].v = (int16_t)in[b - 2 * W + 128];
      tile[2 * P - 2].v = (int16_t)in[b - W + 128];
    }
    if (X + 129 < W - 1) {
      tile[P - 1].v = (int16_t)in[b - 2 * W + 129];
      tile[2 * P - 1].v = (int16_t)in[b - W + 129];
    }
  }
  if (X > 0) {
    if (Y + 32 < H - 1) {
      tile[34 * P].v = (int16_t)in[b + 32LL * W - 2];
      tile[34 * P + 1].v = (int16_t)in[b + 32LL * W - 1];
    }
    if (Y + 33 < H - 1) {
      tile[35 * P].v = (int16_t)in[b + 33LL * W - 2];
      tile[35 * P + 1].v = (int16_t)in[b + 33LL * W - 1];
    }
  }
  if (Y + 32 < H - 1 && X + 129 < W - 1) tile[35 * P - 1].v = (int16_t)in[b + 32LL * W + 129];
  if (Y + 32 < H - 1 && X + 128 < W - 1) tile[35 * P - 2].v = (int16_t)in[b + 32LL * W + 128];
  if (Y + 33 < H - 1 && X + 129 < W - 1) tile[36 * P - 1].v = (int16_t)in[b + 33LL * W + 129];
  if (Y + 33 < H - 1 && X + 128 < W - 1) tile[36 * P - 2].v = (int16_t)in[b + 33LL * W + 128];
  for (int r = 0; r < R; r++) {       /* horizontal pass: tile rows that are frame rows */
    hv[r] = Y + r - 2 >= 0 && Y + r - 2 < H;
    if (!hv[r]) continue;
    for (int c = 2; c < 130; c++) {
      double acc = 0;
      uint8_t p = 0;
      for (int d = -2; d <= 2; d++) {
        const cell_t e = tile[r * P + c + d];
        acc += (double)(e.v < 0 ? 0 : e.v) * t[2 + d];
        p |= e.p;
      }
      hp[r * P + c] = acc;
      hpp[r * P + c] = p;
    }
  }
  for (int r = 0; r < rows; r++)
    for (int c = 0; c < 128; c++) {
      const int y = Y + r, x = X + c;
      int sc = full, poison = 0;
      double v = 0;
      for (int d = -2; d <= 2; d++) {
        const int rr = r + 2 + d;
        if (!hv[rr]) {
          sc -= t[2 + d];
        } else {
          v += hp[rr * P + c + 2] * t[2 + d];
          poison |= hpp[rr * P + c + 2];
        }
      }
      const int otb = y == 0 || y == H - 1, itb = y == 1 || y == H - 2;
      const int olr = x == 0 || x == W - 1, ilr = x == 1 || x == W - 2;
      const int o_corner = otb && olr, i_corner = itb && ilr;
      const int iface = (olr && itb) || (ilr && otb);
      const int o_edge = !o_corner && !iface && (otb || olr);
      const int i_edge = !i_corner && !iface && (itb || ilr);
      if (o_corner) sc = oc;
      if (i_corner) sc = ic;
      if (o_edge) sc = oe;
      if (i_edge) sc = ie;
      if (iface) sc = itf;
      int res;
      if (is_float) res = (int)roundf(ref_fdiv((float)v, sc));
      else res = ((int)v + sc / 2) / sc;
      ov[r * 128 + c] = (int16_t)res;
      op[r * 128 + c] = (uint8_t)poison;
    }
}

/* Run a filter over the frame and write its outputs the way the reference does: every tile
 * stores all 128 columns of its min(32, H - qy) rows by linear index (intra.cl:3027-3038,
 * 3489-3505).  Samples x < W get their OWNING tile's value.  At widths that are not multiples
 * of 128 the last tile column also stores its columns c >= W - qx, which land on the next
 * row, over samples another work-group writes: the two stores race.  Where both values
 * agree the sample is well defined; where they differ (or either is poison) the reference's
 * result depends on the work-groups' timing and the sample is marked undefined.  `undef`
 * (may be NULL) receives, per sample, bit 0 = poison (reads past the frame's end), bit 1 =
 * race with a different value (0 = defined). */
static int filter_run(const uint16_t *in, uint16_t *out, uint8_t *undef, int W, int H, int filter, int kernel_idx) {
  const int five = filter >= MIPO_FILTER_1D_INT_5x5;
  const int sep = filter == MIPO_FILTER_1D_INT || filter == MIPO_FILTER_1D_FLOAT || filter == MIPO_FILTER_1D_INT_5x5 ||
                  filter == MIPO_FILTER_1D_FLOAT_5x5;
  const int is_float = filter == MIPO_FILTER_1D_FLOAT || filter == MIPO_FILTER_2D_FLOAT ||
                       filter == MIPO_FILTER_1D_FLOAT_5x5 || filter == MIPO_FILTER_2D_FLOAT_5x5;
  if (kernel_idx < 0 || kernel_idx >= (five ? 3 : 5)) return -1;
  const uint16_t *taps = five ? TAPS5 + 25 * kernel_idx : TAPS3 + 9 * kernel_idx;
  static int16_t ov[32 * 128];
  static uint8_t op[32 * 128];
  const long long WH = (long long)W * H;
  uint8_t *und = undef ? undef : (uint8_t *)malloc((size_t)WH);
  if (!und) return -1;
  const int tiles_x = (W + 127) / 128, qx_last = 128 * (tiles_x - 1);
  for (int pass = 0; pass < 2; pass++) /* 0: owning stores, 1: the wrapped stores */
    for (int qy = 0; qy < H; qy += 32)
      for (int qx = pass ? qx_last : 0; qx < W; qx += 128) {
        if (pass && W - qx >= 128) continue;
        const int rows = H - qy < 32 ? H - qy : 32;
        if (!sep) tile_2d(in, W, H, qx, qy, taps, five ? 5 : 3, is_float, rows, ov, op);
        else if (five) tile_sep5(in, W, H, qx, qy, taps, is_float, rows, ov, op);
        else tile_sep3(in, W, H, qx, qy, taps, is_float, rows, ov, op);
        for (int r = 0; r < rows; r++)
          for (int c = pass ? W - qx : 0; c < (pass ? 128 : (W - qx < 128 ? W - qx : 128)); c++) {
            const long long idx = (long long)(qy + r) * W + qx + c;
            if (idx >= WH) continue; /* past the frame: the next slot / padding */
            const uint16_t v = (uint16_t)ov[r * 128 + c];
            if (!pass) {
              out[idx] = v;
              und[idx] = op[r * 128 + c];
            } else {
              if (op[r * 128 + c]) und[idx] |= 1;
              if (v != out[idx]) und[idx] |= 2;
            }
          }
      }
  if (!undef) free(und);
  return 0;
}

int mipo_filter_frame_ex(const uint16_t *in, uint16_t *out, uint8_t *undef, int width, int height, int filter,
                         int kernel_idx) {
  if (filter < 0 || filter > 7) return -1;
  return filter_run(in, out, undef, width, height, filter, kernel_idx);
}

int mipo_filter_frame(const uint16_t *in, uint16_t *out, int width, int height, int filter, int kernel_idx) {
  return mipo_filter_frame_ex(in, out, NULL, width, height, filter, kernel_idx);
}

/* CUs whose reference samples (read from a filtered frame, see mipo_cu_boundaries) include
 * an undefined sample of that frame (mipo_filter_frame_ex): 1 per CU in CU order
 * ctu*5380 + shape CU prefix + cu.  CUs the search itself leaves unavailable are not
 * marked. */
void mipo_ref_undefined_cus(const uint8_t *undef, int width, int height, uint8_t *cu_out) {
  const int ctu_cols = (width + 127) / 128, n = mipo_num_ctus(width, height);
  size_t k = 0;
  for (int ctu = 0; ctu < n; ctu++) {
    const int cx = 128 * (ctu % ctu_cols), cy = 128 * (ctu / ctu_cols);
    for (int s = 0; s < MIP_NUM_SHAPES; s++) {
      const mip_shape_desc *sd = &SHAPES[s];
      for (int cu = 0; cu < sd->ncu; cu++, k++) {
        const int x = cx + axis_pos(sd->xb, sd->xs, sd->xd, cu % sd->ncols);
        const int y = cy + axis_pos(sd->yb, sd->ys, sd->yd, cu / sd->ncols);
        int bad = 0;
        if (mipo_cu_defined(width, height, x, y, sd->w, sd->h)) {
          if (y > 0)
            for (int i = 0; i < sd->w; i++) bad |= undef[(size_t)(y - 1) * width + x + i];
          else if (x > 0)
            bad |= undef[x - 1];
          if (x > 0)
            for (int i = 0; i < sd->h; i++) bad |= undef[(size_t)(y + i) * width + x - 1];
          else if (y > 0)
            bad |= undef[(size_t)(y - 1) * width];
        }
        cu_out[k] = (uint8_t)bad;
      }
    }
  }
}

/* ------------------------------------------------------------- synthetic frames --- */

static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Integer-only generators so C and numpy (tests/synth.py) agree bit for bit.
 * kind 0: smooth ramps + triangle-wave texture + per-32x32 DC offsets + noise (+-16);
 * kind 1: uniform 10-bit noise. */
void mipo_synth_frame(uint16_t *out, int width, int height, uint64_t seed, int kind) {
  for (int y = 0; y < height; y++)
    for (int x = 0; x < width; x++) {
      const uint64_t h = splitmix64(seed * 0x100000001B3ull + (uint64_t)y * (uint64_t)width + (uint64_t)x);
      int v;
      if (kind == 1) {
        v = (int)(h & 1023);
      } else if (kind == 2) {
        v = (int)(h % 3);
      } else {
        const uint64_t hb = splitmix64(seed ^ ((uint64_t)(y >> 5) << 32) ^ (uint64_t)(x >> 5));
        const int ramp = ((x * 3 + y * 5) % 512);
        const int tp = (x + 2 * y) % 96;
        const int tri = (tp < 48 ? tp : 96 - tp) * 4;
        const int dc = (int)(hb & 255) - 128;
        const int noise = (int)((h >> 20) & 31) - 16;
        v = 200 + ramp + tri - 96 + dc + noise;
        v = v < 0 ? 0 : (v > 1023 ? 1023 : v);
      }
      out[(size_t)y * width + x] = (uint16_t)v;
    }
}
