// mipgpu.cpp -- C-ABI engine (include/mipgpu.h): device set-up, buffers, work lists and
// the per-batch launch sequence that replaces main.cpp's OpenCL host loop.
#include "mipgpu.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "mip_kernels.h"
#include "mip_tables.h"
#include "chunk_plan.h"
#include "host_stage_hip.h"
#include "numa_place.h"
#include "queue_ring.h"

namespace {

thread_local std::string g_err;

int fail(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return -1;
}

// MIPGPU_SLOW_CALLS=MS (diagnostic): every HIP call made through HIP_TRY / SLOW_CALL that
// blocks the calling thread longer than MS milliseconds is reported on stderr.
double slow_call_ms() {
  static const double v = getenv("MIPGPU_SLOW_CALLS") ? atof(getenv("MIPGPU_SLOW_CALLS")) : 0.0;
  return v;
}
struct SlowCall {
  const char *what;
  std::chrono::steady_clock::time_point t0;
  explicit SlowCall(const char *w) : what(w) {
    if (slow_call_ms() > 0) t0 = std::chrono::steady_clock::now();
  }
  ~SlowCall() {
    if (slow_call_ms() <= 0) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms > slow_call_ms()) fprintf(stderr, "mipgpu slow call: %.3f ms %s\n", ms, what);
  }
};
#define SLOW_CALL(expr) ([&] { SlowCall _sc(#expr); return (expr); }())

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = SLOW_CALL(expr);                                               \
    if (_e != hipSuccess) return fail("%s: %s", #expr, hipGetErrorString(_e));     \
  } while (0)

const mip_shape_desc kShapes[MIP_NUM_SHAPES] = MIP_SHAPE_TABLE;
const char *const kShapeNames[MIP_NUM_SHAPES] = MIP_SHAPE_NAMES;
const uint8_t kW0[16 * 16 * 4] = MIP_WEIGHTS_S0;
const uint8_t kW1[8 * 16 * 8] = MIP_WEIGHTS_S1;
const uint8_t kW2[6 * 64 * 7] = MIP_WEIGHTS_S2;

int axis_pos(int base, int step, int dual, int i) {
  return dual ? base + (i / 2) * step + (i % 2) * dual : base + i * step;
}

// MIP coefficient tables for the MFMA (layout documented in mip_kernels.h).
uint16_t to_half(float f) {
  _Float16 h = (_Float16)f;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

std::vector<uint8_t> build_tables() {
  std::vector<uint8_t> t(mipgpu::kTableBytes, 0);
  uint16_t *w = reinterpret_cast<uint16_t *>(t.data());
  float *ctab = reinterpret_cast<float *>(t.data() + mipgpu::kWeightRows * 16);
  // one matrix row: a0 and w'_1..w'_{nin-1} -> A_j (see mip_kernels.h); returns sum_k A_jk
  auto put = [&](int row, double a0, const double *wp, int nin) {
    double sum_w = 0, sum_a = 0;
    for (int k = 1; k < nin; k++) sum_w += wp[k];
    double a[8] = {a0 - sum_w, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 1; k < nin; k++) a[k] = wp[k];
    for (int k = 0; k < 8; k++) {
      w[row * 8 + k] = to_half((float)a[k]);
      sum_a += a[k];
    }
    return sum_a;
  };
  // sizeId 2: inputs 1..7 use matrix columns 0..6 (p_0 == 0, mip_matrix.cl:441, intra.cl:459-463)
  for (int m = 0; m < 6; m++)
    for (int j = 0; j < 64; j++) {
      double wp[8] = {0};
      for (int k = 1; k < 8; k++) wp[k] = (kW2[(m * 64 + j) * 7 + k - 1] - 32) / 64.0;
      const double sa = put(m * 64 + j, 1.0, wp, 8);
      (void)sa;  // == 1: C' is the constant kAccInitS2
    }
  auto small = [&](int base, int modes, int nin, const uint8_t *src) {
    for (int m = 0; m < modes; m++)
      for (int j = 0; j < 16; j++) {
        const uint8_t *wr = src + (m * 16 + j) * nin;
        double wp[8] = {0};
        for (int k = 1; k < nin; k++) wp[k] = (wr[k] - 32) / 64.0;
        const double sa = put(base + m * 16 + j, (96 - wr[0]) / 64.0, wp, nin);
        ctab[base - mipgpu::kWeightRowOffS1 + m * 16 + j] = (float)(8.0 * (wr[0] - 32) + 0.5 - 1024.0 * sa);
      }
  };
  small(mipgpu::kWeightRowOffS1, 8, 8, kW1);
  small(mipgpu::kWeightRowOffS0, 16, 4, kW0);
  for (int i = 0; i < 4; i++) ctab[384 + i] = mipgpu::kAccInitS2;
  return t;
}

// Per-quadrant work lists.  The CUs of one size class inside quadrant q (several shapes
// share a class) are split into groups of at most class_slots() CUs; a group and a range
// of its mode pairs form a wave task.  Tasks are cut so that none exceeds half of a wave's
// fair share, then assigned longest-first to the least-loaded of the quadrant's `slices`
// lists (one per workgroup); each list stays in decreasing cost order, and the waves of a
// workgroup take its tasks dynamically.  Costs are VALU-instruction estimates per lane.
// MIPGPU_SHAPE_FILTER="i,j,..." (profiling knob) restricts the search to those shapes.
// Edge CTUs: the reference reads samples by linear index (intra.cl:100, 236, 718), so CUs
// right of the frame read the next row (defined costs, searched here too) and only two
// kinds of CU are undefined (MIP_COST_UNAVAILABLE here): CUs below the frame (y + h > H:
// stale LDS, intra.cl:96-98) and CUs whose bottom-right sample's linear index
// (y + h - 1) * W + x + w - 1 is past the frame end (in practice: touching the bottom row
// and reaching past the right edge).  Such CUs get no task.  CTUs with the same set of
// defined CUs share a *variant* (ctu_variants: usually the interior, the last CTU row and
// the last CTU); each variant has its own lists and a fill list of the unavailable cost
// entries (16-byte units inside the CTU's cost block).
struct WorkLists {
  std::vector<mipgpu::WaveTask> tasks;
  std::vector<mipgpu::Job> jobs;
  std::vector<int> list_begin;   // [variant][quadrant][slice] + 1
  std::vector<double> list_cost; // [variant][quadrant][slice]: estimated time of the list on one
                                 // workgroup (VALU instructions per lane, waves share its tasks)
  std::vector<uint32_t> fill;    // unavailable cost entries, uint4 index inside the CTU block
  std::vector<int> fill_begin;   // [variant][quadrant] + 1
  // decisions only: undefined CUs (CU index inside the CTU) per [variant][quadrant], and the
  // CUs whose mode pairs are cut over several tasks per [variant]
  std::vector<uint16_t> dfill, split;
  std::vector<int> dfill_begin, split_begin;
  int max_split = 0;
};

// Profiling knobs that give wrong tables by design (MIPGPU_SHAPE_FILTER, MIPGPU_NO_PAIRS) are
// honoured only by A/B builds made with KNOBS=-DMIPGPU_PROFILING_KNOBS (the option enters the
// build ID, mip_build_id()); a release build refuses to create an engine while they are set
// (mip_engine_create), so no caller -- CLI, C ABI, Python -- gets a silently wrong table.
#ifdef MIPGPU_PROFILING_KNOBS
constexpr bool kProfilingKnobs = true;
#else
constexpr bool kProfilingKnobs = false;
#endif
const char *const kWrongResultKnobs[] = {"MIPGPU_SHAPE_FILTER", "MIPGPU_NO_PAIRS"};

bool shape_selected(int s) {
  if (!kProfilingKnobs) return true;
  const char *flt = getenv("MIPGPU_SHAPE_FILTER");
  if (!flt || !*flt) return true;
  for (const char *p = flt; *p;) {
    char *end;
    const long v = strtol(p, &end, 10);
    if (end == p) break;
    if (v == s) return true;
    p = *end ? end + 1 : end;
  }
  return false;
}

// Task size cap = a wave's fair share / cut_factor (MIPGPU_CUT_FACTOR, tuning knob).
double cut_factor() {
  const char *e = getenv("MIPGPU_CUT_FACTOR");
  return e && atof(e) > 0 ? atof(e) : 2.0;
}

// Wide CUs (32x4, 16x4, 8x4, 32x8, 16x8) searched as their tall transposes (transposed
// classes, mip_kernels.h); MIPGPU_TRANSPOSE=0 (A/B knob) searches them as they are.
bool transpose_wide() {
  const char *e = getenv("MIPGPU_TRANSPOSE");
  return !(e && *e == '0');
}

// MIPGPU_NO_PAIRS=1 (profiling knob): tasks keep their prologue but search no mode pair.
bool no_pairs() {
  const char *e = getenv("MIPGPU_NO_PAIRS");
  return kProfilingKnobs && e && *e == '1';
}

// Estimated VALU instructions per lane for one mode pair of a task of `ncu` CUs.
// Is the cost of the CU at frame position (x, y) defined (mipgpu.layout.cu_defined,
// oracle mipo_cu_defined)?
bool cu_defined(int width, int height, int x, int y, int w, int h) {
  return y + h <= height && (long long)(y + h - 1) * width + x + w - 1 < (long long)width * height;
}

// Reference samples above 10 bits.  At widths that are not multiples of 128 the reference's
// separable filters give the last one or two frame columns values up to ~1.7 x 1023: the
// horizontal pass there sums the wrapped next-row samples while the scale is the frame-edge
// class (intra.cl:3446-3458, 3771-3788).  The search kernel's arithmetic is sized for 10-bit
// samples, so with alternative references the CUs that read columns W-2 or W-1 (their top
// row, left column or padding sample) are left to the exact per-CU kernel (fixup_kernel).
bool reads_last_columns(int width, int height, int x, int y, int w, int h) {
  (void)height;
  auto col_hit = [&](long long li) { const long long c = li % width; return c >= width - 2; };
  if (y > 0) {
    for (int i = 0; i < w; i++)
      if (col_hit((long long)(y - 1) * width + x + i)) return true;
  } else if (x > 0 && col_hit(x - 1)) {
    return true;
  }
  if (x > 0) {
    for (int i = 0; i < h; i++)
      if (col_hit((long long)(y + i) * width + x - 1)) return true;
  } else if (y > 0 && col_hit((long long)(y - 1) * width)) {
    return true;
  }
  return false;
}

// Filtered reference samples the reference leaves undefined because the filter reads memory
// past the frame's end ("poison"; the oracle's mipo_filter_frame_ex models the same and
// tests/test_gpu_parity.py compares the two).  The reference's filters work on 128x32 tiles
// (intra.cl:2873-2879) and address the frame by linear index; halo cells are gated by
// index < W*H (2D intra.cl:2913-2966 / 3103-3189 and float twins; separable 3336-3366,
// 3606-3688), so only interior cells can read past the end:
//   2-D and separable 5-tap: rows inside the frame are read (2904-2909, 3595-3598), so only
//     the last row right of the frame (wrapping past the end) -- at widths that are not
//     multiples of 128;
//   separable 3-tap: interior rows are read unguarded (3330-3332), so every row below the
//     frame (last tile band when H % 32 != 0) too.
// An output depends on the cells of its window (2-D: (2R+1)^2; separable: horizontal taps of
// the vertical taps' rows, 3377-3478 / 3705-3788).  Tiles store all their 128 columns by
// linear index (3027-3038, 3489-3505): the last tile column's columns right of the frame land
// on the next row, so their poison counts there too (where the two stores race with defined
// values, the engine keeps the owning tile's value: one of the reference's outcomes).
// Only the last tile band (rows [y0, H)) holds such cells; returned as a mask over it.
struct Poison {
  int y0 = 0;                  // first frame row of the mask
  std::vector<uint8_t> mask;   // [(H - y0) * W]: 1 = undefined (linear index - y0 * W)
  bool any = false;
  bool at(long long li, int width) const {
    const long long o = li - (long long)y0 * width;
    return o >= 0 && o < (long long)mask.size() && mask[(size_t)o];
  }
};

Poison filter_poison(int width, int height, int filter) {
  Poison ps;
  if (filter < 0) return ps;
  const bool sep = filter == MIP_FILTER_1D_INT || filter == MIP_FILTER_1D_FLOAT || filter == MIP_FILTER_1D_INT_5x5 ||
                   filter == MIP_FILTER_1D_FLOAT_5x5;
  const bool five = filter >= MIP_FILTER_1D_INT_5x5;
  const long long W = width, H = height, WH = W * H;
  ps.y0 = 32 * ((height - 1) / 32);
  ps.mask.assign((size_t)(H - ps.y0) * W, 0);
  const int qy = ps.y0, rows = std::min(32, height - qy);
  // cell poison of tile rows ty (interior 0..31) at tile column tc (0..127)
  auto cell = [&](int qx, int ty, int tc) -> bool {
    if (ty < 0 || ty >= 32 || tc < 0 || tc >= 128) return false;  // halo: gated, never poison
    const long long y = qy + ty;
    if (!(sep && !five) && y >= H) return false;  // 2-D / 5-tap separable: rows below not read
    return y * W + qx + tc >= WH;
  };
  const int R = five ? 2 : 1;
  for (int qx = 0; qx < width; qx += 128) {
    uint8_t out[32][128] = {};
    bool tile_any = false;
    for (int r = 0; r < rows; r++)
      for (int c = 0; c < 128; c++) {
        bool p = false;
        if (!sep) {
          for (int dy = -R; dy <= R && !p; dy++)
            for (int dx = -R; dx <= R && !p; dx++) p = cell(qx, r + dy, c + dx);
        } else {
          // vertical taps over rows r-R..r+R (5-tap: only rows with a horizontal pass,
          // i.e. frame rows, intra.cl:3705-3726), horizontal taps c-R..c+R of each
          for (int dy = -R; dy <= R && !p; dy++) {
            if (five && (qy + r + dy < 0 || qy + r + dy >= height)) continue;
            for (int dx = -R; dx <= R && !p; dx++) p = cell(qx, r + dy, c + dx);
          }
        }
        out[r][c] = p;
        tile_any |= p;
      }
    if (!tile_any) continue;
    for (int r = 0; r < rows; r++)
      for (int c = 0; c < 128; c++) {
        const long long li = (long long)(qy + r) * W + qx + c;  // owning or wrapped store
        if (out[r][c] && li < WH) {
          ps.mask[(size_t)(li - (long long)qy * W)] = 1;
          ps.any = true;
        }
      }
  }
  return ps;
}

// Does the CU at frame position (x, y) read a poisoned reference sample (its top row or the
// top-edge padding sample, its left column or the left-edge padding sample, by linear index
// as the reference's initBoundaries does, intra.cl:96-107, 232-243)?
bool reads_poison(const Poison &ps, int width, int x, int y, int w, int h) {
  if (!ps.any) return false;
  if (y > 0) {
    for (int i = 0; i < w; i++)
      if (ps.at((long long)(y - 1) * width + x + i, width)) return true;
  } else if (x > 0 && ps.at(x - 1, width)) {
    return true;
  }
  if (x > 0) {
    for (int i = 0; i < h; i++)
      if (ps.at((long long)(y + i) * width + x - 1, width)) return true;
  } else if (y > 0 && ps.at((long long)(y - 1) * width, width)) {
    return true;
  }
  return false;
}

// CTU -> variant = index of the CTU's set of CUs the search kernel computes (the others get
// MIP_COST_UNAVAILABLE from the fill lists; the fixup kernel overwrites its CUs after).
// Three maps share the variants (kMapOrig / kMapAltCaller / kMapAltEngine): original
// references (every defined CU); caller-supplied alternative references (minus the fixup CUs
// when the width is not a multiple of 128); the engine filter's references (minus the fixup
// CUs and minus the CUs that read a sample the reference's filter leaves undefined,
// filter_poison -- those are MIP_COST_UNAVAILABLE).
constexpr int kMapOrig = 0, kMapAltCaller = 1, kMapAltEngine = 2, kMaps = 3;
struct CtuVariants {
  std::vector<uint8_t> of_ctu[kMaps];
  std::vector<std::vector<bool>> pattern;         // [variant][CU in CTU order]
  std::vector<mipgpu::FixupCu> fixup[kMaps];      // ALT: CUs computed by the fixup kernel
};

CtuVariants ctu_variants(int width, int height, int filter) {
  CtuVariants v;
  const int cols = (width + 127) / 128, n = cols * ((height + 127) / 128);
  const Poison ps = filter_poison(width, height, filter);
  for (int map = 0; map < kMaps; map++)
    for (int c = 0; c < n; c++) {
      const int cx = 128 * (c % cols), cy = 128 * (c / cols);
      // only CTUs whose CUs reach the last columns can hold fixup CUs (wraps: W < 256)
      const bool near_edge = map != kMapOrig && width % 128 && (cx + 256 >= width || width < 256);
      // only CTUs whose CUs reach the poisoned band (one CTU row up: left columns wrap)
      const bool near_poison = map == kMapAltEngine && ps.any && cy + 256 > ps.y0;
      std::vector<bool> pat;
      pat.reserve(MIP_CUS_PER_CTU);
      int k = 0;
      for (int s = 0; s < MIP_NUM_SHAPES; s++) {
        const mip_shape_desc &sd = kShapes[s];
        for (int cu = 0; cu < sd.ncu; cu++, k++) {
          const int lx = axis_pos(sd.xb, sd.xs, sd.xd, cu % sd.ncols), ly = axis_pos(sd.yb, sd.ys, sd.yd, cu / sd.ncols);
          bool on = cu_defined(width, height, cx + lx, cy + ly, sd.w, sd.h);
          if (on && near_poison && reads_poison(ps, width, cx + lx, cy + ly, sd.w, sd.h)) on = false;
          if (on && near_edge && reads_last_columns(width, height, cx + lx, cy + ly, sd.w, sd.h)) {
            on = false;
            v.fixup[map].push_back(mipgpu::FixupCu{(uint32_t)c, (uint16_t)k, (uint8_t)s, 0});
          }
          pat.push_back(on);
        }
      }
      size_t var = 0;
      while (var < v.pattern.size() && v.pattern[var] != pat) var++;
      if (var == v.pattern.size()) v.pattern.push_back(pat);
      v.of_ctu[map].push_back((uint8_t)std::min<size_t>(var, 255));
    }
  return v;
}

double pair_cost(int cls, int ncu) {
  const int w = mipgpu::kClassW[cls], h = mipgpu::kClassH[cls];
  const int sid = mipgpu::class_size_id(w, h), v = mipgpu::kClassV[cls];
  const int nout = sid == 2 ? 64 : 16;
  const double blocks = (double)h / 4 / v;
  const double mfma = ((ncu + 7) / 8) * (nout / 16);
  return blocks * 200.0 + mfma * 12.0 + 40.0;
}

WorkLists build_work(int slices, int waves, int width, int height, const CtuVariants &cv) {
  WorkLists wl;
  const int cols = (width + 127) / 128;
  (void)cols;
  for (int vq = 0; vq < 4 * (int)cv.pattern.size(); vq++) {
    const int var = vq / 4, q = vq % 4;
    wl.fill_begin.push_back((int)wl.fill.size());
    wl.dfill_begin.push_back((int)wl.dfill.size());
    if (q == 0) {
      if (var > 0) wl.max_split = std::max(wl.max_split, (int)wl.split.size() - wl.split_begin.back());
      wl.split_begin.push_back((int)wl.split.size());
    }
    struct Piece { mipgpu::WaveTask t; double cost; };
    std::vector<Piece> pieces;
    std::vector<std::vector<mipgpu::Job>> cls_cus(mipgpu::kNumClasses);
    int shape_cu0 = 0;  // first CU of the shape inside the CTU (reference order)
    for (int s = 0; s < MIP_NUM_SHAPES; shape_cu0 += kShapes[s].ncu, s++) {
      if (!shape_selected(s)) continue;
      const mip_shape_desc &sd = kShapes[s];
      int cls = mipgpu::size_class(sd.w, sd.h);
      if (transpose_wide() && mipgpu::kClassTransposed[cls] >= 0) cls = mipgpu::kClassTransposed[cls];
      for (int cu = 0; cu < sd.ncu; cu++) {
        const int x = axis_pos(sd.xb, sd.xs, sd.xd, cu % sd.ncols), y = axis_pos(sd.yb, sd.ys, sd.yd, cu / sd.ncols);
        if (x / 64 != (q & 1) || y / 64 != (q >> 1)) continue;
        if (!cv.pattern[var][shape_cu0 + cu]) {
          const uint32_t off = sd.cost_offset + cu * 2 * sd.modes;  // multiple of 4 entries
          for (uint32_t u = 0; u < (uint32_t)(2 * sd.modes) / 4; u++) wl.fill.push_back(off / 4 + u);
          wl.dfill.push_back((uint16_t)(shape_cu0 + cu));
          continue;
        }
        cls_cus[cls].push_back(mipgpu::Job{(uint32_t)(sd.cost_offset + cu * 2 * sd.modes), (uint8_t)(x % 64),
                                           (uint8_t)(y % 64), (uint16_t)(shape_cu0 + cu)});
      }
    }
    double total = 0;
    for (int cls = 0; cls < mipgpu::kNumClasses; cls++) {
      const std::vector<mipgpu::Job> &v = cls_cus[cls];
      if (v.empty()) continue;
      const int nv = (int)v.size(), slots = mipgpu::class_slots(cls);
      const int sid = mipgpu::class_size_id(mipgpu::kClassW[cls], mipgpu::kClassH[cls]);
      const int modes = sid == 2 ? 6 : (sid == 1 ? 8 : 16);
      // groups (class, CUs): full tasks plus a remainder task of the class's row-part variant
      // when the remainder fits it; otherwise equal-sized groups
      // (variant tasks replace one base task when they occupy fewer lane-blocks: a task of
      // V row parts gives every lane H / (4 V) blocks per mode pair)
      std::vector<std::pair<int, int>> groups;
      const int var = mipgpu::kClassVariant[cls], rem = nv % slots;
      const int nvar = var >= 0 ? (rem + mipgpu::class_slots(var) - 1) / mipgpu::class_slots(var) : 0;
      if (rem > 0 && var >= 0 && nvar * mipgpu::kClassV[cls] < mipgpu::kClassV[var]) {
        for (int g = 0; g < nv / slots; g++) groups.push_back({cls, slots});
        for (int g = 0, at = 0; g < nvar; g++) {
          const int n = (rem - at) / (nvar - g);
          groups.push_back({var, n});
          at += n;
        }
      } else {
        const int ng = (nv + slots - 1) / slots;
        for (int g = 0, at = 0; g < ng; g++) {
          const int n = (nv - at) / (ng - g);
          groups.push_back({cls, n});
          at += n;
        }
      }
      for (int g = 0, at = 0; g < (int)groups.size(); g++) {
        const int gc = groups[g].first, n = groups[g].second;
        const uint32_t first = (uint32_t)wl.jobs.size();
        wl.jobs.insert(wl.jobs.end(), v.begin() + at, v.begin() + at + n);
        at += n;
        const double c = pair_cost(gc, n);
        pieces.push_back({mipgpu::WaveTask{(uint8_t)gc, (uint8_t)n, 0, (uint8_t)modes, first}, c});
        total += c * modes;
      }
    }
    // cut long tasks into pair ranges
    const double cap = std::max(1.0, total / (slices * waves) / cut_factor());
    std::vector<Piece> cut;
    for (const Piece &p : pieces) {
      const int np = p.t.q1 - p.t.q0;
      const int parts = std::max(1, std::min(np, (int)std::ceil(p.cost * np / cap)));
      if (parts > 1)
        for (uint32_t j = 0; j < p.t.ncu; j++) wl.split.push_back(wl.jobs[p.t.cu0 + j].cu);
      for (int i = 0; i < parts; i++) {
        Piece c = p;
        c.t.q0 = (uint8_t)(p.t.q0 + np * i / parts);
        c.t.q1 = (uint8_t)(p.t.q0 + np * (i + 1) / parts);
        c.cost = p.cost * (c.t.q1 - c.t.q0) + 150.0;
        if (no_pairs()) c.t.q1 = c.t.q0;  // profiling: task prologues only
        cut.push_back(c);
      }
    }
    std::stable_sort(cut.begin(), cut.end(), [](const Piece &a, const Piece &b) { return a.cost > b.cost; });
    const int bins = slices;
    std::vector<double> load(bins, 0.0);
    std::vector<std::vector<mipgpu::WaveTask>> lists(bins);
    for (const Piece &p : cut) {
      const int b = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      load[b] += p.cost;
      lists[b].push_back(p.t);
    }
    for (int b = 0; b < bins; b++) {
      wl.list_begin.push_back((int)wl.tasks.size());
      wl.tasks.insert(wl.tasks.end(), lists[b].begin(), lists[b].end());
      wl.list_cost.push_back(load[b] / waves);
    }
  }
  wl.list_begin.push_back((int)wl.tasks.size());
  wl.fill_begin.push_back((int)wl.fill.size());
  wl.dfill_begin.push_back((int)wl.dfill.size());
  if (!wl.split_begin.empty())
    wl.max_split = std::max(wl.max_split, (int)wl.split.size() - wl.split_begin.back());
  wl.split_begin.push_back((int)wl.split.size());
  return wl;
}

bool filter_valid(int f, int k) {
  if (f < 0 || f > 7) return false;
  const bool five = f >= 4;
  return k >= 0 && k < (five ? 3 : 5);
}

}  // namespace

struct mip_engine {
  int device = 0, width = 0, height = 0, nctus = 0, ctu_cols = 0;
  // NUMA placement of the engine's host side (numa_place.h): its GPU's node, whose memory
  // holds the engine's page-locked buffers and whose CPUs run its host threads.
  mipgpu::NumaPlace place;
  mip_opts opts{};
  // Host API pipeline (mip_search_frames): `stream` and `stream4` compute (chunks alternate
  // between them, so that one chunk's search takes the CUs its predecessor's drains), `stream2`
  // uploads, `stream3` downloads; per buffer slot, events order upload -> compute -> download
  // and a slot's reuse after its previous chunk (see mip_search_frames).
  hipStream_t stream = nullptr, stream2 = nullptr, stream3 = nullptr, stream4 = nullptr;
  // Buffer slots of the host pipeline: hp_slots regions of hp_cap frames each in the engine
  // buffers (d_frames, d_refs, d_costs, ...).  Large engines (max_batch >= 16): 4 slots of a
  // quarter of max_batch; small ones: 3 slots of max_batch frames (triple buffering, so that a
  // caller searching one frame per call -- the reference's per-frame loop with BUFFER_SLOTS 2,
  // main.cpp:886-898, main_aux_functions.h:5, 617 -- overlaps frame k+1's upload and frame
  // k-1's download with frame k's search).
  static constexpr int kHostSlots = 4;
  int hp_slots = 0, hp_cap = 0, hp_frames = 0;  // hp_frames: frames of the engine buffers
  // Decisions-only chunks: the packed running argmins of the CUs whose mode pairs are cut
  // over several tasks ([hp_frames][nCTUs][5380]); all ones outside the chunks in flight
  // (the unpacking kernel resets the entries it reads), so no initialising kernel runs.
  uint32_t *d_split_acc = nullptr;
  hipEvent_t slot_up[kHostSlots] = {}, slot_comp[kHostSlots] = {}, slot_down[kHostSlots] = {};
  // Chunks run through the slots in one global sequence across host-API calls, so that
  // asynchronous calls (mip_search_frames_async) keep the pipeline full; call k completes
  // at call_done[(k - 1) % kCallRing] (tickets are 1-based call numbers).
  uint64_t host_chunks = 0, host_calls = 0;
  static constexpr int kCallRing = 64;
  hipEvent_t call_done[kCallRing] = {};
  // A host-API call was made: device-API searches that filter into the engine's reference
  // scratch wait for the last call's completion, call_done[(host_calls - 1) % kCallRing]
  // (the host pipeline uses the same buffer; no extra event on the search stream).
  bool host_pending = false;
  // mip_trace_times: per-slot timing events around the chunk's upload and filter launch,
  // the chunk (sequence number, frames) whose events are pending, and the per-frame times
  // read so far.
  bool trace = false;
  hipEvent_t tr_ev[kHostSlots][4] = {};  // upload start / end, filter start / end
  uint64_t tr_chunk[kHostSlots] = {};
  int tr_frames[kHostSlots] = {}, tr_filter[kHostSlots] = {};
  std::vector<std::pair<double, double>> tr_times;
  // Page-locked bounce ring for pageable caller buffers of the host pipeline (host_stage.h).
  mipgpu::HostStage stage;
  uint16_t *d_frames = nullptr, *d_refs = nullptr;
  int32_t *d_costs = nullptr, *d_sad = nullptr, *d_satd = nullptr, *d_best_cost = nullptr;
  uint8_t *d_best = nullptr;
  // Work lists, one set per slice count (workgroups per CTU quadrant): small batches need
  // more, smaller workgroups to fill the chip (see pick_work).
  struct Work {
    int slices = 1;
    bool wide = false;  // lists for one 16-wave workgroup per CU (small launches, pick_work)
    mipgpu::WaveTask *d_tasks = nullptr;
    mipgpu::Job *d_jobs = nullptr;
    int *d_lists = nullptr;
    uint32_t *d_fill = nullptr;
    int *d_fill_begin = nullptr;
    uint16_t *d_dfill = nullptr, *d_split = nullptr;  // decisions only (WorkLists)
    int *d_dfill_begin = nullptr, *d_split_begin = nullptr;
    int max_split = 0;
    // Small launches: the frame's items longest first (SearchArgs::order), their estimated
    // costs in that order (pick_work's makespan model).
    uint32_t *d_order = nullptr;
    std::vector<double> order_cost;
    uint32_t nonempty = 0;  // items of a frame with tasks (original references): the first in d_order
  };
  std::vector<Work> work;
  // pick_work's choice per frame count for small launches (index into `work`), [alt][wide]
  // (the two reference modes have their own resident grids)
  std::vector<int> small_choice[2][2];
  uint8_t *d_tables = nullptr;
  uint8_t *d_ctu_var[kMaps] = {};           // [map][nctus] CTU variant (ctu_variants: orig /
                                            // caller refs / engine-filtered refs)
  mipgpu::FixupCu *d_fixup[kMaps] = {};     // alt refs: CUs of the exact per-CU kernel, per map
  int nfixup[kMaps] = {};
  int resident[2] = {0, 0};  // persistent search grid (workgroups resident on this device), [alt]
  int resident_wide[2] = {0, 0};  // the same for 16-wave workgroups
  int resident_four[2] = {0, 0};  // the four-wave twin's (8-wave workgroups; 0: not available)
  // Engine-owned reference scratch d_refs, written by the engine filter when a device-API
  // search has no caller references: every such search records refs_done on its stream, and
  // the next writer of d_refs (another device-API search, on any stream, or a host-API call)
  // waits for it first.
  hipEvent_t refs_done = nullptr;
  bool refs_pending = false;
  // Item-counter pairs of the persistent search kernel, used round robin; a pair is reused
  // only after the launch that last used it has completed (stream wait on its event), so
  // launches on different streams never share one.
  static constexpr int kQueueSlots = 16;
  uint32_t *d_queue = nullptr;
  hipEvent_t queue_done[kQueueSlots] = {};
  // Three rings: `queue` for device-API launches (any caller stream: reuse ordered by the
  // slot's event) and `hp_queue` / `hp_queue2` for the host pipeline, whose searches run on
  // the engine's own search streams `stream` / `stream4`, one ring each: launches on one
  // in-order stream never overlap, so such a ring needs neither the event record nor the
  // wait (two fewer queue packets per chunk on the search stream's critical path).  The pairs
  // are distinct memory (hp_queue: slots kQueueSlots..2 kQueueSlots-1 of d_queue, hp_queue2
  // the next kQueueSlots).
  struct QueueOps {
    mip_engine *e;
    int base;           // first counter pair of the ring in d_queue
    bool one_stream;    // every launch of the ring is on one stream: no events needed
    int wait(int slot, hipStream_t s) const {
      return one_stream ? 0 : hipStreamWaitEvent(s, e->queue_done[slot], 0) != hipSuccess;
    }
    int record(int slot, hipStream_t s) const {
      return one_stream ? 0 : hipEventRecord(e->queue_done[slot], s) != hipSuccess;
    }
    int clear(int slot, hipStream_t s) const {
      return hipMemsetAsync(e->d_queue + mipgpu::kQueueWords * (base + slot), 0, mipgpu::kQueueWords * sizeof(uint32_t),
                            s) != hipSuccess;
    }
    int sync(hipStream_t s) const { return hipStreamSynchronize(s) != hipSuccess; }
  };
  QueueRing<QueueOps, kQueueSlots> queue{QueueOps{this, 0, false}};
  QueueRing<QueueOps, kQueueSlots> hp_queue{QueueOps{this, kQueueSlots, true}};
  QueueRing<QueueOps, kQueueSlots> hp_queue2{QueueOps{this, 2 * kQueueSlots, true}};  // (stream4)
  // Input contract (10-bit samples): status words the search kernel sets when it stages a
  // sample above 1023 (SearchArgs::status), in page-locked host memory mapped into the
  // device.  One set of kStatusWords per host-API call (call c: set (c - 1) % kCallRing) and
  // one for the device API (set kCallRing), so that a violation is reported for the call
  // that searched the frame: mip_wait(c) reads call c's set (harvest_status), the device API
  // its own set (check_device_status).  status_harvested: calls <= it have had their set
  // read and cleared; call_errors: the flags of harvested calls not yet reported (ticket ->
  // 1 = frame samples, 2 = reference samples).
  uint32_t *h_status = nullptr, *d_status = nullptr;
  uint64_t status_harvested = 0;
  std::map<uint64_t, uint32_t> call_errors;  // (4: the call's merged launch failed)

  // Merged chunks (round 6).  A small host-API call (page-locked buffers, fewer frames than a
  // slot) that arrives while the pipeline is busy is not launched on its own: it opens -- or
  // joins -- the *open chunk*, whose frames are uploaded into one slot's region at the
  // calls' offsets as they arrive, and the chunk is searched by ONE launch of all its frames
  // (open_chunk / flush_open).  One-frame launches run at 0.177 ms against 0.13 ms per frame
  // in 4-frame launches (profiles/r05_small_batch_final.jsonl), so per-frame callers (the
  // reference's loop, main.cpp:678-1241) queueing calls get the multi-frame rate.  The chunk
  // is launched when it is full (merge_cap frames or kMergeCalls calls), when a call that
  // cannot join it arrives, when the next call finds the search launched before it completed
  // (the GPU would idle), at any mip_wait / mip_flush / synchronous call, and before any
  // device-API work of the engine.  (A first version also had a flusher thread that waited
  // for that search with hipEventSynchronize: beside the caller's submissions it made 8 queued
  // calls erratic, 2600-3000 frames/s against 5430 without it, profiles/r06_merge_rates.txt --
  // so there is none.)  MIPGPU_MERGE=0 (A/B knob): off.
  static constexpr int kMergeCalls = 32;
  struct Member {
    uint64_t call;
    int f0, n;  // frames [f0, f0 + n) of the chunk
    int32_t *costs, *sad, *satd, *best_cost;
    uint8_t *best_mode;
  };
  struct OpenChunk {
    bool active = false;
    uint64_t k = 0;       // chunk sequence number (slot k % hp_slots)
    int nb = 0;           // frames so far
    int cap = 0;          // frames it may take (merge_cap)
    unsigned sig = 0;     // outputs and reference source of its calls (merge_sig)
    std::vector<Member> members;
  } open;
  int last_slot = -1;  // slot of the last launched host-pipeline chunk (its slot_comp event)
  int last_frames = 0;  // frames of the last launched host-pipeline chunk (merge_cap)
  uint64_t stat_launches = 0, stat_merged_calls = 0, stat_merged_launches = 0;  // mip_host_stats
  // per-frame status pointers of merged launches ([kCallRing][hp_cap], page-locked, mapped;
  // row (first call - 1) % kCallRing), SearchArgs::frame_status
  uint32_t **h_frame_status = nullptr, **d_frame_status = nullptr;
  // Every public entry point that uses the engine holds `mu`: an engine is used by one thread
  // at a time (include/mipgpu.h); calls from several threads are serialised, not undefined.
  std::recursive_mutex mu;
};

namespace {
// CU count limit of one launch (int32 indices in the decision-list kernel).
constexpr long long kMaxCus = (1LL << 31) - 256;

// Items per workgroup from which a launch cuts its queue into XCD chunks and prefetches
// (mip_search.hip MIP_PREFETCH_MIN_ITEMS); below it, items are taken longest first.
constexpr int kSmallLaunchItemsPerGroup = 32;
// Per-item cost beyond its tasks (window staging, barriers, fills), in the task cost
// model's units (pair_cost: VALU instructions per lane).
constexpr double kItemOverhead = 600.0;

// MIPGPU_DEC_INLINE=1 (A/B knob): decisions-only chunks of the host pipeline initialise and
// unpack their split entries on the search stream (before round 5) instead of the download
// stream.
bool dec_inline() {
  const char *e = getenv("MIPGPU_DEC_INLINE");
  return e && *e == '1';
}

// MIPGPU_GATHER_DOWN=0 (A/B knob): merged decisions-only chunks download member by member.
bool gather_down() {
  const char *e = getenv("MIPGPU_GATHER_DOWN");
  return !(e && *e == '0');
}

// MIPGPU_PIPE_KERNEL (A/B knob) for the host pipeline's chunks: 4 (default) = the four-wave
// twin for small alternating chunks and for decisions-only chunks, 8 = the twin for every
// chunk, 6 = the six-wave kernel on one workgroup per CU for small alternating chunks, 0 = the
// six-wave kernel's full grid throughout.
int pipe_kernel() {
  const char *e = getenv("MIPGPU_PIPE_KERNEL");
  return e && (*e == '0' || *e == '6' || *e == '8') ? *e - '0' : 4;
}

// MIPGPU_EXT_DONE=0 (A/B knob): record the host pipeline's per-chunk completion event as a
// separate marker instead of on the search kernel's dispatch.
bool ext_done_enabled() {
  const char *e = getenv("MIPGPU_EXT_DONE");
  return !(e && *e == '0');
}

// Host pipeline search streams: 2 (chunks alternate between `stream` and `stream4`) or 1
// (MIPGPU_SEARCH_STREAMS=1, A/B knob: every search on `stream`).
int search_streams() {
  const char *e = getenv("MIPGPU_SEARCH_STREAMS");
  return e && *e == '1' ? 1 : 2;
}

bool lpt_order_enabled() {
  const char *e = getenv("MIPGPU_ORDER");  // A/B knob: 0 = raster item order in small launches
  return !(e && *e == '0');
}

// Makespan of `nframes` frames' items taken longest first (SearchArgs::order) by `groups`
// persistent workgroups: greedy list scheduling of the queue order.
double lpt_makespan(const std::vector<double> &order_cost, int nframes, int groups) {
  std::vector<double> fin(groups, 0.0);  // min-heap of finish times
  for (double c : order_cost)
    for (int f = 0; f < nframes; f++) {
      std::pop_heap(fin.begin(), fin.end(), std::greater<double>());
      fin.back() += c;
      std::push_heap(fin.begin(), fin.end(), std::greater<double>());
    }
  return *std::max_element(fin.begin(), fin.end());
}

// Small launches on 16-wave workgroups, one per CU (MIPGPU_WIDE: 0 = never, 1 = every small
// launch; default: below kWideItemsPerGroup items per CU at one slice).  Two 8-wave workgroups (round 4)
// on a CU progress at very different rates when both run an item (the SIMD arbiter serves the
// older waves first: 98 vs 170 us for the two items of a CU in a 1080p frame,
// profiles/r04_item_timeline_1frame.csv), so a launch of ~2 items per CU ends with one
// workgroup running alone; a 16-wave workgroup has all its waves on one item's tasks.
// Measured (profiles/r04_small_batch_wide.jsonl): 1 frame 0.185 -> 0.175 ms, 2 frames
// 0.293 -> 0.314 ms (without a second workgroup the item tails and window stagings idle the
// CU), 8-16 frames -9 %.
// Round 6 (six-wave 12-wave workgroups, tools/experiments/r06/small_ab.sh): 2-frame launches
// (3.98 items per CU) 0.2905 ms on 12-wave workgroups vs 0.2967 wide, 1 frame 0.1758 vs 0.1743
// -- the threshold moved from 4 to 3 items per CU (only one-frame 1080p launches go wide).
constexpr int kWideItemsPerGroup = 3;
bool wide_launch(long long items1, int cus) {
  if (cus < 1) return false;  // no 16-wave workgroup fits a CU of this device
  const char *e = getenv("MIPGPU_WIDE");
  if (e && *e == '0') return false;
  if (e && *e == '1') return true;
  return items1 < (long long)kWideItemsPerGroup * cus;
}

// Work lists for a launch of `nframes`: items (quadrant x slice) for the persistent grid.
// Large launches (>= kSmallLaunchItemsPerGroup items per workgroup at one slice): one slice.
// Small ones take their items longest first, on 8- or 16-wave workgroups (wide_launch); the
// slice count is the one whose predicted makespan (lpt_makespan, per frame count, cached) is
// the shortest.  (Before the LPT order: 1 frame -> 2 slices 5076 frames/s at 1080p (1: 4842,
// 4: 4770).)
const mip_engine::Work &pick_work(mip_engine *e, int nframes, int nrange, bool alt) {
  const int groups = e->resident[alt ? 1 : 0];
  const long long items1 = 4LL * nrange * nframes;  // items at one slice
  if (nrange != e->nctus || items1 >= (long long)kSmallLaunchItemsPerGroup * groups || !lpt_order_enabled()) {
    const int want = items1 < 1000 && nrange != e->nctus ? 2 : 1;
    const mip_engine::Work *best = nullptr;
    for (const mip_engine::Work &w : e->work)
      if (!w.wide && (!best || std::abs(w.slices - want) < std::abs(best->slices - want))) best = &w;
    return *best;
  }
  const bool wide = wide_launch(items1, e->resident_wide[alt ? 1 : 0]);
  std::vector<int> &cache = e->small_choice[alt ? 1 : 0][wide ? 1 : 0];
  if ((int)cache.size() <= nframes) cache.resize(nframes + 1, -1);
  int &ch = cache[nframes];
  if (ch < 0) {
    const int g = wide ? e->resident_wide[alt ? 1 : 0] : groups;
    double best = 0;
    for (size_t i = 0; i < e->work.size(); i++) {
      if (e->work[i].wide != wide) continue;
      const double m = lpt_makespan(e->work[i].order_cost, nframes, g);
      if (ch < 0 || m < best) ch = (int)i, best = m;
    }
  }
  return e->work[ch];
}
}  // namespace

// Samples above 10 bits seen by a search launched before this point (the kernels mark
// SearchArgs::status): the costs of that search are not the reference's, so the call that
// notices reports it (sticky until reported, then cleared).  The reference reads the CSV
// samples into unsigned short and its kernels take short* (main.cpp:364-384, intra.cl:17,
// 545), with 10-bit constants throughout (constants.cl:22-23, valueDC = 512, clip 1023);
// this engine's packed 16-bit / f16 arithmetic is exact for 10-bit samples only.
static uint32_t *status_set(mip_engine *e, int set) { return e->h_status + (size_t)set * mipgpu::kStatusWords; }

// Read and clear a status set: 0, or 1 (frame samples) | 2 (reference samples).
static uint32_t take_status(mip_engine *e, int set) {
  volatile uint32_t *st = status_set(e, set);
  const uint32_t f = (st[mipgpu::kStatusOrig] ? 1u : 0u) | (st[mipgpu::kStatusRefs] ? 2u : 0u);
  if (f) {
    st[mipgpu::kStatusOrig] = 0;
    st[mipgpu::kStatusRefs] = 0;
  }
  return f;
}

static int contract_error(uint32_t flags, const char *what) {
  return fail("input contract: %s samples above 10 bits (> 1023) in a frame searched by %s; its costs are not valid "
              "(samples must be 10-bit values)", (flags & 1) ? "frame" : "reference", what);
}

// Device API: the searches issued since the last check (asynchronous: reported by
// mip_check_input or the next device-API search call).
static int check_device_status(mip_engine *e) {
  const uint32_t f = take_status(e, mip_engine::kCallRing);
  return f ? contract_error(f, "a device-API search of this engine") : 0;
}

// Device pointers of the status sets the kernels mark.
static uint32_t *device_status(mip_engine *e) { return e->d_status + (size_t)mip_engine::kCallRing * mipgpu::kStatusWords; }
static uint32_t *call_status(mip_engine *e, uint64_t call) {
  return e->d_status + (size_t)((call - 1) % mip_engine::kCallRing) * mipgpu::kStatusWords;
}

// Host API: move the status sets of the completed calls (status_harvested, upto] into
// call_errors (only calls that saw a violation are kept, until mip_wait reports them: an
// entry is never dropped, so a call that searched samples above 1023 can never be waited for
// as a success; memory is bounded by the failed calls nobody waits for -- the Python
// binding's tickets wait when dropped).  Every call <= upto must have completed.
static void harvest_status(mip_engine *e, uint64_t upto) {
  for (uint64_t c = e->status_harvested + 1; c <= upto; c++) {
    const uint32_t f = take_status(e, (int)((c - 1) % mip_engine::kCallRing));
    if (f) e->call_errors[c] = f;
  }
  if (upto > e->status_harvested) e->status_harvested = upto;
}

// Host-API calls (synchronous) overwrite engine scratch: order them after the device-API
// searches still reading d_refs; once the call has synchronised both engine streams,
// those searches are complete too.
static int wait_refs_readers(mip_engine *e) {
  if (!e->refs_pending) return 0;
  HIP_TRY(hipStreamWaitEvent(e->stream, e->refs_done, 0));
  HIP_TRY(hipStreamWaitEvent(e->stream4, e->refs_done, 0));
  HIP_TRY(hipStreamWaitEvent(e->stream2, e->refs_done, 0));
  return 0;
}

// Launch the engine's open (merged) chunk, if any (defined with the host pipeline below).
static int flush_open(mip_engine *e);

// Device block cache (round 6).  Freeing a large device allocation halves every later
// host <-> device copy of the process on this platform -- 56.4 -> 28.7 GB/s, SDMA and blit
// copies alike, old and new buffers, whatever the NUMA placement or the number of streams
// (tools/free_repro.hip, profiles/r06_free_repro.txt: a standalone HIP program, no engine) --
// until some later page-locked allocation churn restores it, on some boxes only.  Engines are
// created and destroyed by serving processes (a resolution change), so engine buffers of at
// least kCacheMin bytes are not freed: mip_engine_destroy parks them in a process-wide cache,
// and later engines on the same device take the smallest parked block that fits (blocks are
// not split: the process holds at most its largest engine set).  hipMalloc failing for lack of
// memory releases the device's parked blocks and retries; mip_device_cache(device, 1, ...)
// releases them explicitly.  MIPGPU_DEVICE_CACHE=0 (A/B knob): plain hipMalloc / hipFree.
namespace {
constexpr size_t kCacheMin = 16u << 20;
struct BlockCache {
  std::mutex mu;
  std::map<void *, std::pair<int, size_t>> live;      // blocks handed out: (device, bytes)
  std::multimap<std::pair<int, size_t>, void *> idle;  // parked blocks by (device, bytes)
  uint64_t reused = 0;
};
BlockCache &block_cache() {
  static BlockCache *c = new BlockCache();  // (never destroyed: no hipFree at process exit)
  return *c;
}
bool device_cache_enabled() {
  const char *e = getenv("MIPGPU_DEVICE_CACHE");
  return !(e && *e == '0');
}
// hipMalloc on `device` (the current device) through the cache.
hipError_t dev_malloc(int device, void **p, size_t bytes) {
  if (bytes < kCacheMin || !device_cache_enabled()) return hipMalloc(p, bytes);
  BlockCache &c = block_cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.idle.lower_bound({device, bytes});
    if (it != c.idle.end() && it->first.first == device) {
      *p = it->second;
      c.live[*p] = it->first;
      c.idle.erase(it);
      c.reused++;
      return hipSuccess;
    }
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {  // release the parked blocks, retry
    (void)hipGetLastError();
    std::lock_guard<std::mutex> lk(c.mu);
    for (auto it = c.idle.begin(); it != c.idle.end();)
      if (it->first.first == device) {
        (void)hipFree(it->second);
        it = c.idle.erase(it);
      } else {
        ++it;
      }
    e = hipMalloc(p, bytes);
  }
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> lk(c.mu);
    c.live[*p] = {device, bytes};
  }
  return e;
}
void dev_free(void *p) {
  if (!p) return;
  BlockCache &c = block_cache();
  {
    std::lock_guard<std::mutex> lk(c.mu);
    auto it = c.live.find(p);
    if (it != c.live.end()) {
      c.idle.insert({it->second, p});
      c.live.erase(it);
      return;
    }
  }
  (void)hipFree(p);
}
}  // namespace

// NUMA placement of a device (numa_place.h; none when the bus id or its node is unknown).
static mipgpu::NumaPlace device_place(int device) {
  char bus[64] = {};
  if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) {
    (void)hipGetLastError();
    return mipgpu::NumaPlace();
  }
  return mipgpu::numa_place_of_pci(bus);
}

extern "C" {

void mip_opts_default(mip_opts *o) {
  if (!o) return;
  o->filter = MIP_FILTER_NONE;
  o->kernel_idx = 0;
  o->max_batch = 1;
  o->want_sad_satd = 0;
  o->slices_per_ctu = 0;
  o->best_k = 1;
}

const char *mip_last_error(void) { return g_err.c_str(); }
int mip_abi_version(void) { return MIPGPU_ABI_VERSION; }
#ifndef MIPGPU_BUILD_ID
#define MIPGPU_BUILD_ID "src:unversioned"
#endif
const char *mip_build_id(void) { return MIPGPU_BUILD_ID; }

int mip_num_ctus(int width, int height) { return ((width + 127) / 128) * ((height + 127) / 128); }
int64_t mip_costs_per_frame(int width, int height) { return (int64_t)mip_num_ctus(width, height) * MIP_COSTS_PER_CTU; }
int64_t mip_cus_per_frame(int width, int height) { return (int64_t)mip_num_ctus(width, height) * MIP_CUS_PER_CTU; }

const char *mip_shape_name(int shape) {
  return shape >= 0 && shape < MIP_NUM_SHAPES ? kShapeNames[shape] : "ERROR";
}

int mip_shape_info(int shape, int *w, int *h, int *modes, int *ncu, int *cost_offset) {
  if (shape < 0 || shape >= MIP_NUM_SHAPES) return fail("bad shape index %d", shape);
  const mip_shape_desc &s = kShapes[shape];
  if (w) *w = s.w;
  if (h) *h = s.h;
  if (modes) *modes = s.modes;
  if (ncu) *ncu = s.ncu;
  if (cost_offset) *cost_offset = (int)s.cost_offset;
  return 0;
}

int mip_unavailable_cus(int width, int height, int filter, uint8_t *cu_out) {
  if (!cu_out || width <= 0 || height <= 0 || width % 4 || height % 4) return fail("bad unavailable-CU arguments");
  if (filter < MIP_FILTER_NONE || filter > MIP_FILTER_2D_FLOAT_5x5) return fail("invalid filter %d", filter);
  const Poison ps = filter_poison(width, height, filter);
  const int cols = (width + 127) / 128, n = mip_num_ctus(width, height);
  size_t k = 0;
  for (int c = 0; c < n; c++) {
    const int cx = 128 * (c % cols), cy = 128 * (c / cols);
    for (int s = 0; s < MIP_NUM_SHAPES; s++) {
      const mip_shape_desc &sd = kShapes[s];
      for (int cu = 0; cu < sd.ncu; cu++, k++) {
        const int x = cx + axis_pos(sd.xb, sd.xs, sd.xd, cu % sd.ncols), y = cy + axis_pos(sd.yb, sd.ys, sd.yd, cu / sd.ncols);
        cu_out[k] = !cu_defined(width, height, x, y, sd.w, sd.h) || reads_poison(ps, width, x, y, sd.w, sd.h);
      }
    }
  }
  return 0;
}

int mip_cu_position(int shape, int cu, int *x, int *y) {
  if (shape < 0 || shape >= MIP_NUM_SHAPES) return fail("bad shape index %d", shape);
  const mip_shape_desc &s = kShapes[shape];
  if (cu < 0 || cu >= s.ncu) return fail("bad cu index %d for shape %d", cu, shape);
  if (x) *x = axis_pos(s.xb, s.xs, s.xd, cu % s.ncols);
  if (y) *y = axis_pos(s.yb, s.ys, s.yd, cu / s.ncols);
  return 0;
}

int mip_engine_destroy(mip_engine *e) {
  if (!e) return 0;
  {  // the open chunk is launched (its calls were accepted)
    std::lock_guard<std::recursive_mutex> lk(e->mu);
    (void)hipSetDevice(e->device);
    (void)flush_open(e);
  }
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  if (e->stream2) (void)hipStreamSynchronize(e->stream2);
  if (e->stream3) (void)hipStreamSynchronize(e->stream3);
  if (e->stream4) (void)hipStreamSynchronize(e->stream4);
  e->stage.abandon();
  for (void *p : {(void *)e->d_frames, (void *)e->d_refs, (void *)e->d_costs, (void *)e->d_sad,
                  (void *)e->d_satd, (void *)e->d_best, (void *)e->d_best_cost, (void *)e->d_split_acc,
                  (void *)e->d_tables})
    dev_free(p);
  for (int m = 0; m < kMaps; m++) {
    dev_free(e->d_ctu_var[m]);
    dev_free(e->d_fixup[m]);
  }
  dev_free(e->d_queue);
  if (e->h_status) (void)hipHostFree(e->h_status);
  if (e->h_frame_status) (void)hipHostFree(e->h_frame_status);
  for (hipEvent_t ev : e->queue_done)
    if (ev) (void)hipEventDestroy(ev);
  if (e->refs_done) (void)hipEventDestroy(e->refs_done);
  for (int i = 0; i < mip_engine::kHostSlots; i++)
    for (hipEvent_t ev : {e->slot_up[i], e->slot_comp[i], e->slot_down[i]})
      if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->call_done)
    if (ev) (void)hipEventDestroy(ev);
  for (auto &evs : e->tr_ev)
    for (hipEvent_t ev : evs)
      if (ev) (void)hipEventDestroy(ev);
  for (const mip_engine::Work &w : e->work)
    for (void *p : {(void *)w.d_tasks, (void *)w.d_jobs, (void *)w.d_lists, (void *)w.d_fill, (void *)w.d_fill_begin,
                    (void *)w.d_dfill, (void *)w.d_dfill_begin, (void *)w.d_split, (void *)w.d_split_begin,
                    (void *)w.d_order})
      dev_free(p);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->stream2) (void)hipStreamDestroy(e->stream2);
  if (e->stream3) (void)hipStreamDestroy(e->stream3);
  if (e->stream4) (void)hipStreamDestroy(e->stream4);
  delete e;
  return 0;
}

int mip_engine_create(int device, int width, int height, const mip_opts *opts, mip_engine **out) {
  if (!out) return fail("out is NULL");
  *out = nullptr;
  if (width <= 0 || height <= 0 || width % 4 || height % 4)
    return fail("frame size %dx%d must be positive multiples of 4", width, height);
  // 32-bit linear sample indexes in the kernels (the window reaches 128 columns and 64 rows
  // past the frame)
  if ((long long)(width + 128) * (height + 128) >= (1LL << 31))
    return fail("frame size %dx%d too large (linear sample index beyond 2^31)", width, height);
  mip_opts o;
  mip_opts_default(&o);
  if (opts) o = *opts;
  if (o.max_batch < 1) return fail("max_batch must be >= 1");
  if ((long long)o.max_batch * mip_num_ctus(width, height) * MIP_CUS_PER_CTU > kMaxCus)
    return fail("max_batch %d x %d CTUs exceeds %lld CUs per launch", o.max_batch, mip_num_ctus(width, height), kMaxCus);
  if (o.best_k == 0) o.best_k = 1;
  if (o.best_k < 1 || o.best_k > mipgpu::kMaxBestK) return fail("best_k %d out of range 1..%d", o.best_k, mipgpu::kMaxBestK);
  if (o.filter != MIP_FILTER_NONE) {
    if (!filter_valid(o.filter, o.kernel_idx)) return fail("invalid filter %d / kernel_idx %d", o.filter, o.kernel_idx);
  }
  if (!kProfilingKnobs)
    for (const char *k : kWrongResultKnobs)
      if (const char *v = getenv(k); v && *v)
        return fail("%s is set: a profiling knob that makes wrong cost tables by design, honoured only by A/B builds "
                    "(make KNOBS=-DMIPGPU_PROFILING_KNOBS); this release build refuses to run with it -- unset it", k);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail("device %d out of range (%d devices)", device, ndev);
  HIP_TRY(hipSetDevice(device));

  mip_engine *e = new mip_engine();
  e->device = device;
  e->place = device_place(device);
  e->stage.set_device(device);  // (the bounce ring's completion thread)
  e->stage.set_place(e->place);
  e->width = width;
  e->height = height;
  e->nctus = mip_num_ctus(width, height);
  e->ctu_cols = (width + 127) / 128;
  e->opts = o;
  // host pipeline slots (see mip_engine::hp_slots); the engine buffers hold all of them
  e->hp_slots = o.max_batch >= 16 ? 4 : 3;
  e->hp_cap = o.max_batch >= 16 ? o.max_batch / 4 : o.max_batch;
  e->hp_frames = std::max(o.max_batch, e->hp_slots * e->hp_cap);
  const size_t fs = (size_t)width * height, nb = (size_t)e->hp_frames;
  const size_t ncost = nb * e->nctus * MIP_COSTS_PER_CTU, ncu = nb * e->nctus * MIP_CUS_PER_CTU;
  auto cleanup = [&](int rc) { mip_engine_destroy(e); return rc; };
#define ALLOC(ptr, bytes)                                                               \
  do {                                                                                  \
    hipError_t _e = dev_malloc(device, (void **)&(ptr), (bytes));                       \
    if (_e != hipSuccess) return cleanup(fail("hipMalloc(%zu): %s", (size_t)(bytes), hipGetErrorString(_e))); \
  } while (0)
  {
    // The engine's streams are created with the device's greatest priority.  HIP maps streams
    // onto a few hardware queues per priority (GPU_MAX_HW_QUEUES, 4 on the MI355X boxes); a
    // process that already holds many streams of the default priority -- torch creates a pool
    // of 32 per priority level at its first torch.cuda.Stream() -- then shares those queues
    // with the engine's streams, and the host pipeline's downloads -- blit kernels on the
    // runtime torch's wheel bundles, which then serves the engine (DESIGN.md section 6,
    // pageable host buffers, round 5) -- queued behind the searches on a shared queue:
    // 8 queued 1-frame 1080p full-table calls 830 instead of 1000 frames/s,
    // the configs[2] shape 570-894 instead of 1026 (tools/e2e_probe.py --torch stream,
    // gpurun_out/r05l).  With an explicit priority both rates are restored (high or low alike;
    // high, so that a serving engine is not starved by other work).  MIPGPU_STREAM_PRIO
    // (A/B knob): "low" / "normal" (the plain default streams).
    int lo = 0, hi = 0, prio = 0;
    bool with_prio = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess;
    prio = hi;
    if (const char *sp = getenv("MIPGPU_STREAM_PRIO")) {
      if (!strcmp(sp, "low")) prio = lo;
      else if (!strcmp(sp, "normal")) with_prio = false;
    }
    for (hipStream_t *st : {&e->stream, &e->stream2, &e->stream3, &e->stream4})
      if ((with_prio ? hipStreamCreateWithPriority(st, hipStreamNonBlocking, prio)
                     : hipStreamCreateWithFlags(st, hipStreamNonBlocking)) != hipSuccess)
        return cleanup(fail("hipStreamCreate failed"));
  }
  // The slot events order the engine's own streams on this device only (uploads -> search ->
  // downloads; the kernels' dispatch packets carry the device-scope cache fences).
  // MIPGPU_SLOT_EVENTS (A/B knob): "nofence" drops their system-scope fences
  // (hipEventDisableSystemFence), "device" releases to device scope (hipEventReleaseToDevice).
  unsigned slot_flags = hipEventDisableTiming;
  if (const char *se = getenv("MIPGPU_SLOT_EVENTS")) {
    if (!strcmp(se, "nofence")) slot_flags |= hipEventDisableSystemFence;
    else if (!strcmp(se, "device")) slot_flags |= hipEventReleaseToDevice;
  }
  for (int i = 0; i < mip_engine::kHostSlots; i++)
    for (hipEvent_t *ev : {&e->slot_up[i], &e->slot_comp[i], &e->slot_down[i]})
      if (hipEventCreateWithFlags(ev, slot_flags) != hipSuccess) return cleanup(fail("hipEventCreate failed"));
  for (hipEvent_t &ev : e->call_done)
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return cleanup(fail("hipEventCreate failed"));
  ALLOC(e->d_frames, fs * nb * 2);  // (through the device block cache, dev_malloc)
  if (o.filter != MIP_FILTER_NONE) ALLOC(e->d_refs, fs * nb * 2);
  ALLOC(e->d_costs, ncost * 4);
  if (o.want_sad_satd) {
    ALLOC(e->d_sad, ncost * 4);
    ALLOC(e->d_satd, ncost * 4);
  }
  ALLOC(e->d_best, ncu * o.best_k);
  ALLOC(e->d_queue, mipgpu::kQueueWords * 3 * mip_engine::kQueueSlots * sizeof(uint32_t));
  if (hipMemset(e->d_queue, 0, mipgpu::kQueueWords * 3 * mip_engine::kQueueSlots * sizeof(uint32_t)) != hipSuccess)
    return cleanup(fail("hipMemset failed"));
  // Every engine stream takes its hardware queue now, and the copy streams their copy
  // engines (1 MiB each way through a page-locked buffer): HIP sets these up at their first
  // use (tools/experiments/r05/_r05ao.sh: the CLI's first download started 8-9 ms after the search it
  // waited for).  (The counters are zero: rewriting one is harmless.)
  {
    void *h = nullptr;
    const size_t nbytes = std::min<size_t>(1u << 20, fs * nb * 2);  // (d_frames' size)
    bool ok = hipHostMalloc(&h, nbytes, hipHostMallocDefault) == hipSuccess;
    for (hipStream_t st : {e->stream, e->stream4})
      ok = ok && hipMemsetAsync(e->d_queue, 0, sizeof(uint32_t), st) == hipSuccess;
    ok = ok && hipMemcpyAsync(e->d_frames, h, nbytes, hipMemcpyHostToDevice, e->stream2) == hipSuccess &&
         hipStreamSynchronize(e->stream2) == hipSuccess &&
         hipMemcpyAsync(h, e->d_frames, nbytes, hipMemcpyDeviceToHost, e->stream3) == hipSuccess;
    for (hipStream_t st : {e->stream, e->stream2, e->stream3, e->stream4})
      ok = ok && hipStreamSynchronize(st) == hipSuccess;
    if (h) (void)hipHostFree(h);
    if (!ok) return cleanup(fail("initialising the engine streams failed"));
  }
  for (hipEvent_t &ev : e->queue_done)
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return cleanup(fail("hipEventCreate failed"));
  const size_t status_bytes = (size_t)(mip_engine::kCallRing + 1) * mipgpu::kStatusWords * sizeof(uint32_t);
  const mipgpu::ScopedNodePolicy pol(e->place);  // (the engine's page-locked words on its node)
  const unsigned numa_flag = pol.applied() ? hipHostMallocNumaUser : 0u;
  if (hipHostMalloc((void **)&e->h_status, status_bytes, hipHostMallocMapped | hipHostMallocCoherent | numa_flag) !=
      hipSuccess)
    return cleanup(fail("hipHostMalloc (status words) failed"));
  memset(e->h_status, 0, status_bytes);
  if (hipHostGetDevicePointer((void **)&e->d_status, e->h_status, 0) != hipSuccess || !e->d_status)
    return cleanup(fail("hipHostGetDevicePointer (status words) failed"));
  {  // merged chunks' per-frame status pointers (mip_engine::h_frame_status)
    const size_t bytes = (size_t)mip_engine::kCallRing * e->hp_cap * sizeof(uint32_t *);
    if (hipHostMalloc((void **)&e->h_frame_status, bytes, hipHostMallocMapped | hipHostMallocCoherent | numa_flag) !=
        hipSuccess)
      return cleanup(fail("hipHostMalloc (frame status) failed"));
    memset(e->h_frame_status, 0, bytes);
    if (hipHostGetDevicePointer((void **)&e->d_frame_status, e->h_frame_status, 0) != hipSuccess || !e->d_frame_status)
      return cleanup(fail("hipHostGetDevicePointer (frame status) failed"));
  }
  if (hipEventCreateWithFlags(&e->refs_done, hipEventDisableTiming) != hipSuccess)
    return cleanup(fail("hipEventCreate failed"));
  for (int alt = 0; alt < 2; alt++) {
    if ((e->resident[alt] = mipgpu::search_resident_groups(alt != 0, false)) < 1)
      return cleanup(fail("cannot size the persistent search grid on device %d", device));
    // 16-wave workgroups (small launches) are optional: 0 when one does not fit a CU
    e->resident_wide[alt] = mipgpu::search_resident_groups(alt != 0, true);
    e->resident_four[alt] = mipgpu::search_resident_groups_four(alt != 0, false);
  }
  ALLOC(e->d_best_cost, ncu * o.best_k * 4);
  ALLOC(e->d_split_acc, ncu * 4);
  if (hipMemset(e->d_split_acc, 0xff, ncu * 4) != hipSuccess) return cleanup(fail("hipMemset failed"));
  const CtuVariants cv = ctu_variants(width, height, o.filter);
  if (cv.pattern.size() > (size_t)mipgpu::kMaxCtuVariants)
    return cleanup(fail("too many CTU variants (%zu)", cv.pattern.size()));
  for (int m = 0; m < kMaps; m++) {
    ALLOC(e->d_ctu_var[m], cv.of_ctu[m].size());
    if (hipMemcpy(e->d_ctu_var[m], cv.of_ctu[m].data(), cv.of_ctu[m].size(), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail("uploading CTU variants failed"));
    e->nfixup[m] = (int)cv.fixup[m].size();
    if (e->nfixup[m]) {
      ALLOC(e->d_fixup[m], cv.fixup[m].size() * sizeof(mipgpu::FixupCu));
      if (hipMemcpy(e->d_fixup[m], cv.fixup[m].data(), cv.fixup[m].size() * sizeof(mipgpu::FixupCu),
                    hipMemcpyHostToDevice) != hipSuccess)
        return cleanup(fail("uploading fixup CUs failed"));
    }
  }
  std::vector<int> slice_set;
  if (o.slices_per_ctu > 0) slice_set = {o.slices_per_ctu};
  else slice_set = {1, 2, 4};
  std::vector<std::pair<int, bool>> work_set;  // (slices, wide)
  for (int wide = 0; wide < 2; wide++)
    for (int sl : slice_set) work_set.push_back({sl, wide != 0});
  for (const auto &[sl, wide] : work_set) {
    const WorkLists wl = build_work(sl, wide ? mipgpu::kWideWaves : mipgpu::kSearchWaves, width, height, cv);
    mip_engine::Work w;
    w.slices = sl;
    w.wide = wide;
    e->work.push_back(w);
    mip_engine::Work &ew = e->work.back();
    ALLOC(ew.d_tasks, std::max<size_t>(1, wl.tasks.size()) * sizeof(mipgpu::WaveTask));
    ALLOC(ew.d_jobs, std::max<size_t>(1, wl.jobs.size()) * sizeof(mipgpu::Job));
    ALLOC(ew.d_lists, wl.list_begin.size() * sizeof(int));
    ALLOC(ew.d_fill, std::max<size_t>(1, wl.fill.size()) * sizeof(uint32_t));
    ALLOC(ew.d_fill_begin, wl.fill_begin.size() * sizeof(int));
    if ((!wl.fill.empty() &&
         hipMemcpy(ew.d_fill, wl.fill.data(), wl.fill.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(ew.d_fill_begin, wl.fill_begin.data(), wl.fill_begin.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail("uploading fill lists failed"));
    if ((!wl.tasks.empty() &&
         (hipMemcpy(ew.d_tasks, wl.tasks.data(), wl.tasks.size() * sizeof(mipgpu::WaveTask), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(ew.d_jobs, wl.jobs.data(), wl.jobs.size() * sizeof(mipgpu::Job), hipMemcpyHostToDevice) != hipSuccess)) ||
        hipMemcpy(ew.d_lists, wl.list_begin.data(), wl.list_begin.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail("uploading work lists failed"));
    ew.max_split = wl.max_split;
    {  // small launches: the frame's items longest first (original-reference lists' costs)
      const int per_ctu = 4 * sl;
      std::vector<double> cost((size_t)e->nctus * per_ctu);
      for (int c = 0; c < e->nctus; c++)
        for (int g = 0; g < per_ctu; g++) {
          const int q = g / sl, slc = g % sl, l = (cv.of_ctu[kMapOrig][c] * 4 + q) * sl + slc;
          const bool empty = wl.list_begin[l + 1] == wl.list_begin[l];
          cost[(size_t)c * per_ctu + g] = wl.list_cost[l] + (empty ? kItemOverhead / 8 : kItemOverhead);
        }
      std::vector<uint32_t> order(cost.size());
      for (size_t i = 0; i < order.size(); i++) order[i] = (uint32_t)i;
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
      ew.order_cost.resize(order.size());
      for (size_t i = 0; i < order.size(); i++) ew.order_cost[i] = cost[order[i]];
      for (uint32_t it : order) {  // (the empty items cost kItemOverhead / 8: they come last)
        const int c = (int)(it / per_ctu), g = (int)(it % per_ctu), q = g / sl, slc = g % sl;
        const int l = (cv.of_ctu[kMapOrig][c] * 4 + q) * sl + slc;
        if (wl.list_begin[l + 1] == wl.list_begin[l]) break;
        ew.nonempty++;
      }
      ALLOC(ew.d_order, order.size() * sizeof(uint32_t));
      if (hipMemcpy(ew.d_order, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess)
        return cleanup(fail("uploading the item order failed"));
    }
    if (getenv("MIPGPU_WORK_STATS"))  // diagnostic: list sizes per slice count
      fprintf(stderr, "mipgpu work %dx%d slices %d: %zu tasks, %zu jobs, %zu fill, %zu undefined CUs, %zu split CUs (max %d per CTU)\n",
              width, height, sl, wl.tasks.size(), wl.jobs.size(), wl.fill.size(), wl.dfill.size(), wl.split.size(),
              wl.max_split);
    ALLOC(ew.d_dfill, std::max<size_t>(1, wl.dfill.size()) * sizeof(uint16_t));
    ALLOC(ew.d_dfill_begin, wl.dfill_begin.size() * sizeof(int));
    ALLOC(ew.d_split, std::max<size_t>(1, wl.split.size()) * sizeof(uint16_t));
    ALLOC(ew.d_split_begin, wl.split_begin.size() * sizeof(int));
    if ((!wl.dfill.empty() &&
         hipMemcpy(ew.d_dfill, wl.dfill.data(), wl.dfill.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess) ||
        (!wl.split.empty() &&
         hipMemcpy(ew.d_split, wl.split.data(), wl.split.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(ew.d_dfill_begin, wl.dfill_begin.data(), wl.dfill_begin.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(ew.d_split_begin, wl.split_begin.data(), wl.split_begin.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail("uploading decision lists failed"));
  }
  const std::vector<uint8_t> tab = build_tables();
  ALLOC(e->d_tables, tab.size());
#undef ALLOC
  if (hipMemcpy(e->d_tables, tab.data(), tab.size(), hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail("uploading static tables failed"));
  *out = e;
  return 0;
}

int mip_topk_device(const int32_t *d_costs, int width, int height, int nframes, int k, uint8_t *d_modes,
                    int32_t *d_costs_k, void *stream) {
  if (!d_costs || nframes < 1 || width <= 0 || height <= 0) return fail("bad top-k arguments");
  if (k < 1 || k > mipgpu::kMaxBestK) return fail("k %d out of range 1..%d", k, mipgpu::kMaxBestK);
  if (!d_modes && !d_costs_k) return 0;
  const long long cus = (long long)nframes * mip_num_ctus(width, height) * MIP_CUS_PER_CTU;
  if (cus > kMaxCus) return fail("too many CUs");
  mipgpu::BestArgs b{d_costs, d_modes, d_costs_k, (int)cus, k};
  HIP_TRY(mipgpu::launch_best_modes(b, (hipStream_t)stream));
  return 0;
}

int mip_copy_device(const void *d_src, void *d_dst, size_t bytes, void *stream) {
  if (!d_src || !d_dst) return fail("bad copy arguments");
  HIP_TRY(mipgpu::launch_copy(d_src, d_dst, bytes, (hipStream_t)stream));
  return 0;
}

int mip_filter_device(const uint16_t *d_in, uint16_t *d_out, int width, int height, int nframes,
                      int filter, int kernel_idx, void *stream) {
  if (!d_in || !d_out || nframes < 1) return fail("bad filter arguments");
  if (!filter_valid(filter, kernel_idx)) return fail("invalid filter %d / kernel_idx %d", filter, kernel_idx);
  mipgpu::FilterArgs a{d_in, d_out, width, height, nframes, filter, kernel_idx};
  HIP_TRY(mipgpu::launch_filter(a, (hipStream_t)stream));
  return 0;
}

// caller_refs: d_refs holds caller-supplied reference frames (checked against the 10-bit
// contract like the frames; engine-filtered references are not: the separable filters'
// defined > 10-bit outputs at the last columns go to the fixup kernel).
static int search_device_impl(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs, int nframes,
                              int32_t *d_costs, int32_t *d_sad, int32_t *d_satd, uint8_t *d_best,
                              int32_t *d_best_cost, hipStream_t s, bool caller_refs, uint32_t *d_status,
                              int ctu0 = 0, int nrange = -1, uint32_t *split_acc = nullptr,
                              mipgpu::SplitArgs *defer_split = nullptr, hipEvent_t *done = nullptr,
                              uint32_t *const *frame_status = nullptr, bool alternating = false) {
  if (!e || !d_frames || nframes < 1) return fail("bad search arguments");
  // Decisions only (no cost table): the search writes each CU's decision into d_best /
  // d_best_cost; CUs whose mode pairs are cut over several tasks keep a packed running argmin
  // (cost << 5 | mode) in d_best_cost, set to all ones before and unpacked after the search.
  const bool decisions_only = d_costs == nullptr;
  if (decisions_only) {
    if (!d_best_cost) return fail("a search without d_costs needs d_best_cost (decisions only)");
    if (e->opts.best_k != 1) return fail("a search without d_costs needs best_k == 1 (got %d)", e->opts.best_k);
    if (d_sad || d_satd) return fail("a search without d_costs cannot produce SAD / SATD tables");
  }
  if (nrange < 0) nrange = e->nctus - ctu0;
  if (ctu0 < 0 || nrange < 1 || ctu0 + nrange > e->nctus)
    return fail("CTU range [%d, %d) outside the frame's %d CTUs", ctu0, ctu0 + nrange, e->nctus);
  const long long total_cus = (long long)nframes * e->nctus * MIP_CUS_PER_CTU;
  if (total_cus > kMaxCus) return fail("%d frames x %d CTUs exceed %lld CUs per launch", nframes, e->nctus, kMaxCus);
  const uint16_t *refs = d_refs;
  const bool engine_refs = !refs && e->opts.filter != MIP_FILTER_NONE;
  if (engine_refs) {
    if (nframes > e->opts.max_batch) return fail("nframes %d > max_batch %d", nframes, e->opts.max_batch);
    if (e->refs_pending) HIP_TRY(hipStreamWaitEvent(s, e->refs_done, 0));  // last reader of d_refs
    if (e->host_pending)  // host calls in flight (calls complete in order: the last one)
      HIP_TRY(hipStreamWaitEvent(s, e->call_done[(e->host_calls - 1) % mip_engine::kCallRing], 0));
    if (mip_filter_device(d_frames, e->d_refs, e->width, e->height, nframes, e->opts.filter,
                          e->opts.kernel_idx, s) != 0)
      return -1;
    refs = e->d_refs;
  }
  const bool alt = refs != nullptr && refs != d_frames;
  mipgpu::SearchArgs a{};
  a.orig = d_frames;
  a.refs = alt ? refs : d_frames;
  a.cost = d_costs;
  a.best_mode = decisions_only ? d_best : nullptr;
  a.best_cost = decisions_only ? d_best_cost : nullptr;
  a.sad = d_sad;
  a.satd = d_satd;
  const mip_engine::Work &work = pick_work(e, nframes, nrange, alt);
  int resident = work.wide ? e->resident_wide[alt ? 1 : 0] : e->resident[alt ? 1 : 0];
  // Host-pipeline chunks whose searches alternate between the two search streams and are too
  // small to prefetch (round 6).  At six waves per SIMD a full grid of the batched kernel
  // leaves no room on a CU for the next chunk's workgroups nor for the download stream's
  // unpacking / copy kernels, which wait for the search to drain (a kernel trace of 8 merged
  // one-frame calls: dec_split busy 1.3 ms instead of 28 us).  Such chunks run the four-wave
  // twin (8-wave workgroups, two per CU: the occupancy rounds 1-5 ran the whole pipeline at),
  // or -- MIPGPU_PIPE_KERNEL=6 -- one 12-wave workgroup per CU (8 queued one-frame
  // decisions-only calls 4740 -> 5100 frames/s, 32 calls 5550 -> 6340).
  const bool pipe_small = alternating && !work.wide &&
                          (long long)4 * work.slices * nrange * nframes < (long long)kSmallLaunchItemsPerGroup * resident;
  const int pk = pipe_kernel();
  // (decisions-only pipeline chunks of any size too: their downloads -- blit kernels on torch's
  // runtime -- and split unpacking run beside the next chunk's search; 8 queued 128-frame
  // calls 7097-7121 -> 7191-7247 frames/s, tools/experiments/r06/e2e_twin.sh; full-table
  // chunks are PCIe-bound either way and keep the six-wave kernel)
  const bool four = ((pk == 4 && (pipe_small || (decisions_only && done))) || (pk == 8 && done)) && !work.wide &&
                    e->resident_four[alt ? 1 : 0] > 0;
  if (four) resident = e->resident_four[alt ? 1 : 0];
  else if (pipe_small && pk == 6) resident = std::max(1, resident / 2);
  a.tasks = work.d_tasks;
  a.jobs = work.d_jobs;
  a.list_begin = work.d_lists;
  a.fill = work.d_fill;
  a.fill_begin = work.d_fill_begin;
  a.dfill = work.d_dfill;
  a.dfill_begin = work.d_dfill_begin;
  a.tables = reinterpret_cast<const uint4 *>(e->d_tables);
  // engine-filtered references (here or in the host pipeline) leave the CUs that read the
  // filter's undefined samples unavailable; caller-supplied references are taken as they are
  const int map = !alt ? kMapOrig : (caller_refs ? kMapAltCaller : kMapAltEngine);
  a.ctu_var = e->d_ctu_var[map];
  a.width = e->width;
  a.height = e->height;
  a.ctu_cols = e->ctu_cols;
  a.nctus = e->nctus;
  a.ctu0 = ctu0;
  a.nrange = nrange;
  a.slices = work.slices;
  a.status = d_status;  // the calling API's status set (mip_engine::h_status)
  a.frame_status = frame_status;  // merged chunks: each frame's own call's set
  a.check_refs = alt && caller_refs;
  a.order = lpt_order_enabled() ? work.d_order : nullptr;  // launch_search drops it for large / range launches
  // pair mode of 16-wave launches (original references; launch_search checks the rest)
  const char *pv = getenv("MIPGPU_PAIR");  // A/B knob: 0 = 16-wave launches take items one at a time
  a.nonempty = work.wide && !alt && a.order && !(pv && *pv == '0') ? work.nonempty * (uint32_t)nframes : 0;
  // MIPGPU_WAVE_TIMING=file (profiling): per-task cycles appended to `file` (synchronous;
  // one binary record of uint64 [workgroup][wave][kClockSlots] per launch), and the task
  // lists to `file`.tasks once.
  static const char *timing = getenv("MIPGPU_WAVE_TIMING");
  std::vector<uint64_t> clocks;
  if (timing) {
    const size_t n = (size_t)4 * work.slices * nrange * nframes * mipgpu::kClockSlots;
    HIP_TRY(hipMalloc((void **)&a.wave_clock, n * 8));
    HIP_TRY(hipMemsetAsync(a.wave_clock, 0, n * 8, s));
    clocks.resize(n);
    static std::atomic<bool> dumped{false};
    if (!dumped.exchange(true)) {
      const WorkLists wl = build_work(work.slices, work.wide ? mipgpu::kWideWaves : mipgpu::kSearchWaves, e->width, e->height,
                                      ctu_variants(e->width, e->height, e->opts.filter));
      if (FILE *f = fopen((std::string(timing) + ".tasks").c_str(), "w")) {
        fprintf(f, "{\"slices\": %d, \"list_begin\": [", work.slices);
        for (size_t i = 0; i < wl.list_begin.size(); i++) fprintf(f, "%s%d", i ? ", " : "", wl.list_begin[i]);
        fprintf(f, "], \"tasks\": [");
        for (size_t i = 0; i < wl.tasks.size(); i++)
          fprintf(f, "%s[%d, %d, %d, %d]", i ? ", " : "", wl.tasks[i].cls, wl.tasks[i].ncu, wl.tasks[i].q0, wl.tasks[i].q1);
        fprintf(f, "]}\n");
        fclose(f);
      }
    }
  }
  // split_acc + defer_split (host pipeline): the split CUs meet in split_acc, which holds all
  // ones outside the launches in flight, and the caller unpacks (and re-initialises) it on
  // its download stream -- no kernel but the search on the search stream
  if (decisions_only && split_acc && defer_split) a.split_acc = split_acc;
  else defer_split = nullptr;
  const mipgpu::SplitArgs sa{work.d_split, work.d_split_begin, a.ctu_var, d_best, d_best_cost,
                             e->nctus, ctu0, nrange, work.max_split, a.split_acc};
  if (defer_split) *defer_split = sa;
  if (decisions_only && !defer_split) HIP_TRY(mipgpu::launch_dec_split(sa, nframes, true, s));
  // the host pipeline's launches (on the engine's search streams) use their own rings
  auto &ring = s == e->stream ? e->hp_queue : s == e->stream4 ? e->hp_queue2 : e->queue;
  const int qbase = s == e->stream ? mip_engine::kQueueSlots : s == e->stream4 ? 2 * mip_engine::kQueueSlots : 0;
  const int slot = ring.acquire(s);
  if (slot < 0) return fail("ordering the search's item counter failed: %s", hipGetErrorString(hipGetLastError()));
  a.queue = e->d_queue + mipgpu::kQueueWords * (qbase + slot);
  // done (host pipeline): the chunk's completion event, recorded by the search kernel's own
  // dispatch when nothing follows it on s (saves a marker packet between two chunks'
  // searches); *done = nullptr tells the caller it was recorded
  const bool last = !(alt && e->nfixup[map]) && !engine_refs && !timing &&
                    (decisions_only ? defer_split != nullptr : !(d_best || d_best_cost)) && ext_done_enabled();
  hipEvent_t stop = done && last ? *done : nullptr;
  const hipError_t le = four ? SLOW_CALL(mipgpu::launch_search_four(a, nframes, alt, resident, false, s, stop))
                             : SLOW_CALL(mipgpu::launch_search(a, nframes, alt, resident, work.wide, s, stop));
  if (le == hipSuccess && stop) *done = nullptr;
  if (le != hipSuccess) {
    ring.failed(slot);  // the pair is cleared before its next use
    return fail("search launch failed: %s", hipGetErrorString(le));
  }
  if (ring.launched(slot, s) != 0) return fail("hipEventRecord failed");
  if (alt && e->nfixup[map]) HIP_TRY(mipgpu::launch_fixup(a, e->d_fixup[map], e->nfixup[map], nframes, s));
  if (engine_refs) {
    HIP_TRY(hipEventRecord(e->refs_done, s));
    e->refs_pending = true;
  }
  if (timing) {
    HIP_TRY(hipMemcpyAsync(clocks.data(), a.wave_clock, clocks.size() * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    (void)hipFree(a.wave_clock);
    if (FILE *f = fopen(timing, "ab")) {
      fwrite(clocks.data(), 8, clocks.size(), f);
      fclose(f);
    }
  }
  if (decisions_only) {
    if (!defer_split) HIP_TRY(mipgpu::launch_dec_split(sa, nframes, false, s));
  } else if (d_best || d_best_cost) {
    mipgpu::BestArgs b{d_costs, d_best, d_best_cost, (int)total_cus, e->opts.best_k};
    HIP_TRY(mipgpu::launch_best_modes(b, s));
  }
  return 0;
}

int mip_search_device(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs, int nframes,
                      int32_t *d_costs, int32_t *d_sad, int32_t *d_satd, uint8_t *d_best_mode,
                      int32_t *d_best_cost, void *stream) {
  if (!e) return fail("engine is NULL");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (check_device_status(e) != 0) return -1;
  HIP_TRY(hipSetDevice(e->device));
  if (flush_open(e) != 0) return -1;  // (device-API work orders itself after the host calls)
  return search_device_impl(e, d_frames, d_refs, nframes, d_costs, d_sad, d_satd, d_best_mode, d_best_cost,
                            (hipStream_t)stream, d_refs != nullptr && d_refs != d_frames, device_status(e));
}

int mip_check_input(mip_engine *e, void *stream) {
  if (!e) return fail("engine is NULL");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return check_device_status(e);
}

int mip_search_device_range(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs, int nframes,
                            int ctu_begin, int ctu_end, int32_t *d_costs, int32_t *d_sad, int32_t *d_satd,
                            void *stream) {
  if (!e) return fail("engine is NULL");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (!d_costs) return fail("d_costs is NULL");
  // an empty range (more CTU-row bands than CTU rows, mipgpu.split) is a successful no-op
  if (ctu_begin == ctu_end && ctu_begin >= 0 && ctu_end <= e->nctus) return 0;
  if (check_device_status(e) != 0) return -1;
  HIP_TRY(hipSetDevice(e->device));
  if (flush_open(e) != 0) return -1;
  return search_device_impl(e, d_frames, d_refs, nframes, d_costs, d_sad, d_satd, nullptr, nullptr,
                            (hipStream_t)stream, d_refs != nullptr && d_refs != d_frames, device_status(e), ctu_begin,
                            ctu_end - ctu_begin);
}

static int search_frames_chunks(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null, int nframes,
                                int32_t *costs_out, uint8_t *best_mode_out, int32_t *best_cost_out, int32_t *sad_out,
                                int32_t *satd_out, uint64_t call, bool sync);

// mip_trace_times: read the pending chunk times of slot `sl` (waits for its events).
static int drain_trace(mip_engine *e, int sl) {
  if (!e->tr_frames[sl]) return 0;
  float up = 0, fl = 0;
  HIP_TRY(hipEventSynchronize(e->tr_ev[sl][1]));
  HIP_TRY(hipEventElapsedTime(&up, e->tr_ev[sl][0], e->tr_ev[sl][1]));
  if (e->tr_filter[sl]) {
    HIP_TRY(hipEventSynchronize(e->tr_ev[sl][3]));
    HIP_TRY(hipEventElapsedTime(&fl, e->tr_ev[sl][2], e->tr_ev[sl][3]));
  }
  const int n = e->tr_frames[sl];
  for (int i = 0; i < n; i++) e->tr_times.push_back({(double)up / n, (double)fl / n});
  e->tr_frames[sl] = 0;
  return 0;
}

// ---- Merged chunks (mip_engine::open, round 6) ----
// Outputs and reference source of a host-API call: calls merge into one launch only when
// these agree (one kernel variant, one set of output tables for the chunk).
enum : unsigned { kSigCost = 1, kSigSad = 2, kSigSatd = 4, kSigBestMode = 8, kSigBestCost = 16, kSigRefs = 32, kSigDec = 64 };

// MIPGPU_MERGE (A/B / test knob): 0 = every call launches on its own; "hold" = small calls
// open a chunk even into an idle pipeline and only a full chunk, an incompatible call, a wait
// or a device-API call launch it (deterministic merges for tests).
static int merge_mode() {
  const char *e = getenv("MIPGPU_MERGE");
  if (e && *e == '0') return 0;
  return e && !strcmp(e, "hold") ? 2 : 1;
}

// Launch the open chunk: the engine filter over its frames (engine references), ONE search
// of all its frames -- each frame marking its own call's status set (SearchArgs::frame_status)
// -- each member call's downloads from its own frames, and each member call's completion
// event.  After a failure the members' tickets report it (call_errors flag 4).
static int flush_open(mip_engine *e) {
  mip_engine::OpenChunk &o = e->open;
  if (!o.active) return 0;
  o.active = false;  // (whatever happens below, the chunk is over)
  if (o.members.empty()) return 0;
  const uint64_t k = o.k, first = o.members.front().call;
  const int sl = (int)(k % e->hp_slots), nb = o.nb;
  const unsigned sig = o.sig;
  const bool dec = (sig & kSigDec) != 0;
  const size_t fs = (size_t)e->width * e->height, fo = (size_t)sl * e->hp_cap;
  const size_t cpf = (size_t)e->nctus * MIP_COSTS_PER_CTU, upf = (size_t)e->nctus * MIP_CUS_PER_CTU * e->opts.best_k;
  const hipStream_t up = e->stream2, down = e->stream3;
  const hipStream_t comp = search_streams() == 2 && (k & 1) ? e->stream4 : e->stream;
  auto run = [&]() -> int {
    uint16_t *d_frames = e->d_frames + fo * fs;
    const uint16_t *d_refs = (sig & kSigRefs) ? e->d_refs + fo * fs : nullptr;
    if (!(sig & kSigRefs) && e->opts.filter != MIP_FILTER_NONE) {  // on the upload stream, as a chunk's
      if (mip_filter_device(d_frames, e->d_refs + fo * fs, e->width, e->height, nb, e->opts.filter, e->opts.kernel_idx,
                            up) != 0)
        return -1;
      d_refs = e->d_refs + fo * fs;
    }
    HIP_TRY(hipEventRecord(e->slot_up[sl], up));
    HIP_TRY(hipStreamWaitEvent(comp, e->slot_up[sl], 0));
    // row (first - 1) % kCallRing: its previous user, the chunk of call first - kCallRing, has
    // completed (search_frames_call waits for that call before accepting call `first`)
    const size_t row = (size_t)((first - 1) % mip_engine::kCallRing) * e->hp_cap;
    for (const mip_engine::Member &m : o.members)
      for (int i = 0; i < m.n; i++) e->h_frame_status[row + m.f0 + i] = call_status(e, m.call);
    int32_t *d_costs = dec ? nullptr : e->d_costs + fo * cpf;
    int32_t *d_sad = (sig & kSigSad) ? e->d_sad + fo * cpf : nullptr;
    int32_t *d_satd = (sig & kSigSatd) ? e->d_satd + fo * cpf : nullptr;
    uint8_t *d_best = (sig & kSigBestMode) ? e->d_best + fo * upf : nullptr;
    int32_t *d_best_cost = (sig & kSigBestCost) || dec ? e->d_best_cost + fo * upf : nullptr;
    mipgpu::SplitArgs split{};
    const bool defer = dec && !dec_inline();
    hipEvent_t comp_done = e->slot_comp[sl];
    if (search_device_impl(e, d_frames, d_refs, nb, d_costs, d_sad, d_satd, d_best, d_best_cost, comp,
                           (sig & kSigRefs) != 0, call_status(e, first), 0, -1,
                           defer ? e->d_split_acc + fo * e->nctus * MIP_CUS_PER_CTU : nullptr, defer ? &split : nullptr,
                           &comp_done, e->d_frame_status + row, search_streams() == 2) != 0)
      return -1;
    if (comp_done) HIP_TRY(hipEventRecord(e->slot_comp[sl], comp));
    e->last_slot = sl;
    e->last_frames = nb;
    e->stat_launches++;
    e->stat_merged_launches++;
    e->stat_merged_calls += o.members.size();
    HIP_TRY(hipStreamWaitEvent(down, e->slot_comp[sl], 0));
    if (defer) HIP_TRY(mipgpu::launch_dec_split(split, nb, false, down));
    // Decisions-only members' downloads as one copy kernel writing straight into their
    // device-mapped page-locked buffers: one dispatch per chunk instead of two copies per
    // member.  Fewer queued commands, fewer of the runtime's host stalls (section 6 of
    // DESIGN.md): 32 queued one-frame calls' rounds 6397-6419 frames/s at the 25th percentile
    // instead of 4033-6187 (medians 6451-6477 vs 6423-6628; tools/experiments/r06/gather.sh).
    bool gathered = false;
    if (dec && gather_down() && 2 * o.members.size() <= (size_t)mipgpu::kMaxCopyPieces) {
      mipgpu::CopyPieces cp{};
      gathered = true;
      for (const mip_engine::Member &m : o.members) {
        const size_t f = (size_t)m.f0, n = (size_t)m.n;
        auto add = [&](void *host, const void *dev, size_t bytes) {
          void *dp = nullptr;
          if (!host) return;
          if (hipHostGetDevicePointer(&dp, host, 0) != hipSuccess || !dp) {
            (void)hipGetLastError();
            gathered = false;
            return;
          }
          cp.p[cp.n++] = mipgpu::CopyPiece{static_cast<const uint8_t *>(dev), static_cast<uint8_t *>(dp), bytes};
        };
        add(m.best_mode, d_best + f * upf, n * upf);
        add(m.best_cost, d_best_cost + f * upf, n * upf * 4);
      }
      if (gathered) HIP_TRY(mipgpu::launch_gather_copy(cp, down));
    }
    for (const mip_engine::Member &m : o.members) {
      if (gathered) break;
      const size_t f = (size_t)m.f0, n = (size_t)m.n;
      if (m.costs) HIP_TRY(hipMemcpyAsync(m.costs, d_costs + f * cpf, n * cpf * 4, hipMemcpyDeviceToHost, down));
      if (m.sad) HIP_TRY(hipMemcpyAsync(m.sad, d_sad + f * cpf, n * cpf * 4, hipMemcpyDeviceToHost, down));
      if (m.satd) HIP_TRY(hipMemcpyAsync(m.satd, d_satd + f * cpf, n * cpf * 4, hipMemcpyDeviceToHost, down));
      if (m.best_mode) HIP_TRY(hipMemcpyAsync(m.best_mode, d_best + f * upf, n * upf, hipMemcpyDeviceToHost, down));
      if (m.best_cost)
        HIP_TRY(hipMemcpyAsync(m.best_cost, d_best_cost + f * upf, n * upf * 4, hipMemcpyDeviceToHost, down));
    }
    HIP_TRY(hipEventRecord(e->slot_down[sl], down));
    return 0;
  };
  const int rc = run();
  if (rc != 0) {  // (as a failed call: wait for what was queued, restore the split accumulator)
    const std::string err = g_err;
    for (hipStream_t st : {e->stream2, e->stream, e->stream4, e->stream3}) (void)hipStreamSynchronize(st);
    (void)hipMemset(e->d_split_acc, 0xff, (size_t)e->hp_frames * e->nctus * MIP_CUS_PER_CTU * 4);
    g_err = err;
  }
  for (const mip_engine::Member &m : o.members) {  // completion of every member (its ticket)
    if (rc != 0) e->call_errors[m.call] |= 4u;
    (void)hipEventRecord(e->call_done[(m.call - 1) % mip_engine::kCallRing], down);
  }
  o.members.clear();
  o.nb = 0;
  return rc;
}

// Frames an open chunk may take: its search can start only when all of its frames are
// uploaded, and the uploads run during the search launched before it -- one 1080p frame
// uploads in ~80 us, a launch of n frames searches in ~130 n + 47 us --
// so a chunk after one of n frames takes at most 1.625 n + 0.6 frames (1, 2, 3, 5, 8, 13, ...:
// a chunk of a whole slot right after a one-frame launch left the GPU idle for six uploads).
// MIPGPU_MERGE=hold: up to a slot.
static int merge_cap(const mip_engine *e) {
  if (merge_mode() == 2) return e->hp_cap;
  return std::max(2, std::min(e->hp_cap, (13 * std::max(1, e->last_frames) + 5) / 8));
}

// Add a call to the open chunk (opening one if there is none): its frames (and caller
// references) are uploaded into the chunk's slot region at the chunk's next frame.
static int merge_call(mip_engine *e, const uint16_t *frames, const uint16_t *refs, int nframes, int32_t *costs,
                      uint8_t *best_mode, int32_t *best_cost, int32_t *sad, int32_t *satd, unsigned sig, uint64_t call) {
  mip_engine::OpenChunk &o = e->open;
  const size_t fs = (size_t)e->width * e->height;
  const hipStream_t up = e->stream2;
  if (!o.active) {
    if ((refs || e->opts.filter != MIP_FILTER_NONE) && !e->d_refs)
      HIP_TRY(dev_malloc(e->device, (void **)&e->d_refs, fs * e->hp_frames * 2));
    if (wait_refs_readers(e) != 0) return -1;
    e->refs_pending = false;
    o.k = e->host_chunks++;
    const int sl = (int)(o.k % e->hp_slots);
    o.active = true;
    o.nb = 0;
    o.cap = merge_cap(e);
    o.sig = sig;
    o.members.clear();
    // the slot's previous chunk is over once its downloads are (as search_frames_chunks)
    if (o.k >= (uint64_t)e->hp_slots) HIP_TRY(hipStreamWaitEvent(up, e->slot_down[sl], 0));
  }
  const size_t f = (size_t)(o.k % e->hp_slots) * e->hp_cap + o.nb;
  HIP_TRY(hipMemcpyAsync(e->d_frames + f * fs, frames, nframes * fs * 2, hipMemcpyHostToDevice, up));
  if (refs) HIP_TRY(hipMemcpyAsync(e->d_refs + f * fs, refs, nframes * fs * 2, hipMemcpyHostToDevice, up));
  o.members.push_back(mip_engine::Member{call, o.nb, nframes, costs, sad, satd, best_cost, best_mode});
  o.nb += nframes;
  return 0;
}

// One host-API call (mip_search_frames_async; mip_search_frames with sync = true: it waits for
// the call before returning, so no later call can queue behind its last chunks).
static int search_frames_call(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null, int nframes,
                              int32_t *costs_out, uint8_t *best_mode_out, int32_t *best_cost_out, int32_t *sad_out,
                              int32_t *satd_out, uint64_t *ticket, bool sync) {
  if (!e || !frames || nframes < 1 || !ticket) return fail("bad search arguments");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  *ticket = 0;
  if ((sad_out || satd_out) && !e->opts.want_sad_satd) return fail("engine created without want_sad_satd");
  HIP_TRY(hipSetDevice(e->device));
  const uint64_t next = e->host_calls + 1;
  // MIPGPU_MAX_INFLIGHT=D (A/B knob): call `next` waits on the host until call next - D has
  // completed (bounds the commands queued in the HIP runtime).
  if (const char *mi = getenv("MIPGPU_MAX_INFLIGHT"); mi && atoi(mi) > 0 && next > (uint64_t)atoi(mi)) {
    const uint64_t c = next - (uint64_t)atoi(mi);
    if (e->open.active && e->open.members.front().call <= c && flush_open(e) != 0) return -1;
    HIP_TRY(hipEventSynchronize(e->call_done[(c - 1) % mip_engine::kCallRing]));
  }
  // call `next` marks status set (next - 1) % kCallRing: the call that used it before (more
  // than kCallRing calls in flight) must have completed and been harvested first
  if (next > (uint64_t)mip_engine::kCallRing && e->status_harvested < next - mip_engine::kCallRing) {
    if (e->open.active && e->open.members.front().call <= next - mip_engine::kCallRing && flush_open(e) != 0) return -1;
    HIP_TRY(hipEventSynchronize(e->call_done[(next - 1) % mip_engine::kCallRing]));
    harvest_status(e, next - mip_engine::kCallRing);
  }
  // Merged chunks (mip_engine::open): a call with page-locked buffers and fewer frames than a
  // slot joins the open chunk (same outputs, room left), or opens one while the pipeline is
  // busy; anything else launches the open chunk first and takes the chunked path.
  {
    using mipgpu::host_pinned;
    const bool pinned = host_pinned(frames) && (!refs_or_null || host_pinned(refs_or_null)) &&
                        (!costs_out || host_pinned(costs_out)) && (!sad_out || host_pinned(sad_out)) &&
                        (!satd_out || host_pinned(satd_out)) && (!best_mode_out || host_pinned(best_mode_out)) &&
                        (!best_cost_out || host_pinned(best_cost_out));
    const bool dec = !costs_out && !sad_out && !satd_out && e->opts.best_k == 1 && (best_mode_out || best_cost_out);
    const unsigned sig = (costs_out ? kSigCost : 0) | (sad_out ? kSigSad : 0) | (satd_out ? kSigSatd : 0) |
                         (best_mode_out ? kSigBestMode : 0) | (best_cost_out ? kSigBestCost : 0) |
                         (refs_or_null ? kSigRefs : 0) | (dec ? kSigDec : 0);
    const int mode = merge_mode();
    const bool small = pinned && mode && !e->trace && nframes < e->hp_cap;
    mip_engine::OpenChunk &o = e->open;
    bool join = false;
    // the search launched before the open chunk has completed: the GPU would idle -- launch
    // the chunk now (this call then opens the next one)
    if (o.active && mode == 1 && e->last_slot >= 0 &&
        SLOW_CALL(hipEventQuery(e->slot_comp[e->last_slot])) == hipSuccess && flush_open(e) != 0)
      return -1;
    if (o.active) {
      join = small && o.sig == sig && o.nb + nframes <= o.cap && (int)o.members.size() < mip_engine::kMergeCalls;
      if (!join && flush_open(e) != 0) return -1;
    }
    if (!o.active && small && !sync && nframes <= merge_cap(e) &&
               (mode == 2 || (e->host_calls > 0 && SLOW_CALL(hipEventQuery(e->call_done[(e->host_calls - 1) %
                                                                              mip_engine::kCallRing])) == hipErrorNotReady))) {
      join = true;  // the pipeline is busy: open a chunk
    }
    if (join) {
      if (merge_call(e, frames, refs_or_null, nframes, costs_out, best_mode_out, best_cost_out, sad_out, satd_out, sig,
                     next) != 0)
        return -1;
      *ticket = ++e->host_calls;
      e->host_pending = true;
      if ((o.nb >= o.cap || (int)o.members.size() >= mip_engine::kMergeCalls || sync) && flush_open(e) != 0)
        return -1;
      return 0;
    }
  }
  const int rc = search_frames_chunks(e, frames, refs_or_null, nframes, costs_out, best_mode_out, best_cost_out,
                                      sad_out, satd_out, next, sync);
  // After a failure part-way through the chunks, the chunks already queued are waited for
  // here (no ticket covers them).
  if (rc != 0) {
    const std::string err = g_err;
    (void)hipStreamSynchronize(e->stream2);
    (void)hipStreamSynchronize(e->stream);
    (void)hipStreamSynchronize(e->stream4);
    (void)hipStreamSynchronize(e->stream3);
    // staged downloads of the calls before this one complete normally; this call's are dropped
    (void)e->stage.drain(e->host_calls);
    e->stage.abandon();
    (void)take_status(e, (int)((next - 1) % mip_engine::kCallRing));  // the failed call's chunks: no ticket
    // a decisions-only chunk may have been searched without its unpacking (which resets its
    // split_acc entries): restore all ones (the streams are idle now)
    (void)hipMemset(e->d_split_acc, 0xff, (size_t)e->hp_frames * e->nctus * MIP_CUS_PER_CTU * 4);
    g_err = err;
    return rc;
  }
  // completion on the download stream (every chunk ends there, after its search and
  // downloads, outputs or not): calls complete in order
  const uint64_t call = ++e->host_calls;
  HIP_TRY(hipEventRecord(e->call_done[(call - 1) % mip_engine::kCallRing], e->stream3));
  e->host_pending = true;
  *ticket = call;
  return 0;
}

int mip_search_frames_async(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null, int nframes,
                            int32_t *costs_out, uint8_t *best_mode_out, int32_t *best_cost_out, int32_t *sad_out,
                            int32_t *satd_out, uint64_t *ticket) {
  return search_frames_call(e, frames, refs_or_null, nframes, costs_out, best_mode_out, best_cost_out, sad_out,
                            satd_out, ticket, false);
}

static int search_frames_chunks(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null, int nframes,
                                int32_t *costs_out, uint8_t *best_mode_out, int32_t *best_cost_out, int32_t *sad_out,
                                int32_t *satd_out, uint64_t call, bool sync) {
  const size_t fs = (size_t)e->width * e->height;
  if ((refs_or_null || e->opts.filter != MIP_FILTER_NONE) && !e->d_refs)
    HIP_TRY(dev_malloc(e->device, (void **)&e->d_refs, fs * e->hp_frames * 2));
  if (wait_refs_readers(e) != 0) return -1;
  e->refs_pending = false;  // the waits above order every later use of the engine streams
  const size_t cpf = (size_t)e->nctus * MIP_COSTS_PER_CTU, upf = (size_t)e->nctus * MIP_CUS_PER_CTU * e->opts.best_k;
  // Chunks of `sb` frames rotate over the engine's hp_slots buffer slots (mip_engine::hp_slots:
  // 4 slots of a quarter of max_batch, or 3 slots of max_batch for engines below 16 frames)
  // through a three-stream pipeline: stream2 uploads chunk k+1 while `stream` searches chunk k
  // and stream3 downloads chunk k-1, so the copy engines (H2D and D2H) and the compute run
  // concurrently and the search kernels keep the whole GPU.  Per slot: the upload waits until
  // the previous chunk of the slot has been searched (its frames / refs are free), the search
  // waits for the upload and for the previous download of the slot's outputs, the download
  // waits for the search.  The chunk sequence (and so the slot rotation and these waits)
  // continues across calls, so asynchronous calls queue behind each other without draining
  // the pipeline -- with three slots even one-frame calls overlap (the reference's
  // BUFFER_SLOTS 2 loop: frame curr+1's upload during frame curr's kernels, main.cpp:886-898,
  // and a non-blocking read-back of slot curr % 2, main_aux_functions.h:617).  Transfers run
  // at DMA rate from page-locked host memory (mip_host_alloc); pageable buffers go through the
  // engine's page-locked bounce ring (host_stage.h), their downloads finished by mip_wait.
  const int nslots = e->hp_slots;
  // a slot is a fixed region of slot_cap frames of the engine buffers (chunk sizes differ
  // between calls -- outputs requested, call length -- but a slot's region never moves, so
  // the per-slot events order every reuse of it)
  const int slot_cap = e->hp_cap;
  // A call into an idle pipeline (nothing queued before it) is cut in two (at most a slot's
  // frames each), so that its own upload, search and download overlap; calls queued behind
  // others keep whole-slot chunks (the overlap comes from the neighbouring calls, and larger
  // launches are more efficient).  sb only shrinks below.
  const bool idle = e->host_calls == 0 ||
                    SLOW_CALL(hipEventQuery(e->call_done[(e->host_calls - 1) % mip_engine::kCallRing])) == hipSuccess;
  int sb = mipgpu::call_chunk_cap(nframes, slot_cap, nslots, idle);
  // Full tables to the host (PCIe-bound): chunks of at most ~1 GiB of downloads, so the
  // first download starts early and, for pageable outputs, the bounce ring's copy-out keeps
  // up (1080p, 8 calls of 128 frames: 96-frame chunks 831 frames/s pageable, 32-frame 892,
  // 16-frame 1018; page-locked 990 / 963 / 1036).  Decisions only keeps the larger chunks
  // (its rate is the search's, whose launches are more efficient with more frames).
  const size_t down_per_frame = (size_t)((costs_out ? 1 : 0) + (sad_out ? 1 : 0) + (satd_out ? 1 : 0)) * cpf * 4;
  if (down_per_frame) {
    const char *cm = getenv("MIPGPU_CHUNK_MB");  // tuning knob: download bytes per chunk
    const size_t cap = (size_t)(cm && atoi(cm) > 0 ? atoi(cm) : 1024) << 20;
    sb = std::max(1, std::min<int>(sb, (int)(cap / down_per_frame)));
  }
  const hipStream_t up = e->stream2, down = e->stream3;
  const bool pin_in = mipgpu::host_pinned(frames) && (!refs_or_null || mipgpu::host_pinned(refs_or_null));
  const bool pin_cost = !costs_out || mipgpu::host_pinned(costs_out);
  const bool pin_sad = !sad_out || mipgpu::host_pinned(sad_out);
  const bool pin_satd = !satd_out || mipgpu::host_pinned(satd_out);
  const bool pin_bm = !best_mode_out || mipgpu::host_pinned(best_mode_out);
  const bool pin_bc = !best_cost_out || mipgpu::host_pinned(best_cost_out);
  auto equal_chunks = [&] {  // a short last chunk would leave the search waiting for the next upload
    const int nch = (nframes + sb - 1) / sb;
    sb = (nframes + nch - 1) / nch;
  };
  equal_chunks();
  if (!(pin_in && pin_cost && pin_sad && pin_satd && pin_bm && pin_bc)) {
    // pieces sized for a whole slot of the buffers this call moves (not for this call's
    // chunk: a call into an idle pipeline is cut in two, and growing the ring later drains
    // it and pins new memory)
    const size_t per_frame = std::max({fs * 2, down_per_frame ? cpf * 4 : 0,
                                       best_cost_out ? upf * 4 : (best_mode_out ? upf : 0)});
    HIP_TRY(e->stage.reserve(std::min<size_t>((size_t)slot_cap * per_frame, mipgpu::HostStage::kMaxPiece)));
    // Pageable transfers take ring bytes per buffer: a chunk's downloads must fit the ring
    // beside the next chunk's uploads (host_stage.h kMaxChunkPieces), else enqueueing them
    // waits on the host for the chunk's own search.
    const size_t piece = e->stage.piece();
    auto bytes = [&](bool pinned, size_t bytes_per_frame) -> size_t {
      return pinned ? 0 : e->stage.footprint((size_t)sb * bytes_per_frame);
    };
    auto fits = [&] {
      const size_t down_b = bytes(pin_cost, costs_out ? cpf * 4 : 0) + bytes(pin_sad, sad_out ? cpf * 4 : 0) +
                            bytes(pin_satd, satd_out ? cpf * 4 : 0) + bytes(pin_bm, best_mode_out ? upf : 0) +
                            bytes(pin_bc, best_cost_out ? upf * 4 : 0);
      const size_t up_b = bytes(pin_in, fs * 2) * (refs_or_null ? 2 : 1);
      return down_b <= mipgpu::HostStage::kMaxChunkPieces * piece &&
             up_b <= mipgpu::HostStage::kMaxChunkUploadPieces * piece;
    };
    while (sb > 1 && !fits()) sb--;
    equal_chunks();
  }
  // host <-> device copy on stream s: DMA from / to page-locked memory, else the bounce ring
  auto to_dev = [&](void *d, const void *h, size_t n, bool pinned) {
    return pinned ? hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, up) : e->stage.upload(d, h, n, up, call);
  };
  auto to_host = [&](void *h, const void *d, size_t n, bool pinned) {
    return pinned ? hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, down) : e->stage.download(h, d, n, down, call);
  };
  // A longer call into an idle pipeline ramps its first chunks up from a few frames: the
  // search starts after one small upload instead of a whole chunk's (64 frames: 4.7 ms at
  // 56 GB/s), and each chunk's upload still fits under the previous chunk's search (upload
  // 74 us per 1080p frame, search ~131 us: growth x1.75).  A synchronous decisions-only call
  // (mip_search_frames: nothing can queue behind it) ramps its last chunks down the same way,
  // so the download left after the last search is a few frames' (decision lists: 67 us per
  // frame, under the next chunk's search; full tables are download-bound throughout, where a
  // ramp-down changes nothing).  The rest of the call keeps equal chunks of at most sb.
  // MIPGPU_RAMP=0 (A/B knob): no ramps; MIPGPU_RAMP=up: no ramp-down.
  int nhead = 0, ntail = 0;
  std::vector<int> plan;
  {
    const char *rv = getenv("MIPGPU_RAMP");
    const bool ramps = nslots == 4 && sb >= 16 && !(rv && !strcmp(rv, "0"));
    plan = mipgpu::chunk_plan(nframes, sb, ramps && idle && nframes >= 2 * sb,
                              ramps && sync && !down_per_frame && !(rv && !strcmp(rv, "up")), &nhead, &ntail);
  }
  const bool ramped = nhead + ntail > 0;
  // Searches of consecutive chunks alternate between two search streams, so that a chunk's
  // search takes the CUs as its predecessor's persistent grid drains -- except in ramped
  // calls, whose short chunks are sized to run one after the other (device API, 1080p,
  // tools/overlap_probe.py: one-frame launches +10 % decisions-only / +5 % full tables on
  // two streams; host pipeline: 8 queued one-frame calls decisions-only +5 %, 4-frame +4 %,
  // one synchronous ramped 128-frame call -2 %, so ramped calls keep one stream).
  const bool alt_streams = search_streams() == 2 && !ramped;
  for (const int nb : plan)  // (chunk_plan never exceeds sb <= slot_cap: a slot's region)
    if (nb < 1 || nb > slot_cap) return fail("internal: a chunk of %d frames for a slot of %d", nb, slot_cap);
  int f0 = 0;
  for (const int nb : plan) {
    const uint64_t k = e->host_chunks++;
    const int sl = (int)(k % nslots);
    const hipStream_t comp = alt_streams && (k & 1) ? e->stream4 : e->stream;
    const bool reuse = k >= (uint64_t)nslots;  // the slot served chunk k - nslots (this or an earlier call)
    const size_t fo = (size_t)sl * slot_cap;  // first engine frame of this chunk's slot
    uint16_t *d_frames = e->d_frames + fo * fs;
    // the slot's previous chunk is over once its downloads are (they wait for its search):
    // then its frames / refs may be overwritten here, and -- through this upload -- its
    // outputs by this chunk's search, which waits for nothing else (one cross-stream wait
    // on the search stream per chunk)
    if (reuse) HIP_TRY(hipStreamWaitEvent(up, e->slot_down[sl], 0));
    if (e->trace) {
      if (drain_trace(e, sl) != 0) return -1;
      HIP_TRY(hipEventRecord(e->tr_ev[sl][0], up));
    }
    HIP_TRY(to_dev(d_frames, frames + f0 * fs, nb * fs * 2, pin_in));
    if (e->trace) HIP_TRY(hipEventRecord(e->tr_ev[sl][1], up));
    const uint16_t *d_refs = nullptr;
    if (refs_or_null) {
      HIP_TRY(to_dev(e->d_refs + fo * fs, refs_or_null + f0 * fs, nb * fs * 2, pin_in));
      d_refs = e->d_refs + fo * fs;
    }
    // the engine filter runs on the upload stream behind the chunk's upload: it overlaps the
    // previous chunk's search (its workgroups take CUs as the persistent search grid drains)
    // and the slot's refs region is free once the slot's previous search is (waited above)
    const bool filt = !refs_or_null && e->opts.filter != MIP_FILTER_NONE;
    if (filt) {
      if (e->trace) HIP_TRY(hipEventRecord(e->tr_ev[sl][2], up));
      if (mip_filter_device(d_frames, e->d_refs + fo * fs, e->width, e->height, nb, e->opts.filter,
                            e->opts.kernel_idx, up) != 0)
        return -1;
      if (e->trace) HIP_TRY(hipEventRecord(e->tr_ev[sl][3], up));
      d_refs = e->d_refs + fo * fs;
    }
    HIP_TRY(hipEventRecord(e->slot_up[sl], up));
    HIP_TRY(hipStreamWaitEvent(comp, e->slot_up[sl], 0));
    if (e->trace) {
      e->tr_frames[sl] = nb;
      e->tr_filter[sl] = filt;
      e->tr_chunk[sl] = k;
    }
    // decisions only (no cost / SAD / SATD table requested, K = 1): the fused argmin, no table
    const bool decisions_only = !costs_out && !sad_out && !satd_out && e->opts.best_k == 1 &&
                                (best_mode_out || best_cost_out);
    int32_t *d_costs = decisions_only ? nullptr : e->d_costs + fo * cpf;
    int32_t *d_sad = sad_out ? e->d_sad + fo * cpf : nullptr, *d_satd = satd_out ? e->d_satd + fo * cpf : nullptr;
    uint8_t *d_best = best_mode_out ? e->d_best + fo * upf : nullptr;
    int32_t *d_best_cost = best_cost_out || decisions_only ? e->d_best_cost + fo * upf : nullptr;
    // Decisions only: the split CUs' packed running minima live in d_split_acc, which holds
    // all ones outside the chunks in flight (the unpacking resets what it reads), so the
    // search stream runs the search kernel alone and the unpacking runs on the download
    // stream before the download -- the initialising and unpacking kernels and their launch
    // gaps leave the search stream's critical path (one-frame calls: ~20 us of ~190 us).
    mipgpu::SplitArgs split{};
    const bool defer = decisions_only && !dec_inline();
    hipEvent_t comp_done = e->slot_comp[sl];  // (nullptr after the call: the search recorded it)
    if (search_device_impl(e, d_frames, d_refs, nb, d_costs, d_sad, d_satd, d_best, d_best_cost, comp,
                           refs_or_null != nullptr, call_status(e, call), 0, -1,
                           defer ? e->d_split_acc + fo * e->nctus * MIP_CUS_PER_CTU : nullptr,
                           defer ? &split : nullptr, &comp_done, nullptr, alt_streams) != 0)
      return -1;
    if (comp_done) HIP_TRY(hipEventRecord(e->slot_comp[sl], comp));
    e->last_slot = sl;
    e->last_frames = nb;
    e->stat_launches++;
    HIP_TRY(hipStreamWaitEvent(down, e->slot_comp[sl], 0));  // (also without outputs: slot_down ends the chunk)
    if (defer) HIP_TRY(mipgpu::launch_dec_split(split, nb, false, down));
    if (costs_out) HIP_TRY(to_host(costs_out + f0 * cpf, d_costs, nb * cpf * 4, pin_cost));
    if (sad_out) HIP_TRY(to_host(sad_out + f0 * cpf, d_sad, nb * cpf * 4, pin_sad));
    if (satd_out) HIP_TRY(to_host(satd_out + f0 * cpf, d_satd, nb * cpf * 4, pin_satd));
    if (best_mode_out) HIP_TRY(to_host(best_mode_out + f0 * upf, d_best, nb * upf, pin_bm));
    if (best_cost_out) HIP_TRY(to_host(best_cost_out + f0 * upf, d_best_cost, nb * upf * 4, pin_bc));
    HIP_TRY(hipEventRecord(e->slot_down[sl], down));
    f0 += nb;
  }
  return 0;
}

int mip_wait(mip_engine *e, uint64_t ticket) {
  if (!e) return fail("engine is NULL");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (ticket == 0 || ticket > e->host_calls) return fail("unknown ticket %llu", (unsigned long long)ticket);
  HIP_TRY(hipSetDevice(e->device));
  // the caller is about to block: an open chunk can gain no more calls from it (launched now,
  // behind the searches in flight; a failure is reported by its members' tickets)
  (void)flush_open(e);
  // a ticket older than the ring shares its event with a later call: waiting for that one
  // is later than needed, never too early
  HIP_TRY(hipEventSynchronize(e->call_done[(ticket - 1) % mip_engine::kCallRing]));
  // pageable outputs: copy the call's staged downloads out (and everything queued before)
  HIP_TRY(e->stage.drain(ticket));
  // input contract of this call only (every call <= ticket has completed: calls complete in
  // order); the flags of earlier calls stay with their own tickets
  harvest_status(e, ticket);
  const auto it = e->call_errors.find(ticket);
  if (it == e->call_errors.end()) return 0;
  const uint32_t f = it->second;
  e->call_errors.erase(it);
  if (f & 4u)
    return fail("host-API call %llu of this engine: its merged launch failed", (unsigned long long)ticket);
  char what[64];
  snprintf(what, sizeof what, "host-API call %llu of this engine", (unsigned long long)ticket);
  return contract_error(f, what);
}

int mip_search_frames(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null, int nframes,
                      int32_t *costs_out, uint8_t *best_mode_out, int32_t *best_cost_out, int32_t *sad_out,
                      int32_t *satd_out) {
  if (!e) return fail("engine is NULL");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  uint64_t ticket = 0;
  if (search_frames_call(e, frames, refs_or_null, nframes, costs_out, best_mode_out, best_cost_out, sad_out,
                         satd_out, &ticket, true) != 0)
    return -1;
  return mip_wait(e, ticket);
}

int mip_trace_times(mip_engine *e, int enable) {
  if (!e) return fail("engine is NULL");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  if (flush_open(e) != 0) return -1;  // (merged chunks are not traced)
  if (enable && !e->tr_ev[0][0]) {
    // all events or none: a partial set would turn tracing on with null events
    hipEvent_t ev[mip_engine::kHostSlots][4] = {};
    for (auto &row : ev)
      for (hipEvent_t &x : row)
        if (hipEventCreate(&x) != hipSuccess) {
          for (auto &r2 : ev)
            for (hipEvent_t y : r2)
              if (y) (void)hipEventDestroy(y);
          return fail("hipEventCreate failed (tracing stays off)");
        }
    memcpy(e->tr_ev, ev, sizeof ev);
  }
  e->trace = enable != 0;
  return 0;
}

int mip_pop_times(mip_engine *e, double *upload_ms, double *filter_ms, int max, int *n) {
  if (!e || !n || max < 0) return fail("bad arguments");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  // pending chunks in sequence order (frame order)
  std::vector<int> order;
  for (int sl = 0; sl < mip_engine::kHostSlots; sl++)
    if (e->tr_frames[sl]) order.push_back(sl);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return e->tr_chunk[a] < e->tr_chunk[b]; });
  for (int sl : order)
    if (drain_trace(e, sl) != 0) return -1;
  const int k = std::min<int>(max, (int)e->tr_times.size());
  for (int i = 0; i < k; i++) {
    if (upload_ms) upload_ms[i] = e->tr_times[i].first;
    if (filter_ms) filter_ms[i] = e->tr_times[i].second;
  }
  e->tr_times.erase(e->tr_times.begin(), e->tr_times.begin() + k);
  *n = k;
  return 0;
}

int mip_device_cache(int device, int release, uint64_t *idle_bytes, uint64_t *reused_blocks) {
  BlockCache &c = block_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  uint64_t idle = 0;
  for (auto it = c.idle.begin(); it != c.idle.end();) {
    if (it->first.first == device && release) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(device);
      (void)hipFree(it->second);
      (void)hipSetDevice(cur);
      it = c.idle.erase(it);
      continue;
    }
    if (it->first.first == device) idle += it->first.second;
    ++it;
  }
  if (idle_bytes) *idle_bytes = idle;
  if (reused_blocks) *reused_blocks = c.reused;
  return 0;
}

int mip_flush(mip_engine *e) {
  if (!e) return fail("engine is NULL");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  return flush_open(e);
}

int mip_host_stats(mip_engine *e, uint64_t *out, int n) {
  if (!e || !out || n < 0 || n > 4) return fail("bad arguments");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  const uint64_t v[4] = {e->host_calls, e->stat_launches, e->stat_merged_calls, e->stat_merged_launches};
  for (int i = 0; i < n; i++) out[i] = v[i];
  return 0;
}

int mip_host_alloc(size_t bytes, void **out) {
  if (!out) return fail("out is NULL");
  *out = nullptr;
  HIP_TRY(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  return 0;
}

int mip_host_alloc_near(int device, size_t bytes, void **out) {
  if (!out) return fail("out is NULL");
  *out = nullptr;
  const mipgpu::NumaPlace p = device_place(device);
  const mipgpu::ScopedNodePolicy pol(p);
  HIP_TRY(hipHostMalloc(out, bytes ? bytes : 1, pol.applied() ? hipHostMallocNumaUser : hipHostMallocDefault));
  return 0;
}

int mip_numa_node_of_pci(const char *pci_bus_id) {
  if (!pci_bus_id) return fail("pci_bus_id is NULL");
  return mipgpu::numa_place_of_pci(pci_bus_id).node;
}

int mip_numa_node(int device) { return device_place(device).node; }

int mip_bind_thread(int device) { return mipgpu::bind_current_thread(device_place(device)) ? 1 : 0; }

int mip_host_free(void *p) {
  if (p) HIP_TRY(hipHostFree(p));
  return 0;
}

int mip_filter_frames(mip_engine *e, const uint16_t *frames, int nframes, int filter, int kernel_idx,
                      uint16_t *out) {
  if (!e || !frames || !out || nframes < 1) return fail("bad filter arguments");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  HIP_TRY(hipSetDevice(e->device));
  if (flush_open(e) != 0) return -1;
  const size_t fs = (size_t)e->width * e->height;
  if (!e->d_refs) HIP_TRY(dev_malloc(e->device, (void **)&e->d_refs, fs * e->hp_frames * 2));
  if (wait_refs_readers(e) != 0) return -1;
  // asynchronous host searches still in flight use d_frames / d_refs: let them finish
  HIP_TRY(hipStreamSynchronize(e->stream2));
  HIP_TRY(hipStreamSynchronize(e->stream));
  HIP_TRY(hipStreamSynchronize(e->stream4));
  HIP_TRY(hipStreamSynchronize(e->stream3));
  for (int f0 = 0; f0 < nframes; f0 += e->opts.max_batch) {
    const int nb = std::min(e->opts.max_batch, nframes - f0);
    HIP_TRY(hipMemcpyAsync(e->d_frames, frames + f0 * fs, nb * fs * 2, hipMemcpyHostToDevice, e->stream));
    if (mip_filter_device(e->d_frames, e->d_refs, e->width, e->height, nb, filter, kernel_idx, e->stream) != 0)
      return -1;
    HIP_TRY(hipMemcpyAsync(out + f0 * fs, e->d_refs, nb * fs * 2, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  HIP_TRY(hipStreamSynchronize(e->stream2));
  e->refs_pending = false;
  return 0;
}

double mip_time_search_device(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs, int nframes,
                              int32_t *d_costs, int reps) {
  if (!e || reps < 1) return fail("bad timing arguments");
  std::lock_guard<std::recursive_mutex> lk(e->mu);
  if (hipSetDevice(e->device) != hipSuccess) return fail("hipSetDevice");
  if (flush_open(e) != 0) return -1;
  hipEvent_t t0, t1;
  if (hipEventCreate(&t0) != hipSuccess || hipEventCreate(&t1) != hipSuccess) return fail("hipEventCreate");
  (void)hipEventRecord(t0, e->stream);
  for (int r = 0; r < reps; r++)
    if (search_device_impl(e, d_frames, d_refs, nframes, d_costs, nullptr, nullptr, nullptr, nullptr, e->stream,
                           d_refs != nullptr && d_refs != d_frames, device_status(e)) != 0) {
      (void)hipEventDestroy(t0);
      (void)hipEventDestroy(t1);
      return -1;
    }
  (void)hipEventRecord(t1, e->stream);
  (void)hipEventSynchronize(t1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, t0, t1);
  (void)hipEventDestroy(t0);
  (void)hipEventDestroy(t1);
  if (check_device_status(e) != 0) return -1;
  return ms / reps;
}

}  // extern "C"
