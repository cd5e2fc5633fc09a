// mipgpu.cpp -- C-ABI engine (include/mipgpu.h): device set-up, buffers, work lists and
// the per-batch launch sequence that replaces main.cpp's OpenCL host loop.
#include "mipgpu.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mip_kernels.h"
#include "mip_tables.h"

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

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
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

// Expanded weights, layout documented in mip_kernels.h.
std::vector<int16_t> expand_weights() {
  std::vector<int16_t> w(mipgpu::kWeightWords, 0);
  for (int m = 0; m < 6; m++)
    for (int j = 0; j < 64; j++)
      for (int i = 0; i < 7; i++) w[(m * 64 + j) * 8 + 1 + i] = kW2[(m * 64 + j) * 7 + i];
  for (int m = 0; m < 8; m++)
    for (int j = 0; j < 16; j++)
      for (int i = 0; i < 8; i++) w[(mipgpu::kWeightRowOffS1 + m * 16 + j) * 8 + i] = kW1[(m * 16 + j) * 8 + i];
  for (int m = 0; m < 16; m++)
    for (int j = 0; j < 16; j++)
      for (int i = 0; i < 4; i++) w[(mipgpu::kWeightRowOffS0 + m * 16 + j) * 8 + i] = kW0[(m * 16 + j) * 4 + i];
  return w;
}

// Per-quadrant work lists.  Jobs (CU, mode pair) of a shape inside quadrant q are grouped
// into wave tasks of up to 64/S jobs (S = W/4 strips per CU; at most 16 jobs for shapes
// that stage reduced predictions in LDS, see mip_search.hip).  Jobs are CU-major for
// those shapes (lanes of one CU read the same samples) and pair-major for the shapes
// that compute their matrix products per lane (lanes of a wave share weight rows).
// Shapes are ordered by rows per strip (descending) so the round-robin assignment of
// tasks to waves balances, and tasks of one shape stay adjacent.
// MIPGPU_SHAPE_FILTER="i,j,..." (profiling knob) restricts the search to those shapes.
struct WorkLists {
  std::vector<mipgpu::WaveTask> tasks;
  std::vector<mipgpu::Job> jobs;
  int task_begin[5];
};

bool shape_selected(int s) {
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

WorkLists build_work() {
  std::vector<int> order;
  for (int i = 0; i < MIP_NUM_SHAPES; i++)
    if (shape_selected(i)) order.push_back(i);
  std::stable_sort(order.begin(), order.end(), [](int a, int b) { return kShapes[a].h > kShapes[b].h; });
  WorkLists wl;
  for (int q = 0; q < 4; q++) {
    wl.task_begin[q] = (int)wl.tasks.size();
    for (int s : order) {
      const mip_shape_desc &sd = kShapes[s];
      const int r = sd.size_id == 2 ? 8 : 4;
      const bool direct = sd.w == r;
      const int strips = sd.w / 4;
      // shapes staging reduced predictions: the wave scratch holds 16 x 65 dwords
      const int per_task = direct ? 64 / strips : std::min(64 / strips, 1040 / (r * r + 1));
      std::vector<int> cus;
      for (int cu = 0; cu < sd.ncu; cu++) {
        const int x = axis_pos(sd.xb, sd.xs, sd.xd, cu % sd.ncols), y = axis_pos(sd.yb, sd.ys, sd.yd, cu / sd.ncols);
        if (x / 64 == (q & 1) && y / 64 == (q >> 1)) cus.push_back(cu);
      }
      const int nout = r * r;
      const int wrow0 = sd.size_id == 2 ? 0 : (sd.size_id == 1 ? mipgpu::kWeightRowOffS1 : mipgpu::kWeightRowOffS0);
      auto make_job = [&](int cu, int p) {
        const int x = axis_pos(sd.xb, sd.xs, sd.xd, cu % sd.ncols), y = axis_pos(sd.yb, sd.ys, sd.yd, cu / sd.ncols);
        const bool tr = 2 * p >= sd.modes;
        const int mw = tr ? 2 * p - sd.modes : 2 * p;
        return mipgpu::Job{(uint32_t)(sd.cost_offset + cu * 2 * sd.modes + 2 * p), (uint8_t)(x % 64), (uint8_t)(y % 64),
                           (uint16_t)((wrow0 + mw * nout) | (tr ? mipgpu::kJobTransposed : 0))};
      };
      std::vector<mipgpu::Job> jobs;
      if (direct) {
        for (int p = 0; p < sd.modes; p++)
          for (int cu : cus) jobs.push_back(make_job(cu, p));
      } else {
        for (int cu : cus)
          for (int p = 0; p < sd.modes; p++) jobs.push_back(make_job(cu, p));
      }
      for (size_t j = 0; j < jobs.size(); j += per_task) {
        const int n = (int)std::min<size_t>(per_task, jobs.size() - j);
        wl.tasks.push_back({(uint8_t)s, (uint8_t)n, 0, (uint32_t)(wl.jobs.size() + j)});
      }
      wl.jobs.insert(wl.jobs.end(), jobs.begin(), jobs.end());
    }
  }
  wl.task_begin[4] = (int)wl.tasks.size();
  return wl;
}

bool filter_supported(int f) { return f == 2 || f == 3 || f == 6 || f == 7; }
bool filter_valid(int f, int k) {
  if (f < 0 || f > 7) return false;
  const bool five = f >= 4;
  return k >= 0 && k < (five ? 3 : 5);
}

}  // namespace

struct mip_engine {
  int device = 0, width = 0, height = 0, nctus = 0, ctu_cols = 0;
  mip_opts opts{};
  hipStream_t stream = nullptr;
  uint16_t *d_frames = nullptr, *d_refs = nullptr;
  int32_t *d_costs = nullptr, *d_sad = nullptr, *d_satd = nullptr, *d_best_cost = nullptr;
  uint8_t *d_best = nullptr;
  mipgpu::WaveTask *d_tasks = nullptr;
  mipgpu::Job *d_jobs = nullptr;
  int task_begin[5] = {0, 0, 0, 0, 0};
  int16_t *d_weights = nullptr;
  int slices = 8;
};

extern "C" {

void mip_opts_default(mip_opts *o) {
  if (!o) return;
  o->filter = MIP_FILTER_NONE;
  o->kernel_idx = 0;
  o->max_batch = 1;
  o->want_sad_satd = 0;
  o->slices_per_ctu = 0;
}

const char *mip_last_error(void) { return g_err.c_str(); }
int mip_abi_version(void) { return MIPGPU_ABI_VERSION; }

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
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (void *p : {(void *)e->d_frames, (void *)e->d_refs, (void *)e->d_costs, (void *)e->d_sad,
                  (void *)e->d_satd, (void *)e->d_best, (void *)e->d_best_cost, (void *)e->d_tasks,
                  (void *)e->d_jobs, (void *)e->d_weights})
    if (p) (void)hipFree(p);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return 0;
}

int mip_engine_create(int device, int width, int height, const mip_opts *opts, mip_engine **out) {
  if (!out) return fail("out is NULL");
  *out = nullptr;
  if (width <= 0 || height <= 0 || width % 4 || height % 4)
    return fail("frame size %dx%d must be positive multiples of 4", width, height);
  mip_opts o;
  mip_opts_default(&o);
  if (opts) o = *opts;
  if (o.max_batch < 1) return fail("max_batch must be >= 1");
  if (o.filter != MIP_FILTER_NONE) {
    if (!filter_valid(o.filter, o.kernel_idx)) return fail("invalid filter %d / kernel_idx %d", o.filter, o.kernel_idx);
    if (!filter_supported(o.filter)) return fail("filter %d (separable) is not available on the HIP path yet", o.filter);
  }
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail("device %d out of range (%d devices)", device, ndev);
  HIP_TRY(hipSetDevice(device));

  mip_engine *e = new mip_engine();
  e->device = device;
  e->width = width;
  e->height = height;
  e->nctus = mip_num_ctus(width, height);
  e->ctu_cols = (width + 127) / 128;
  e->opts = o;
  const size_t fs = (size_t)width * height, nb = (size_t)o.max_batch;
  const size_t ncost = nb * e->nctus * MIP_COSTS_PER_CTU, ncu = nb * e->nctus * MIP_CUS_PER_CTU;
  auto cleanup = [&](int rc) { mip_engine_destroy(e); return rc; };
#define ALLOC(ptr, bytes)                                                               \
  do {                                                                                  \
    hipError_t _e = hipMalloc((void **)&(ptr), (bytes));                                \
    if (_e != hipSuccess) return cleanup(fail("hipMalloc(%zu): %s", (size_t)(bytes), hipGetErrorString(_e))); \
  } while (0)
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail("hipStreamCreate failed"));
  ALLOC(e->d_frames, fs * nb * 2);
  if (o.filter != MIP_FILTER_NONE) ALLOC(e->d_refs, fs * nb * 2);
  ALLOC(e->d_costs, ncost * 4);
  if (o.want_sad_satd) {
    ALLOC(e->d_sad, ncost * 4);
    ALLOC(e->d_satd, ncost * 4);
  }
  ALLOC(e->d_best, ncu);
  ALLOC(e->d_best_cost, ncu * 4);
  const WorkLists wl = build_work();
  for (int q = 0; q < 5; q++) e->task_begin[q] = wl.task_begin[q];
  ALLOC(e->d_tasks, std::max<size_t>(1, wl.tasks.size()) * sizeof(mipgpu::WaveTask));
  ALLOC(e->d_jobs, std::max<size_t>(1, wl.jobs.size()) * sizeof(mipgpu::Job));
  const std::vector<int16_t> w = expand_weights();
  ALLOC(e->d_weights, w.size() * 2);
#undef ALLOC
  if ((!wl.tasks.empty() &&
       (hipMemcpy(e->d_tasks, wl.tasks.data(), wl.tasks.size() * sizeof(mipgpu::WaveTask), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(e->d_jobs, wl.jobs.data(), wl.jobs.size() * sizeof(mipgpu::Job), hipMemcpyHostToDevice) != hipSuccess)) ||
      hipMemcpy(e->d_weights, w.data(), w.size() * 2, hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail("uploading static tables failed"));
  e->slices = o.slices_per_ctu > 0 ? o.slices_per_ctu : 1;
  *out = e;
  return 0;
}

int mip_filter_device(const uint16_t *d_in, uint16_t *d_out, int width, int height, int nframes,
                      int filter, int kernel_idx, void *stream) {
  if (!d_in || !d_out || nframes < 1) return fail("bad filter arguments");
  if (!filter_valid(filter, kernel_idx)) return fail("invalid filter %d / kernel_idx %d", filter, kernel_idx);
  if (!filter_supported(filter)) return fail("filter %d (separable) is not available on the HIP path yet", filter);
  mipgpu::FilterArgs a{d_in, d_out, width, height, nframes, filter, kernel_idx};
  HIP_TRY(mipgpu::launch_filter(a, (hipStream_t)stream));
  return 0;
}

static int search_device_impl(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs, int nframes,
                              int32_t *d_costs, int32_t *d_sad, int32_t *d_satd, uint8_t *d_best,
                              int32_t *d_best_cost, hipStream_t s) {
  if (!e || !d_frames || !d_costs || nframes < 1) return fail("bad search arguments");
  const uint16_t *refs = d_refs;
  if (!refs && e->opts.filter != MIP_FILTER_NONE) {
    if (nframes > e->opts.max_batch) return fail("nframes %d > max_batch %d", nframes, e->opts.max_batch);
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
  a.sad = d_sad;
  a.satd = d_satd;
  a.tasks = e->d_tasks;
  a.jobs = e->d_jobs;
  a.weights = e->d_weights;
  a.width = e->width;
  a.height = e->height;
  a.ctu_cols = e->ctu_cols;
  a.nctus = e->nctus;
  for (int q = 0; q < 5; q++) a.task_begin[q] = e->task_begin[q];
  a.slices = e->slices;
  HIP_TRY(mipgpu::launch_search(a, nframes, alt, s));
  if (d_best || d_best_cost) {
    mipgpu::BestArgs b{d_costs, d_best, d_best_cost, nframes * e->nctus * MIP_CUS_PER_CTU};
    HIP_TRY(mipgpu::launch_best_modes(b, s));
  }
  return 0;
}

int mip_search_device(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs, int nframes,
                      int32_t *d_costs, int32_t *d_sad, int32_t *d_satd, uint8_t *d_best_mode,
                      int32_t *d_best_cost, void *stream) {
  if (!e) return fail("engine is NULL");
  HIP_TRY(hipSetDevice(e->device));
  return search_device_impl(e, d_frames, d_refs, nframes, d_costs, d_sad, d_satd, d_best_mode, d_best_cost,
                            (hipStream_t)stream);
}

int mip_search_frames(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null, int nframes,
                      int32_t *costs_out, uint8_t *best_mode_out, int32_t *best_cost_out, int32_t *sad_out,
                      int32_t *satd_out) {
  if (!e || !frames || nframes < 1) return fail("bad search arguments");
  if ((sad_out || satd_out) && !e->opts.want_sad_satd) return fail("engine created without want_sad_satd");
  if (refs_or_null && e->opts.filter == MIP_FILTER_NONE && !e->d_refs) {
    const size_t fs = (size_t)e->width * e->height;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMalloc((void **)&e->d_refs, fs * e->opts.max_batch * 2));
  }
  HIP_TRY(hipSetDevice(e->device));
  const size_t fs = (size_t)e->width * e->height;
  const size_t cpf = (size_t)e->nctus * MIP_COSTS_PER_CTU, upf = (size_t)e->nctus * MIP_CUS_PER_CTU;
  for (int f0 = 0; f0 < nframes; f0 += e->opts.max_batch) {
    const int nb = std::min(e->opts.max_batch, nframes - f0);
    HIP_TRY(hipMemcpyAsync(e->d_frames, frames + f0 * fs, nb * fs * 2, hipMemcpyHostToDevice, e->stream));
    const uint16_t *d_refs = nullptr;
    if (refs_or_null) {
      HIP_TRY(hipMemcpyAsync(e->d_refs, refs_or_null + f0 * fs, nb * fs * 2, hipMemcpyHostToDevice, e->stream));
      d_refs = e->d_refs;
    }
    if (search_device_impl(e, e->d_frames, d_refs, nb, e->d_costs, sad_out ? e->d_sad : nullptr,
                           satd_out ? e->d_satd : nullptr, best_mode_out ? e->d_best : nullptr,
                           best_cost_out ? e->d_best_cost : nullptr, e->stream) != 0)
      return -1;
    if (costs_out) HIP_TRY(hipMemcpyAsync(costs_out + f0 * cpf, e->d_costs, nb * cpf * 4, hipMemcpyDeviceToHost, e->stream));
    if (sad_out) HIP_TRY(hipMemcpyAsync(sad_out + f0 * cpf, e->d_sad, nb * cpf * 4, hipMemcpyDeviceToHost, e->stream));
    if (satd_out) HIP_TRY(hipMemcpyAsync(satd_out + f0 * cpf, e->d_satd, nb * cpf * 4, hipMemcpyDeviceToHost, e->stream));
    if (best_mode_out) HIP_TRY(hipMemcpyAsync(best_mode_out + f0 * upf, e->d_best, nb * upf, hipMemcpyDeviceToHost, e->stream));
    if (best_cost_out) HIP_TRY(hipMemcpyAsync(best_cost_out + f0 * upf, e->d_best_cost, nb * upf * 4, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  return 0;
}

int mip_filter_frames(mip_engine *e, const uint16_t *frames, int nframes, int filter, int kernel_idx,
                      uint16_t *out) {
  if (!e || !frames || !out || nframes < 1) return fail("bad filter arguments");
  HIP_TRY(hipSetDevice(e->device));
  const size_t fs = (size_t)e->width * e->height;
  if (!e->d_refs) HIP_TRY(hipMalloc((void **)&e->d_refs, fs * e->opts.max_batch * 2));
  for (int f0 = 0; f0 < nframes; f0 += e->opts.max_batch) {
    const int nb = std::min(e->opts.max_batch, nframes - f0);
    HIP_TRY(hipMemcpyAsync(e->d_frames, frames + f0 * fs, nb * fs * 2, hipMemcpyHostToDevice, e->stream));
    if (mip_filter_device(e->d_frames, e->d_refs, e->width, e->height, nb, filter, kernel_idx, e->stream) != 0)
      return -1;
    HIP_TRY(hipMemcpyAsync(out + f0 * fs, e->d_refs, nb * fs * 2, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
  }
  return 0;
}

double mip_time_search_device(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs, int nframes,
                              int32_t *d_costs, int reps) {
  if (!e || reps < 1) return fail("bad timing arguments");
  if (hipSetDevice(e->device) != hipSuccess) return fail("hipSetDevice");
  hipEvent_t t0, t1;
  if (hipEventCreate(&t0) != hipSuccess || hipEventCreate(&t1) != hipSuccess) return fail("hipEventCreate");
  (void)hipEventRecord(t0, e->stream);
  for (int r = 0; r < reps; r++)
    if (search_device_impl(e, d_frames, d_refs, nframes, d_costs, nullptr, nullptr, nullptr, nullptr, e->stream) != 0) {
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
  return ms / reps;
}

}  // extern "C"
