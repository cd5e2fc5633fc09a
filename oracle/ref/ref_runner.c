/* ref_runner.c -- TEST INFRASTRUCTURE: run the reference's OpenCL kernels on a GPU.
 *
 * Loads the code objects ref_build made from /root/reference/intra.cl and replays the
 * reference host sequence of main.cpp:678-1241 for each frame:
 *     [filterFrame_<type>] -> initBoundaries -> MIP_ReducedPred -> upsampleDistortion x3
 * with the reference's launch shapes (main.cpp:311-313, 696-697, 837, 938, 1036, 1115,
 * 1192) and buffer sizes (main.cpp:420-453).  Unlike main.cpp it fences every step
 * (SURVEY.md section 5 lists the races of the original host loop) and always passes
 * rep = frame % 2 so that the filter and the boundary kernels agree on the slot.
 *
 * Output: int32 little-endian cost table(s) in the reference layout, optional filtered
 * frame, and a JSON line with per-kernel device times (CL profiling events).
 *
 * usage: ref_runner --bins DIR --width W --height H [--frames N] [--synth KIND:SEED]
 *                   [--input FILE.u16] [--filter NAME] [--kernel-idx K] [--full-dist]
 *                   [--out-cost F] [--out-sad F] [--out-satd F] [--out-filtered F]
 *                   [--reps R] [--fill V]
 *
 * --fill V: every device buffer (frame slots and their padding, filtered frames, the
 * boundary / prediction scratch, the cost tables) starts as the 16-bit pattern V instead
 * of zero.  Outputs that change with V depend on memory the reference never wrote for
 * this frame (out-of-frame reads, stale scratch): tools/ref_fill_experiment.py runs the
 * reference with two fill values to find them.
 */
#define CL_TARGET_OPENCL_VERSION 120
#include <CL/cl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../mip_oracle.h"

#define CHECK(e, what)                                                       \
  do {                                                                       \
    cl_int _e = (e);                                                         \
    if (_e != CL_SUCCESS) {                                                  \
      fprintf(stderr, "OpenCL error %d at %s (%s:%d)\n", _e, what, __FILE__, \
              __LINE__);                                                     \
      exit(3);                                                               \
    }                                                                        \
  } while (0)

/* Per-CTU strides of the reference's unified buffers (constants.h:568-570, 1041, 1111,
 * 1556, 1631). */
enum { RED_PER_CTU = 4356 * 4 + 1024 * 2, REF_PER_CTU = 48640, PRED_PER_CTU = 2231296,
       COST_PER_CTU = 97840 };

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static unsigned char *slurp(const char *path, size_t *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long len = ftell(f);
  rewind(f);
  unsigned char *buf = (unsigned char *)malloc((size_t)len);
  if (fread(buf, 1, (size_t)len, f) != (size_t)len) { fclose(f); free(buf); return NULL; }
  fclose(f);
  *n = (size_t)len;
  return buf;
}

static void sanitize(const char *in, char *out) {
  for (; *in; in++, out++) *out = *in == ':' ? '_' : (*in == '+' ? 'p' : (*in == '-' ? 'm' : *in));
  *out = 0;
}

static cl_program load_program(cl_context ctx, cl_device_id dev, const char *dir,
                               const char *tag, int sid, int dist) {
  char path[4096];
  snprintf(path, sizeof path, "%s/intra_%s_s%d_d%d.bin", dir, tag, sid, dist);
  size_t n = 0;
  unsigned char *bin = slurp(path, &n);
  if (!bin) { fprintf(stderr, "missing reference binary %s (run make -C oracle ref)\n", path); exit(4); }
  cl_int err, st;
  const unsigned char *b = bin;
  cl_program p = clCreateProgramWithBinary(ctx, 1, &dev, &n, &b, &st, &err);
  CHECK(err, "clCreateProgramWithBinary");
  CHECK(st, "binary status");
  CHECK(clBuildProgram(p, 1, &dev, "", NULL, NULL), "clBuildProgram(binary)");
  free(bin);
  return p;
}

/* Device time of a finished command from its profiling timestamps; falls back to the
 * host wall time around enqueue+clFinish (passed in) when the timestamps are unusable. */
static int g_event_fallbacks = 0;
static char g_fallback_reason[256] = "";
static double ev_ms(cl_event e, double wall_ms) {
  cl_ulong a = 0, b = 0, qd = 0, sb = 0, cp = 0;
  cl_int e1 = clGetEventProfilingInfo(e, CL_PROFILING_COMMAND_START, sizeof a, &a, NULL);
  cl_int e2 = clGetEventProfilingInfo(e, CL_PROFILING_COMMAND_END, sizeof b, &b, NULL);
  if (e1 != CL_SUCCESS || e2 != CL_SUCCESS || b < a || (double)(b - a) * 1e-6 > 1e3 * wall_ms + 1e3) {
    (void)clGetEventProfilingInfo(e, CL_PROFILING_COMMAND_QUEUED, sizeof qd, &qd, NULL);
    (void)clGetEventProfilingInfo(e, CL_PROFILING_COMMAND_SUBMIT, sizeof sb, &sb, NULL);
    (void)clGetEventProfilingInfo(e, 0x1284 /* CL_PROFILING_COMMAND_COMPLETE, OpenCL 2.0 */, sizeof cp, &cp, NULL);
    if (!g_event_fallbacks) /* the first one, for the report (relative to QUEUED, ns) */
      snprintf(g_fallback_reason, sizeof g_fallback_reason,
               "start err %d, end err %d; ns after queued: submit %lld start %lld end %lld complete %lld; wall %.4f ms",
               (int)e1, (int)e2, (long long)(sb - qd), (long long)(a - qd), (long long)(b - qd), (long long)(cp - qd),
               wall_ms);
    g_event_fallbacks++;
    return wall_ms;
  }
  return (double)(b - a) * 1e-6;
}

static void write_file(const char *path, const void *data, size_t bytes) {
  FILE *f = fopen(path, "wb");
  if (!f || fwrite(data, 1, bytes, f) != bytes) { fprintf(stderr, "cannot write %s\n", path); exit(5); }
  fclose(f);
}

int main(int argc, char **argv) {
  const char *bins = "oracle/_ref", *input = NULL, *filter = NULL;
  const char *out_cost = NULL, *out_sad = NULL, *out_satd = NULL, *out_filt = NULL;
  int W = 0, H = 0, frames = 1, kidx = 0, full = 0, reps = 1, kind = 0, fill = 0;
  unsigned long long seed = 0x1080;
  for (int i = 1; i < argc; i++) {
    const char *a = argv[i], *v = i + 1 < argc ? argv[i + 1] : "";
    if (!strcmp(a, "--bins")) bins = v, i++;
    else if (!strcmp(a, "--width")) W = atoi(v), i++;
    else if (!strcmp(a, "--height")) H = atoi(v), i++;
    else if (!strcmp(a, "--frames")) frames = atoi(v), i++;
    else if (!strcmp(a, "--synth")) { sscanf(v, "%d:%llx", &kind, &seed); i++; }
    else if (!strcmp(a, "--input")) input = v, i++;
    else if (!strcmp(a, "--filter")) filter = v, i++;
    else if (!strcmp(a, "--kernel-idx")) kidx = atoi(v), i++;
    else if (!strcmp(a, "--full-dist")) full = 1;
    else if (!strcmp(a, "--out-cost")) out_cost = v, i++;
    else if (!strcmp(a, "--out-sad")) out_sad = v, i++;
    else if (!strcmp(a, "--out-satd")) out_satd = v, i++;
    else if (!strcmp(a, "--out-filtered")) out_filt = v, i++;
    else if (!strcmp(a, "--reps")) reps = atoi(v), i++;
    else if (!strcmp(a, "--fill")) fill = (int)strtol(v, NULL, 0), i++;
    else { fprintf(stderr, "unknown argument %s\n", a); return 2; }
  }
  if (W <= 0 || H <= 0 || frames <= 0) { fprintf(stderr, "need --width/--height\n"); return 2; }
  if ((out_sad || out_satd) && !full) { fprintf(stderr, "--out-sad/--out-satd need --full-dist\n"); return 2; }

  const size_t fs = (size_t)W * H;
  const int nctus = ((W + 127) / 128) * ((H + 127) / 128);
  uint16_t *host = (uint16_t *)malloc(fs * 2 * frames);
  if (input) {
    size_t n = 0;
    unsigned char *b = slurp(input, &n);
    if (!b || n < fs * 2 * frames) { fprintf(stderr, "input too small\n"); return 2; }
    memcpy(host, b, fs * 2 * frames);
    free(b);
  } else {
    for (int f = 0; f < frames; f++) mipo_synth_frame(host + fs * f, W, H, seed + f, kind);
  }

  cl_platform_id plat;
  CHECK(clGetPlatformIDs(1, &plat, NULL), "platform");
  cl_device_id dev;
  CHECK(clGetDeviceIDs(plat, CL_DEVICE_TYPE_GPU, 1, &dev, NULL), "gpu device");
  char dname[256], tag[256];
  clGetDeviceInfo(dev, CL_DEVICE_NAME, sizeof dname, dname, NULL);
  sanitize(dname, tag);
  cl_int err;
  cl_context ctx = clCreateContext(NULL, 1, &dev, NULL, NULL, &err);
  CHECK(err, "context");
  cl_command_queue q = clCreateCommandQueue(ctx, dev, CL_QUEUE_PROFILING_ENABLE, &err);
  CHECK(err, "queue");

  cl_program p2 = load_program(ctx, dev, bins, tag, 2, full ? 0 : 1);
  cl_program p1 = load_program(ctx, dev, bins, tag, 1, full ? 0 : 1);
  cl_program p0 = load_program(ctx, dev, bins, tag, 0, full ? 0 : 1);

  const size_t slots = 2;
  /* The filter kernels' surplus work-groups (nCTUs*4 > quarter-CTU tiles) and the
   * separable kernels' unguarded bottom fetch (intra.cl:3330-3332) read up to ~100 rows
   * past the last frame slot; main.cpp gets away with it by luck.  Pad the frame
   * buffers so those reads stay inside the allocation (their results are discarded). */
  const size_t pad = (size_t)W * 256 + 4096;
  cl_mem m_ref = clCreateBuffer(ctx, CL_MEM_READ_WRITE, (slots * fs + pad) * 2, NULL, &err); CHECK(err, "buf");
  cl_mem m_filt = clCreateBuffer(ctx, CL_MEM_READ_WRITE, (slots * fs + pad) * 2, NULL, &err); CHECK(err, "buf");
  /* Both frame buffers start as the fill pattern (zero by default): the separable filters
   * read rows below the frame unguarded (intra.cl:3330-3332), and at widths that are not
   * multiples of 128 the linear indexes of the last CTU / tile column run past the frame
   * end (intra.cl:100, 718, 2905); with --fill those reads see V. */
  const cl_short fillv = (cl_short)fill;
  CHECK(clEnqueueFillBuffer(q, m_ref, &fillv, sizeof fillv, 0, (slots * fs + pad) * 2, 0, NULL, NULL), "fill");
  CHECK(clEnqueueFillBuffer(q, m_filt, &fillv, sizeof fillv, 0, (slots * fs + pad) * 2, 0, NULL, NULL), "fill");
  cl_mem m_redT = clCreateBuffer(ctx, CL_MEM_READ_WRITE, slots * nctus * RED_PER_CTU * 2, NULL, &err); CHECK(err, "buf");
  cl_mem m_redL = clCreateBuffer(ctx, CL_MEM_READ_WRITE, slots * nctus * RED_PER_CTU * 2, NULL, &err); CHECK(err, "buf");
  cl_mem m_refT = clCreateBuffer(ctx, CL_MEM_READ_WRITE, slots * nctus * REF_PER_CTU * 2, NULL, &err); CHECK(err, "buf");
  cl_mem m_refL = clCreateBuffer(ctx, CL_MEM_READ_WRITE, slots * nctus * REF_PER_CTU * 2, NULL, &err); CHECK(err, "buf");
  cl_mem m_pred = clCreateBuffer(ctx, CL_MEM_READ_WRITE, slots * (size_t)nctus * PRED_PER_CTU * 2, NULL, &err); CHECK(err, "buf");
  const size_t cost_bytes = slots * (size_t)nctus * COST_PER_CTU * 8;
  cl_mem m_min = clCreateBuffer(ctx, CL_MEM_READ_WRITE, cost_bytes, NULL, &err); CHECK(err, "buf");
  cl_mem m_sad = clCreateBuffer(ctx, CL_MEM_READ_WRITE, cost_bytes, NULL, &err); CHECK(err, "buf");
  cl_mem m_satd = clCreateBuffer(ctx, CL_MEM_READ_WRITE, cost_bytes, NULL, &err); CHECK(err, "buf");
  {
    cl_mem scratch[] = {m_redT, m_redL, m_refT, m_refL, m_pred, m_min, m_sad, m_satd};
    size_t bytes[] = {slots * nctus * RED_PER_CTU * 2, slots * nctus * RED_PER_CTU * 2, slots * nctus * REF_PER_CTU * 2,
                      slots * nctus * REF_PER_CTU * 2, slots * (size_t)nctus * PRED_PER_CTU * 2, cost_bytes, cost_bytes,
                      cost_bytes};
    for (int b = 0; b < 8; b++)
      CHECK(clEnqueueFillBuffer(q, scratch[b], &fillv, sizeof fillv, 0, bytes[b], 0, NULL, NULL), "fill scratch");
    CHECK(clFinish(q), "fill finish");
  }

  cl_kernel k_filt = NULL;
  if (filter) { k_filt = clCreateKernel(p2, filter, &err); CHECK(err, "filter kernel"); }
  cl_kernel k_init = clCreateKernel(p2, "initBoundaries", &err); CHECK(err, "initBoundaries");
  cl_kernel k_red = clCreateKernel(p2, "MIP_ReducedPred", &err); CHECK(err, "MIP_ReducedPred");
  cl_kernel k_up[3];
  k_up[0] = clCreateKernel(p2, "upsampleDistortion", &err); CHECK(err, "up2");
  k_up[1] = clCreateKernel(p1, "upsampleDistortion", &err); CHECK(err, "up1");
  k_up[2] = clCreateKernel(p0, "upsampleDistortion", &err); CHECK(err, "up0");
  const int up_wgs[3] = {nctus * 28, nctus * 18, nctus * 8};

  int32_t *costs = out_cost ? (int32_t *)malloc((size_t)frames * nctus * COST_PER_CTU * 4) : NULL;
  int32_t *sads = out_sad ? (int32_t *)malloc((size_t)frames * nctus * COST_PER_CTU * 4) : NULL;
  int32_t *satds = out_satd ? (int32_t *)malloc((size_t)frames * nctus * COST_PER_CTU * 4) : NULL;
  int64_t *tmp = (int64_t *)malloc((size_t)nctus * COST_PER_CTU * 8);
  uint16_t *filtered = out_filt ? (uint16_t *)malloc(fs * 2 * frames) : NULL;

  double t_filt = 0, t_init = 0, t_red = 0, t_up[3] = {0, 0, 0};
  double wall0 = 0, wall = 0;
  for (int rep_i = 0; rep_i < reps; rep_i++) {
    if (rep_i == reps - 1 || reps == 1) { t_filt = t_init = t_red = t_up[0] = t_up[1] = t_up[2] = 0; }
    wall0 = now_s();
    for (int f = 0; f < frames; f++) {
      cl_int rep = f % 2;
      cl_event e;
      CHECK(clEnqueueWriteBuffer(q, m_ref, CL_TRUE, rep * fs * 2, fs * 2, host + fs * f, 0, NULL, NULL), "H2D");
      if (k_filt) {
        clSetKernelArg(k_filt, 0, sizeof(cl_mem), &m_ref);
        clSetKernelArg(k_filt, 1, sizeof(cl_mem), &m_filt);
        clSetKernelArg(k_filt, 2, sizeof(cl_int), &W);
        clSetKernelArg(k_filt, 3, sizeof(cl_int), &H);
        clSetKernelArg(k_filt, 4, sizeof(cl_int), &kidx);
        clSetKernelArg(k_filt, 5, sizeof(cl_int), &rep);
        size_t l = 256, g = (size_t)nctus * 4 * 256;
        double w0 = now_s();
        CHECK(clEnqueueNDRangeKernel(q, k_filt, 1, NULL, &g, &l, 0, NULL, &e), "filter");
        CHECK(clFinish(q), "finish filter");
        t_filt += ev_ms(e, (now_s() - w0) * 1e3);
        clReleaseEvent(e);
        if (filtered)
          CHECK(clEnqueueReadBuffer(q, m_filt, CL_TRUE, rep * fs * 2, fs * 2, filtered + fs * f, 0, NULL, NULL), "D2H filt");
      }
      cl_mem src = k_filt ? m_filt : m_ref; /* main.cpp:818-822 */
      clSetKernelArg(k_init, 0, sizeof(cl_mem), &src);
      clSetKernelArg(k_init, 1, sizeof(cl_int), &W);
      clSetKernelArg(k_init, 2, sizeof(cl_int), &H);
      clSetKernelArg(k_init, 3, sizeof(cl_mem), &m_redT);
      clSetKernelArg(k_init, 4, sizeof(cl_mem), &m_redL);
      clSetKernelArg(k_init, 5, sizeof(cl_mem), &m_refT);
      clSetKernelArg(k_init, 6, sizeof(cl_mem), &m_refL);
      clSetKernelArg(k_init, 7, sizeof(cl_int), &rep);
      size_t l = 128, g = (size_t)nctus * 47 * 128;
      double w0 = now_s();
      CHECK(clEnqueueNDRangeKernel(q, k_init, 1, NULL, &g, &l, 0, NULL, &e), "initBoundaries");
      CHECK(clFinish(q), "finish init");
      t_init += ev_ms(e, (now_s() - w0) * 1e3);
      clReleaseEvent(e);

      clSetKernelArg(k_red, 0, sizeof(cl_mem), &m_pred);
      clSetKernelArg(k_red, 1, sizeof(cl_int), &W);
      clSetKernelArg(k_red, 2, sizeof(cl_int), &H);
      clSetKernelArg(k_red, 3, sizeof(cl_mem), &m_ref);
      clSetKernelArg(k_red, 4, sizeof(cl_mem), &m_redT);
      clSetKernelArg(k_red, 5, sizeof(cl_mem), &m_redL);
      clSetKernelArg(k_red, 6, sizeof(cl_int), &rep);
      l = 256;
      g = (size_t)nctus * 47 * 256;
      w0 = now_s();
      CHECK(clEnqueueNDRangeKernel(q, k_red, 1, NULL, &g, &l, 0, NULL, &e), "MIP_ReducedPred");
      CHECK(clFinish(q), "finish reduced");
      t_red += ev_ms(e, (now_s() - w0) * 1e3);
      clReleaseEvent(e);

      for (int s = 0; s < 3; s++) {
        cl_kernel k = k_up[s];
        int a = 0;
        clSetKernelArg(k, a++, sizeof(cl_mem), &m_pred);
        clSetKernelArg(k, a++, sizeof(cl_int), &W);
        clSetKernelArg(k, a++, sizeof(cl_int), &H);
        if (full) {
          clSetKernelArg(k, a++, sizeof(cl_mem), &m_sad);
          clSetKernelArg(k, a++, sizeof(cl_mem), &m_satd);
        }
        clSetKernelArg(k, a++, sizeof(cl_mem), &m_min);
        clSetKernelArg(k, a++, sizeof(cl_mem), &m_ref); /* originals, main.cpp:1006 */
        clSetKernelArg(k, a++, sizeof(cl_mem), &m_refT);
        clSetKernelArg(k, a++, sizeof(cl_mem), &m_refL);
        clSetKernelArg(k, a++, sizeof(cl_int), &rep);
        g = (size_t)up_wgs[s] * 256;
        w0 = now_s();
        CHECK(clEnqueueNDRangeKernel(q, k, 1, NULL, &g, &l, 0, NULL, &e), "upsampleDistortion");
        CHECK(clFinish(q), "finish upsample");
        t_up[s] += ev_ms(e, (now_s() - w0) * 1e3);
        clReleaseEvent(e);
      }
      const size_t off = (size_t)rep * nctus * COST_PER_CTU * 8, cnt = (size_t)nctus * COST_PER_CTU;
      if (costs) {
        CHECK(clEnqueueReadBuffer(q, m_min, CL_TRUE, off, cnt * 8, tmp, 0, NULL, NULL), "D2H cost");
        for (size_t i = 0; i < cnt; i++) costs[(size_t)f * cnt + i] = (int32_t)tmp[i];
      }
      if (sads) {
        CHECK(clEnqueueReadBuffer(q, m_sad, CL_TRUE, off, cnt * 8, tmp, 0, NULL, NULL), "D2H sad");
        for (size_t i = 0; i < cnt; i++) sads[(size_t)f * cnt + i] = (int32_t)tmp[i];
      }
      if (satds) {
        CHECK(clEnqueueReadBuffer(q, m_satd, CL_TRUE, off, cnt * 8, tmp, 0, NULL, NULL), "D2H satd");
        for (size_t i = 0; i < cnt; i++) satds[(size_t)f * cnt + i] = (int32_t)tmp[i];
      }
    }
    wall = now_s() - wall0;
  }
  const size_t cnt = (size_t)frames * nctus * COST_PER_CTU;
  if (costs) write_file(out_cost, costs, cnt * 4);
  if (sads) write_file(out_sad, sads, cnt * 4);
  if (satds) write_file(out_satd, satds, cnt * 4);
  if (filtered) write_file(out_filt, filtered, fs * 2 * frames);
  const double dev_ms = t_filt + t_init + t_red + t_up[0] + t_up[1] + t_up[2];
  printf("{\"device\": \"%s\", \"width\": %d, \"height\": %d, \"frames\": %d, \"filter\": \"%s\", "
         "\"kernel_ms\": {\"filter\": %.4f, \"initBoundaries\": %.4f, \"MIP_ReducedPred\": %.4f, "
         "\"upsampleDistortion_s2\": %.4f, \"upsampleDistortion_s1\": %.4f, \"upsampleDistortion_s0\": %.4f}, "
         "\"device_ms_per_frame\": %.4f, \"wall_ms_per_frame\": %.4f, \"event_fallbacks\": %d, "
         "\"event_fallback_reason\": \"%s\"}\n",
         dname, W, H, frames, filter ? filter : "", t_filt / frames, t_init / frames, t_red / frames,
         t_up[0] / frames, t_up[1] / frames, t_up[2] / frames, dev_ms / frames, wall * 1e3 / frames,
         g_event_fallbacks, g_fallback_reason);
  return 0;
}
