/* ref_build.c -- TEST INFRASTRUCTURE: compile the reference's own OpenCL kernels.
 *
 * Builds /root/reference/intra.cl (read in place, never copied) with the AMD OpenCL
 * runtime's offline-device support (CL_CONTEXT_OFFLINE_DEVICES_AMD), using the build
 * options of main.cpp:486-530 ("-DSIZEID=s -DTRACE_POWER=1 -DN_FRAMES=n
 * -DMAX_PERFORMANCE_DIST=d") plus an include path for intra.cl:9-10.  The resulting
 * gfx950 code objects go to oracle/_ref/ and are loaded on the GPU box by ref_runner
 * through clCreateProgramWithBinary -- the reference kernels, compiled by the vendor
 * OpenCL compiler, running on the real device.
 *
 * usage: ref_build <reference_dir> <out_dir> <device_name> [device_name...]
 */
#define CL_TARGET_OPENCL_VERSION 120
#include <CL/cl.h>
#include <CL/cl_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static char *slurp(const char *path, size_t *n) {
  FILE *f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long len = ftell(f);
  rewind(f);
  char *buf = (char *)malloc((size_t)len + 1);
  if (fread(buf, 1, (size_t)len, f) != (size_t)len) { fclose(f); free(buf); return NULL; }
  buf[len] = 0;
  fclose(f);
  *n = (size_t)len;
  return buf;
}

static void sanitize(const char *in, char *out) {
  for (; *in; in++, out++) *out = (*in == ':' || *in == '+' || *in == '-') ? (*in == '+' ? 'p' : (*in == '-' ? 'm' : '_')) : *in;
  *out = 0;
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <reference_dir> <out_dir> <device_name>...\n", argv[0]);
    return 2;
  }
  char path[4096];
  snprintf(path, sizeof path, "%s/intra.cl", argv[1]);
  size_t n = 0;
  char *src = slurp(path, &n);
  if (!src) { fprintf(stderr, "cannot read %s\n", path); return 1; }

  cl_platform_id plat;
  cl_uint np = 0;
  if (clGetPlatformIDs(1, &plat, &np) != CL_SUCCESS || np == 0) { fprintf(stderr, "no OpenCL platform\n"); return 1; }
  cl_context_properties props[] = {CL_CONTEXT_PLATFORM, (cl_context_properties)plat,
                                   CL_CONTEXT_OFFLINE_DEVICES_AMD, 1, 0};
  cl_int err;
  cl_context ctx = clCreateContextFromType(props, CL_DEVICE_TYPE_ALL, NULL, NULL, &err);
  if (err != CL_SUCCESS) { fprintf(stderr, "offline context failed: %d\n", err); return 1; }
  size_t sz = 0;
  clGetContextInfo(ctx, CL_CONTEXT_DEVICES, 0, NULL, &sz);
  int nd = (int)(sz / sizeof(cl_device_id));
  cl_device_id *devs = (cl_device_id *)malloc(sz);
  clGetContextInfo(ctx, CL_CONTEXT_DEVICES, sz, devs, NULL);

  int failures = 0;
  for (int a = 3; a < argc; a++) {
    cl_device_id dev = 0;
    for (int k = 0; k < nd; k++) {
      char name[256];
      clGetDeviceInfo(devs[k], CL_DEVICE_NAME, sizeof name, name, NULL);
      if (!strcmp(name, argv[a])) dev = devs[k];
    }
    if (!dev) { fprintf(stderr, "offline device %s not offered\n", argv[a]); failures++; continue; }
    char tag[256];
    sanitize(argv[a], tag);
    for (int dist = 0; dist <= 1; dist++)
      for (int sid = 2; sid >= 0; sid--) {
        char opts[8192];
        snprintf(opts, sizeof opts,
                 "-I%s -DSIZEID=%d -DTRACE_POWER=1 -DN_FRAMES=2 -DMAX_PERFORMANCE_DIST=%d",
                 argv[1], sid, dist);
        const char *s = src;
        cl_program prog = clCreateProgramWithSource(ctx, 1, &s, &n, &err);
        err = clBuildProgram(prog, 1, &dev, opts, NULL, NULL);
        if (err != CL_SUCCESS) {
          size_t ls = 0;
          clGetProgramBuildInfo(prog, dev, CL_PROGRAM_BUILD_LOG, 0, NULL, &ls);
          char *log = (char *)malloc(ls + 1);
          clGetProgramBuildInfo(prog, dev, CL_PROGRAM_BUILD_LOG, ls, log, NULL);
          fprintf(stderr, "build %s sid=%d failed (%d):\n%s\n", argv[a], sid, err, log);
          free(log);
          failures++;
          continue;
        }
        size_t bs = 0;
        clGetProgramInfo(prog, CL_PROGRAM_BINARY_SIZES, sizeof bs, &bs, NULL);
        unsigned char *bin = (unsigned char *)malloc(bs);
        unsigned char *bp[1] = {bin};
        clGetProgramInfo(prog, CL_PROGRAM_BINARIES, sizeof bp, bp, NULL);
        snprintf(path, sizeof path, "%s/intra_%s_s%d_d%d.bin", argv[2], tag, sid, dist);
        FILE *o = fopen(path, "wb");
        if (!o || fwrite(bin, 1, bs, o) != bs) { fprintf(stderr, "write %s failed\n", path); failures++; }
        if (o) fclose(o);
        printf("wrote %s (%zu bytes)\n", path, bs);
        free(bin);
        clReleaseProgram(prog);
      }
  }
  free(devs);
  free(src);
  clReleaseContext(ctx);
  return failures ? 1 : 0;
}
