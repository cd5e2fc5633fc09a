/* cl_cpu_shim.cl -- TEST INFRASTRUCTURE: the OpenCL C builtins the reference's intra.cl
 * calls, for running its kernels on the host CPU (BASELINE
 * configs[0]).  Compiled by the same clang, for the same x86-64 target and options as
 * /root/reference/intra.cl (oracle/Makefile ref-cpu), so every definition below gets the
 * mangled name and vector ABI the compiled kernels call.  Work-item / work-group ids and
 * barrier() come from the work-group executor (ref/ref_cpu_runner.cpp: one fiber per work-item).
 * Semantics follow the OpenCL 1.2 specification (select: per-component MSB for vectors,
 * abs returns the unsigned type, shuffle takes mask components modulo the vector size).
 */
ulong shim_group_id(uint d);
ulong shim_local_id(uint d);
ulong shim_local_size(uint d);
void shim_barrier(void);

#define OVL __attribute__((overloadable))

size_t OVL get_group_id(uint d) { return shim_group_id(d); }
size_t OVL get_local_id(uint d) { return shim_local_id(d); }
size_t OVL get_local_size(uint d) { return shim_local_size(d); }
void OVL barrier(cl_mem_fence_flags f) { shim_barrier(); }

uint OVL abs(int x) { return x < 0 ? (uint)(-(long)x) : (uint)x; }
int OVL max(int a, int b) { return a > b ? a : b; }
int OVL min(int a, int b) { return a < b ? a : b; }
int OVL clamp(int x, int lo, int hi) { return x < lo ? lo : (x > hi ? hi : x); }

short OVL select(short a, short b, short c) { return c ? b : a; }
int OVL select(int a, int b, int c) { return c ? b : a; }
uint OVL select(uint a, uint b, uint c) { return c ? b : a; }
float OVL select(float a, float b, int c) { return c ? b : a; }
float OVL select(float a, float b, uint c) { return c ? b : a; }
short4 OVL select(short4 a, short4 b, short4 c) { return c < (short4)0 ? b : a; }
short8 OVL select(short8 a, short8 b, short8 c) { return c < (short8)0 ? b : a; }

int16 OVL convert_int16(short16 v) { return __builtin_convertvector(v, int16); }
float4 OVL convert_float4(short4 v) { return __builtin_convertvector(v, float4); }
float4 OVL convert_float4(uchar4 v) { return __builtin_convertvector(v, float4); }

float OVL dot(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

float OVL ceil(float x) { return __builtin_ceilf(x); }
double OVL ceil(double x) { return __builtin_ceil(x); }
float OVL floor(float x) { return __builtin_floorf(x); }
float OVL round(float x) { return __builtin_roundf(x); }
float OVL log2(float x) { return __builtin_log2f(x); }

short2 OVL vload2(size_t o, const __global short *p) { p += 2 * o; return (short2)(p[0], p[1]); }
short4 OVL vload4(size_t o, const __global short *p) { p += 4 * o; return (short4)(p[0], p[1], p[2], p[3]); }
short4 OVL vload4(size_t o, const __local short *p) { p += 4 * o; return (short4)(p[0], p[1], p[2], p[3]); }
uchar4 OVL vload4(size_t o, const __constant uchar *p) { p += 4 * o; return (uchar4)(p[0], p[1], p[2], p[3]); }
uchar8 OVL vload8(size_t o, const __constant uchar *p) {
  p += 8 * o;
  return (uchar8)(p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7]);
}

uchar8 OVL shuffle(uchar8 x, uchar8 mask) {
  uchar8 r;
  r.s0 = x[mask.s0 & 7];
  r.s1 = x[mask.s1 & 7];
  r.s2 = x[mask.s2 & 7];
  r.s3 = x[mask.s3 & 7];
  r.s4 = x[mask.s4 & 7];
  r.s5 = x[mask.s5 & 7];
  r.s6 = x[mask.s6 & 7];
  r.s7 = x[mask.s7 & 7];
  return r;
}
