/* ref_cpu_runner.cpp -- TEST INFRASTRUCTURE: the reference's own OpenCL kernels on the host CPU
 * (BASELINE configs[0]).  A baseline, never a target.
 *
 * /root/reference/intra.cl is compiled by clang for x86-64 (oracle/Makefile ref-cpu: one
 * shared library per SIZEID build, with the OpenCL builtins of ref/cl_cpu_shim.cl) and its
 * kernels run here with the reference's launch shapes and buffer layout (main.cpp:420-453,
 * 802-1199; the same sequence as ref/ref_runner.c replays on the GPU):
 *     initBoundaries -> MIP_ReducedPred -> upsampleDistortion (SIZEID 2, 1, 0)
 * Work-groups: the reference's __local arrays are static variables of each kernel in the
 * compiled code, so work-groups run in separate worker processes (fork; every worker has its
 * own copy of them), which share the device buffers (MAP_SHARED memory); inside a
 * work-group every work-item is a fiber (its own stack; a 14-instruction x86-64 switch of the
 * callee-saved registers -- ucontext's signal-mask system calls made 256-item work-groups
 * 10x slower) and barrier() switches to the next work-item (round robin: all work-items
 * reach every barrier, as OpenCL requires).
 *
 * usage: ref_cpu_runner --libs DIR --width W --height H [--frames N] [--synth KIND:SEED]
 *                       [--workers N] [--out-cost F]
 * prints one JSON line: wall time per kernel and per frame, workers (= host cores used).
 */
#include <dlfcn.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

extern "C" {
#include "../mip_oracle.h"
}

// ---------------------------------------------------------------- work-group executor
// ctx_switch(&from_sp, to_sp): save the callee-saved registers on the current stack, store
// its pointer in *from_sp, continue on to_sp (System V x86-64).
extern "C" void ctx_switch(void **from_sp, void *to_sp);
asm(R"(
  .text
  .globl ctx_switch
  .type ctx_switch, @function
ctx_switch:
  pushq %rbp
  pushq %rbx
  pushq %r12
  pushq %r13
  pushq %r14
  pushq %r15
  movq %rsp, (%rdi)
  movq %rsi, %rsp
  popq %r15
  popq %r14
  popq %r13
  popq %r12
  popq %rbx
  popq %rbp
  ret
  .size ctx_switch, .-ctx_switch
)");

namespace {
size_t g_group = 0, g_lsize = 0;
int g_cur = 0, g_done = 0;
struct Fiber {
  void *sp = nullptr;
  char *stack = nullptr;
  bool done = false;
};
std::vector<Fiber> g_fib;
void *g_sched_sp = nullptr, *g_dead_sp = nullptr;
std::function<void()> g_body;
constexpr size_t kStack = 256 << 10;
void fiber_entry();
// first activation of a fiber (reached by ctx_switch's `ret`, stack aligned as after a call)
void fiber_trampoline() {
  fiber_entry();
  abort();  // (never returns: fiber_entry switches away)
}
void *fresh_stack(char *stack) {
  uintptr_t slot = ((uintptr_t)(stack + kStack) & ~(uintptr_t)15) - 16;  // return-address slot, 16-aligned
  *(void **)slot = (void *)&fiber_trampoline;
  for (int i = 1; i <= 6; i++) *(void **)(slot - 8 * i) = nullptr;  // rbp rbx r12 r13 r14 r15
  return (void *)(slot - 48);
}

int next_live(int from) {
  const int n = (int)g_fib.size();
  for (int k = 1; k <= n; k++) {
    const int j = (from + k) % n;
    if (!g_fib[j].done) return j;
  }
  return -1;
}

void fiber_entry() {
  g_body();
  const int me = g_cur;
  g_fib[me].done = true;
  g_done++;
  const int nx = next_live(me);
  if (nx < 0) {
    ctx_switch(&g_dead_sp, g_sched_sp);
  } else {
    g_cur = nx;
    ctx_switch(&g_dead_sp, g_fib[nx].sp);
  }
}

// One work-group of `lsize` work-items running `body` (the kernel call).
void run_group(size_t group, size_t lsize, const std::function<void()> &body) {
  g_group = group;
  g_lsize = lsize;
  g_body = body;
  if (g_fib.size() != lsize) {
    for (Fiber &f : g_fib) free(f.stack);
    g_fib.assign(lsize, Fiber());
    for (Fiber &f : g_fib) f.stack = (char *)malloc(kStack);
  }
  for (Fiber &f : g_fib) {
    f.done = false;
    f.sp = fresh_stack(f.stack);
  }
  g_done = 0;
  g_cur = 0;
  ctx_switch(&g_sched_sp, g_fib[0].sp);
  if (g_done != (int)lsize) {
    fprintf(stderr, "work-group %zu ended with %d of %zu work-items\n", group, g_done, lsize);
    exit(6);
  }
}
}  // namespace

extern "C" {
unsigned long shim_group_id(unsigned d) { return d == 0 ? g_group : 0; }
unsigned long shim_local_id(unsigned d) { return d == 0 ? (unsigned long)g_cur : 0; }
unsigned long shim_local_size(unsigned d) { return d == 0 ? g_lsize : 1; }
void shim_barrier(void) {
  const int me = g_cur, nx = next_live(me);
  if (nx < 0 || nx == me) return;
  g_cur = nx;
  ctx_switch(&g_fib[me].sp, g_fib[nx].sp);  // (resumed with g_cur == me)
}
}

// ---------------------------------------------------------------- launches
namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// `ngroups` work-groups of `lsize` work-items over `workers` processes (group g on worker
// g % workers); returns the wall time.
double launch(int workers, size_t ngroups, size_t lsize, const std::function<void()> &body) {
  const double t0 = now_s();
  std::vector<pid_t> kids;
  for (int w = 0; w < workers; w++) {
    const pid_t p = fork();
    if (p == 0) {
      for (size_t g = (size_t)w; g < ngroups; g += (size_t)workers) run_group(g, lsize, body);
      _exit(0);
    }
    if (p < 0) {
      perror("fork");
      exit(7);
    }
    kids.push_back(p);
  }
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
      fprintf(stderr, "worker failed (status %d)\n", st);
      exit(8);
    }
  }
  return now_s() - t0;
}

template <class T>
T *shared(size_t count) {
  void *p = mmap(nullptr, count * sizeof(T), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) {
    perror("mmap");
    exit(9);
  }
  return (T *)p;
}

void *sym(void *lib, const char *name) {
  void *f = dlsym(lib, name);
  if (!f) {
    fprintf(stderr, "missing %s: %s\n", name, dlerror());
    exit(4);
  }
  return f;
}

// Per-CTU strides of the reference's unified buffers (as ref/ref_runner.c).
enum : size_t { RED_PER_CTU = 4356 * 4 + 1024 * 2, REF_PER_CTU = 48640, PRED_PER_CTU = 2231296, COST_PER_CTU = 97840 };

typedef void (*InitFn)(short *, int, int, short *, short *, short *, short *, int);
typedef void (*RedFn)(short *, int, int, short *, short *, short *, int);
typedef void (*UpFn)(short *, int, int, long *, short *, short *, short *, int);  // MAX_PERFORMANCE_DIST=1
}  // namespace

int main(int argc, char **argv) {
  const char *libs = "oracle/_ref", *out_cost = nullptr;
  int W = 0, H = 0, frames = 1, kind = 0, workers = (int)sysconf(_SC_NPROCESSORS_ONLN);
  unsigned long long seed = 0x1080;
  for (int i = 1; i < argc; i++) {
    const char *a = argv[i], *v = i + 1 < argc ? argv[i + 1] : "";
    if (!strcmp(a, "--libs")) libs = v, i++;
    else if (!strcmp(a, "--width")) W = atoi(v), i++;
    else if (!strcmp(a, "--height")) H = atoi(v), i++;
    else if (!strcmp(a, "--frames")) frames = atoi(v), i++;
    else if (!strcmp(a, "--synth")) { sscanf(v, "%d:%llx", &kind, &seed); i++; }
    else if (!strcmp(a, "--workers")) workers = atoi(v), i++;
    else if (!strcmp(a, "--out-cost")) out_cost = v, i++;
    else { fprintf(stderr, "unknown argument %s\n", a); return 2; }
  }
  if (W <= 0 || H <= 0 || frames < 1 || workers < 1) { fprintf(stderr, "need --width/--height\n"); return 2; }
  void *lib[3];
  for (int s = 0; s < 3; s++) {
    const std::string p = std::string(libs) + "/intra_cpu_s" + std::to_string(s) + ".so";
    if (!(lib[s] = dlopen(p.c_str(), RTLD_NOW | RTLD_LOCAL))) {
      fprintf(stderr, "cannot load %s: %s (make -C oracle ref-cpu)\n", p.c_str(), dlerror());
      return 4;
    }
  }
  InitFn k_init = (InitFn)sym(lib[2], "__clang_ocl_kern_imp_initBoundaries");
  RedFn k_red = (RedFn)sym(lib[2], "__clang_ocl_kern_imp_MIP_ReducedPred");
  UpFn k_up[3] = {(UpFn)sym(lib[2], "__clang_ocl_kern_imp_upsampleDistortion"),
                  (UpFn)sym(lib[1], "__clang_ocl_kern_imp_upsampleDistortion"),
                  (UpFn)sym(lib[0], "__clang_ocl_kern_imp_upsampleDistortion")};

  const size_t fs = (size_t)W * H, slots = 2, pad = (size_t)W * 256 + 4096;
  const size_t nctus = (size_t)((W + 127) / 128) * ((H + 127) / 128);
  short *m_ref = shared<short>(slots * fs + pad);  // zero-filled (ref_runner's default fill)
  short *m_redT = shared<short>(slots * nctus * RED_PER_CTU), *m_redL = shared<short>(slots * nctus * RED_PER_CTU);
  short *m_refT = shared<short>(slots * nctus * REF_PER_CTU), *m_refL = shared<short>(slots * nctus * REF_PER_CTU);
  short *m_pred = shared<short>(slots * nctus * PRED_PER_CTU);
  long *m_min = shared<long>(slots * nctus * COST_PER_CTU);
  std::vector<uint16_t> host(fs);
  std::vector<int32_t> costs;
  if (out_cost) costs.resize((size_t)frames * nctus * COST_PER_CTU);
  const int up_wgs[3] = {(int)nctus * 28, (int)nctus * 18, (int)nctus * 8};
  double t_init = 0, t_red = 0, t_up[3] = {0, 0, 0};
  const double wall0 = now_s();
  for (int f = 0; f < frames; f++) {
    const int rep = f % 2;
    mipo_synth_frame(host.data(), W, H, seed + f, kind);
    memcpy(m_ref + (size_t)rep * fs, host.data(), fs * 2);
    t_init += launch(workers, nctus * 47, 128, [&] { k_init(m_ref, W, H, m_redT, m_redL, m_refT, m_refL, rep); });
    t_red += launch(workers, nctus * 47, 256, [&] { k_red(m_pred, W, H, m_ref, m_redT, m_redL, rep); });
    for (int s = 0; s < 3; s++)
      t_up[s] += launch(workers, (size_t)up_wgs[s], 256,
                        [&, s] { k_up[s](m_pred, W, H, m_min, m_ref, m_refT, m_refL, rep); });
    if (out_cost) {
      const size_t cnt = nctus * COST_PER_CTU;
      for (size_t i = 0; i < cnt; i++) costs[(size_t)f * cnt + i] = (int32_t)m_min[(size_t)rep * cnt + i];
    }
  }
  const double wall = now_s() - wall0;
  if (out_cost) {
    FILE *o = fopen(out_cost, "wb");
    if (!o || fwrite(costs.data(), 4, costs.size(), o) != costs.size()) { fprintf(stderr, "cannot write %s\n", out_cost); return 5; }
    fclose(o);
  }
  printf("{\"device\": \"host CPU (x86-64, clang-compiled intra.cl)\", \"width\": %d, \"height\": %d, \"frames\": %d, "
         "\"workers\": %d, \"kernel_s\": {\"initBoundaries\": %.4f, \"MIP_ReducedPred\": %.4f, "
         "\"upsampleDistortion_s2\": %.4f, \"upsampleDistortion_s1\": %.4f, \"upsampleDistortion_s0\": %.4f}, "
         "\"wall_s_per_frame\": %.4f, \"frames_per_s\": %.5f}\n",
         W, H, frames, workers, t_init / frames, t_red / frames, t_up[0] / frames, t_up[1] / frames, t_up[2] / frames,
         wall / frames, frames / wall);
  return 0;
}
