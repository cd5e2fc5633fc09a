// mfma_probe.hip -- checks the operand layout of v_mfma_f32_32x32x16_f16 on gfx950 and that
// f16 inputs given as raw bit patterns 0..2047 (k * 2^-24: subnormals and exponent-1 normals)
// multiply exactly (no denormal flush) -- the representation the SATD-on-MFMA design uses.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/bin/mfma_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A[i][k] (32x16) row-major f16 bits, B[k][n] (16x32) f16 bits, D[i][n] (32x32) f32
__global__ void mm(const unsigned short *A, const unsigned short *B, const float *C, float *D) {
  const int l = threadIdx.x;
  h8 a, b;
  for (int j = 0; j < 8; j++) {
    const int k = 8 * (l / 32) + j;
    unsigned short av = A[(l % 32) * 16 + k], bv = B[k * 32 + (l % 32)];
    a[j] = __builtin_bit_cast(_Float16, av);
    b[j] = __builtin_bit_cast(_Float16, bv);
  }
  f16v c;
  for (int v = 0; v < 16; v++) {
    const int row = 8 * (v / 4) + 4 * (l / 32) + v % 4;
    c[v] = C[row * 32 + l % 32];
  }
  const f16v d = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  for (int v = 0; v < 16; v++) {
    const int row = 8 * (v / 4) + 4 * (l / 32) + v % 4;
    D[row * 32 + l % 32] = d[v];
  }
}

static float h2f(unsigned short h) {
  const int e = (h >> 10) & 31, m = h & 1023, s = h >> 15;
  float v = e == 0 ? ldexpf((float)m, -24) : ldexpf((float)(1024 + m), e - 25);
  return s ? -v : v;
}

int main() {
  unsigned short hA[32 * 16], hB[16 * 32];
  float hC[32 * 32], hD[32 * 32];
  srand(1);
  // A: +-1 and small integers (f16 normal), B: bit patterns 0..2047 (k * 2^-24)
  for (int i = 0; i < 32 * 16; i++) {
    const int v = (rand() % 7) - 3;  // -3..3
    _Float16 f = (_Float16)v;
    memcpy(&hA[i], &f, 2);
  }
  for (int i = 0; i < 16 * 32; i++) hB[i] = (unsigned short)(rand() % 2048);
  for (int i = 0; i < 32 * 32; i++) hC[i] = ldexpf((float)((rand() % 4001) - 2000), -24);
  unsigned short *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dC, sizeof hC);
  hipMalloc(&dD, sizeof hD);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32; i++)
    for (int n = 0; n < 32; n++) {
      double s = hC[i * 32 + n];
      for (int k = 0; k < 16; k++) s += (double)h2f(hA[i * 16 + k]) * (double)h2f(hB[k * 32 + n]);
      if ((double)hD[i * 32 + n] != s) {
        if (bad < 5) printf("mismatch D[%d][%d] = %.10g (x2^24 %.3f) expected %.10g (x2^24 %.3f)\n", i, n, hD[i * 32 + n],
                            ldexp(hD[i * 32 + n], 24), s, ldexp(s, 24));
        bad++;
      }
    }
  printf("32x32x16 f16 layout + subnormal exactness: %d mismatches of 1024\n", bad);
  return bad != 0;
}
