// fetch_probe.hip -- calibrate rocprofv3 FETCH_SIZE on gfx950 for the load widths the kernels
// use (GPU box, under rocprofv3 --pmc FETCH_SIZE).  Each kernel reads the same 1 GiB buffer
// once (coalesced, every byte once) and writes one word per workgroup:
//   read8    8-byte loads per lane (the search kernel's window / lattice staging)
//   read16   16-byte loads per lane (the filter's staging; the MI355X guide's x2 case)
//   window8  the search kernel's quadrant windows: rows of 68 samples starting 4 samples
//            before each 64-sample quadrant, 65 rows, 8-byte chunks (tile_load's pattern)
//   write8   8-byte stores per lane, coalesced (1 GiB)
//   wstride  the search kernel's cost stores: lane = CU with a 128-byte row of 32 int32
//            costs, each store instruction writes 8 bytes (one mode pair) of 64 rows, 16
//            instructions fill the rows (1 GiB)
// FETCH_SIZE / WRITE_SIZE (KiB) x 1024 / bytes = the correction factor for that access.
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void read8(const uint2 *in, size_t n, unsigned *out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += in[i].x ^ in[i].y;
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ void read16(const uint4 *in, size_t n, unsigned *out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += in[i].x ^ in[i].y ^ in[i].z ^ in[i].w;
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ void write8(uint2 *o, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    o[i] = make_uint2((unsigned)i, 1u);
}

__global__ void wstride(uint2 *o, size_t rows) {  // rows of 16 uint2
  for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x)
    for (int p = 0; p < 16; p++) o[r * 16 + p] = make_uint2((unsigned)r, (unsigned)p);
}

// frame W x H of uint16 (W multiple of 128); one workgroup per 64x64 quadrant
__global__ void window8(const uint16_t *frame, int W, int H, unsigned *out) {
  const int qx = 64 * (blockIdx.x % (W / 64)), qy = 64 * (blockIdx.x / (W / 64));
  unsigned acc = 0;
  for (int i = threadIdx.x; i < 65 * 17; i += blockDim.x) {
    const int row = i / 17, ch = i % 17, fy = qy - 1 + row, fx = qx - 4 + 4 * ch;
    if (fy >= 0 && fy < H && fx >= 0) {
      const uint2 v = *reinterpret_cast<const uint2 *>(frame + (size_t)fy * W + fx);
      acc += v.x ^ v.y;
    }
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  void *buf;
  unsigned *out;
  hipMalloc(&buf, bytes);
  hipMalloc(&out, 1 << 20);
  hipMemset(buf, 1, bytes);
  hipDeviceSynchronize();
  read8<<<4096, 256>>>((const uint2 *)buf, bytes / 8, out);
  read16<<<4096, 256>>>((const uint4 *)buf, bytes / 16, out);
  const int W = 7680, H = (int)(bytes / 2 / 7680) / 64 * 64;  // 1 GiB of 8K-wide rows
  window8<<<(W / 64) * (H / 64), 256>>>((const uint16_t *)buf, W, H, out);
  write8<<<4096, 256>>>((uint2 *)buf, bytes / 8);
  wstride<<<4096, 256>>>((uint2 *)buf, bytes / 128);
  hipDeviceSynchronize();
  printf("bytes per kernel: read8 %zu, read16 %zu, window8 unique %zu (rows read %zu)\n", bytes, bytes,
         (size_t)W * H * 2, (size_t)(W / 64) * (H / 64) * 65 * 136);
  return 0;
}
