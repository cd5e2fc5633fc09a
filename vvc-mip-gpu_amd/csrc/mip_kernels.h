// mip_kernels.h -- launch interface between the C-ABI host code (mipgpu.cpp) and the
// gfx950 kernels (mip_search.hip, mip_filter.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mipgpu {

// Work is organised per 64x64 quadrant of a CTU (no CU of the 47 shapes straddles a
// quadrant).  A *job* is one (CU, mode pair) of a shape inside the quadrant; a *wave task*
// is up to 64/S jobs of one shape (S = W/4 strips per CU), one lane per (job, strip).
// Job geometry is resolved on the host (no integer division in the kernel).
struct Job {
  uint32_t cost;  // entry of mode 2q inside the CTU's cost block: shape offset + cu*2*modes + 2q
                  // (CU index in reference order, constants.h:1235-1354 / 1558-1631)
  uint8_t lx, ly; // CU origin inside the 64x64 quadrant
  uint16_t wrow;  // weight row of mode (2q mod modes); bit 15: pair is transposed (2q >= modes)
};
constexpr uint16_t kJobTransposed = 0x8000;
struct WaveTask {
  uint8_t shape;
  uint8_t njobs;
  uint16_t pad;
  uint32_t job0;  // index into the quadrant's job array
};

struct SearchArgs {
  const uint16_t *orig;   // [frames][height][width] original samples (distortion)
  const uint16_t *refs;   // reference-sample source: == orig, or the filtered frames
  int32_t *cost;          // [frames][nctus][97840]  min(2*SAD, SATD)
  int32_t *sad;           // optional, same layout
  int32_t *satd;          // optional, same layout
  const WaveTask *tasks;  // 4 per-quadrant task lists, concatenated (heaviest first)
  const Job *jobs;        // 4 per-quadrant job arrays, concatenated
  const int16_t *weights; // expanded MIP weights, see kWeightWords
  int width, height;
  int ctu_cols, nctus;
  int task_begin[5];      // quadrant q's tasks: [task_begin[q], task_begin[q+1])
  int slices;             // workgroups per CTU quadrant
};

// Expanded weight table (int16): 16-byte rows of 8 taps, index (mode*outputs + j)*8.
//   sizeId 2: rows [0, 384)    taps (0, w0..w6)   (mip_matrix.cl:441, intra.cl:459-463)
//   sizeId 1: rows [384, 512)  taps w0..w7
//   sizeId 0: rows [512, 768)  taps w0..w3, 0, 0, 0, 0
constexpr int kWeightRowsS2 = 6 * 64, kWeightRowsS1 = 8 * 16, kWeightRowsS0 = 16 * 16;
constexpr int kWeightRowOffS1 = kWeightRowsS2, kWeightRowOffS0 = kWeightRowsS2 + kWeightRowsS1;
constexpr int kWeightWords = (kWeightRowsS2 + kWeightRowsS1 + kWeightRowsS0) * 8;

struct BestArgs {
  const int32_t *cost;
  uint8_t *best_mode;
  int32_t *best_cost;
  int total_cus;          // frames * nctus * 5380
};

struct FilterArgs {
  const uint16_t *in;
  uint16_t *out;
  int width, height, nframes;
  int filter;             // reference whitelist index (constants.h:25-34)
  int kernel_idx;
};

hipError_t launch_search(const SearchArgs &a, int nframes, bool alt_refs, hipStream_t s);
hipError_t launch_best_modes(const BestArgs &a, hipStream_t s);
hipError_t launch_filter(const FilterArgs &a, hipStream_t s);

}  // namespace mipgpu
