// mip_kernels.h -- launch interface between the C-ABI host code (mipgpu.cpp) and the
// gfx950 kernels (mip_search.hip, mip_filter.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mipgpu {

// Work is organised per 64x64 quadrant of a CTU (no CU of the 47 shapes straddles a
// quadrant).  CUs of one size class (W x H; several shapes share a class) are grouped into
// wave *tasks*: up to 64/(S*V) CUs (S = W/4 column strips, V = row parts, see
// mip_search.hip) and a range of mode pairs; one lane per (CU, strip, row part) walks
// the pairs one after another.
struct Job {      // one CU of a task (geometry resolved on the host: no division in kernels)
  uint32_t cost;  // entry of mode 0 inside the CTU's cost block: shape offset + cu*2*modes
                  // (CU index in reference order, constants.h:1235-1354 / 1558-1631)
  uint8_t lx, ly; // CU origin inside the 64x64 quadrant
  uint16_t cu;    // CU index inside the CTU (reference order, 0..5379): decision entries
};
struct WaveTask {
  uint8_t cls;    // size class, kClassW/kClassH
  uint8_t ncu;    // CUs in the task
  uint8_t q0, q1; // mode pairs [q0, q1): pair q = modes 2q, 2q+1 (transposed when 2q >= modes)
  uint32_t cu0;   // first CU in the job array
};

// Size classes: W x H with V row parts per CU.  Classes 0-16 are the base class of each CU
// size (row parts: classes with few CUs per quadrant split each CU's rows over V lanes per
// strip so that a task still fills the wave); 17-20 are variants with more row parts, used
// for the remainder group of a class whose CU count per quadrant is not a multiple of its
// task size (e.g. 28 CUs of 32x8 = 3 tasks of 8 + one task of 4 CUs with V = 2; 84 CUs of
// 8x16 = 2 tasks of 32 + three tasks of 7, 7, 6 CUs with V = 4; 12 CUs of 32x16 = one task of
// 8 + one task of 4 with V = 2, classes 27-28).  21-26 are *transposed*
// classes (kClassTR): tasks of wide CUs (32x4, 16x4, 8x4, 32x8, 16x8 -- one upsampling
// direction only) searched as their tall transposes W x H listed here (mip_search.hip
// run_task; the CU position sets of a size and its transpose are transposes of each other).
constexpr int kNumClasses = 29;
constexpr int kNumBaseClasses = 17;
constexpr int kClassW[kNumClasses] = {64, 32, 32, 16, 32, 8, 16, 16, 8, 32, 4, 16, 4, 8, 8, 4, 4, 32, 16, 16, 8,
                                      4, 4, 4, 8, 8, 8, 32, 16};
constexpr int kClassH[kNumClasses] = {64, 32, 16, 32, 8, 32, 16, 8, 16, 4, 32, 4, 16, 8, 4, 8, 4, 8, 16, 8, 16,
                                      32, 16, 8, 32, 16, 16, 16, 32};
// MIP_SIX_WAVES: the search kernel's occupancy design.
//   3 (default since round 6): 12-wave workgroups, two per CU -- six waves per SIMD (80 VGPRs)
//     -- with the MIP tables and the next item's window in LDS beside a 768-word per-wave
//     scratch: 16x16 / 16x8 and the 64-slot 4x4 / 4x8 tasks produce their reduced predictions
//     in halves, 8xH tasks in quarters (mip_search.hip Geo, phase_a_half, walk_pairs_chunked).
//   0: 8-wave workgroups, two per CU, four waves per SIMD, 1280-word scratch (rounds 1-5).
//   1, 2 (round 5 experiments): 12-wave workgroups with the tables in global memory, 1152-word
//     scratch, no prefetch / three 8-wave workgroups.
#ifndef MIP_SIX_WAVES
#define MIP_SIX_WAVES 3
#endif
constexpr int kV16 = MIP_SIX_WAVES == 1 || MIP_SIX_WAVES == 2 ? 2 : 1;  // row parts of the 16x16 / 16x8 base classes
constexpr int kClassV[kNumClasses] = {4, 2, 1, 2, 1, 1, kV16, kV16, 1, 1, 2, 1, 2, 1, 1, 1, 1, 2, 4, 2, 4,
                                      2, 2, 1, 1, 1, 4, 2, 4};
constexpr bool kClassTR[kNumClasses] = {false, false, false, false, false, false, false, false, false, false, false,
                                        false, false, false, false, false, false, false, false, false, false,
                                        true, true, true, true, true, true, false, false};
constexpr int kClassVariant[kNumClasses] = {-1, -1, 27, 28, 17, -1, 18, 19, 20, -1, -1, -1, -1, -1, -1, -1, -1,
                                            -1, -1, -1, -1, -1, -1, -1, -1, 26, -1, -1, -1};  // remainder-task class
// base class -> its transposed class (-1: searched as it is)
constexpr int kClassTransposed[kNumBaseClasses] = {-1, -1, -1, -1, 24, -1, -1, 25, -1, 21, -1, 22, -1, -1, 23, -1, -1};
constexpr int size_class(int w, int h) {  // base class of a CU size
  for (int i = 0; i < kNumBaseClasses; i++)
    if (kClassW[i] == w && kClassH[i] == h) return i;
  return -1;
}
constexpr int class_size_id(int w, int h) { return (w == 4 && h == 4) ? 0 : ((w == 4 || h == 4 || (w == 8 && h == 8)) ? 1 : 2); }
constexpr int class_slots(int cls) { return 64 / ((kClassW[cls] / 4) * kClassV[cls]); }

struct SearchArgs {
  const uint16_t *orig;   // [frames][height][width] original samples (distortion)
  const uint16_t *refs;   // reference-sample source: == orig, or the filtered frames
  int32_t *cost;          // [frames][nctus][97840]  min(2*SAD, SATD); null: decisions only
  // Decisions only ([frames][nctus][5380] per-CU best mode / cost): a task that searches
  // all of a CU's mode pairs writes the CU's decision directly; CUs whose pairs are cut over
  // several tasks (the `split` lists) meet in best_cost as a packed running argmin
  // (cost << 5 | mode, all ones before the launch, atomicMin), unpacked after it
  // (launch_dec_split); CUs the reference leaves undefined get 0xff / kUnavailable from the
  // `dfill` lists.
  uint8_t *best_mode;     // optional
  int32_t *best_cost;
  // optional: the split CUs' packed running argmins go here instead of best_cost (same CU
  // indexing; all ones before the launch, reset to all ones by the unpacking launch_dec_split
  // -- the host pipeline keeps it initialised across launches, so no init kernel runs)
  uint32_t *split_acc;
  const uint16_t *dfill;  // undefined CUs of (v, q): CU indices inside the CTU,
  const int *dfill_begin; // [dfill_begin[4v+q], dfill_begin[4v+q+1])
  int32_t *sad;           // optional, same layout
  int32_t *satd;          // optional, same layout
  const WaveTask *tasks;  // per (quadrant, wave) task lists, concatenated
  const Job *jobs;
  const int *list_begin;  // task list of (CTU variant v, quadrant q, slice s), index l = (4v+q)*slices+s:
                          // [list_begin[l], list_begin[l+1])
  const uint32_t *fill;   // unavailable cost entries of (v, q) (uint4 units inside the CTU's cost
  const int *fill_begin;  // block): [fill_begin[4v+q], fill_begin[4v+q+1])
  const uint8_t *ctu_var; // [nctus] CTU variant (mipgpu.cpp ctu_variants): which CUs are defined
  const uint4 *tables;    // kTableBytes: MIP matrices for the MFMA, see below
  int width, height;
  int ctu_cols, nctus;
  int ctu0, nrange;       // CTUs searched: [ctu0, ctu0 + nrange) of every frame (whole frame:
                          // 0, nctus); cost entries of the other CTUs are not written
  int slices;             // workgroups (task lists) per CTU quadrant
  uint32_t *queue;        // kQueueWords counters, zero at launch (the kernel leaves them zero
                          // again): [c] next item of chunk c (c < kQueueChunks), then
                          // [kQueueChunks] workgroups done
  uint32_t nitems;        // frames * nrange * 4 * slices (set by launch_search)
  // Small launches (one queue chunk): item order longest first (LPT).  order[i] = the i-th
  // (CTU, quadrant, slice) item of a frame, index ctu * 4 * slices + quadrant * slices +
  // slice, by decreasing estimated cost; queue index q -> item order[q / nframes] of frame
  // q % nframes.  Null: raster order (frame-major).  Whole-frame launches only.
  const uint32_t *order;
  uint32_t nframes;
  uint32_t chunks;        // queue chunks, 1..kQueueChunks (set by launch_search)
  uint64_t *wave_clock;   // profiling (MIPGPU_WAVE_TIMING): [workgroup][kClockSlots] cycles per
                          // task of the workgroup's list; else null
  // Input contract (samples are 10-bit): a workgroup that stages an original sample above
  // 1023 stores 1 to status[kStatusOrig], a caller-supplied reference sample above 1023
  // (check_refs) 1 to status[kStatusRefs].  status is engine-owned page-locked host memory
  // (read by the host after the search; only ever written when the contract is broken).
  uint32_t *status;
  // Merged host-pipeline chunks (several host-API calls in one launch, mipgpu.cpp
  // open_chunk): frame f of the launch marks frame_status[f] (its own call's status set)
  // instead of status; null otherwise.  Read only when the contract is broken.
  uint32_t *const *frame_status;
  int check_refs;
  // 16-wave launches with the longest-first order and original references (pair mode,
  // mip_search.hip pair_loop): the first `nonempty` queue positions hold the items with
  // tasks, the rest only fills.  0: items one at a time.
  uint32_t nonempty;
};
constexpr int kStatusOrig = 0, kStatusRefs = 1, kStatusWords = 4;
constexpr uint32_t kAbove10Bits = 0xfc00fc00u;  // any of bits 10..15 in either half
constexpr int kClockSlots = 128;
// Item queue of one launch: the items are cut into kQueueChunks contiguous chunks, one per
// XCD (workgroups b and b + 8 share an XCD), each with its own counter (mip_search.hip
// take_item).
constexpr int kQueueChunks = 8;
constexpr int kQueueWords = 16;  // 8 chunk counters, the done counter, padding to 64 bytes
// CTU variants (mipgpu.cpp ctu_variants): CTUs with the same set of defined CUs share work /
// fill lists; the lists omit the CUs whose cost the reference leaves undefined.
constexpr int kMaxCtuVariants = 255;

// MIP matrices, restated for an exact f16 MFMA (mip_search.hip, phase A).  The reference
// computes pred_j = clamp(((32 - 32*sum_k p_k + sum_k p_k*w_jk) >> 6) + b0, 0, 1023) with
// p_k = b_k - b0 (p_0 = 0 for sizeId 2, 512 - b0 otherwise; intra.cl:415-482).  With
// w'_k = (w_jk - 32)/64 and a0 = 1 (sizeId 2; its matrix has no column for input 0) or
// (96 - w_j0)/64 (sizeId 1/0: p_0 = 512 - b0 folded), that is
//     pred_j = clamp(floor(C_j + a0*b0 + sum_{k>=1} w'_k (b_k - b0)))
// with C_j = 0.5 (sizeId 2) or 8*(w_j0 - 32) + 0.5.  The MFMA is fed x_k = 1024 + b_k (f16
// bit pattern 0x6400 | b_k, no conversion), so the stored coefficients are
//     A_j0 = a0 - sum_{k>=1} w'_k,   A_jk = w'_k (k >= 1),   C'_j = C_j - 1024 * sum_k A_jk.
// All values are multiples of 1/64 below 2^5 (f16-exact); every partial sum stays below
// 2^18 in units of 1/64, so the f32 accumulation is exact.
//   f16 rows [768][8], row = base(sizeId) + mode*R*R + j, base = 0 / 384 / 512 for sizeId
//   2 / 1 / 0 (sizeId 0: 4 inputs, halves 4..7 zero).
//   f32 rows [388] (sizeId 1 and 0, from row 384): C'_j; then 4 x kAccInitS2, the sizeId 2
//   C' = 0.5 - 1024 of every row (read from LDS so it stays in registers).
constexpr float kAccInitS2 = 0.5f - 1024.0f;
constexpr int kWeightRows = 768, kWeightRowOffS1 = 384, kWeightRowOffS0 = 512;
constexpr int kCtabRows = 384 + 4;  // + 4 copies of kAccInitS2 (row 384..387)
constexpr int kTableBytes = kWeightRows * 16 + kCtabRows * 4;

// One CU searched by the exact per-CU kernel (fixup_kernel): alternative references whose
// samples may exceed 10 bits (mipgpu.cpp reads_last_columns).
struct FixupCu {
  uint32_t ctu;
  uint16_t cu;     // CU index inside the CTU (reference order, 0..5379)
  uint8_t shape;
  uint8_t pad;
};

struct BestArgs {
  const int32_t *cost;
  uint8_t *best_mode;     // [total_cus][k]
  int32_t *best_cost;     // [total_cus][k]
  int total_cus;          // frames * nctus * 5380
  int k;                  // decision list length, 1..kMaxBestK
};
constexpr int kMaxBestK = 32;

struct FilterArgs {
  const uint16_t *in;
  uint16_t *out;
  int width, height, nframes;
  int filter;             // reference whitelist index (constants.h:25-34)
  int kernel_idx;
};

// Waves per search workgroup: two 12-wave workgroups share a CU in batched launches (MIP_SIX_WAVES
// 3; 8-wave ones with MIP_SIX_WAVES 0, three per CU with 2); small launches can run one 16-wave
// workgroup per CU instead ("wide"), whose waves share one item's tasks (launch_search).
constexpr int kSearchWaves = MIP_SIX_WAVES == 1 || MIP_SIX_WAVES == 3 ? 12 : 8, kWideWaves = 16;
// Workgroups of the search kernel resident on the current device at once (persistent grid
// size); computed once per engine (mip_engine_create), 0 on error.
int search_resident_groups(bool alt_refs, bool wide);
// The four-wave twin (mip_search.hip compiled again with -DMIP_SIX_WAVES=0
// -DMIP_FOUR_WAVE_TWIN=1): 8-wave workgroups, two per CU, for the host pipeline's small
// alternating chunks; same arguments, no wide launches (0 / hipErrorInvalidValue).
#if !defined(MIP_FOUR_WAVE_TWIN) || !MIP_FOUR_WAVE_TWIN  // (in the twin the names above are these)
int search_resident_groups_four(bool alt_refs, bool wide);
#endif
// done: optional event recorded by the kernel's own dispatch (hipExtLaunchKernel's stop
// event) instead of a separate marker packet behind it.
hipError_t launch_search(const SearchArgs &a, int nframes, bool alt_refs, int resident, bool wide, hipStream_t s,
                         hipEvent_t done = nullptr);
#if !defined(MIP_FOUR_WAVE_TWIN) || !MIP_FOUR_WAVE_TWIN
hipError_t launch_search_four(const SearchArgs &a, int nframes, bool alt_refs, int resident, bool wide, hipStream_t s,
                         hipEvent_t done = nullptr);
#endif
hipError_t launch_best_modes(const BestArgs &a, hipStream_t s);
// Decisions only, CUs whose mode pairs are cut over several tasks (split CUs of the CTU's
// variant: [split_begin[v], split_begin[v+1]) of `split`, at most max_split per variant):
// init = true sets their best_cost entries to all ones (before the search); init = false
// unpacks the packed argmin in place into best_mode / best_cost (after it).  With `acc`
// (SearchArgs::split_acc) the packed argmins are read from acc, which the unpacking resets
// to all ones (init is then never needed).
struct SplitArgs {
  const uint16_t *split;
  const int *split_begin;
  const uint8_t *ctu_var;
  uint8_t *best_mode;
  int32_t *best_cost;
  int nctus, ctu0, nrange, max_split;
  uint32_t *acc;
};
hipError_t launch_dec_split(const SplitArgs &a, int nframes, bool init, hipStream_t s);
hipError_t launch_filter(const FilterArgs &a, hipStream_t s);
// Streaming device-to-device copy (16-byte aligned, multiple of 16 bytes): HBM calibration.
hipError_t launch_copy(const void *src, void *dst, size_t bytes, hipStream_t s);
// Several copies in one launch (the merged chunks' downloads into the members' page-locked,
// device-mapped host buffers: one dispatch instead of one per buffer).
struct CopyPiece {
  const uint8_t *src;
  uint8_t *dst;
  uint64_t bytes;
};
constexpr int kMaxCopyPieces = 64;
struct CopyPieces {
  CopyPiece p[kMaxCopyPieces];
  int n;
};
hipError_t launch_gather_copy(const CopyPieces &a, hipStream_t s);
// Exact per-CU search of `n` CUs of every frame (same outputs as the search kernel: cost /
// SAD / SATD tables or, decisions only, the decision in a.best_mode / a.best_cost).
hipError_t launch_fixup(const SearchArgs &a, const FixupCu *cus, int n, int nframes, hipStream_t s);

}  // namespace mipgpu
