/* mip_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar C restatement of the reference's MIP cost pipeline and low-pass filters
 * (iagostorch/VVC-MIP-GPU: intra.cl, kernel_aux_functions.cl, constants.cl).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / CPU baseline.  The product path (libmipgpu.so) never links it.
 *
 * Parity pinning: the outputs of this oracle are checked against golden fixtures that
 * were produced by running the reference's own OpenCL kernels (compiled from
 * /root/reference/intra.cl by oracle/ref/Makefile) on an MI355X, see
 * tests/golden/README.md and tests/test_oracle_golden.py.
 */
#ifndef MIP_ORACLE_H
#define MIP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIPO_UNAVAILABLE 0x7fffffff

/* Filter identifiers, in the order of the reference whitelist constants.h:25-34. */
enum {
  MIPO_FILTER_1D_INT = 0,
  MIPO_FILTER_1D_FLOAT = 1,
  MIPO_FILTER_2D_INT = 2,        /* filterFrame_2d_int_quarterCtu   intra.cl:2856 */
  MIPO_FILTER_2D_FLOAT = 3,      /* filterFrame_2d_float_quarterCtu intra.cl:1639 */
  MIPO_FILTER_1D_INT_5x5 = 4,
  MIPO_FILTER_1D_FLOAT_5x5 = 5,
  MIPO_FILTER_2D_INT_5x5 = 6,    /* filterFrame_2d_int_5x5_quarterCtu   intra.cl:3042 */
  MIPO_FILTER_2D_FLOAT_5x5 = 7,  /* filterFrame_2d_float_5x5_quarterCtu intra.cl:2311 */
};

int mipo_num_ctus(int width, int height);
int64_t mipo_costs_per_frame(int width, int height);

/* Full MIP search of one frame (all CTUs).  `refs` is the frame the reference samples
 * are taken from (== orig for USE_ALTERNATIVE_SAMPLES=0, the filtered frame otherwise).
 * Outputs use the reference cost layout ALL_stridedDistortionsPerCtu (constants.h:1558):
 * index = ctu*97840 + shape.cost_offset + cu*2*modes + mode.  sad/satd may be NULL.
 * CUs whose cost the reference leaves undefined (mipo_cu_defined) get MIPO_UNAVAILABLE.
 * nthreads<=0: all OpenMP threads. */
void mipo_search_frame(const uint16_t *orig, const uint16_t *refs, int width, int height,
                       int32_t *cost, int32_t *sad, int32_t *satd, int nthreads);

/* Search a subset of CTUs [ctu0, ctu1) (for bounded CPU samples); same layout, the
 * output pointers address the full-frame table. */
void mipo_search_ctus(const uint16_t *orig, const uint16_t *refs, int width, int height,
                      int ctu0, int ctu1, int32_t *cost, int32_t *sad, int32_t *satd,
                      int nthreads);

/* Per-CU argmin over the cost table (lowest mode index wins ties); one byte per CU in
 * CU order ctu*5380 + shape CU prefix + cu.  Unavailable CUs -> 0xff. */
void mipo_best_modes(const int32_t *cost, int nctus, uint8_t *best_mode, int32_t *best_cost);

/* Reduced boundaries / reduced prediction of one CU, stage-level helpers for tests. */
void mipo_cu_boundaries(const uint16_t *refs, int width, int height, int x, int y, int w,
                        int h, int16_t *top, int16_t *left, int16_t *red_top,
                        int16_t *red_left);
void mipo_reduced_pred(int size_id, int mode, int transposed, const int16_t *red_top,
                       const int16_t *red_left, int16_t *pred);

/* Low-pass filters (2-D quarter-CTU kernels and separable kernels). */
/* Counts of reduced-prediction clip events since the last reset ([0] < 0, [1] > 1023). */
void mipo_clip_counts(long long *out, int reset);

int mipo_filter_frame(const uint16_t *in, uint16_t *out, int width, int height,
                      int filter, int kernel_idx);

/* Same, plus undef[i] = 1 for samples the reference leaves undefined: they depend on memory
 * past the frame's end (the separable filters' unguarded interior rows, intra.cl:3330; the
 * wrapped columns of the last tile column in the last rows) or on the order of two
 * work-groups' stores (the last tile column's wrapped stores at widths that are not
 * multiples of 128).  Defined samples are the reference's own output bit for bit. */
int mipo_filter_frame_ex(const uint16_t *in, uint16_t *out, uint8_t *undef, int width, int height,
                         int filter, int kernel_idx);

/* 1 = the reference defines the cost of the CU at frame position (x, y) of size w x h. */
int mipo_cu_defined(int width, int height, int x, int y, int w, int h);

/* Per CU (CU order ctu*5380 + shape prefix + cu): 1 if the CU is defined but one of its
 * reference samples is an undefined sample of the filtered frame. */
void mipo_ref_undefined_cus(const uint8_t *undef, int width, int height, uint8_t *cu_out);

/* Synthetic 10-bit frames: kind 0 = structured, 1 = uniform noise. */
void mipo_synth_frame(uint16_t *out, int width, int height, uint64_t seed, int kind);

#ifdef __cplusplus
}
#endif
#endif
