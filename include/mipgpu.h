/* mipgpu.h -- C ABI of the MI355X-native VVC MIP search engine (libmipgpu.so).
 *
 * Drop-in boundary for the hot path of iagostorch/VVC-MIP-GPU.  The reference has no
 * FFI layer: its path is main.cpp's OpenCL dispatch of
 *     filterFrame_<type>  (intra.cl:1639-3823, dispatched main.cpp:700-761)
 *     initBoundaries      (intra.cl:17,   main.cpp:802-843)
 *     MIP_ReducedPred     (intra.cl:349,  main.cpp:909-945)
 *     upsampleDistortion  (intra.cl:545,  main.cpp:995-1199, built 3x with -DSIZEID)
 * plus the cost read-back readMemobjsIntoArray_Distortion (main_aux_functions.h:585-630).
 * Each entry point below replaces one of those steps (cited per function); the C++ CLI
 * (vvc-mip-gpu_amd/cli/mipgpu_cli.cpp) replaces main.cpp on top of it.
 *
 * Conventions: plain pointers and sizes, int status (0 = ok, <0 = error, message via
 * mip_last_error()), no exceptions cross the boundary.  Host buffers are owned by the
 * caller; device buffers of the engine are owned by the engine.  One engine per device;
 * an engine must be used by one host thread at a time.  Samples are 10-bit values in
 * uint16; frames are row-major, consecutive frames are concatenated.
 *
 * Input contract: every sample of a frame (and of caller-supplied reference frames) is at
 * most 1023, like the reference's 10-bit constants (valueDC 512, clip 1023,
 * constants.cl:22-23).  The search kernel detects a staged sample above 1023 and the engine
 * reports it as an error (costs of such a frame are not valid): mip_search_frames /
 * mip_wait fail for the call that searched it; device-API searches are asynchronous, so
 * their violation is reported by mip_check_input or by the engine's next search call.
 *
 * Cost layout (identical to the reference's ALL_stridedDistortionsPerCtu,
 * constants.h:1558-1631): int32 [frames][nCTUs][97840], entry
 *     ctu*97840 + shape_offset + cu*2*modes + mode
 * with the 47 CU shapes in reference order.  Samples are addressed like the reference does,
 * by linear index y * width + x, so CUs right of the frame (widths that are not multiples
 * of 128) read the next row's samples and get the reference's costs.  CUs whose cost the
 * reference leaves undefined -- below the frame (stale LDS, intra.cl:96-98), reading past
 * the frame's end, or (engine filter) reading a filtered sample computed from past the
 * frame's end -- are reported as MIP_COST_UNAVAILABLE (mip_unavailable_cus lists them).
 */
#ifndef MIPGPU_H
#define MIPGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIPGPU_ABI_VERSION 7
#define MIP_COSTS_PER_CTU_ABI 97840
#define MIP_CUS_PER_CTU_ABI 5380
#define MIP_COST_UNAVAILABLE 0x7fffffff

/* Reference filter whitelist order, constants.h:25-34. */
typedef enum {
  MIP_FILTER_NONE = -1,               /* USE_ALTERNATIVE_SAMPLES=0: references = originals */
  MIP_FILTER_1D_INT = 0,              /* filterFrame_1d_int            intra.cl:3267 */
  MIP_FILTER_1D_FLOAT = 1,            /* filterFrame_1d_float          intra.cl:1828 */
  MIP_FILTER_2D_INT = 2,              /* filterFrame_2d_int_quarterCtu intra.cl:2856 */
  MIP_FILTER_2D_FLOAT = 3,            /* filterFrame_2d_float_quarterCtu intra.cl:1639 */
  MIP_FILTER_1D_INT_5x5 = 4,          /* filterFrame_1d_int_5x5        intra.cl:3508 */
  MIP_FILTER_1D_FLOAT_5x5 = 5,        /* filterFrame_1d_float_5x5      intra.cl:2539 */
  MIP_FILTER_2D_INT_5x5 = 6,          /* filterFrame_2d_int_5x5_quarterCtu intra.cl:3042 */
  MIP_FILTER_2D_FLOAT_5x5 = 7         /* filterFrame_2d_float_5x5_quarterCtu intra.cl:2311 */
} mip_filter_type;

typedef struct {
  int filter;          /* mip_filter_type; MIP_FILTER_NONE for original references */
  int kernel_idx;      /* --KernelIdx: tap set index (0..4 for 3x3, 0..2 for 5x5) */
  int max_batch;       /* frames per device batch (device buffers sized for this); >= 1 */
  int want_sad_satd;   /* also produce the SAD / SATD tables (MAX_PERFORMANCE_DIST=0) */
  int slices_per_ctu;  /* workgroups per 64x64 CTU quadrant in the search kernel; 0 = auto
                          (chosen per launch: more, smaller workgroups for small batches) */
  int best_k;          /* decision list length K of best_mode_out / best_cost_out (1..32;
                          0 = 1): the K lowest-cost modes of every CU, see mip_topk_device */
} mip_opts;

typedef struct mip_engine mip_engine;

/* Defaults: no filter, kernel_idx 0, max_batch 1, no SAD/SATD, auto slicing. */
void mip_opts_default(mip_opts *opts);

/* Create an engine on HIP device `device` for width x height frames (width, height
 * multiples of 4).  Replaces main.cpp:90-598 (device/context/queue/buffer/program set-up).
 * Returns 0 and *out, or <0. */
int mip_engine_create(int device, int width, int height, const mip_opts *opts, mip_engine **out);
int mip_engine_destroy(mip_engine *e);

/* Geometry helpers. */
int mip_num_ctus(int width, int height);                     /* intra.cl:31-33 */
int64_t mip_costs_per_frame(int width, int height);          /* nCTUs * 97840 */
int64_t mip_cus_per_frame(int width, int height);            /* nCTUs * 5380 */
const char *mip_shape_name(int shape);                       /* main_aux_functions.h:296-401 */
/* Geometry of CU shape `shape` (0..46): w, h, modes (without transposition), CU count per
 * CTU, cost offset inside the CTU block.  Returns 0 or <0 for a bad index. */
int mip_shape_info(int shape, int *w, int *h, int *modes, int *ncu, int *cost_offset);
/* CTU-relative position of CU `cu` of `shape` (ALL_X_POS / ALL_Y_POS, constants.h:1235-1354). */
int mip_cu_position(int shape, int cu, int *x, int *y);

/* CUs whose costs this engine reports as MIP_COST_UNAVAILABLE for width x height frames,
 * with references from the engine's own filter `filter` (MIP_FILTER_NONE: original
 * references): 1 per CU in the order ctu*5380 + shape CU prefix + cu, for nCTUs*5380 CUs.
 * They are the CUs the reference leaves undefined geometrically (below the frame, stale LDS
 * intra.cl:96-98; reading past the frame's end) and, with a filter, the CUs that read a
 * filtered sample the reference's filter computes from memory past the frame's end (its
 * linear tile addressing, intra.cl:2904-2909 / 3330-3332; e.g. the last frame row of the
 * separable 3-tap filters when the height is not a multiple of 32).  Filtered samples that
 * two of the reference's tiles store with different values (widths that are not multiples
 * of 128, intra.cl:3037) are not undefined here: the engine uses the owning tile's value,
 * one of the reference's two outcomes.  Host only; returns 0 or <0. */
int mip_unavailable_cus(int width, int height, int filter, uint8_t *cu_out);

/* Low-pass filter of `nframes` host frames (filterFrame_<type>, main.cpp:700-761).
 * out must hold nframes frames.  Synchronous. */
int mip_filter_frames(mip_engine *e, const uint16_t *frames, int nframes, int filter,
                      int kernel_idx, uint16_t *out);

/* Full MIP search of `nframes` host frames: H2D, [filter], search, D2H, in chunks through
 * the engine's three streams (uploads, search, downloads) and buffer slots -- 4 slots of
 * max_batch/4 frames (max_batch >= 16), else 3 slots of max_batch frames (the engine's
 * buffers hold 3 x max_batch frames then) -- so that one chunk's upload, the previous
 * chunk's search and the one before's download run at the same time, also across calls:
 * an engine searching one frame per call (max_batch 1, the reference's per-frame loop with
 * BUFFER_SLOTS 2, main.cpp:886-898, main_aux_functions.h:5, 617) overlaps frame k+1's
 * upload and frame k-1's download with frame k's search when the calls are queued with
 * mip_search_frames_async.  A call into an idle pipeline is cut into two chunks.
 * Replaces the per-frame loop main.cpp:678-1241 + readMemobjsIntoArray_Distortion.
 * refs_or_null: caller-provided reference-sample frames (alternative samples computed
 * elsewhere); NULL = originals, or the engine's filter when opts.filter != NONE.
 * costs_out: int32 [nframes][nCTUs*97840] (may be NULL if only best modes are wanted).
 * best_mode_out / best_cost_out: optional per-CU decision lists, [nframes][nCTUs*5380][K]
 * with K = opts.best_k (K = 1: the argmin; mip_topk_device gives the ordering rules;
 * 0xff / MIP_COST_UNAVAILABLE for unavailable CUs).
 * sad_out / satd_out: optional (need opts.want_sad_satd).  Synchronous.
 * Host buffers: page-locked memory (mip_host_alloc, hipHostRegister) is transferred by DMA
 * directly; pageable memory (malloc, the reference's return_minSadHad, main.cpp:656-668)
 * goes through the engine's page-locked bounce ring (one arena of 16 pieces of up to 64 MB,
 * parallel host copies), allocated at its first use. */
int mip_search_frames(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null,
                      int nframes, int32_t *costs_out, uint8_t *best_mode_out,
                      int32_t *best_cost_out, int32_t *sad_out, int32_t *satd_out);

/* mip_search_frames without the final wait: enqueues the call's chunks behind the calls
 * still in flight (the upload / search / download pipeline stays full from one call to the
 * next) and returns a ticket (> 0) in *ticket.  The host buffers must stay valid and
 * unmodified (inputs) / unread (outputs) until mip_wait(e, ticket) returns.  Calls complete
 * in order.  mip_filter_frames waits for every call in flight.
 * Merged launches (ABI 7): a call with page-locked buffers and fewer frames than one buffer
 * slot (opts.max_batch below 16, else max_batch / 4) that arrives while the pipeline is busy
 * joins the engine's open chunk -- calls with the same outputs and reference source share ONE
 * search launch (one-frame calls then run at the multi-frame launch rate).  The chunk is
 * launched when full, when an incompatible call arrives, when a later call finds the GPU idle,
 * at any mip_wait / mip_flush / synchronous call / device-API call of the engine.  Every call
 * keeps its own ticket, outputs and input-contract status.  A caller that queues a call and
 * then neither waits nor calls again should call mip_flush (launches the open chunk now). */
int mip_search_frames_async(mip_engine *e, const uint16_t *frames, const uint16_t *refs_or_null,
                            int nframes, int32_t *costs_out, uint8_t *best_mode_out,
                            int32_t *best_cost_out, int32_t *sad_out, int32_t *satd_out,
                            uint64_t *ticket);

/* Block until the call with this ticket (and every earlier one) has completed: its outputs
 * are in host memory.  Pageable output buffers are complete (copied out of the bounce ring by
 * its completion thread) when this returns -- an asynchronous call with pageable outputs
 * must be waited for.  Fails
 * if THIS call's search staged a sample above 1023 (input contract; every call has its own
 * status, so an earlier or later call's violation is reported by that call's own wait). */
int mip_wait(mip_engine *e, uint64_t ticket);

/* Launch the engine's open (merged) chunk now, if any (see mip_search_frames_async); no wait. */
int mip_flush(mip_engine *e);

/* Device block cache (ABI 7).  Freeing a large device allocation halves every later host <->
 * device copy of the process on the MI355X platform (profiles/r06_free_repro.txt), so
 * mip_engine_destroy parks its buffers of >= 16 MB in a process-wide cache that later engines
 * on the same device reuse (the smallest block that fits).  mip_device_cache reports the
 * parked bytes of `device` and the blocks reused so far; release = 1 frees the parked blocks
 * first (hipFree: the copies of the process may slow down afterwards). */
int mip_device_cache(int device, int release, uint64_t *idle_bytes, uint64_t *reused_blocks);

/* Device-resident variant (inputs already in HBM; all pointers are device pointers,
 * `stream` is a hipStream_t; NULL means the default (null) stream, as in HIP).
 * Asynchronous on `stream`.
 * d_refs NULL: originals, or the engine filter applied into engine scratch.
 * d_costs NULL = decisions only (no cost table is written): needs d_best_cost and
 * opts.best_k == 1, no SAD / SATD; the search kernel keeps every CU's argmin itself (packed
 * in d_best_cost, unpacked in place).  mip_search_frames takes this path whenever no table
 * (costs / SAD / SATD) is requested and best_k == 1.  The optional outputs may be NULL. */
int mip_search_device(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs,
                      int nframes, int32_t *d_costs, int32_t *d_sad, int32_t *d_satd,
                      uint8_t *d_best_mode, int32_t *d_best_cost, void *stream);

/* Input-contract check of the device-API searches issued on `stream` (a hipStream_t, NULL =
 * the null stream): synchronises the stream, returns <0 (mip_last_error names it) if a
 * search of this engine staged a sample above 1023 since the last check, else 0. */
int mip_check_input(mip_engine *e, void *stream);

/* mip_search_device restricted to the CTUs [ctu_begin, ctu_end) (raster order) of every
 * frame: writes exactly those CTUs' blocks of the full-size cost / SAD / SATD tables and
 * leaves the others untouched.  The frames are complete (CUs at the range's top and left
 * edge read their reference samples from the rows / columns outside the range, the filter
 * runs over whole frames), so ranges that tile the frame give the full table: one large
 * frame split into CTU-row bands over several GPUs.  No decision
 * lists (run mip_topk_device on the assembled table). */
int mip_search_device_range(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs,
                            int nframes, int ctu_begin, int ctu_end, int32_t *d_costs,
                            int32_t *d_sad, int32_t *d_satd, void *stream);

/* Per-CU decision lists (no reference counterpart; what an encoder's full-RD stage takes
 * from the cost table, e.g. VTM's numModesForFullRD MIP candidates): for every CU of
 * `nframes` device cost tables (reference layout), the k lowest-cost modes in increasing
 * cost order, ties to the lower mode index.  Modes are numbered as the log's Mode column
 * (0..2*modes-1, transposed modes >= modes).  Entries past the CU's 2*modes modes and all
 * entries of unavailable CUs are 0xff / MIP_COST_UNAVAILABLE.  k in 1..32.
 * d_modes: uint8 [nframes][nCTUs*5380][k]; d_costs_k: int32, same shape (either may be
 * NULL).  Asynchronous on `stream`. */
int mip_topk_device(const int32_t *d_costs, int width, int height, int nframes, int k,
                    uint8_t *d_modes, int32_t *d_costs_k, void *stream);

/* Streaming device-to-device copy of `bytes` (a multiple of 16, 16-byte aligned pointers),
 * asynchronous on `stream`: 16 bytes per lane, four loads in flight per lane -- the HBM copy
 * rate bench.py prices the filter kernel against (no reference counterpart). */
int mip_copy_device(const void *d_src, void *d_dst, size_t bytes, void *stream);

/* Device-resident filter (asynchronous on `stream`). */
int mip_filter_device(const uint16_t *d_in, uint16_t *d_out, int width, int height,
                      int nframes, int filter, int kernel_idx, void *stream);

/* Kernel-only timing of the search on resident buffers: runs `reps` launches of the
 * fused search for `nframes` device frames on the engine's own stream, returns the mean
 * device time per launch in milliseconds (HIP events on that stream), or <0. */
double mip_time_search_device(mip_engine *e, const uint16_t *d_frames, const uint16_t *d_refs,
                              int nframes, int32_t *d_costs, int reps);

/* Per-frame device times of the host pipeline, for the reference's stdout report
 * ("FilterSamples took %f ms" and the filter TIMING REPORT, main.cpp:749-775; the frame
 * write time, main.cpp:580-595).  mip_trace_times(e, 1): mip_search_frames[_async] brackets
 * every chunk's upload and filter launch with HIP timing events (a buffer slot is then reused
 * only after its times were read: tracing costs some overlap).  mip_pop_times returns the
 * per-frame times (the chunk's time / its frames, frame order) of the calls completed so
 * far: up to `max` frames into upload_ms / filter_ms (either may be NULL; filter 0 without
 * a filter), the count in *n. */
int mip_trace_times(mip_engine *e, int enable);
int mip_pop_times(mip_engine *e, double *upload_ms, double *filter_ms, int max, int *n);

/* Host-pipeline counters of the engine (diagnostics, tests): out[0] host-API calls, out[1]
 * search launches of the host pipeline (chunks), out[2] calls that went through merged
 * chunks, out[3] merged launches (n entries of out are written, n <= 4). */
int mip_host_stats(mip_engine *e, uint64_t *out, int n);

/* Page-locked host memory (hipHostMalloc): host buffers for mip_search_frames /
 * mip_filter_frames allocated here are transferred by DMA at full PCIe rate (pageable
 * buffers are staged through the runtime -- the cost table is 52.8 MB per 1080p frame).
 * Replaces the reference's malloc'd return_minSadHad etc. (main.cpp:656-668). */
int mip_host_alloc(size_t bytes, void **out);
int mip_host_free(void *p);

/* NUMA placement (ABI 7).  Each GPU hangs off one socket of a multi-socket host; an engine
 * keeps its page-locked buffers on that GPU's NUMA node and runs its host threads (bounce-ring
 * copies, completion, merge flusher) on the node's CPUs.  mip_host_alloc_near allocates the
 * caller's page-locked buffers on `device`'s node (else as mip_host_alloc);
 * mip_bind_thread runs the calling thread on the node's CPUs (1 bound, 0 nothing to do: one
 * node or unknown); mip_numa_node gives the node (-1 unknown / one node);
 * mip_numa_node_of_pci the node of a PCI bus id ("0000:c1:00.0"), read from sysfs
 * (MIPGPU_SYSFS_ROOT overrides /sys). */
int mip_host_alloc_near(int device, size_t bytes, void **out);
int mip_bind_thread(int device);
int mip_numa_node(int device);
int mip_numa_node_of_pci(const char *pci_bus_id);

/* Last error message of the calling thread ("" if none). */
const char *mip_last_error(void);
int mip_abi_version(void);
/* Build ID of this library: "src:<hash of the sources and compiler flags> git:<commit>"
 * (+ "knobs:<-D options>" for A/B variants).  bench.py prints it and ties profiles/ to it. */
const char *mip_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
