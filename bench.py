#!/usr/bin/env python3
"""bench.py -- 1080p frames/s of the full MIP mode search over all 47 CU shapes.

One *step* = one pass of the fused HIP search over a batch of B (default 384) synthetic
1920x1080 frames resident in HBM (original references, BASELINE.json configs[1]), writing the complete
int32 cost table (97840 entries per CTU, the reference's minSadHad table).  Frames shard
across GPUs (one process per GPU, no data-path collective; RCCL only carries the barrier
and the max-over-ranks of the timing) -> weak scaling.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames-per-step B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Without a launcher (WORLD_SIZE unset), `--gpus N` > 1 starts the N ranks itself (one child
process per GPU, before anything touches the GPU) and exits with their status; under a
launcher, `--gpus` must equal WORLD_SIZE.

Rank 0 prints one JSON line (contract in the task statement), plus:
  roofline      HBM roofline of the search kernel (algorithmic bytes = frame read + int32
                cost write, per launch) with the launch time from HIP events on the stream
                the kernel runs on, and the PMC-measured traffic when profiles/ holds it;
  valu          the bound that actually applies to this path: VALU instruction issue.
                Wave64 VALU instructions per launch (PMC SQ_INSTS_VALU, profiles/traffic.json)
                over the live launch time against the single-issue rate (1024 SIMDs x one
                wave64 instruction per quad-cycle at 2.4 GHz), the PMC issue rate per SIMD
                quad-cycle and its dual-issued share (SQ_ACTIVE_INST_VALU2).  gfx950 issues a
                second VALU instruction in the same quad-cycle only for simple VOP1/VOP2 forms
                from another wave; measured ceilings (profiles/r02_dual_census.txt, 4 waves per
                SIMD): 1.37 per quad-cycle for an all-eligible stream, 0.86 for a stream of none;
                the SURVEY 8d algorithmic op count is reported alongside;
  filter        the alternative-reference low-pass filter of BASELINE configs[2]
                (filterFrame_2d_float_5x5_quarterCtu, KernelIdx 2) on the same frames:
                HBM roofline (one frame read + one write per frame) and the alt-refs
                search rate (filter + search per step);
  cpu_baseline  the C oracle (oracle/mip_oracle.c, OpenMP) on the host cores, one full frame;
  reference_gpu the reference's own OpenCL kernels (oracle/_ref, compiled from intra.cl)
                timed on the same MI355X, when their code objects are present;
  end_to_end    host-buffer API rate including PCIe transfers (never `value`).
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "1080p frames/sec, full MIP mode search over all CU sizes; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md, HBM3E peak (spec)
MFMA_F16_PEAK_TFLOPS = 2500.0    # MI355X_MICROARCH.md, dense f16/bf16 matrix peak
# VALU issue: 256 CUs x 4 SIMDs, one wave64 instruction per quad-cycle (4 clocks) each, 2.4 GHz
# (MI355X_MICROARCH.md) = 614.4 G wave-instructions/s.  Dual issue (two eligible instructions
# in one quad-cycle) raises it for simple VOP1/VOP2 forms only: measured ceilings per SIMD
# quad-cycle at 4 waves/SIMD (tools/dual_census.sh, profiles/r02_dual_census.txt).
VALU_PEAK_INSTS = 256 * 4 * 2.4e9 / 4
DUAL_CEILINGS = {"all_dual_eligible": 1.37, "none_dual_eligible": 0.86, "unit": "VALU instructions per SIMD quad-cycle",
                 "source": "profiles/r02_dual_census.txt (4 waves/SIMD)"}
# SURVEY.md section 8d algorithmic op model per CTU: GEMV 40.4 M MAC (on MFMA here) and
# 99.6 M vector ops (upsampling 13.8 + 19.9 M, SAD 19.3 M, SATD 46.6 M) -- the VALU share.
VECTOR_OPS_PER_CTU = 99.6e6
E2E_CALLS = 8  # host-buffer calls queued per end-to-end measurement round
E2E_ROUNDS = 3  # timed rounds per end-to-end leg (median reported)
E2E_FRAMES_MULTI = 32  # frames per host-buffer call at N > 1 (bounds each rank's page-locked memory)


def metric_name(width, height):
    """BASELINE.json's metric for the 1080p workload; the same metric named for the frame size
    otherwise (the config sweep's 4K / 8K lines are not 1080p frames)."""
    if (width, height) == (1920, 1080):
        return METRIC
    return "%dx%d frames/sec, full MIP mode search over all CU sizes; 1/2/4/8 GPU" % (width, height)


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus n` without a launcher: start n ranks of this script (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1), wait for them and
    return the worst exit status.  Nothing in this process touches the GPU.  A rank that
    fails ends the others (they would wait at the barrier)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0:
                rc = rc or code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


def gather_ranks(values, world, device=None):
    """All ranks' `values` (list of floats) -> [world][len(values)] (nccl or gloo)."""
    if world <= 1:
        return [list(values)]
    import torch
    import torch.distributed as dist
    t = torch.tensor(values, dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [[float(v) for v in o.cpu()] for o in out]


def dist_max(value, world, device=None):
    """Max over ranks (works for nccl with a device tensor and for gloo on CPU)."""
    if world <= 1:
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def choose_backend(world, local_rank, ndev):
    """(backend, device index) of a rank.  One rank per GPU: rank LOCAL_RANK on device
    LOCAL_RANK, barriers and timing reductions over nccl (RCCL).  More ranks than GPUs (a
    rehearsal of the N-GPU path on a smaller box) put rank r on device r % count and carry
    them over gloo (RCCL needs a device per rank).  Frames stay sharded per rank either way."""
    return ("nccl" if world <= ndev else "gloo"), local_rank % max(1, ndev)


def init_ranks(world, local_rank, ndev):
    """Process group of a multi-rank run (no-op for one rank); returns (backend, device index,
    device of the collectives' tensors: None for gloo)."""
    import torch
    backend, dev_index = choose_backend(world, local_rank, ndev)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
    return backend, dev_index, (None if backend == "gloo" else torch.device("cuda", dev_index))


def shard_seed(base_seed, rank):
    """Each rank processes its own frames (frame sharding, no overlap)."""
    return base_seed + 1000003 * rank


def aggregate(frames_per_step, steps, world, max_elapsed_s):
    total = frames_per_step * steps * world
    return total / max_elapsed_s, 1000.0 * max_elapsed_s / steps


def algorithmic_bytes_per_frame(w, h):
    from mipgpu.layout import COSTS_PER_CTU, num_ctus
    return w * h * 2 + num_ctus(w, h) * COSTS_PER_CTU * 4


def load_pmc(width, height, frames, build):
    """PMC summary (tools/profile_round.sh -> tools/traffic_json.py) for this workload, or {}.
    Only a profile of THIS build counts: the entry's build ID must name the same sources and
    flags as the loaded library (mip_build_id), else the PMC fields are left null."""
    from mipgpu import source_id
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        rec = json.load(open(path)).get("%dx%dx%d" % (width, height, frames), {})
    except Exception:
        return {}, "no profiles/traffic.json entry for this workload"
    if not rec:
        return {}, "no profiles/traffic.json entry for this workload"
    if source_id(rec.get("build_id", "")) != source_id(build):
        return {}, "profiles/traffic.json was collected on build %r, not this one" % rec.get("build_id")
    return rec, "profiles/traffic.json, same build"


# Environment knobs of libmipgpu.so that change the work or the launch shape (profiling / A/B
# tools).  A headline number is refused while any of them is set; --allow-knobs (the A/B
# scripts) records them in the line instead.  Print-only diagnostics are harmless.
HARMLESS_KNOBS = {"MIPGPU_STAGE_STATS", "MIPGPU_WORK_STATS", "MIPGPU_STAGE_TRACE", "MIPGPU_NO_TORCH", "MIPGPU_SLOW_CALLS"}


def active_knobs():
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("MIPGPU_") and k not in HARMLESS_KNOBS}


def valu_section(pmc, kernel_ms, alg_ops):
    insts = pmc.get("valu_insts_per_launch")
    out = {"bound": "valu-issue", "unit": "G wave64 VALU instructions/s", "peak": round(VALU_PEAK_INSTS / 1e9, 1),
           "achieved": None, "frac": None, "valu_insts_per_launch": insts,
           "issue_utilization": pmc.get("valu_issue_utilization"),
           "issue_per_simd_quad_cycle": pmc.get("valu_insts_per_simd_quad_cycle"),
           "dual_issue_share": pmc.get("valu_dual_issue_share"),
           "issue_ceilings": DUAL_CEILINGS,
           "algorithmic_vector_ops_per_s": round(alg_ops / (kernel_ms * 1e-3) / 1e12, 2),
           "algorithmic_unit": "T int ops/s (SURVEY 8d model, 99.6 M vector ops per CTU)"}
    if insts:
        rate = insts / (kernel_ms * 1e-3)
        out["achieved"], out["frac"] = round(rate / 1e9, 1), round(rate / VALU_PEAK_INSTS, 4)
        # against the two-per-quad-cycle ceiling (dual issue: both eligible, from two waves)
        out["dual_peak"] = round(2 * VALU_PEAK_INSTS / 1e9, 1)
        out["frac_of_dual_peak"] = round(rate / (2 * VALU_PEAK_INSTS), 4)
    flops = pmc.get("mfma_f16_flops_per_launch")
    if flops:
        # phase A (the MIP matrix products) on the matrix cores: f16 MFMA rate vs the dense peak
        tf = flops / (kernel_ms * 1e-3) / 1e12
        out["mfma"] = {"unit": "TFLOP/s", "achieved": round(tf, 2), "peak": MFMA_F16_PEAK_TFLOPS,
                       "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 5),
                       "insts_per_launch": pmc.get("mfma_insts_per_launch"),
                       "busy_utilization": pmc.get("mfma_busy_utilization"),
                       "note": "block-diagonal K: half of each 16x16x16 product multiplies zeros"}
    return out


def filter_section(eng_cls, frames, W, H, B, stream, dev, steps, pmc):
    """BASELINE configs[2] filter (2-D float 5x5, KernelIdx 2) on the resident frames: HBM
    roofline of the filter kernel and the alternative-reference search rate."""
    import torch
    from mipgpu import filter_device
    name, kidx = "filterFrame_2d_float_5x5_quarterCtu", 2
    out = torch.empty_like(frames)
    for _ in range(3):
        filter_device(frames, out, name, kidx, stream=stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        filter_device(frames, out, name, kidx, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    # calibration: a streaming copy of the same bytes on the same stream (mip_copy_device:
    # 16 bytes per lane, four loads in flight -- the guide's achievable-copy form; 384 frames
    # are far past the last-level cache); torch's copy_ beside it (round 5's calibration)
    from mipgpu import copy_device
    copy_device(frames, out, stream=stream)
    e0.record(stream)
    for _ in range(steps):
        copy_device(frames, out, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    copy_ms = e0.elapsed_time(e1) / steps
    with torch.cuda.stream(stream):
        out.copy_(frames)
        e0.record(stream)
        for _ in range(steps):
            out.copy_(frames)
        e1.record(stream)
    torch.cuda.synchronize(dev)
    torch_copy_ms = e0.elapsed_time(e1) / steps
    alg = 2 * 2 * W * H * B
    res = {"kernel": "filter_kernel<2, true, false>", "filter": name, "kernel_idx": kidx, "bound": "hbm",
           "kernel_ms_per_launch": round(ms, 4), "algorithmic_bytes_per_launch": alg,
           "achieved": round(alg / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "copy_GBps": round(alg / (copy_ms * 1e-3) / 1e9, 1), "frac_of_copy": round(copy_ms / ms, 4),
           "copy_kernel": "mip_copy_device (16 B per lane, 4 loads in flight)",
           "torch_copy_GBps": round(alg / (torch_copy_ms * 1e-3) / 1e9, 1),
           "traffic": (pmc.get("filter") or {}).get("hbm_bytes_per_launch")}
    alt = eng_cls(W, H, device=dev.index, filter=name, kernel_idx=kidx, max_batch=B)
    costs = torch.empty((B, alt.costs_per_frame), dtype=torch.int32, device=dev)
    for _ in range(2):
        alt.search_device(frames, costs=costs, stream=stream)
    e0.record(stream)
    for _ in range(steps):
        alt.search_device(frames, costs=costs, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    res["alt_refs_search"] = {"value": round(B * steps / (e0.elapsed_time(e1) * 1e-3), 1), "unit": "frames/s",
                              "note": "filter + search per step, device time (BASELINE configs[2] path)"}
    alt.close()
    return res


def cpu_baseline(width, height, seed, budget_s=10.0):
    """The C oracle on the host cores for ~budget_s seconds (whole frames, at least one)."""
    import numpy as np
    import oracle_lib
    from mipgpu.synth import synth_frame
    threads = min(16, os.cpu_count() or 1)
    frames = [synth_frame(width, height, seed + i, 0) for i in range(4)]
    oracle_lib.lib()
    n, t0 = 0, time.perf_counter()
    while n == 0 or time.perf_counter() - t0 < budget_s:
        oracle_lib.search(frames[n % len(frames)], nthreads=threads)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 4), "unit": "1080p frames/s" if (width, height) == (1920, 1080) else
            "%dx%d frames/s" % (width, height), "cores": threads, "kind": "port",
            "configs0": "BASELINE configs[0] names the reference's OpenCL kernels on the host CPU's OpenCL device; "
                        "this image has no CPU OpenCL device (SURVEY.md 8c: the AMD ICD lists 0 CPU devices, no "
                        "PoCL), so this figure is the C port of the reference pipeline (oracle/mip_oracle.c); the "
                        "reference's own kernels compiled for the CPU are `reference_kernels`",
            "sample": "%d synthetic %dx%d frames (all CTUs, full search, same generator as the GPU run) through "
                      "the C oracle oracle/mip_oracle.c, OpenMP %d threads, %.1f s" % (n, width, height, threads, dt)}


def reference_kernels_cpu(width, height, seed):
    """BASELINE configs[0] / SURVEY 8d C1: the reference's own kernels (/root/reference's
    intra.cl compiled by clang for the host CPU with oracle/ref/cl_cpu_shim.cl's builtins --
    oracle/_ref/ref_cpu_runner, built in the container) on one 1080p frame, original
    references, every work-group, on the host cores; None when the runner was not built."""
    runner = os.path.join(REPO, "oracle", "_ref", "ref_cpu_runner")
    if not os.path.exists(runner):
        return None
    workers = min(16, os.cpu_count() or 1)
    try:
        out = subprocess.run([runner, "--libs", os.path.join(REPO, "oracle", "_ref"), "--width", str(width),
                              "--height", str(height), "--synth", "0:%x" % seed, "--workers", str(workers)],
                             capture_output=True, timeout=300, check=True).stdout.decode()
        d = json.loads(out.strip().splitlines()[-1])
    except Exception as exc:  # informative only
        return {"error": str(exc)[:200]}
    return {"value": round(d["frames_per_s"], 5),
            "unit": "1080p frames/s" if (width, height) == (1920, 1080) else "%dx%d frames/s" % (width, height),
            "cores": workers, "kind": "reference",
            "kernel_s_per_frame": d["kernel_s"], "wall_s_per_frame": round(d["wall_s_per_frame"], 3),
            "sample": "one synthetic %dx%d frame, original references (BASELINE configs[0]), every work-group of "
                      "initBoundaries, MIP_ReducedPred and the three upsampleDistortion builds" % (width, height),
            "note": "the reference's own intra.cl kernels compiled by clang for x86-64 (oracle/Makefile ref-cpu) with "
                    "the OpenCL builtins of oracle/ref/cl_cpu_shim.cl, work-groups over %d worker processes, "
                    "work-items as fibers (oracle/ref/ref_cpu_runner.cpp); its tables hash like the golden fixtures "
                    "the same kernels made on the MI355X (tests/test_ref_cpu.py).  A baseline, not a target" % workers}


def reference_kernel_trace(cmd, frames, reps):
    """Device time per frame of the reference's kernels from a rocprofv3 kernel trace of
    ref_runner (its CL profiling timestamps are unusable on this runtime: END precedes
    START), or None when rocprofv3 is not available."""
    import csv
    import shutil
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    d = tempfile.mkdtemp(prefix="refprof_")
    try:
        subprocess.run([prof, "--kernel-trace", "--stats", "-d", d, "-o", "ref", "--output-format", "csv", "--"] + cmd,
                       capture_output=True, timeout=240, check=True, env=dict(os.environ, TMPDIR="/tmp"))
        stats = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith("kernel_stats.csv")]
        per = {}
        for row in csv.DictReader(open(stats[0])):
            if row["Name"] in ("initBoundaries", "MIP_ReducedPred", "upsampleDistortion") or row["Name"].startswith("filterFrame"):
                per[row["Name"]] = float(row["TotalDurationNs"]) * 1e-6 / (frames * reps)
        return per if per else None
    except Exception:
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def reference_gpu(width, height, frames, seed):
    runner = os.path.join(REPO, "oracle", "_ref", "ref_runner")
    if not os.path.exists(runner):
        return None
    try:
        cmd = [runner, "--bins", os.path.join(REPO, "oracle", "_ref"), "--width", str(width),
               "--height", str(height), "--frames", str(frames), "--synth", "0:%x" % seed, "--reps", "2"]
        out = subprocess.run(cmd, capture_output=True, timeout=180, check=True).stdout.decode()
        d = json.loads(out.strip().splitlines()[-1])
        trace = reference_kernel_trace(cmd, frames, 2)
        if trace:
            ms = sum(trace.values())
            return {"value": round(1000.0 / ms, 3), "unit": "frames/s (device time: rocprofv3 kernel trace of the reference's kernels)",
                    "kernel_ms_per_frame": {k: round(v, 4) for k, v in trace.items()},
                    "host_timed_value": round(1000.0 / d["device_ms_per_frame"], 3),
                    "wall_value": round(1000.0 / d["wall_ms_per_frame"], 2),
                    "event_fallbacks": int(d.get("event_fallbacks", 0)),
                    "event_fallback_reason": d.get("event_fallback_reason") or None, "device": d["device"],
                    "note": "reference intra.cl kernels (initBoundaries, MIP_ReducedPred, 3x upsampleDistortion) "
                            "compiled by the AMD OpenCL compiler, same GPU, same synthetic frames; host_timed_value: "
                            "enqueue + clFinish around each kernel (CL profiling events unusable)"}
        if not d["device_ms_per_frame"] > 0:
            return {"error": "no device timing", "raw": d}
        # device time from the CL profiling timestamps of every kernel; a kernel whose
        # timestamps are unusable is timed by the host around enqueue + clFinish instead, and
        # then the figure is labelled as such
        fb = int(d.get("event_fallbacks", 0))
        unit = "frames/s (device time, CL profiling events)" if fb == 0 else \
            "frames/s (host wall time around each kernel: %d CL profiling events unusable)" % fb
        return {"value": round(1000.0 / d["device_ms_per_frame"], 3), "unit": unit, "event_fallbacks": fb,
                "event_fallback_reason": d.get("event_fallback_reason") or None,
                "wall_value": round(1000.0 / d["wall_ms_per_frame"], 2),
                "kernel_ms_per_frame": d["kernel_ms"], "device": d["device"],
                "note": "reference intra.cl kernels (initBoundaries, MIP_ReducedPred, 3x upsampleDistortion) "
                        "compiled by the AMD OpenCL compiler, same GPU, same synthetic frames"}
    except Exception as exc:  # the comparison is informative only
        return {"error": str(exc)[:200]}


def ranks_section(per_rank, frames_per_step, steps, backend, devices=None):
    """Rank count actually running (dist.get_world_size()) and each rank's own rate (its own
    search launches' device time: the wall time between the barriers is the slowest rank's
    for every rank).  devices: GPUs visible to a rank (ranks share a GPU when world > devices)."""
    world = len(per_rank)
    if world > 1:
        import torch.distributed as dist
        world = dist.get_world_size()
    return {"world_size": world, "backend": backend, "devices": devices,
            "shared_devices": bool(devices) and world > devices,
            "per_rank_frames_per_s": [round(frames_per_step / (r[1] * 1e-3), 2) for r in per_rank],
            "per_rank_kernel_ms": [round(r[1], 4) for r in per_rank]}


def timed_rounds(run_round, world, coll_dev, frames_per_round, rounds=E2E_ROUNDS):
    """End-to-end leg over all ranks: one warm-up round, then `rounds` timed rounds, each
    aligned by a barrier (N > 1) and timed by its slowest rank (max over ranks).  Returns the
    median whole-job rate (all ranks' frames / the slowest rank's time), every round's rate,
    and this rank's own median rate (its frames / its own time)."""
    import statistics
    agg, own = [], []
    for r in range(1 + rounds):
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        t0 = time.perf_counter()
        run_round()
        dt = time.perf_counter() - t0
        slowest = dist_max(dt, world, coll_dev)
        if r:
            agg.append(world * frames_per_round / slowest)
            own.append(frames_per_round / dt)
    return round(statistics.median(agg), 2), [round(x, 1) for x in agg], round(statistics.median(own), 2)


def e2e_multi_section(legs, world, coll_dev, frames_per_call, note):
    """`end_to_end` at N > 1: each leg's whole-job rate (`aggregate`) and every rank's own rate
    (`ranks`), gathered on every rank (collective), for rank 0 to print."""
    res = {"unit": "frames/s", "world_size": world, "frames_per_call": frames_per_call, "calls_per_round": E2E_CALLS,
           "aggregate": {}, "rounds": {}, "ranks": {}, "note": note}
    for name, (value, rounds, own) in legs.items():
        res["aggregate"][name] = value
        res["rounds"][name] = rounds
        res["ranks"][name] = [round(r[0], 2) for r in gather_ranks([own], world, coll_dev)]
    return res


def plumbing_check(args):
    """--plumbing-check: the multi-rank path of main() on CPU (gloo), a sleep per step."""
    import torch.distributed as dist
    rank, _, world = dist_env()
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.01 * (1 + rank))  # rank r is the (r+1)-times slower one
    own = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_rank = gather_ranks([elapsed, 1e3 * own / args.steps], world)
    max_elapsed = max(r[0] for r in per_rank)
    value, ms_per_step = aggregate(args.frames_per_step, args.steps, world, max_elapsed)
    # the end-to-end legs' aggregation at N > 1 (a sleep per round; rank r the (r+1)-times slower)
    e2e = None
    if world > 1 and not args.no_end_to_end:
        legs = {"value": timed_rounds(lambda: time.sleep(0.01 * (1 + rank)), world, None, E2E_CALLS * E2E_FRAMES_MULTI),
                "decisions_value": timed_rounds(lambda: time.sleep(0.005 * (1 + rank)), world, None,
                                                E2E_CALLS * E2E_FRAMES_MULTI)}
        e2e = e2e_multi_section(legs, world, None, E2E_FRAMES_MULTI, "plumbing check (sleep per round)")
    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 4), "unit": "frames/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
                "data": "plumbing check (no GPU, sleep per step)",
                "ranks": ranks_section(per_rank, args.frames_per_step, args.steps, "gloo" if world > 1 else None)}
        if e2e:
            line["end_to_end"] = e2e
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames-per-step", type=int, default=384)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x1080)
    ap.add_argument("--slices", type=int, default=0, help="workgroups per CTU (0 = engine default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-reference-gpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip the single-frame latency launches")
    ap.add_argument("--no-filter", action="store_true", help="skip the filter / alternative-refs measurement")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="skip the host-buffer measurement (its launches are half batches; keep them out of profiles)")
    ap.add_argument("--refs-filter", default=None,
                    help="alternative references: run this reference filter (e.g. filterFrame_2d_int_quarterCtu) "
                         "inside every step (BASELINE configs[2]/[4]); default: original references")
    ap.add_argument("--kernel-idx", type=int, default=0, help="KernelIdx of --refs-filter")
    ap.add_argument("--allow-knobs", action="store_true",
                    help="A/B tooling only: run although MIPGPU_* work knobs are set (they are recorded in the "
                         "line, which is then marked as no headline)")
    ap.add_argument("--plumbing-check", action="store_true",
                    help="CPU only (gloo): run the rank launch, timing reduction and JSON line with a "
                         "sleep in place of the search (tests/test_bench_dist.py)")
    args = ap.parse_args()

    knobs = active_knobs()
    if knobs and not args.allow_knobs:
        print("bench.py: refusing to measure with libmipgpu work knobs set (%s): they change the work or the "
              "launch shape; unset them (A/B tools pass --allow-knobs)" % ", ".join(knobs), file=sys.stderr)
        sys.exit(3)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks" % (args.gpus, os.environ["WORLD_SIZE"]),
              file=sys.stderr)
        sys.exit(2)
    if args.plumbing_check:
        return plumbing_check(args)

    import numpy as np
    import torch

    from mipgpu import MipEngine
    from mipgpu.layout import num_ctus
    from mipgpu.synth import synth_frames_torch

    rank, local_rank, world = dist_env()
    ndev = torch.cuda.device_count()
    backend, dev_index, coll_dev = init_ranks(world, local_rank, ndev)
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    # the rank's host side on its GPU's NUMA node (mip_bind_thread; no-op on a one-node host):
    # its page-locked buffers (pinned_empty(device=...)) and the engine's threads are placed too
    from mipgpu import bind_thread, numa_node
    numa = {"node": numa_node(dev_index), "thread_bound": bind_thread(dev_index)}
    W, H, B = args.width, args.height, args.frames_per_step

    # synthetic frames generated on the GPU (bit-identical to mipgpu.synth.synth_frames)
    frames = synth_frames_torch(W, H, B, shard_seed(args.seed, rank), 0, device=dev)
    eng = MipEngine(W, H, device=dev_index, max_batch=B, slices_per_ctu=args.slices, filter=args.refs_filter,
                    kernel_idx=args.kernel_idx)
    costs = torch.empty((B, eng.costs_per_frame), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)  # the search kernels and the timing events share it

    for _ in range(args.warmup):
        eng.search_device(frames, costs=costs, stream=stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        eng.search_device(frames, costs=costs, stream=stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one search launch per step, same stream

    per_rank = gather_ranks([elapsed, kernel_ms], world, coll_dev)
    max_elapsed = max(r[0] for r in per_rank)
    max_kernel_ms = max(r[1] for r in per_rank)
    value, ms_per_step = aggregate(B, args.steps, world, max_elapsed)

    e2e_multi = None
    if world > 1 and not args.no_end_to_end:
        # Host-fed rate of the whole job (informative, never `value`): every rank feeds its own
        # GPU from page-locked host buffers on that GPU's NUMA node -- E2E_CALLS asynchronous
        # calls of E2E_FRAMES_MULTI frames per round, rounds aligned by a barrier and timed by
        # the slowest rank.  Full int32 cost tables (52.8 MB per 1080p frame over PCIe) and
        # decisions only.
        from mipgpu import pinned_empty
        Bm = min(B, E2E_FRAMES_MULTI)
        hp = pinned_empty((Bm, H, W), np.uint16, device=dev_index)
        hp[:] = frames[:Bm].cpu().numpy().view(np.uint16)
        cost_out = {"cost": pinned_empty((Bm, eng.costs_per_frame), np.int32, device=dev_index)}
        dec_out = {"best_mode": pinned_empty((Bm, eng.cus_per_frame), np.uint8, device=dev_index),
                   "best_cost": pinned_empty((Bm, eng.cus_per_frame), np.int32, device=dev_index)}

        def leg(**kw):
            return timed_rounds(lambda: eng.wait([eng.search_async(hp, **kw) for _ in range(E2E_CALLS)][-1]),
                                world, coll_dev, E2E_CALLS * Bm)
        legs = {"value": leg(out=cost_out), "decisions_value": leg(costs=False, best=True, out=dec_out)}
        e2e_multi = e2e_multi_section(
            legs, world, coll_dev, Bm,
            "host frames in (page-locked, on the rank's GPU's NUMA node), per rank %d asynchronous calls of %d "
            "frames per round, rounds aligned by a barrier; aggregate = all ranks' frames / the slowest rank's "
            "time (median of %d rounds after a warm-up round); value: int32 cost tables out (%.1f MB per frame), "
            "decisions_value: per-CU best mode + cost out" % (E2E_CALLS, Bm, E2E_ROUNDS,
                                                              algorithmic_bytes_per_frame(W, H) / 1e6))
        del hp, cost_out, dec_out

    cfg = {(1920, 1080, None): 1, (1920, 1080, "filterFrame_2d_float_5x5_quarterCtu"): 2, (3840, 2160, None): 3,
           (7680, 4320, "filterFrame_2d_int_quarterCtu"): 4}.get((W, H, args.refs_filter))
    refs_desc = ("original references" if args.refs_filter is None else
                 "alternative references %s KernelIdx %d filtered inside the step" % (args.refs_filter, args.kernel_idx))
    if cfg is not None:
        refs_desc += " (BASELINE configs[%d])" % cfg
    if rank == 0:
        alg_bytes = algorithmic_bytes_per_frame(W, H) * B
        achieved = alg_bytes / (max_kernel_ms * 1e-3) / 1e9
        ops = VECTOR_OPS_PER_CTU * num_ctus(W, H) * B
        from mipgpu import build_id
        build = build_id()
        pmc, pmc_src = load_pmc(W, H, B, build)
        res = {
            "metric": metric_name(W, H), "value": round(value, 2), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16x2/int32",
            "data": "synthetic (seeded integer generator, mipgpu/synth.py, generated on the GPU)",
            "config": {"workload": "%dx%d frames, %s; %d frames per step per GPU resident in HBM; full int32 "
                                   "cost table written" % (W, H, refs_desc, B),
                       "width": W, "height": H, "frames_per_step": B, "parallelism": "frames sharded over %d GPU(s)" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": pmc.get("hbm_bytes_per_launch"),
                         "kernel": "mip_search_kernel" if args.refs_filter is None else "filter_kernel + mip_search_kernel",
                         "kernel_ms_per_launch": round(max_kernel_ms, 4),
                         "algorithmic_bytes_per_launch": alg_bytes},
            # The bound that applies: VALU issue (see the module docstring).
            "valu": valu_section(pmc, max_kernel_ms, ops),
            "ranks": ranks_section(per_rank, B, args.steps, backend if world > 1 else None,
                                   devices=ndev),
            "build_id": build, "pmc_source": pmc_src, "numa": numa,
        }
        if e2e_multi is not None:
            res["end_to_end"] = e2e_multi
        if world > max(1, ndev):  # a rehearsal: ranks time-share GPUs
            note = ("%d ranks share %d GPU(s): each kernel time is a time-shared one, so the roofline / VALU fields "
                    "are not meaningful here (the rank bookkeeping and aggregation are what this line checks)"
                    % (world, ndev))
            for key in ("roofline", "valu"):
                res[key]["meaningful"] = False
                res[key]["note"] = note
        if knobs:
            res["knobs"] = knobs
            res["headline"] = False  # measured with work knobs set (A/B tooling)
        if world == 1 and not args.no_filter:
            res["filter"] = filter_section(MipEngine, frames, W, H, B, stream, dev, 5, pmc)
        if world == 1 and not args.no_latency:
            # Latency of a single-frame launch (informative; `value` is batch throughput).
            f1 = torch.empty((1, eng.costs_per_frame), dtype=torch.int32, device=dev)
            for _ in range(3):
                eng.search_device(frames[:1], costs=f1, stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                eng.search_device(frames[:1], costs=f1, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            res["single_frame_ms"] = round(e0.elapsed_time(e1) / 20, 4)
        if world == 1 and not args.no_latency:
            # Decisions only (the serving path): the same B resident frames, no cost table --
            # the per-CU argmin is fused into the search (mip_search_device with d_costs NULL).
            bm = torch.empty((B, eng.cus_per_frame), dtype=torch.uint8, device=dev)
            bc = torch.empty((B, eng.cus_per_frame), dtype=torch.int32, device=dev)
            for _ in range(2):
                eng.search_device(frames, costs=False, best_mode=bm, best_cost=bc, stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(5):
                eng.search_device(frames, costs=False, best_mode=bm, best_cost=bc, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            res["decisions_device"] = {"value": round(5 * B / (e0.elapsed_time(e1) * 1e-3), 1), "unit": "frames/s",
                                       "note": "per-CU best mode + cost of the same resident frames, no cost table "
                                               "(argmin fused into the search kernel), device time"}
        if world == 1:
            if not args.no_cpu_baseline:
                res["cpu_baseline"] = cpu_baseline(W, H, args.seed)
                rk = reference_kernels_cpu(W, H, args.seed)
                if rk is not None:
                    res["cpu_baseline"]["reference_kernels"] = rk
        if world == 1 and not args.no_end_to_end:
            # Host-buffer path incl. PCIe (informative, never `value`): page-locked buffers
            # (mip_host_alloc; transfers overlap the next chunk's search) and pageable ones.
            # Each leg: one warm-up round, then E2E_ROUNDS timed rounds of E2E_CALLS
            # asynchronous calls queued back to back (mip_search_frames_async) and one wait for
            # the last; the median round is reported (the first round after an engine's or a
            # buffer's first use runs up to ~40 % slow: tools/e2e_probe.py fps_all).
            import statistics
            from mipgpu import pinned_empty
            Be = min(B, 128)  # frames per call (bounded host memory: 6.8 GB of int32 costs per call)
            host = frames[:Be].cpu().numpy().view(np.uint16)
            hp = pinned_empty(host.shape, np.uint16, device=dev_index)
            hp[:] = host

            def e2e_leg(fr, **kw):
                rates = []
                for r in range(1 + E2E_ROUNDS):
                    t0 = time.perf_counter()
                    eng.wait([eng.search_async(fr, **kw) for _ in range(E2E_CALLS)][-1])
                    if r:
                        rates.append(E2E_CALLS * Be / (time.perf_counter() - t0))
                return round(statistics.median(rates), 2), [round(x, 1) for x in rates]

            pinned_fps, pinned_all = e2e_leg(hp, out={"cost": pinned_empty((Be, eng.costs_per_frame), np.int32,
                                                                           device=dev_index)})
            # pageable (malloc'd) buffers, staged through the engine's page-locked bounce ring:
            # steady state with outputs the caller reuses (touched, like pinned ones above) and
            # a cold call into a fresh allocation (first-touch page faults of 6.8 GB included)
            qout = {"cost": np.empty((Be, eng.costs_per_frame), np.int32)}
            qout["cost"].fill(0)
            pageable_fps, pageable_all = e2e_leg(host, out=qout)
            del qout
            t0 = time.perf_counter()
            eng.search(host)
            pageable_cold_fps = Be / (time.perf_counter() - t0)
            # decisions only: frames in, per-CU best mode + cost out (no cost table: fused argmin)
            dout = {"best_mode": pinned_empty((Be, eng.cus_per_frame), np.uint8, device=dev_index),
                    "best_cost": pinned_empty((Be, eng.cus_per_frame), np.int32, device=dev_index)}
            decisions_fps, decisions_all = e2e_leg(hp, costs=False, best=True, out=dout)
            res["end_to_end"] = {"value": pinned_fps, "unit": "frames/s",
                                 "pageable_value": pageable_fps,
                                 "pageable_cold_value": round(pageable_cold_fps, 2),
                                 "decisions_value": decisions_fps,
                                 "rounds": {"value": pinned_all, "pageable_value": pageable_all,
                                            "decisions_value": decisions_all},
                                 "note": "host frames in, host int32 cost tables out (H2D + search + D2H, "
                                         "%.1f MB per frame over PCIe), %d asynchronous calls of %d frames queued back to back "
                                         "(the pipeline's fill and drain included), median of %d rounds after a warm-up round; "
                                         "value: page-locked buffers; pageable_value: malloc'd buffers "
                                         "(bounce ring), outputs reused; pageable_cold_value: one call into a "
                                         "fresh allocation; "
                                         "decisions_value: page-locked frames in, per-CU best mode + cost out "
                                         "(%.1f MB per frame)" %
                                         (algorithmic_bytes_per_frame(W, H) / 1e6, E2E_CALLS, Be, E2E_ROUNDS,
                                          (2 * W * H + 5 * eng.cus_per_frame) / 1e6)}
        if world == 1 and not args.no_reference_gpu:
            ref = reference_gpu(W, H, min(B, 4), args.seed)
            if ref is not None:
                res["reference_gpu"] = ref
                if ref.get("value"):
                    res["speedup_vs_reference_gpu"] = round(value / ref["value"], 2)
        print(json.dumps(res), flush=True)
    eng.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
