"""CLI surface: vvc-mip-gpu_amd/bin/mipgpu_cli against the reference's main.cpp contract.

* argument handling and exit codes of main.cpp:47-83 / main_aux_functions.h:113-162
  (CPU: these paths end before an engine is created);
* the cost log, byte for byte, against a restatement of exportAllDistortionValues_File
  (main_aux_functions.h:735-798) filled with the C oracle's costs (GPU)."""
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from mipgpu import layout
from mipgpu.synth import synth_frames

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "vvc-mip-gpu_amd", "bin", "mipgpu_cli")

needs_cli = pytest.mark.skipif(not os.path.exists(CLI), reason="CLI not built (make -C vvc-mip-gpu_amd)")


def run(args, timeout=300):
    return subprocess.run([CLI] + args, capture_output=True, text=True, timeout=timeout)


def reference_log(cost, width, sad=None, satd=None) -> bytes:
    """exportAllDistortionValues_File (main_aux_functions.h:735-798) for one frame: header,
    then per CTU the SizeId2, SizeId1 and SizeId0 shapes in table order, every CU, every
    mode (transposed ones included); X/Y from ALL_X_POS/ALL_Y_POS, 4x4 CUs from
    4*(cu%32), 4*(cu/32) (785-786); SAD, SATD, minSadHad printed with %ld."""
    nctus = cost.size // layout.COSTS_PER_CTU
    ctu_cols = -(-width // 128)
    out = ["CTU,cuSizeName,W,H,CU,X,Y,Mode,SAD,SATD,minSadHad\n"]
    for ctu in range(nctus):
        cx, cy = 128 * (ctu % ctu_cols), 128 * (ctu // ctu_cols)
        for s in layout.SHAPES:
            if s.size_id == 0:
                xs = 4 * (np.arange(s.ncu) % 32)
                ys = 4 * (np.arange(s.ncu) // 32)
            else:
                xs, ys = s.positions()
            for cu in range(s.ncu):
                head = f"{ctu},{s.name},{s.w},{s.h},{cu},{cx + xs[cu]},{cy + ys[cu]},"
                base = ctu * layout.COSTS_PER_CTU + s.cost_offset + cu * s.total_modes
                for m in range(s.total_modes):
                    i = base + m
                    a = 0 if sad is None else sad[i]
                    b = 0 if satd is None else satd[i]
                    out.append(f"{head}{m},{a},{b},{cost[i]}\n")
    return "".join(out).encode()


def write_csv(path, frames):
    with open(path, "w") as f:
        for fr in frames:
            for row in fr:
                f.write(",".join(map(str, row.tolist())) + "\n")


def mask_unavailable(cost, width, height):
    m = layout.available_mask(width, height)
    return np.where(m, cost, layout.UNAVAILABLE).astype(np.int32)


# ---------------------------------------------------------------- CPU: arguments
@needs_cli
def test_help_exits_1():
    r = run(["-h"])
    assert r.returncode == 1 and "--FramesToBeEncoded" in r.stdout


@needs_cli
def test_missing_parameters_are_reported():
    r = run(["-s", "64x64"])
    assert r.returncode == 1
    assert "[!] ERROR: FramesToBeEncoded not set." in r.stdout
    assert "[!] ERROR: Input original frames not set." in r.stdout
    assert "Exiting after finding errors in input parameters" in r.stdout


@needs_cli
def test_unsupported_filter_exits_0():
    r = run(["-f", "1", "-s", "64x64", "-o", "x.csv", "--FilterType=notAFilter"])
    assert r.returncode == 0 and "Filter type notAFilter not supported" in r.stdout


@needs_cli
def test_unknown_and_ambiguous_options():
    assert run(["--Bogus", "1"]).returncode == 1
    assert "ambiguous" in run(["--F", "1"]).stderr  # FramesToBeEncoded / FilterType


@needs_cli
def test_extension_arguments_are_validated():
    for bad in (["--TopK", "0"], ["--TopK", "33"], ["--InputFormat", "rgb"], ["--TopK", "x"]):
        r = run(["-f", "1", "-s", "128x128", "-o", "x.csv"] + bad)
        assert r.returncode == 1 and "is invalid" in r.stderr, bad
    r = run(["-h"])
    assert all(k in r.stdout for k in ("--TopK", "--BinaryLog", "--InputFormat"))


@needs_cli
@pytest.mark.parametrize("args,size", [([], "130x64"), (["--StrictResolution"], "640x480")])
def test_unsupported_resolution_message(tmp_path, args, size):
    """main.cpp:301-309: an unsupported size prints the reference's error and its resolution
    table, and exits 0 (sizes not multiples of 4; with --StrictResolution every size outside
    the reference's table)."""
    r = run(["-f", "1", "-s", size, "-o", str(tmp_path / "none.csv")] + args)
    assert r.returncode == 0
    assert f"[!] ERROR: Unsupported resolution {size}\nSupported resolutions are:\n" in r.stdout
    for res in ("3840x2160", "1920x1080", "1280x720", "832x480", "416x240"):
        assert f"  {res}\n" in r.stdout
    assert "Current frame" not in r.stdout


# ------------------------------------------------------------ GPU: the cost log
@pytest.mark.gpu
@needs_cli
def test_device_list_shards_frames(gpu_available, tmp_path):
    """--DeviceIndex 0,0: two engines (one per list entry, here both on GPU 0) each search a
    contiguous half of the frames; the log of frame 0 is unchanged and --AllFrames shows
    every frame's rows in order."""
    W, H, N = 128, 128, 3
    frames = synth_frames(W, H, N, 0xC12, 0)
    write_csv(tmp_path / "in.csv", frames)
    logs = {}
    for dev in ("0", "0,0"):
        prefix = str(tmp_path / ("out_" + dev.replace(",", "_")))
        r = run(["-f", str(N), "-s", f"{W}x{H}", "-o", str(tmp_path / "in.csv"), "-l", prefix,
                 "--DeviceIndex", dev, "--AllFrames"])
        assert r.returncode == 0, r.stdout + r.stderr
        assert f"Device Index={dev}" in r.stdout
        logs[dev] = open(prefix + ".csv", "rb").read()
    assert logs["0"] == logs["0,0"]
    want = b"".join(reference_log(O.search(frames[f]), W).split(b"\n", 1)[1] if f else reference_log(O.search(frames[f]), W)
                    for f in range(N))
    assert logs["0,0"] == want


@pytest.mark.gpu
@needs_cli
@pytest.mark.parametrize("extra,filt,kidx,sad_satd", [
    ([], None, 0, False),
    (["--FilterType", "filterFrame_2d_int_quarterCtu", "--KernelIdx", "1"], "filterFrame_2d_int_quarterCtu", 1, False),
    (["--Filter=filterFrame_1d_float_5x5", "--KernelIdx=2", "--ReportSadSatd"], "filterFrame_1d_float_5x5", 2, True),
])
def test_cost_log_is_byte_identical(gpu_available, tmp_path, extra, filt, kidx, sad_satd):
    W, H, N = 256, 136, 2
    frames = synth_frames(W, H, N, 0xC11, 1)
    write_csv(tmp_path / "in.csv", frames)
    prefix = str(tmp_path / "out")
    r = run(["-f", str(N), "-s", f"{W}x{H}", "-o", str(tmp_path / "in.csv"), "-l", prefix] + extra)
    assert r.returncode == 0, r.stdout + r.stderr
    for f in range(N):
        assert f"Current frame {f}\n" in r.stdout
    # the reference's per-frame report: stages (fused here) and, with a filter, its device time
    stages = ("Performing initBoundaries kernel...\nPerforming MIP_ReducedPred kernel...\n" +
              "Performing upsampleDistortion kernel...\n" * 3)
    assert r.stdout.count(stages) == N
    took = re.findall(r"FilterSamples took ([0-9.]+) ms\n\nTIMING REPORT\nWrite\(ns\): [0-9.]+\nExecution\(ns\):([0-9.]+)\n"
                      r"Read\(ns\): 0.000000\nTotalFilterTime\(ms\): [0-9.]+\n", r.stdout)
    assert len(took) == (N if filt else 0)
    assert all(float(ms) > 0 and abs(float(ms) * 1e6 - float(ns)) < 1 for ms, ns in took)
    assert re.search(rf"Elapsed time \(ms\) from writing samples to reading distortion \({N}x\), \d+\n", r.stdout)
    res = O.engine_search(frames[0], filt, kidx, want_sad_satd=sad_satd)
    cost, sad, satd = res if sad_satd else (res, None, None)
    cost = mask_unavailable(cost, W, H)
    if sad_satd:
        sad, satd = mask_unavailable(sad, W, H), mask_unavailable(satd, W, H)
    got = open(prefix + ".csv", "rb").read()
    want = reference_log(cost, W, sad, satd)
    assert len(got) == len(want) and got == want


@pytest.mark.gpu
@needs_cli
def test_raw_inputs_binary_log_and_topk(gpu_available, tmp_path):
    """--InputFormat u16 / yuv420p10 (luma plane) give the CSV input's log; --BinaryLog holds
    every frame's cost table; --TopK 4 lists each CU's 4 best modes in rank order."""
    W, H, N, K = 264, 136, 2, 4
    frames = synth_frames(W, H, N, 0xC13, 0)
    write_csv(tmp_path / "in.csv", frames)
    frames.astype("<u2").tofile(tmp_path / "in.u16")
    rng = np.random.default_rng(3)
    with open(tmp_path / "in.yuv", "wb") as f:
        for fr in frames:
            f.write(fr.astype("<u2").tobytes())
            f.write(rng.integers(0, 1024, size=2 * (W // 2) * (H // 2), dtype=np.uint16).astype("<u2").tobytes())
    logs = {}
    for name, extra in (("csv", []), ("u16", []), ("yuv", ["--InputFormat", "yuv420p10"])):
        prefix = str(tmp_path / ("out_" + name))
        r = run(["-f", str(N), "-s", f"{W}x{H}", "-o", str(tmp_path / ("in." + name)), "-l", prefix,
                 "--BinaryLog", prefix + ".bin", "--BestModes", prefix + "_best.csv", "--TopK", str(K)] + extra)
        assert r.returncode == 0, r.stdout + r.stderr
        logs[name] = open(prefix + ".csv", "rb").read()
    assert logs["csv"] == logs["u16"] == logs["yuv"]
    want = [mask_unavailable(O.search(frames[f]), W, H) for f in range(N)]
    b = layout.read_binary_log(str(tmp_path / "out_yuv.bin"))
    assert (b["width"], b["height"], b["frames"]) == (W, H, N) and "sad" not in b
    assert np.array_equal(np.asarray(b["cost"]), np.stack(want))
    # decision lists: rows of the BestModes CSV vs the numpy statement
    import csv
    rows = list(csv.DictReader(open(tmp_path / "out_yuv_best.csv")))
    n = layout.num_ctus(W, H)
    got = {}
    for r in rows:
        got.setdefault((int(r["Frame"]), int(r["CTU"]), r["cuSizeName"], int(r["CU"])), []).append(
            (int(r["Rank"]), int(r["Mode"]), int(r["Transposed"]), int(r["Cost"])))
    shapes = {s.name: s for s in layout.SHAPES}
    for f in range(N):
        wm, wc = layout.topk_modes(want[f], n, K)
        k = 0
        for ctu in range(n):
            for s in layout.SHAPES:
                for cu in range(s.ncu):
                    lst = got[(f, ctu, s.name, cu)]
                    if wm[k, 0] == 0xFF:
                        assert lst == [(0, -1, -1, layout.UNAVAILABLE)]
                    else:
                        exp = [(r, int(m) % s.modes, int(m >= s.modes), int(c))
                               for r, (m, c) in enumerate(zip(wm[k], wc[k])) if m != 0xFF]
                        assert lst == exp
                    k += 1
    assert set(shapes) == {key[2] for key in got}


@pytest.mark.gpu
@needs_cli
def test_streaming_chunks_multi_device(gpu_available, tmp_path):
    """More frames than one chunk (--BatchFrames 2 over two engines: chunks of 4 frames,
    the last one partial): frames are read, searched and written chunk by chunk through the
    3-slot pipeline.  The log of every frame (--AllFrames), the binary log with SAD / SATD
    (written out of order into its three regions) and the decision rows must equal the
    oracle's, frame by frame and in order."""
    W, H, N = 128, 136, 7
    frames = synth_frames(W, H, N, 0xC14, 1)
    write_csv(tmp_path / "in.csv", frames)
    prefix = str(tmp_path / "out")
    r = run(["-f", str(N), "-s", f"{W}x{H}", "-o", str(tmp_path / "in.csv"), "-l", prefix, "--AllFrames",
             "--ReportSadSatd", "--BatchFrames", "2", "--DeviceIndex", "0,0", "--BinaryLog", prefix + ".bin",
             "--BestModes", prefix + "_best.csv"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert [int(x) for x in re.findall(r"Current frame (\d+)", r.stdout)] == list(range(N))
    want = [tuple(mask_unavailable(t, W, H) for t in O.search(frames[f], want_sad_satd=True)) for f in range(N)]
    log = b"".join(reference_log(c, W, s, t).split(b"\n", 1)[1] if f else reference_log(c, W, s, t)
                   for f, (c, s, t) in enumerate(want))
    assert open(prefix + ".csv", "rb").read() == log
    b = layout.read_binary_log(prefix + ".bin")
    assert b["frames"] == N
    for key, i in (("cost", 0), ("sad", 1), ("satd", 2)):
        assert np.array_equal(np.asarray(b[key]), np.stack([w[i] for w in want])), key
    import csv
    rows = list(csv.DictReader(open(prefix + "_best.csv")))
    assert len(rows) == N * layout.num_ctus(W, H) * layout.CUS_PER_CTU
    assert [int(x["Frame"]) for x in rows[::layout.CUS_PER_CTU]] == sorted(
        [f for f in range(N) for _ in range(layout.num_ctus(W, H))])
    n = layout.num_ctus(W, H)
    for f in range(N):
        bm, bc = layout.best_modes(want[f][0], n)
        got = rows[f * n * layout.CUS_PER_CTU:(f + 1) * n * layout.CUS_PER_CTU]
        assert [int(x["Cost"]) for x in got] == bc.tolist()


@pytest.mark.gpu
@needs_cli
def test_truncated_input_fails(gpu_available, tmp_path):
    """A CSV with fewer frames than -f asks for: exit 1 with the reference's message
    (main.cpp:366-368 perror), even when the shortfall is in a later chunk."""
    W, H = 128, 128
    frames = synth_frames(W, H, 2, 0xC15, 0)
    write_csv(tmp_path / "in.csv", frames)
    r = run(["-f", "5", "-s", f"{W}x{H}", "-o", str(tmp_path / "in.csv"), "-l", str(tmp_path / "o"),
             "--BatchFrames", "1"])
    assert r.returncode == 1
    assert "error while opening samples files" in r.stderr


@pytest.mark.gpu
@needs_cli
def test_best_modes_of_unlogged_frames(gpu_available, tmp_path):
    """--BestModes without --AllFrames / --BinaryLog: only frame 0's cost table is needed (the
    reference's log), so frames 1.. are searched decisions-only (the argmin fused into the
    search kernel, no cost table).  Every frame's decision rows must equal the oracle's argmin
    (ties to the lower mode, unavailable CUs Mode -1)."""
    import csv
    W, H, N = 264, 200, 4
    frames = synth_frames(W, H, N, 0xC16, 1)
    write_csv(tmp_path / "in.csv", frames)
    prefix = str(tmp_path / "out")
    r = run(["-f", str(N), "-s", f"{W}x{H}", "-o", str(tmp_path / "in.csv"), "-l", prefix, "--BatchFrames", "3",
             "--BestModes", prefix + "_best.csv"])
    assert r.returncode == 0, r.stdout + r.stderr
    rows = list(csv.DictReader(open(prefix + "_best.csv")))
    n = layout.num_ctus(W, H)
    assert len(rows) == N * n * layout.CUS_PER_CTU
    for f in range(N):
        bm, bc = layout.best_modes(O.search(frames[f]), n)
        got = rows[f * n * layout.CUS_PER_CTU:(f + 1) * n * layout.CUS_PER_CTU]
        assert [int(x["Cost"]) for x in got] == bc.tolist(), f
        shapes = [s for s in layout.SHAPES for _ in range(s.ncu)] * n
        want = [(-1, -1) if m == 0xFF else (int(m) % s.modes, int(m >= s.modes)) for m, s in zip(bm, shapes)]
        assert [(int(x["BestMode"]), int(x["Transposed"])) for x in got] == want, f


@pytest.mark.gpu
@needs_cli
def test_samples_above_10_bits_are_refused(gpu_available, tmp_path):
    """Input contract (include/mipgpu.h): a 12-bit sample (4095) in the CSV stops the CLI with
    exit 1 and its position; in a raw input (no CPU check) the engine's kernel-side check fails
    the search: exit 1, no log of wrong costs."""
    W, H, N = 128, 128, 2
    frames = synth_frames(W, H, N, 0xC17, 0)
    frames[1, 37, 101] = 4095
    write_csv(tmp_path / "in.csv", frames)
    r = run(["-f", str(N), "-s", f"{W}x{H}", "-o", str(tmp_path / "in.csv"), "-l", str(tmp_path / "o")])
    assert r.returncode == 1 and "1:37:101 (frame:row:column) is above 10 bits" in r.stdout, r.stdout + r.stderr
    frames.astype("<u2").tofile(tmp_path / "in.u16")
    r = run(["-f", str(N), "-s", f"{W}x{H}", "-o", str(tmp_path / "in.u16"), "-l", str(tmp_path / "o2")])
    assert r.returncode == 1 and "above 10 bits" in r.stdout, r.stdout + r.stderr


@needs_cli
def test_wrong_result_knob_stops_the_cli(tmp_path):
    """`MIPGPU_NO_PAIRS=1 mipgpu_cli ...` (a profiling knob of A/B builds: no mode pair
    searched) exits with an error naming the knob and writes no cost log (CPU: the release
    library refuses the knob before touching the GPU)."""
    frames = synth_frames(128, 128, 1, 0xC18, 0)
    write_csv(tmp_path / "in.csv", frames)
    env = dict(os.environ, MIPGPU_NO_PAIRS="1")
    r = subprocess.run([CLI, "-f", "1", "-s", "128x128", "-o", str(tmp_path / "in.csv"), "-l", str(tmp_path / "o")],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "MIPGPU_NO_PAIRS" in r.stdout + r.stderr, r.stdout + r.stderr
    assert not (tmp_path / "o.csv").exists()
