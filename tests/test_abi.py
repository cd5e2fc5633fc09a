"""C-ABI boundary: the library loads and exports exactly what include/mipgpu.h declares.
Only host-side geometry helpers are called (no GPU needed)."""
import ctypes
import os
import re
import sys
import subprocess

import pytest

import mipgpu
from mipgpu import layout

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mipgpu.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mip_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(mipgpu.LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "vvc-mip-gpu_amd"), "lib/libmipgpu.so"])
    return mipgpu.library()


def test_exports_every_declared_symbol(lib):
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    out = subprocess.check_output(["nm", "-D", "--defined-only", mipgpu.LIB_PATH]).decode()
    exported = set(re.findall(r" T (mip_\w+)", out))
    assert set(syms) <= exported


def test_geometry_helpers(lib):
    assert lib.mip_abi_version() == 7
    assert lib.mip_num_ctus(1920, 1080) == 135
    assert lib.mip_num_ctus(3840, 2160) == 510
    assert lib.mip_num_ctus(7680, 4320) == 2040
    assert lib.mip_costs_per_frame(1920, 1080) == 135 * 97840
    assert lib.mip_cus_per_frame(1920, 1080) == 135 * 5380
    for s in layout.SHAPES:
        assert lib.mip_shape_name(s.index).decode() == s.name
        w, h, m, n, o = (ctypes.c_int() for _ in range(5))
        assert lib.mip_shape_info(s.index, *(ctypes.byref(v) for v in (w, h, m, n, o))) == 0
        assert (w.value, h.value, m.value, n.value, o.value) == (s.w, s.h, s.modes, s.ncu, s.cost_offset)
        xs, ys = s.positions()
        for cu in (0, s.ncu // 2, s.ncu - 1):
            x, y = ctypes.c_int(), ctypes.c_int()
            assert lib.mip_cu_position(s.index, cu, ctypes.byref(x), ctypes.byref(y)) == 0
            assert (x.value, y.value) == (xs[cu], ys[cu])
    assert lib.mip_shape_info(47, None, None, None, None, None) != 0
    assert b"bad shape" in lib.mip_last_error()


def test_filter_names_follow_reference_whitelist():
    assert mipgpu.filter_index("filterFrame_2d_float_5x5_quarterCtu") == 7
    assert mipgpu.filter_index(None) == mipgpu.FILTER_NONE
    with pytest.raises(mipgpu.MipError):
        mipgpu.filter_index("filterFrame_2d")  # half-CTU kernel, not whitelisted (constants.h:25-34)


def test_missing_library_fails_loudly(tmp_path):
    """The product path has no CPU fallback: without libmipgpu.so the binding raises."""
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import mipgpu\n"
            "try:\n    mipgpu.MipEngine(128, 128)\nexcept mipgpu.MipError as e:\n    print('MipError', e)\n"
            % os.path.join(REPO, "vvc-mip-gpu_amd"))
    env = dict(os.environ, MIPGPU_LIB=str(tmp_path / "absent.so"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert "MipError" in out.stdout and "no CPU fallback" in out.stdout, out.stdout + out.stderr


def test_engine_create_rejects_bad_arguments_before_touching_the_gpu(lib):
    """Argument checks in mip_engine_create run before any HIP call (safe without a GPU):
    frame size, max_batch, best_k, and the per-launch CU count (2^31 - 256), which an 8K
    batch of ~200 frames would overflow in int (mipgpu.cpp kMaxCus)."""
    cases = [
        ((1922, 1080, 1, 1), b"multiples of 4"),
        ((0, 1080, 1, 1), b"multiples of 4"),
        ((1920, 1080, 0, 1), b"max_batch"),
        ((7680, 4320, 200, 1), b"CUs per launch"),
        ((1920, 1080, 1, 33), b"best_k"),
    ]
    for (w, h, batch, k), msg in cases:
        o = mipgpu._Opts()
        lib.mip_opts_default(ctypes.byref(o))
        o.max_batch, o.best_k = batch, k
        e = ctypes.c_void_p()
        assert lib.mip_engine_create(0, w, h, ctypes.byref(o), ctypes.byref(e)) != 0
        assert not e.value
        assert msg in lib.mip_last_error(), lib.mip_last_error()
    # 195 frames of 8K fit (195 * 2040 * 5380 < 2^31 - 256); 196 do not
    assert 195 * 2040 * 5380 <= (1 << 31) - 256 < 196 * 2040 * 5380
    with pytest.raises(mipgpu.MipError, match="CUs per launch"):
        mipgpu.MipEngine(7680, 4320, max_batch=196)


def test_build_id_names_the_sources(lib):
    """mip_build_id(): the hash of the sources + flags the library was built from (the Makefile
    computes it the same way), so a bench line / profile can be tied to its build."""
    bid = mipgpu.build_id()
    assert bid.startswith("src:") and " git:" in bid, bid
    want = subprocess.check_output(["make", "-s", "-C", os.path.join(REPO, "vvc-mip-gpu_amd"), "build-id"]).decode()
    assert mipgpu.source_id(bid) == mipgpu.source_id(want.strip())


@pytest.mark.parametrize("knob", ["MIPGPU_NO_PAIRS", "MIPGPU_SHAPE_FILTER"])
def test_wrong_result_knobs_are_refused_by_the_release_library(lib, monkeypatch, knob):
    """Profiling knobs that make wrong tables by design (MIPGPU_NO_PAIRS: no mode pair searched;
    MIPGPU_SHAPE_FILTER: a subset of the shapes) are honoured only by A/B builds with
    -DMIPGPU_PROFILING_KNOBS (named in the build ID); the release library refuses to create an
    engine while one is set -- before any HIP call -- instead of returning silently wrong
    costs through the C ABI, the Python binding or the CLI."""
    assert "knobs:" not in mipgpu.build_id()
    monkeypatch.setenv(knob, "1")
    o = mipgpu._Opts()
    lib.mip_opts_default(ctypes.byref(o))
    e = ctypes.c_void_p()
    assert lib.mip_engine_create(0, 256, 136, ctypes.byref(o), ctypes.byref(e)) != 0 and not e.value
    assert knob.encode() in lib.mip_last_error() and b"profiling knob" in lib.mip_last_error()
    with pytest.raises(mipgpu.MipError, match="profiling knob"):
        mipgpu.MipEngine(256, 136)


def test_one_hip_runtime_per_process():
    """Loading libmipgpu.so and then importing torch leaves ONE HIP runtime in the process
    (torch's wheel bundles its own libamdhip64, loaded by path; mipgpu preloads that runtime by
    path so the engine binds to it) -- two runtimes in one process made torch report no GPU
    once the engine had opened it (round 5).  Loading the library does not import torch
    (a multi-second import for numpy-only callers)."""
    code = ("import sys; sys.path.insert(0, %r); import mipgpu; mipgpu.library(); "
            "t = 'torch' in sys.modules; import torch; "
            "print(len(mipgpu.hip_runtimes()), t, mipgpu.hip_runtimes())" % os.path.join(REPO, "vvc-mip-gpu_amd"))
    out = subprocess.check_output([sys.executable, "-c", code], text=True, timeout=300).strip()
    assert out.startswith("1 False "), out
    if mipgpu._torch_hip_runtime():
        assert os.path.realpath(mipgpu._torch_hip_runtime()) in out, out
