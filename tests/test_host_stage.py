"""The pageable bounce ring (vvc-mip-gpu_amd/csrc/host_stage.h) on CPU: its queue and
completion-thread logic over a simulated device (tests/cpp/test_host_stage.cpp), built with
g++ (no GPU), and once more under ThreadSanitizer on a smaller workload."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "test_host_stage.cpp")
INC = os.path.join(REPO, "vvc-mip-gpu_amd", "csrc")


def _build(exe, extra):
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-pthread", *extra,
                           "-I", INC, "-o", str(exe), SRC])


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_stage(tmp_path):
    exe = tmp_path / "test_host_stage"
    _build(exe, [])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_stage: ok" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_stage_thread_sanitizer(tmp_path):
    exe = tmp_path / "test_host_stage_tsan"
    try:
        _build(exe, ["-g", "-fsanitize=thread"])
    except subprocess.CalledProcessError:
        pytest.skip("compiler without ThreadSanitizer")
    r = subprocess.run([str(exe), "quick"], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "host_stage: ok" in r.stdout
