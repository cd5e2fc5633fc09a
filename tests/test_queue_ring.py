"""The search kernel's item-counter bookkeeping (csrc/queue_ring.h) on CPU: a C++ unit test
with mock stream operations, built with g++ (no GPU)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_queue_ring_bookkeeping(tmp_path):
    exe = tmp_path / "test_queue_ring"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I",
                           os.path.join(REPO, "vvc-mip-gpu_amd", "csrc"), "-o", str(exe),
                           os.path.join(REPO, "tests", "cpp", "test_queue_ring.cpp")])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "queue_ring: ok" in r.stdout
