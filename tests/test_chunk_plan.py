"""The host pipeline's chunk plan (vvc-mip-gpu_amd/csrc/chunk_plan.h: equal chunks, ramps up
for calls into an idle pipeline and down for synchronous decisions-only calls) on CPU: a C++
unit test built with g++ (no GPU)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_chunk_plan(tmp_path):
    exe = tmp_path / "test_chunk_plan"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I",
                           os.path.join(REPO, "vvc-mip-gpu_amd", "csrc"), "-o", str(exe),
                           os.path.join(REPO, "tests", "cpp", "test_chunk_plan.cpp")])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "chunk_plan: ok" in r.stdout
