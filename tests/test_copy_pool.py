"""The bounce ring's parallel host memcpy (vvc-mip-gpu_amd/csrc/copy_pool.h) on CPU: a C++
unit test built with g++ (no GPU)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_copy_pool(tmp_path):
    exe = tmp_path / "test_copy_pool"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-pthread", "-I",
                           os.path.join(REPO, "vvc-mip-gpu_amd", "csrc"), "-o", str(exe),
                           os.path.join(REPO, "tests", "cpp", "test_copy_pool.cpp")])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "copy_pool: ok" in r.stdout
