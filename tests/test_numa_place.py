"""NUMA placement of an engine's host side (vvc-mip-gpu_amd/csrc/numa_place.h, round 6) on CPU:
a fake sysfs tree (two nodes, GPUs on node 0 and 1, one without a node), read by the C++ unit
test (g++) and by the library's mip_numa_node_of_pci through MIPGPU_SYSFS_ROOT (no GPU)."""
import ctypes
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fake_sysfs(root):
    def put(rel, text):
        p = root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)
    put("bus/pci/devices/0000:c1:00.0/numa_node", "1\n")
    put("bus/pci/devices/0000:41:00.0/numa_node", "0\n")
    put("bus/pci/devices/0000:05:00.0/numa_node", "-1\n")
    put("devices/system/node/online", "0-1\n")
    put("devices/system/node/node0/cpulist", "0-1,4-5\n")
    put("devices/system/node/node1/cpulist", "2-3,6-7\n")
    # a one-node host
    put("one_node/bus/pci/devices/0000:c1:00.0/numa_node", "0\n")
    put("one_node/devices/system/node/online", "0\n")
    put("one_node/devices/system/node/node0/cpulist", "0-7\n")
    return root


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_numa_place_unit(tmp_path):
    exe = tmp_path / "test_numa_place"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-pthread", "-I",
                           os.path.join(REPO, "vvc-mip-gpu_amd", "csrc"), "-o", str(exe),
                           os.path.join(REPO, "tests", "cpp", "test_numa_place.cpp")])
    r = subprocess.run([str(exe), str(fake_sysfs(tmp_path / "sys"))], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "numa_place: ok" in r.stdout


def test_library_reads_the_gpu_node_from_sysfs(tmp_path):
    """mip_numa_node_of_pci through the C ABI, in a child process whose MIPGPU_SYSFS_ROOT is
    the fake tree (the node exists only when its CPUs intersect the process's)."""
    root = fake_sysfs(tmp_path / "sys")
    code = ("import sys, os; sys.path.insert(0, %r); import mipgpu; L = mipgpu.library(); "
            "ok = os.sched_getaffinity(0); "
            "print(L.mip_numa_node_of_pci(b'0000:C1:00.0'), L.mip_numa_node_of_pci(b'0000:41:00.0'), "
            "L.mip_numa_node_of_pci(b'0000:05:00.0'), L.mip_numa_node_of_pci(b'0000:77:00.0'), "
            "int(bool(ok & {2, 3, 6, 7})), int(bool(ok & {0, 1, 4, 5})))" % os.path.join(REPO, "vvc-mip-gpu_amd"))
    out = subprocess.check_output([sys.executable, "-c", code], text=True, timeout=300,
                                  env=dict(os.environ, MIPGPU_SYSFS_ROOT=str(root), MIPGPU_NO_TORCH="1")).split()
    n1, n0, nm, nu, has1, has0 = map(int, out)
    assert n1 == (1 if has1 else -1) and n0 == (0 if has0 else -1) and nm == -1 and nu == -1, out
