"""Build-time resource checks of the gfx950 kernels in libmipgpu.so (CPU: reads the code
objects' metadata, tests/kernel_resources.py).

* No kernel spills to scratch (an out-of-line device helper in the search loop once cost
  192 bytes per lane of scratch, 12 % of the search time and 2x its HBM traffic) -- except the
  12-wave search kernels, which at 80 VGPRs keep up to 24 dwords of per-item state in scratch
  (item setup and window staging, once per quadrant item: none inside the size classes' code,
  tools/isa_dump.py); they are held to 96 bytes per lane.
* mip_search_kernel: the 12-wave variants <= 80 VGPRs, i.e. 6 waves per SIMD -- two 12-wave
  workgroups per CU; the 16-wave variants (small launches, one workgroup per CU) and the
  four-wave twin's 8-wave ones (the host pipeline's small chunks, two per CU) <= 128 VGPRs,
  4 waves per SIMD: the occupancy the persistent grid is sized for.
* filter_kernel: 2-D filters (128-thread tiles) <= 64 VGPRs, i.e. 8 waves per SIMD; the
  separable ones run one-wave 64-thread tiles (round 6) whose ~10 KB of LDS each allow 16 per
  CU, 4 waves per SIMD: <= 128 VGPRs.
"""
import os
import re

import pytest

import kernel_resources

LIB = os.path.join(os.path.dirname(__file__), "..", "vvc-mip-gpu_amd", "lib", "libmipgpu.so")


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("libmipgpu.so not built")
    return kernel_resources.kernels(LIB)


def _named(kernels, part):
    found = {n: k for n, k in kernels.items() if part in n}
    assert found, part
    return found


def test_every_kernel_variant_present(kernels):
    # {orig, alt} x {table, decisions} x prefetch (orig), and the 16-wave variants of small
    # launches ({orig, alt} x {table, decisions}, no prefetch)
    # + the four-wave twin's 8-wave variants ({orig, alt} x {table, decisions}, orig x prefetch)
    assert len(_named(kernels, "mip_search_kernel")) == 16
    assert len(_named(kernels, "filter_kernel")) == 8      # radius x int/float x 2-D/separable
    for part in ("fixup_kernel", "best_mode_kernel", "dec_split_kernel"):
        _named(kernels, part)


def _search_waves(name):
    return int(re.search(r"mip_search_kernelILb\dELb\dELb\dELi(\d+)EE", name).group(1))  # <ALT, DEC, PF, NW>


def test_no_scratch_spills(kernels):
    spilled = {n: k[".private_segment_fixed_size"] for n, k in kernels.items() if k[".private_segment_fixed_size"]}
    bounded = {n: b for n, b in spilled.items() if "mip_search_kernel" in n and _search_waves(n) == 12 and b <= 96}
    assert spilled == bounded, spilled


def test_search_kernel_occupancy(kernels):
    waves = set()
    for name, k in _named(kernels, "mip_search_kernel").items():
        nw = _search_waves(name)
        waves.add(nw)
        limit = 80 if nw == 12 else 128  # 6 / 4 waves per SIMD (8: the four-wave twin)
        assert k[".vgpr_count"] + k.get(".agpr_count", 0) <= limit, (name, k[".vgpr_count"])
    assert waves == {8, 12, 16}


def test_filter_kernel_occupancy(kernels):
    for name, k in _named(kernels, "filter_kernel").items():
        sep = re.search(r"filter_kernelILi\dELb\dELb(\d)EE", name).group(1) == "1"  # <RAD, FLOAT, SEP>
        assert k[".vgpr_count"] <= (128 if sep else 64), (name, k[".vgpr_count"])
