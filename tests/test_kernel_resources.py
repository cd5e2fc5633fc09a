"""Build-time resource checks of the gfx950 kernels in libmipgpu.so (CPU: reads the code
objects' metadata, tests/kernel_resources.py).

* No kernel spills to scratch (an out-of-line device helper in the search loop once cost
  192 bytes per lane of scratch, 12 % of the search time and 2x its HBM traffic).
* mip_search_kernel: <= 128 VGPRs, i.e. 4 waves per SIMD -- two 8-wave workgroups per CU
  (or one 16-wave workgroup in small launches), the occupancy the persistent grid is sized
  for.
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
    assert len(_named(kernels, "mip_search_kernel")) == 10
    assert len(_named(kernels, "filter_kernel")) == 8      # radius x int/float x 2-D/separable
    for part in ("fixup_kernel", "best_mode_kernel", "dec_split_kernel"):
        _named(kernels, part)


def test_no_scratch_spills(kernels):
    spilled = {n: k[".private_segment_fixed_size"] for n, k in kernels.items() if k[".private_segment_fixed_size"]}
    assert not spilled


def test_search_kernel_occupancy(kernels):
    for name, k in _named(kernels, "mip_search_kernel").items():
        assert k[".vgpr_count"] + k.get(".agpr_count", 0) <= 128, (name, k[".vgpr_count"])


def test_filter_kernel_occupancy(kernels):
    for name, k in _named(kernels, "filter_kernel").items():
        sep = re.search(r"filter_kernelILi\dELb\dELb(\d)EE", name).group(1) == "1"  # <RAD, FLOAT, SEP>
        assert k[".vgpr_count"] <= (128 if sep else 64), (name, k[".vgpr_count"])
