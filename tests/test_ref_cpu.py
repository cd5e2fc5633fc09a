"""The reference's own kernels on the host CPU (oracle/ref/ref_cpu_runner.cpp: /root/reference's
intra.cl compiled by clang for x86-64 with the OpenCL builtins of oracle/ref/cl_cpu_shim.cl;
BASELINE configs[0], the `cpu_baseline.reference_kernels` figure of bench.py).  Test
infrastructure pinned twice: its cost tables must hash like the golden fixtures the same
kernels produced on the MI355X (AMD OpenCL), and equal the C oracle on every defined entry.
Needs the libraries `make -C oracle ref-cpu` builds where the reference tree is mounted."""
import os
import subprocess

import numpy as np
import pytest

import golden_utils as G
import oracle_lib as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref")
RUNNER = os.path.join(REF, "ref_cpu_runner")

pytestmark = pytest.mark.skipif(
    not (os.path.exists(RUNNER) and all(os.path.exists(os.path.join(REF, "intra_cpu_s%d.so" % s)) for s in range(3))),
    reason="reference-on-CPU libraries not built (make -C oracle ref-cpu, needs /root/reference)")


@pytest.mark.parametrize("name", ["small_structured", "small_uniform_partial", "w416_orig"])
def test_reference_on_cpu_matches_its_gpu_fixture_and_the_oracle(tmp_path, name):
    fx = G.load(name)
    c = fx["config"]
    out = tmp_path / "cost.bin"
    r = subprocess.run([RUNNER, "--libs", REF, "--width", str(c["width"]), "--height", str(c["height"]),
                        "--frames", str(c["frames"]), "--synth", "%d:%x" % (c["kind"], c["seed"]),
                        "--workers", str(min(8, os.cpu_count() or 1)), "--out-cost", str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    cpf = (c["width"] + 127) // 128 * ((c["height"] + 127) // 128) * 97840
    costs = np.fromfile(out, "<i4").reshape(c["frames"], cpf)
    frames = G.inputs(fx)
    for f in range(c["frames"]):
        _, _, mask = G.refs_and_mask(fx, frames, f)
        assert G.sha(G.masked(costs[f], mask)) == fx["frames"][f]["cost_sha256"], (name, f)
        want = O.search(frames[f])
        assert np.array_equal(costs[f][mask.reshape(-1)], want.reshape(-1)[mask.reshape(-1)]), (name, f)
