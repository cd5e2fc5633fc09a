"""The C oracle against the reference kernels' own outputs (golden fixtures)."""
import numpy as np
import pytest

import golden_utils as G
import oracle_lib as O
from mipgpu import layout
from mipgpu.synth import synth_frame

SMALL = [n for n in G.names() if n.startswith("small_")]
LARGE = [n for n in G.names() if not n.startswith("small_")]


def _refs(fx, frames, f):
    c = fx["config"]
    return O.filter_frame(frames[f], c["filter"], c["kernel_idx"]) if c["filter"] else None


def test_synth_generators_agree():
    for kind in (0, 1, 2):
        assert (O.synth(136, 72, 0xABC, kind) == synth_frame(136, 72, 0xABC, kind)).all()


@pytest.mark.parametrize("name", SMALL)
def test_oracle_matches_reference_small(name):
    fx = G.load(name)
    c = fx["config"]
    frames = G.inputs(fx)
    for f, fr in enumerate(fx["frames"]):
        refs = _refs(fx, frames, f)
        if refs is not None:
            assert G.sha(refs) == fr["filtered_sha256"]
        cost, sad, satd = O.search(frames[f], refs, want_sad_satd=True)
        assert G.sha(G.masked(cost, c["width"], c["height"])) == fr["cost_sha256"]
        if "sad_sha256" in fr:
            assert G.sha(G.masked(sad, c["width"], c["height"])) == fr["sad_sha256"]
            assert G.sha(G.masked(satd, c["width"], c["height"])) == fr["satd_sha256"]


@pytest.mark.parametrize("name", LARGE)
def test_oracle_matches_reference_ctu_rows(name):
    """Full-size configs: the stored CTU rows, recomputed for just those CTUs."""
    fx = G.load(name)
    c = fx["config"]
    frames = G.inputs(fx)
    mask = layout.available_mask(c["width"], c["height"])
    for f, fr in enumerate(fx["frames"]):
        refs = _refs(fx, frames, f)
        if refs is not None:
            assert G.sha(refs) == fr["filtered_sha256"]
        for ctu in map(int, fr["ctu_rows"]):
            cost = O.search(frames[f], refs, ctus=(ctu, ctu + 1))
            sl = slice(ctu * 97840, (ctu + 1) * 97840)
            got = np.where(mask[sl], cost[sl], layout.UNAVAILABLE)
            assert (got == G.ctu_row(fx, f, ctu)).all()


@pytest.mark.slow
def test_oracle_matches_reference_full_1080p():
    fx = G.load("c2_1080p_orig")
    frames = G.inputs(fx)
    cost = O.search(frames[0])
    assert G.sha(G.masked(cost, 1920, 1080)) == fx["frames"][0]["cost_sha256"]


def test_oracle_fixture_generation_was_clean():
    for n in G.names():
        for ck in G.load(n).get("oracle_check", []):
            assert all(v == 0 for k, v in ck.items() if k.endswith("mismatches") or k.endswith("maxdiff")), (n, ck)
