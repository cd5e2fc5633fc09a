"""The C oracle against the reference kernels' own outputs (golden fixtures)."""
import numpy as np
import pytest

import golden_utils as G
import oracle_lib as O
from mipgpu import layout
from mipgpu.synth import synth_frame

SMALL = [n for n in G.names() if n.startswith(("small_", "w416", "w832", "w1280"))]
LARGE = [n for n in G.names() if n not in SMALL]


def test_synth_generators_agree():
    for kind in (0, 1, 2):
        assert (O.synth(136, 72, 0xABC, kind) == synth_frame(136, 72, 0xABC, kind)).all()


@pytest.mark.parametrize("name", SMALL)
def test_oracle_matches_reference_small(name):
    fx = G.load(name)
    c = fx["config"]
    frames = G.inputs(fx)
    for f, fr in enumerate(fx["frames"]):
        refs, und, mask = G.refs_and_mask(fx, frames, f)
        assert int(mask.sum()) == fr["defined_entries"]
        if refs is not None:
            assert G.filtered_sha(refs, und) == fr["filtered_sha256"]
        cost, sad, satd = O.search(frames[f], refs, want_sad_satd=True)
        assert G.sha(G.masked(cost, mask)) == fr["cost_sha256"]
        if "sad_sha256" in fr:
            assert G.sha(G.masked(sad, mask)) == fr["sad_sha256"]
            assert G.sha(G.masked(satd, mask)) == fr["satd_sha256"]


@pytest.mark.parametrize("name", LARGE)
def test_oracle_matches_reference_ctu_rows(name):
    """Full-size configs: the stored CTU rows, recomputed for just those CTUs."""
    fx = G.load(name)
    c = fx["config"]
    frames = G.inputs(fx)
    for f, fr in enumerate(fx["frames"]):
        refs, und, mask = G.refs_and_mask(fx, frames, f)
        assert int(mask.sum()) == fr["defined_entries"]
        if refs is not None:
            assert G.filtered_sha(refs, und) == fr["filtered_sha256"]
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
    assert G.sha(G.masked(cost, layout.available_mask(1920, 1080))) == fx["frames"][0]["cost_sha256"]


def test_oracle_fixture_generation_was_clean():
    """At generation (tools/ref_golden.py) the oracle matched the reference on every
    defined entry, and every entry that changed across the fill experiment's runs was in
    the oracle's undefined set."""
    for n in G.names():
        fx = G.load(n)
        assert fx.get("format") == 2, n
        for ck in fx["oracle_check"] + fx["fill_check"]:
            assert all(v == 0 for k, v in ck.items() if k.endswith("mismatches")), (n, ck)
        assert len(fx["fill_check"]) == fx["config"]["frames"], n
