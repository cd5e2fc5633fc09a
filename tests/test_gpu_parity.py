"""HIP path parity: libmipgpu.so (gfx950 kernels) against the C oracle and against the
reference kernels' golden outputs.  Integer path -> bit-exact everywhere; the float
filters are also required to be bit-exact (tolerance 0): both sides divide exactly as
the reference's compiled kernels do (frexp / v_rcp_f32 / v_mul / v_ldexp, see
oracle/mip_oracle.c ref_fdiv), which the golden fixtures with tie-prone scales pin."""
import numpy as np
import pytest

import golden_utils as G
import oracle_lib as O
from mipgpu import MipEngine, MipError, filter_index, layout
from mipgpu.synth import synth_frame, synth_frames

pytestmark = pytest.mark.gpu

FILTERS = [("filterFrame_1d_int", 5), ("filterFrame_1d_float", 5), ("filterFrame_2d_int_quarterCtu", 5),
           ("filterFrame_2d_float_quarterCtu", 5), ("filterFrame_1d_int_5x5", 3), ("filterFrame_1d_float_5x5", 3),
           ("filterFrame_2d_int_5x5_quarterCtu", 3), ("filterFrame_2d_float_5x5_quarterCtu", 3)]


def _engine(c, **kw):
    return MipEngine(c["width"], c["height"], filter=c["filter"], kernel_idx=c["kernel_idx"],
                     max_batch=c["frames"], **kw)


SMALL = [n for n in G.names() if n.startswith(("small_", "w416", "w832", "w1280"))]


@pytest.mark.parametrize("name", SMALL)
def test_small_configs_vs_oracle_and_reference(gpu_available, name):
    """Small sizes and the reference's own resolutions whose width is not a multiple of 128
    (416x240, 832x480, 1280x720: CUs right of the frame read the next row, the filters'
    racing stores): bit-exact vs the oracle everywhere, and the defined entries hash to the
    reference's."""
    fx = G.load(name)
    c = fx["config"]
    frames = G.inputs(fx)
    with _engine(c, want_sad_satd=True) as eng:
        out = eng.search(frames, sad_satd=True)
        filt = eng.filter_frames(frames, c["filter"], c["kernel_idx"]) if c["filter"] else None
    for f, fr in enumerate(fx["frames"]):
        refs, und, mask = G.refs_and_mask(fx, frames, f)
        oc, osad, osatd = O.engine_search(frames[f], c["filter"], c["kernel_idx"], want_sad_satd=True)
        assert np.array_equal(out["cost"][f], oc)
        assert np.array_equal(out["sad"][f], osad)
        assert np.array_equal(out["satd"][f], osatd)
        # UNAVAILABLE: the geometrically undefined CUs and (engine filter) the CUs reading a
        # filtered sample the reference computes from memory past the frame's end -- a subset
        # of the reference's undefined entries (the rest only race, see oracle_lib)
        unav = out["cost"][f] == layout.UNAVAILABLE
        assert np.array_equal(unav, O.engine_unavailable_mask(frames[f], c["filter"], c["kernel_idx"]))
        assert not (unav & mask).any()
        assert G.sha(G.masked(out["cost"][f], mask)) == fr["cost_sha256"]
        if "sad_sha256" in fr:
            assert G.sha(G.masked(out["sad"][f], mask)) == fr["sad_sha256"]
            assert G.sha(G.masked(out["satd"][f], mask)) == fr["satd_sha256"]
        if filt is not None:
            assert np.array_equal(filt[f], refs)
            assert G.filtered_sha(filt[f], und) == fr["filtered_sha256"]


@pytest.mark.parametrize("name", [n for n in G.names() if n not in SMALL])
def test_full_size_configs_vs_reference(gpu_available, name):
    """1080p / 4K: the whole cost table, defined entries, hashes to the reference's."""
    fx = G.load(name)
    c = fx["config"]
    frames = G.inputs(fx)
    with _engine(c) as eng:
        out = eng.search(frames)
        if c["filter"]:
            filt = eng.filter_frames(frames, c["filter"], c["kernel_idx"])
    for f, fr in enumerate(fx["frames"]):
        refs, und, mask = G.refs_and_mask(fx, frames, f)
        # the engine's UNAVAILABLE entries: the geometrically undefined CUs and, with the engine's
        # filter, the CUs that read a filtered sample computed from past the frame's end
        unav = out["cost"][f] == layout.UNAVAILABLE
        assert np.array_equal(unav, O.engine_unavailable_mask(frames[f], c["filter"], c["kernel_idx"]))
        assert not (unav & mask).any()
        assert G.sha(G.masked(out["cost"][f], mask)) == fr["cost_sha256"]
        for ctu in map(int, fr["ctu_rows"]):
            sl = slice(ctu * 97840, (ctu + 1) * 97840)
            assert np.array_equal(G.masked(out["cost"][f][sl], mask[sl]), G.ctu_row(fx, f, ctu))
        if c["filter"]:
            assert G.filtered_sha(filt[f], und) == fr["filtered_sha256"]


@pytest.mark.parametrize("w,h", [(392, 136), (648, 232), (300, 68), (292, 36)])
@pytest.mark.parametrize("filt,nk", FILTERS)
def test_filters_vs_oracle(gpu_available, filt, nk, w, h):
    # partial tiles on both axes; 648x232 has 6 interior tiles (vectorised staging path);
    # widths 300 and 292 are not multiples of 8 (sample-by-sample staging)
    frame = synth_frame(w, h, 0x51, 1)
    # near-black samples: quotients around 1/2 (sum == scale/2 is the case where the
    # reference's fp32 division can fall just below the tie)
    dark = np.random.default_rng(5).integers(0, 3, (h, w)).astype(np.uint16)
    with MipEngine(w, h) as eng:
        for k in range(nk):
            for fr in (frame, dark):
                got = eng.filter_frames(fr, filt, k)[0]
                assert np.array_equal(got, O.filter_frame(fr, filt, k)), (filt, k)


@pytest.mark.parametrize("w,h,kind", [(136, 72, 0), (8, 8, 1), (132, 260, 1), (128, 4, 0), (640, 384, 1)])
def test_edge_frame_sizes(gpu_available, w, h, kind):
    frame = synth_frame(w, h, 0x77 + w + h, kind)
    with MipEngine(w, h, want_sad_satd=True) as eng:
        out = eng.search(frame, sad_satd=True, best=True)
    oc, osad, osatd = O.search(frame, want_sad_satd=True)
    assert np.array_equal(out["cost"][0], oc)
    assert np.array_equal(out["sad"][0], osad)
    assert np.array_equal(out["satd"][0], osatd)
    bm, bc = layout.best_modes(oc, layout.num_ctus(w, h))
    assert np.array_equal(out["best_mode"][0], bm)
    assert np.array_equal(out["best_cost"][0], bc)
    avail = layout.available_mask(w, h)
    assert (oc[~avail] == layout.UNAVAILABLE).all()


def test_alt_refs_supplied_by_caller(gpu_available):
    frame = synth_frame(256, 136, 0x99, 0)
    refs = synth_frame(256, 136, 0x9A, 1)
    with MipEngine(256, 136) as eng:
        out = eng.search(frame, refs=refs)
    assert np.array_equal(out["cost"][0], O.search(frame, refs))


def test_batched_device_api_matches_host_api(gpu_available):
    import torch
    w, h, n = 384, 256, 3
    frames = synth_frames(w, h, n, 0x123, 0)
    with MipEngine(w, h, max_batch=n, filter="filterFrame_2d_float_5x5_quarterCtu", kernel_idx=2) as eng:
        host = eng.search(frames, best=True)
        d = torch.from_numpy(frames.astype(np.int16)).cuda()
        costs = eng.search_device(d)
        bm = torch.empty((n, eng.cus_per_frame), dtype=torch.uint8, device="cuda")
        eng.search_device(d, costs=costs, best_mode=bm)
        torch.cuda.synchronize()
        assert np.array_equal(costs.cpu().numpy(), host["cost"])
        assert np.array_equal(bm.cpu().numpy(), host["best_mode"])
    for f in range(n):
        assert np.array_equal(host["cost"][f], O.engine_search(frames[f], "filterFrame_2d_float_5x5_quarterCtu", 2))


def test_many_launches_on_two_streams(gpu_available):
    """The persistent search kernel takes its items from one of 16 device counters per
    engine; 40 back-to-back launches alternating between two streams (and frame counts, so
    the grids differ) must reuse the counters safely and all give the same tables."""
    import torch
    w, h = 264, 200  # edge CTUs in both directions
    frames = synth_frames(w, h, 3, 0x51, 0)
    want = np.stack([O.search(frames[f]) for f in range(3)])
    d = torch.from_numpy(frames.astype(np.int16)).cuda()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    with MipEngine(w, h, max_batch=3) as eng:
        outs = []
        for i in range(40):
            n = 1 + i % 3
            outs.append((n, eng.search_device(d[:n], stream=streams[i % 2])))
        torch.cuda.synchronize()
        for n, c in outs:
            assert np.array_equal(c.cpu().numpy(), want[:n])


@pytest.mark.parametrize("k", [1, 3, 13, 32])
def test_topk_decision_lists(gpu_available, k):
    """mip_topk_device / engine best_k vs the numpy statement on oracle cost tables (edge
    CTUs: unavailable CUs; k = 13 and 32 exceed the 12 / 16 modes of some shapes)."""
    import torch
    from mipgpu import topk_device
    w, h = 264, 136
    frames = synth_frames(w, h, 2, 0x7C, 0)
    want = [O.search(frames[f]) for f in range(2)]
    n = layout.num_ctus(w, h)
    d = torch.from_numpy(np.stack(want)).cuda()
    modes, costs = topk_device(d, w, h, k)
    torch.cuda.synchronize()
    with MipEngine(w, h, max_batch=2, best_k=k) as eng:
        out = eng.search(frames, best=True)
    for f in range(2):
        wm, wc = layout.topk_modes(want[f], n, k)
        assert np.array_equal(modes[f].cpu().numpy(), wm)
        assert np.array_equal(costs[f].cpu().numpy(), wc)
        em = out["best_mode"][f].reshape(-1, k)
        ec = out["best_cost"][f].reshape(-1, k)
        assert np.array_equal(em, wm) and np.array_equal(ec, wc)
    if k == 1:
        bm, bc = layout.best_modes(want[0], n)
        assert np.array_equal(modes[0, :, 0].cpu().numpy(), bm)


def test_full_size_ctu_shift_and_batch_invariance(gpu_available):
    """Size-independent properties at the bench's 1080p size: (a) shifting a frame right by
    one CTU (128 columns) shifts every CTU's cost block by one CTU, except CTUs whose left
    reference column changes (first column); (b) a frame's table does not depend on the
    batch it is searched in (persistent item queue, edge-CTU lists, slice choice)."""
    W, H = 1920, 1080
    a = synth_frame(W, H, 0xB1, 0)
    b = np.empty_like(a)
    b[:, 128:] = a[:, :W - 128]
    b[:, :128] = synth_frame(128, H, 0xB2, 1)
    cols, rows = layout.ctu_grid(W, H)
    batch = np.stack([a, b, synth_frame(W, H, 0xB3, 0)])
    with MipEngine(W, H, max_batch=3) as eng:
        ca = eng.search(a)["cost"][0].reshape(-1, layout.COSTS_PER_CTU)
        cb = eng.search(b)["cost"][0].reshape(-1, layout.COSTS_PER_CTU)
        cbatch = eng.search(batch)["cost"]
    for r in range(rows):
        for c in range(1, cols - 1):
            assert np.array_equal(ca[r * cols + c], cb[r * cols + c + 1]), (r, c)
    assert np.array_equal(cbatch[0].reshape(ca.shape), ca)
    assert np.array_equal(cbatch[1].reshape(cb.shape), cb)


def test_errors_are_loud(gpu_available):
    with pytest.raises(MipError):
        MipEngine(130, 64)  # width not a multiple of 4
    with pytest.raises(MipError):
        MipEngine(128, 64, filter="filterFrame_2d_int_quarterCtu", kernel_idx=7)
    with pytest.raises(MipError):
        filter_index("filterFrame_2d_float")  # not whitelisted
    with pytest.raises(MipError):
        MipEngine(128, 64, best_k=33)


def _extreme(pattern, w, h):
    y, x = np.mgrid[0:h, 0:w]
    if pattern == "checker1":
        return np.where((x + y) % 2, 1023, 0)
    if pattern == "checker4":
        return np.where((x // 4 + y // 4) % 2, 1023, 0)
    if pattern == "stripes":
        return np.where((x // 2) % 2, 1023, 0)
    if pattern == "binary_noise":
        return np.random.default_rng(7).integers(0, 2, (h, w)) * 1023
    if pattern == "lattice8":  # dark frame, bright lines every 8 samples
        return np.where((x % 8 == 7) | (y % 8 == 5), 1023, 0)
    return np.full((h, w), 1023 if pattern == "white" else 0)


@pytest.mark.parametrize("pattern", ["checker1", "checker4", "stripes", "binary_noise", "lattice8", "white", "black"])
def test_extreme_content_clipping(gpu_available, pattern):
    """0/1023 patterns drive the unclipped MIP predictions far outside [0, 1023] (both
    clipping directions of intra.cl:481-482 and the saturating conversion in phase A)."""
    w, h = 192, 136
    frame = _extreme(pattern, w, h).astype(np.uint16)
    with MipEngine(w, h, want_sad_satd=True) as eng:
        out = eng.search(frame, sad_satd=True)
    O.clip_counts(reset=True)
    oc, osad, osatd = O.search(frame, want_sad_satd=True)
    low, high = O.clip_counts()
    if pattern not in ("white", "black"):
        assert low > 0 and high > 0, (low, high)
    assert np.array_equal(out["cost"][0], oc)
    assert np.array_equal(out["sad"][0], osad)
    assert np.array_equal(out["satd"][0], osatd)


def test_8k_alt_int_whole_table(gpu_available):
    """BASELINE configs[4]: one 7680x4320 frame per GPU with alternative references
    (filterFrame_2d_int_quarterCtu, KernelIdx 0), "integer bit-exact at 8K".  The reference
    cannot search the whole frame in one run -- its int32 reduced-prediction index overflows
    (2040 CTUs x 2 231 296 entries > 2^31, intra.cl:519-537) -- so it ran as overlapping
    crops of <= 960 CTUs (tests/golden/c6_4320p_alt_int.json, tools/ref_golden_8k.py): the
    whole filtered frame and the WHOLE cost table (all 2040 CTUs, 199.6 M entries) must equal
    the oracle bit for bit and, on the entries the reference defines, the stitched reference
    table; the decisions-only path must give the table's argmin."""
    w, h, filt = 7680, 4320, "filterFrame_2d_int_quarterCtu"
    frame = synth_frame(w, h, 0x8E, 1)
    with MipEngine(w, h, filter=filt, kernel_idx=0) as eng:
        out = eng.search(frame, best=True)
        dec = eng.search(frame, costs=False, best=True)
        got_refs = eng.filter_frames(frame, filt, 0)[0]
    assert np.array_equal(got_refs, O.filter_frame(frame, filt, 0))
    want = O.engine_search(frame, filt, 0)
    assert np.array_equal(out["cost"][0], want)
    if "c6_4320p_alt_int" in G.names():  # the reference's own kernels (stitched crops)
        fx = G.load("c6_4320p_alt_int")
        assert (fx["config"]["seed"], fx["config"]["kind"]) == (0x8E, 1)
        _, und, mask = G.refs_and_mask(fx, frame[None], 0)
        fr = fx["frames"][0]
        assert G.sha(G.masked(out["cost"][0], mask)) == fr["cost_sha256"]
        assert G.filtered_sha(got_refs, und) == fr["filtered_sha256"]
        for ctu in map(int, fr["ctu_rows"]):
            sl = slice(ctu * 97840, (ctu + 1) * 97840)
            assert np.array_equal(G.masked(out["cost"][0][sl], mask[sl]), G.ctu_row(fx, 0, ctu)), ctu
    bm, bc = layout.best_modes(want, layout.num_ctus(w, h))
    assert np.array_equal(out["best_mode"][0], bm) and np.array_equal(out["best_cost"][0], bc)
    assert np.array_equal(dec["best_mode"][0], bm) and np.array_equal(dec["best_cost"][0], bc)


def test_4k_four_frame_batch_each_frame(gpu_available):
    """BASELINE configs[3]'s per-GPU share: 4 frames of 3840x2160 (original references) in ONE
    device launch (the bench's resident-frame path), every frame's whole table checked against
    the oracle, and the same frames searched one per launch give the same tables."""
    import torch
    w, h, n = 3840, 2160, 4
    frames = synth_frames(w, h, n, 0x4F40, 0)
    frames[3] = synth_frame(w, h, 0x4F44, 1)  # one uniform-noise frame in the batch
    d = torch.from_numpy(frames.astype(np.int16)).cuda()
    with MipEngine(w, h, max_batch=n) as eng:
        batch = eng.search_device(d).cpu().numpy()
        single = [eng.search_device(d[f:f + 1]).cpu().numpy()[0] for f in range(n)]
        eng.check_input()
    for f in range(n):
        want = O.search(frames[f])
        assert np.array_equal(batch[f], want), f
        assert np.array_equal(single[f], want), f


@pytest.mark.parametrize("filt,k", [(None, 0), ("filterFrame_2d_float_5x5_quarterCtu", 2)])
def test_host_pipeline_four_slots_uneven_chunks(gpu_available, filt, k):
    """mip_search_frames with max_batch >= 16: 4 engine buffer slots over 2 streams, chunks
    of max_batch/4 frames, an uneven last chunk (19 frames = 4+4+4+4+3), all outputs.
    Every frame must equal the device API on the same frames and the oracle."""
    import torch
    w, h, n = 264, 136, 19
    frames = synth_frames(w, h, n, 0x4F0, 0)
    with MipEngine(w, h, max_batch=16, filter=filt, kernel_idx=k, want_sad_satd=True) as eng:
        host = eng.search(frames, best=True, sad_satd=True)
        d = torch.from_numpy(frames.astype(np.int16)).cuda()
        dev = np.concatenate([eng.search_device(d[:16]).cpu().numpy(), eng.search_device(d[16:]).cpu().numpy()])
    assert np.array_equal(host["cost"], dev)
    nct = layout.num_ctus(w, h)
    for f in range(n):
        oc, osad, osatd = O.engine_search(frames[f], filt, k, want_sad_satd=True)
        assert np.array_equal(host["cost"][f], oc), f
        assert np.array_equal(host["sad"][f], osad), f
        assert np.array_equal(host["satd"][f], osatd), f
        bm, bc = layout.best_modes(oc, nct)
        assert np.array_equal(host["best_mode"][f], bm), f
        assert np.array_equal(host["best_cost"][f], bc), f


@pytest.mark.parametrize("filt,k", [(None, 0), ("filterFrame_2d_float_5x5_quarterCtu", 2)])
def test_host_pipeline_ramped_first_chunks(gpu_available, filt, k):
    """A call into an idle pipeline with max_batch 64 (4 slots of 16 frames) ramps its first
    chunks up (4, 7, 12 frames, then 14 + 14 + 13: mipgpu.cpp search_frames_chunks), a call
    queued behind it does not; full tables + decisions, then decisions only.  Every frame must
    equal the oracle."""
    w, h, n = 136, 72, 64
    frames = synth_frames(w, h, n, 0x7A3, 0)
    nct = layout.num_ctus(w, h)
    want = [O.engine_search(frames[f], filt, k) for f in range(n)]
    with MipEngine(w, h, max_batch=n, filter=filt, kernel_idx=k) as eng:
        t1 = eng.search_async(frames, best=True)
        t2 = eng.search_async(frames[::-1].copy(), best=True)
        r1, r2 = eng.wait(t1), eng.wait(t2)
        dec = eng.search(frames, costs=False, best=True)
    for f in range(n):
        bm, bc = layout.best_modes(want[f], nct)
        assert np.array_equal(r1["cost"][f], want[f]), f
        assert np.array_equal(r2["cost"][n - 1 - f], want[f]), f
        assert np.array_equal(r1["best_mode"][f], bm), f
        assert np.array_equal(dec["best_mode"][f], bm), f
        assert np.array_equal(dec["best_cost"][f], bc), f


def test_engine_filter_scratch_shared_by_two_streams(gpu_available):
    """Device-API searches that filter into the engine's reference scratch (no caller
    references) on two streams, with different frames per launch: each launch must wait
    for the previous reader of the scratch (refs_done), so every table matches the oracle;
    a host-API call in between must wait as well."""
    import torch
    filt, k = "filterFrame_2d_float_5x5_quarterCtu", 2
    w, h = 264, 200
    frames = synth_frames(w, h, 4, 0x5C, 0)
    want = np.stack([O.engine_search(frames[f], filt, k) for f in range(4)])
    d = torch.from_numpy(frames.astype(np.int16)).cuda()
    pairs = [d[[f0, (f0 + 1) % 4]].contiguous() for f0 in range(4)]
    torch.cuda.synchronize()  # the gathers ran on the current stream
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    with MipEngine(w, h, max_batch=2, filter=filt, kernel_idx=k) as eng:
        outs = []
        for i in range(24):
            f0 = (i * 3) % 4
            sel = [f0, (f0 + 1) % 4]
            outs.append((sel, eng.search_device(pairs[f0], stream=streams[i % 2])))
            if i == 11:
                mid = eng.search(frames[2:4])["cost"]
        torch.cuda.synchronize()
        for sel, c in outs:
            assert np.array_equal(c.cpu().numpy(), want[sel])
        assert np.array_equal(mid, want[2:4])


def test_host_pipeline_decisions_only_with_caller_refs(gpu_available):
    """mip_search_frames with two buffer slots (max_batch 4: chunks of 2 frames), caller
    references uploaded through the pipeline next to the frames, 7 frames (slots reused,
    uneven last chunk) and decisions only (no cost-table download): each slot's upload must
    wait for the previous search of that slot, each search for its upload."""
    w, h, n = 256, 136, 7
    frames = synth_frames(w, h, n, 0x7D1, 0)
    refs = synth_frames(w, h, n, 0x7D2, 0)
    with MipEngine(w, h, max_batch=4) as eng:
        out = eng.search(frames, refs=refs, costs=False, best=True)
    assert "cost" not in out
    nct = layout.num_ctus(w, h)
    for f in range(n):
        bm, bc = layout.best_modes(O.search(frames[f], refs[f]), nct)
        assert np.array_equal(out["best_mode"][f], bm), f
        assert np.array_equal(out["best_cost"][f], bc), f


def test_async_host_calls_in_flight(gpu_available):
    """mip_search_frames_async: four calls queued back to back (different frames, outputs
    and reference sources; slots reused across calls) complete in order with the oracle's
    tables; waiting for an earlier ticket after a later one is a no-op; unknown tickets are
    errors."""
    w, h = 256, 136
    frames = synth_frames(w, h, 9, 0xA51, 0)
    refs = synth_frames(w, h, 3, 0xA52, 0)
    nct = layout.num_ctus(w, h)
    with MipEngine(w, h, max_batch=4) as eng:
        t1 = eng.search_async(frames[0:3], best=True)
        t2 = eng.search_async(frames[3:5], costs=False, best=True)
        t3 = eng.search_async(frames[5:8], refs=refs)
        t4 = eng.search_async(frames[8:9])
        o4 = eng.wait(t4)
        o1, o2, o3 = eng.wait(t1), eng.wait(t2), eng.wait(t3)
        with pytest.raises(MipError):
            eng.wait(type(t4)(t4.value + 1, {}, None))
    for f in range(3):
        oc = O.search(frames[f])
        assert np.array_equal(o1["cost"][f], oc), f
        assert np.array_equal(o1["best_mode"][f], layout.best_modes(oc, nct)[0]), f
    for f in range(2):
        bm, bc = layout.best_modes(O.search(frames[3 + f]), nct)
        assert np.array_equal(o2["best_mode"][f], bm) and np.array_equal(o2["best_cost"][f], bc), f
    for f in range(3):
        assert np.array_equal(o3["cost"][f], O.search(frames[5 + f], refs[f])), f
    assert np.array_equal(o4["cost"][0], O.search(frames[8]))


def test_pageable_and_pinned_host_buffers_agree(gpu_available):
    """mip_search_frames with pageable (numpy) buffers -- staged through the engine's
    page-locked bounce ring -- and with page-locked buffers give identical outputs; several
    asynchronous calls with pageable outputs are in flight at once (ring pieces recycled
    across calls, copied out by wait)."""
    from mipgpu import pinned_empty
    w, h, n = 392, 264, 21
    frames = synth_frames(w, h, n, 0x9A6, 0)
    with MipEngine(w, h, max_batch=16, want_sad_satd=True) as eng:
        pf = pinned_empty(frames.shape, np.uint16)
        pf[:] = frames
        out = {k: pinned_empty((n, eng.costs_per_frame), np.int32) for k in ("cost", "sad", "satd")}
        out.update(best_mode=pinned_empty((n, eng.cus_per_frame), np.uint8),
                   best_cost=pinned_empty((n, eng.cus_per_frame), np.int32))
        pinned = eng.search(pf, best=True, sad_satd=True, out=out)
        paged = eng.search(frames, best=True, sad_satd=True)
        tickets = [eng.search_async(frames[i:i + 7], best=True) for i in range(0, n, 7)]
        parts = [eng.wait(t) for t in tickets]
    for k in ("cost", "sad", "satd", "best_mode", "best_cost"):
        assert np.array_equal(pinned[k], paged[k]), k
    assert np.array_equal(np.concatenate([p["cost"] for p in parts]), pinned["cost"])
    assert np.array_equal(np.concatenate([p["best_mode"] for p in parts]), pinned["best_mode"])
    assert np.array_equal(pinned["cost"][3], O.search(frames[3]))


def test_async_calls_with_different_chunk_sizes(gpu_available):
    """Asynchronous host calls whose chunk sizes differ (call lengths 5 / 7 / 3 / 11 frames are
    cut into equal chunks of up to a slot's 4 frames; decisions-only and full-table calls
    interleaved) all in flight at once: every chunk uses its slot's fixed region of the engine
    buffers, ordered by the slot's events, so each call's outputs equal a synchronous search
    of the same frames."""
    w, h = 392, 264
    frames = synth_frames(w, h, 26, 0xC5A, 0)
    with MipEngine(w, h, max_batch=16, want_sad_satd=True) as eng:
        want = eng.search(frames, best=True, sad_satd=True)
        spans = [(0, 5, "full"), (5, 12, "dec"), (12, 15, "sad"), (15, 26, "dec"), (0, 11, "full")]
        tickets = []
        for a0, a1, kind in spans:
            if kind == "dec":
                tickets.append(eng.search_async(frames[a0:a1], costs=False, best=True))
            else:
                tickets.append(eng.search_async(frames[a0:a1], best=True, sad_satd=kind == "sad"))
        outs = [eng.wait(t) for t in tickets]
    for (a0, a1, kind), o in zip(spans, outs):
        assert np.array_equal(o["best_mode"], want["best_mode"][a0:a1]), (a0, a1, kind)
        assert np.array_equal(o["best_cost"], want["best_cost"][a0:a1]), (a0, a1, kind)
        if kind != "dec":
            assert np.array_equal(o["cost"], want["cost"][a0:a1]), (a0, a1, kind)
        if kind == "sad":
            assert np.array_equal(o["sad"], want["sad"][a0:a1]) and np.array_equal(o["satd"], want["satd"][a0:a1])
    assert np.array_equal(want["cost"][7], O.search(frames[7]))


def test_dropped_ticket_waits(gpu_available):
    """A search_async ticket dropped without wait(): its finaliser waits, so the output and
    input arrays it keeps alive are not freed while the engine's copies use them; the
    engine stays usable."""
    import gc
    w, h = 256, 136
    frames = synth_frames(w, h, 4, 0xD70, 0)
    with MipEngine(w, h, max_batch=2) as eng:
        for _ in range(3):
            eng.search_async(frames)  # dropped at once
        gc.collect()
        assert np.array_equal(eng.search(frames[1])["cost"][0], O.search(frames[1]))


def test_async_host_calls_and_device_filter_scratch(gpu_available):
    """An engine with a filter: asynchronous host calls (filtering into the reference
    scratch per slot) in flight while a device-API search filters into the same scratch on
    another stream -- the device search waits for the host pipeline, every table matches."""
    import torch
    filt, k = "filterFrame_2d_int_quarterCtu", 1
    w, h = 264, 136
    frames = synth_frames(w, h, 6, 0xA61, 0)
    want = np.stack([O.engine_search(frames[f], filt, k) for f in range(6)])
    d = torch.from_numpy(frames[4:6].astype(np.int16)).cuda()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with MipEngine(w, h, max_batch=2, filter=filt, kernel_idx=k) as eng:
        t1 = eng.search_async(frames[0:2])
        t2 = eng.search_async(frames[2:4])
        dc = eng.search_device(d, stream=s)
        o1, o2 = eng.wait(t1), eng.wait(t2)
        torch.cuda.synchronize()
        assert np.array_equal(dc.cpu().numpy(), want[4:6])
    assert np.array_equal(o1["cost"], want[0:2])
    assert np.array_equal(o2["cost"], want[2:4])


@pytest.mark.parametrize("w,h,filt,k", [(264, 200, None, 0), (136, 72, None, 0),
                                        (392, 264, "filterFrame_2d_float_5x5_quarterCtu", 2),
                                        (416, 240, "filterFrame_1d_int_5x5", 2)])
def test_device_decisions_only_fused_argmin(gpu_available, w, h, filt, k):
    """mip_search_device without a cost table (costs=False): a task with all of a CU's mode
    pairs writes the CU's decision directly; tasks that cut a CU's pairs meet in a packed
    argmin (cost << 5 | mode, atomicMin) unpacked after the launch; undefined CUs are written
    from the decisions-only fill lists.  Must equal the argmin of the oracle's table (ties to
    the lower mode, unavailable CUs 0xff / MIP_COST_UNAVAILABLE) on every entry (outputs start
    as a sentinel: an entry nobody writes fails), for 1..3-frame batches (different task cuts
    per slice count).  416x240 with a separable filter: reference samples above 10 bits in the
    last columns (the exact per-CU kernel's CUs write their decision directly)."""
    import torch
    n = 3
    frames = synth_frames(w, h, n, 0xD0 + w, 1)
    if w == 416:
        assert max(O.filter_frame(frames[f], filt, k).max() for f in range(n)) > 1023
    nct = layout.num_ctus(w, h)
    want = []
    for f in range(n):
        want.append(layout.best_modes(O.engine_search(frames[f], filt, k), nct))
    d = torch.from_numpy(frames.astype(np.int16)).cuda()
    with MipEngine(w, h, max_batch=n, filter=filt, kernel_idx=k) as eng:
        for nb in (1, 2, 3):
            bm = torch.full((nb, eng.cus_per_frame), 0x5a, dtype=torch.uint8, device="cuda")
            bc = torch.full((nb, eng.cus_per_frame), -5, dtype=torch.int32, device="cuda")
            assert eng.search_device(d[:nb], costs=False, best_mode=bm, best_cost=bc) is None
            torch.cuda.synchronize()
            for f in range(nb):
                assert np.array_equal(bm[f].cpu().numpy(), want[f][0]), (nb, f)
                assert np.array_equal(bc[f].cpu().numpy(), want[f][1]), (nb, f)
        with pytest.raises(MipError):  # the packed argmin needs the cost output as scratch
            eng.search_device(d[:1], costs=False, best_mode=bm[:1])


@pytest.mark.parametrize("w,h,filt,k", [(392, 264, None, 0), (416, 240, "filterFrame_1d_int_5x5", 2)])
def test_transposed_classes_equal_direct_search(gpu_available, monkeypatch, w, h, filt, k):
    """Wide single-direction CUs (32x4, 16x4, 8x4, 32x8, 16x8) are searched as their tall
    transposes (transposed classes, mip_kernels.h).  Engines built with MIPGPU_TRANSPOSE=0
    (searched as they are) and =1 (default) must give identical cost / SAD / SATD tables and
    decisions, equal to the oracle's; partial CTUs on both axes and, at 416x240 with a
    separable filter, the fixup CUs."""
    frames = synth_frames(w, h, 2, 0x7A + w, 1)
    out = {}
    for t in ("0", "1"):
        monkeypatch.setenv("MIPGPU_TRANSPOSE", t)
        with MipEngine(w, h, max_batch=2, filter=filt, kernel_idx=k, want_sad_satd=True) as eng:
            out[t] = eng.search(frames, best=True, sad_satd=True)
            out[t + "dec"] = eng.search(frames, costs=False, best=True)
    for key in ("cost", "sad", "satd", "best_mode", "best_cost"):
        assert np.array_equal(out["0"][key], out["1"][key]), key
    for key in ("best_mode", "best_cost"):
        assert np.array_equal(out["0dec"][key], out["1"][key]), key
    for f in range(2):
        cost, sad, satd = O.engine_search(frames[f], filt, k, want_sad_satd=True)
        assert np.array_equal(out["1"]["cost"][f], cost)
        assert np.array_equal(out["1"]["sad"][f], sad) and np.array_equal(out["1"]["satd"][f], satd)


@pytest.mark.parametrize("slices", [1, 2, 3, 4])
def test_slice_counts_agree(gpu_available, slices):
    """Engines with a fixed number of workgroups per CTU quadrant (mip_opts.slices_per_ctu:
    the task lists are cut into more pair ranges, so more CUs are split over tasks -- the
    decisions-only path's packed atomicMin entries) give the oracle's tables and argmins,
    with alternative references (fixup CUs) at a width that is not a multiple of 128."""
    w, h, filt, k = 416, 240, "filterFrame_2d_int_quarterCtu", 1
    frames = synth_frames(w, h, 2, 0x51C + slices, 1)
    with MipEngine(w, h, max_batch=2, filter=filt, kernel_idx=k, slices_per_ctu=slices) as eng:
        full = eng.search(frames, best=True)
        dec = eng.search(frames, costs=False, best=True)
    for f in range(2):
        cost = O.engine_search(frames[f], filt, k)
        assert np.array_equal(full["cost"][f], cost), f
        bm, bc = layout.best_modes(cost, layout.num_ctus(w, h))
        assert np.array_equal(dec["best_mode"][f], bm) and np.array_equal(dec["best_cost"][f], bc), f


def test_decisions_only_full_size_matches_table_argmin(gpu_available):
    """1080p (the bench size), 2 frames: the fused decisions-only search gives exactly the
    decision lists of the full cost table (best_mode_kernel over it)."""
    W, H = 1920, 1080
    frames = synth_frames(W, H, 2, 0xDEC, 0)
    with MipEngine(W, H, max_batch=2) as eng:
        full = eng.search(frames, best=True)
        dec = eng.search(frames, costs=False, best=True)
    assert "cost" not in dec
    assert np.array_equal(dec["best_mode"], full["best_mode"])
    assert np.array_equal(dec["best_cost"], full["best_cost"])
    bm, bc = layout.best_modes(full["cost"][1], layout.num_ctus(W, H))
    assert np.array_equal(dec["best_mode"][1], bm) and np.array_equal(dec["best_cost"][1], bc)


def test_prefetching_launch_equals_small_launches(gpu_available):
    """Launches with >= 32 items per workgroup run the prefetching kernel variant (next item's
    window staged by the first idle wave, late takes in the last rounds; mip_search.hip).
    34 1080p frames in one launch (18 360 items) must give exactly the tables of the same
    frames searched two at a time (the non-prefetching variant, pinned to the oracle by the
    other tests), and the decisions-only variant of the big launch the argmin of its table."""
    import torch
    from mipgpu import topk_device
    W, H, n = 1920, 1080, 34
    frames = torch.from_numpy(synth_frames(W, H, n, 0x9F0, 0).astype(np.int16)).cuda()
    with MipEngine(W, H, max_batch=n) as eng:
        big = eng.search_device(frames)
        small = torch.empty_like(big)
        for f in range(0, n, 2):
            eng.search_device(frames[f:f + 2], costs=small[f:f + 2])
        bm = torch.full((n, eng.cus_per_frame), 0x5a, dtype=torch.uint8, device="cuda")
        bc = torch.full((n, eng.cus_per_frame), -5, dtype=torch.int32, device="cuda")
        eng.search_device(frames, costs=False, best_mode=bm, best_cost=bc)
        tm, tc = topk_device(big, W, H, 1)
        torch.cuda.synchronize()
        assert torch.equal(big, small)
        assert torch.equal(bm, tm[..., 0]) and torch.equal(bc, tc[..., 0])


def test_tickets_dropped_on_another_thread(gpu_available):
    """_Ticket.__del__ waits for its call (mip_wait drains the engine's bounce ring): tickets
    dropped on a second thread while the first thread runs searches on the same engine are
    serialised by the engine's lock; every result stays the oracle's."""
    import gc
    import threading
    w, h = 264, 136
    frames = synth_frames(w, h, 4, 0x7E1, 0)
    want = np.stack([O.search(frames[f]) for f in range(4)])
    errors = []
    with MipEngine(w, h, max_batch=4) as eng:
        def dropper():
            try:
                for i in range(20):
                    t = eng.search_async(frames[i % 4:i % 4 + 1])  # pageable output: ring drained by wait
                    del t
                    gc.collect()
            except Exception as exc:  # noqa: BLE001
                errors.append(exc)
        th = threading.Thread(target=dropper)
        th.start()
        for i in range(10):
            out = eng.search(frames)
            assert np.array_equal(out["cost"], want), i
        th.join()
    assert not errors, errors


@pytest.mark.parametrize("w,h,n,filt,k", [(1920, 1080, 1, None, 0), (416, 240, 3, "filterFrame_2d_int_quarterCtu", 1),
                                          (264, 136, 2, None, 0)])
def test_small_launch_shapes_agree(gpu_available, monkeypatch, w, h, n, filt, k):
    """Small launches run one 16-wave workgroup per CU below 4 items
    per CU (MIPGPU_WIDE; mip_search_kernel<..., 16>) -- with original references and the
    longest-first order two items at a time (pair mode, MIPGPU_PAIR; the fill-only items
    ride along) -- and 8-wave workgroups above, with the items longest first or in raster
    order (MIPGPU_ORDER).  The knobs are read per launch (mipgpu.cpp wide_launch,
    lpt_order_enabled, the pair knob): one engine runs every combination, and every
    combination must give the same cost / SAD / SATD tables and decisions (full table and
    fused decisions-only), equal to the oracle's."""
    frames = synth_frames(w, h, n, 0x5A11 + w, 1)
    outs = []
    with MipEngine(w, h, max_batch=n, filter=filt, kernel_idx=k, want_sad_satd=True) as eng:
        for wide, pair, order in (("1", "1", "1"), ("1", "0", "1"), ("0", "1", "1"), ("1", "1", "0"),
                                  ("0", "1", "0")):
            monkeypatch.setenv("MIPGPU_WIDE", wide)
            monkeypatch.setenv("MIPGPU_PAIR", pair)
            monkeypatch.setenv("MIPGPU_ORDER", order)
            full = eng.search(frames, best=True, sad_satd=True)
            dec = eng.search(frames, costs=False, best=True)
            outs.append(((wide, pair, order), full, dec))
    ref = outs[0][1]
    for knobs, full, dec in outs:
        for key in ("cost", "sad", "satd", "best_mode", "best_cost"):
            assert np.array_equal(full[key], ref[key]), (knobs, key)
        for key in ("best_mode", "best_cost"):
            assert np.array_equal(dec[key], ref[key]), (knobs, "dec", key)
    cost, sad, satd = O.engine_search(frames[n - 1], filt, k, want_sad_satd=True)
    assert np.array_equal(ref["cost"][n - 1], cost)
    assert np.array_equal(ref["sad"][n - 1], sad) and np.array_equal(ref["satd"][n - 1], satd)


@pytest.mark.parametrize("w,filt,k", [(264, None, 0), (256, "filterFrame_2d_float_5x5_quarterCtu", 2)])
def test_per_frame_calls_triple_buffered(gpu_available, w, filt, k):
    """The drop-in's per-frame loop (main.cpp:678-1241 searches one frame per iteration):
    default options (max_batch 1: three one-frame buffer slots), ten asynchronous one-frame
    calls in flight at once with mixed outputs -- full table + decisions, decisions only,
    caller references, page-locked and pageable buffers -- each equal to the oracle."""
    from mipgpu import pinned_empty
    h = 136
    frames = synth_frames(w, h, 10, 0xF1A, 0)
    refs = synth_frames(w, h, 10, 0xF1B, 0)
    nct = layout.num_ctus(w, h)
    kinds = ["full", "dec", "refs", "pinned_dec", "full", "refs_dec", "dec", "pinned_full", "full", "dec"]
    with MipEngine(w, h, filter=filt, kernel_idx=k) as eng:
        assert eng.max_batch == 1
        tickets = []
        for i, kind in enumerate(kinds):
            f = frames[i:i + 1]
            if kind.startswith("pinned"):
                pf = pinned_empty(f.shape, np.uint16)
                pf[:] = f
                f = pf
            r = refs[i:i + 1] if kind.startswith("refs") else None
            if kind.endswith("dec"):
                tickets.append(eng.search_async(f, refs=r, costs=False, best=True))
            else:
                tickets.append(eng.search_async(f, refs=r, best=True))
        outs = [eng.wait(t) for t in tickets]
    for i, (kind, o) in enumerate(zip(kinds, outs)):
        if kind.startswith("refs"):
            oc = O.search(frames[i], refs[i])
        elif filt is None:
            oc = O.search(frames[i])
        else:
            oc = O.search(frames[i], O.filter_frame(frames[i], filt, k))
        bm, bc = layout.best_modes(oc, nct)
        if "cost" in o:
            assert np.array_equal(o["cost"][0], oc), (i, kind)
        assert np.array_equal(o["best_mode"][0], bm), (i, kind)
        assert np.array_equal(o["best_cost"][0], bc), (i, kind)


def test_per_frame_pipeline_stress_1080p(gpu_available):
    """Ordering of the host pipeline's three streams under load at the bench size: 48
    asynchronous one-frame 1080p calls in flight (three buffer slots reused 16 times each;
    decisions only and full tables interleaved, page-locked buffers), frames drawn from a pool
    of four -- every call's outputs equal a synchronous search of the same frame (a slot read
    before its upload landed, or downloaded before its search finished, would show as a
    mismatch)."""
    from mipgpu import pinned_empty
    W, H = 1920, 1080
    pool = synth_frames(W, H, 4, 0x5F1, 0)
    with MipEngine(W, H, max_batch=4) as ref_eng:
        want = ref_eng.search(pool, best=True)
    with MipEngine(W, H) as eng:
        pf = pinned_empty(pool.shape, np.uint16)
        pf[:] = pool
        tickets, kinds = [], []
        for i in range(48):
            f = pf[i % 4:i % 4 + 1]
            if i % 6 == 5:
                out = {"cost": pinned_empty((1, eng.costs_per_frame), np.int32),
                       "best_mode": pinned_empty((1, eng.cus_per_frame), np.uint8),
                       "best_cost": pinned_empty((1, eng.cus_per_frame), np.int32)}
                tickets.append(eng.search_async(f, best=True, out=out))
                kinds.append("full")
            else:
                out = {"best_mode": pinned_empty((1, eng.cus_per_frame), np.uint8),
                       "best_cost": pinned_empty((1, eng.cus_per_frame), np.int32)}
                tickets.append(eng.search_async(f, costs=False, best=True, out=out))
                kinds.append("dec")
        outs = [eng.wait(t) for t in tickets]
    for i, (kind, o) in enumerate(zip(kinds, outs)):
        j = i % 4
        assert np.array_equal(o["best_mode"][0], want["best_mode"][j]), (i, kind)
        assert np.array_equal(o["best_cost"][0], want["best_cost"][j]), (i, kind)
        if kind == "full":
            assert np.array_equal(o["cost"][0], want["cost"][j]), i


@pytest.mark.parametrize("max_batch,n", [(1, 3), (1, 5), (4, 9), (4, 13)])
def test_idle_call_chunks_fit_their_slot(gpu_available, max_batch, n):
    """Small engines (max_batch < 16: three slots of max_batch frames) cut a call into an idle
    pipeline in two -- but never into chunks larger than a slot (a call of more
    than 2 x max_batch frames had spilled into the next slot's region).  Calls start at every
    slot offset (0, 1 or 2 earlier one-frame chunks), so the first chunk lands in each slot,
    incl. the last one; full tables + decisions, then decisions only; every frame equals the
    oracle."""
    w, h = 264, 136
    frames = synth_frames(w, h, n, 0x1DC + 7 * max_batch + n, 0)
    nct = layout.num_ctus(w, h)
    want = [O.search(frames[f]) for f in range(n)]
    for offset in range(3):
        with MipEngine(w, h, max_batch=max_batch) as eng:
            for i in range(offset):  # host_chunks = offset before the call under test
                eng.search(frames[i:i + 1], costs=False, best=True)
            full = eng.search(frames, best=True)
            dec = eng.search(frames, costs=False, best=True)
        for f in range(n):
            bm, bc = layout.best_modes(want[f], nct)
            assert np.array_equal(full["cost"][f], want[f]), (offset, f)
            assert np.array_equal(full["best_mode"][f], bm), (offset, f)
            assert np.array_equal(dec["best_mode"][f], bm) and np.array_equal(dec["best_cost"][f], bc), (offset, f)


@pytest.mark.parametrize("filt,k,pk,gather", [(None, 0, "4", "1"), ("filterFrame_2d_float_5x5_quarterCtu", 2, "4", "1"),
                                              (None, 0, "6", "1"), (None, 0, "0", "0")])
def test_merged_launches_keep_each_call_its_own(gpu_available, monkeypatch, filt, k, pk, gather):
    """Merged launches (mipgpu.cpp open chunk, ABI 7): small page-locked calls share one search
    launch.  MIPGPU_MERGE=hold makes the grouping deterministic (chunks open even into an idle
    pipeline and are launched only by the other triggers): four decisions-only calls, three
    full-table calls, caller references (1 + 2 frames), then four decisions-only calls of which
    one holds a sample above 1023, then an 8-frame call (a whole slot: not merged).  Every call
    equals the oracle, the bad call -- and only it -- fails at its own wait, and the counters
    show exactly four merged launches of 13 calls.  pk: the kernel of these small alternating
    chunks (MIPGPU_PIPE_KERNEL: 4 the four-wave twin, 6 the six-wave kernel on half the grid,
    0 its full grid) -- the per-frame status pointers work in each; gather: the merged
    decisions-only downloads as one copy kernel (default) or one copy per member buffer."""
    from mipgpu import pinned_empty
    monkeypatch.setenv("MIPGPU_MERGE", "hold")
    monkeypatch.setenv("MIPGPU_PIPE_KERNEL", pk)
    monkeypatch.setenv("MIPGPU_GATHER_DOWN", gather)  # merged decisions-only downloads: one copy kernel / per member
    w, h = 264, 136
    n = 23
    frames = synth_frames(w, h, n, 0x3E6 + (k or 0), 0)
    refs = synth_frames(w, h, 3, 0x3E7, 0)
    bad = 14  # frame of the bad call
    pf = pinned_empty(frames.shape, np.uint16)
    pf[:] = frames
    pf[bad, 40, 77] = 1024
    pr = pinned_empty(refs.shape, np.uint16)
    pr[:] = refs
    nct = layout.num_ctus(w, h)

    def outs(nf, full):
        o = {"best_mode": pinned_empty((nf, nct * layout.CUS_PER_CTU), np.uint8),
             "best_cost": pinned_empty((nf, nct * layout.CUS_PER_CTU), np.int32)}
        if full:
            o["cost"] = pinned_empty((nf, nct * layout.COSTS_PER_CTU), np.int32)
        return o
    # (first frame, frames, kind): dec / full / refs (full table, caller references)
    calls = [(0, 1, "dec"), (1, 1, "dec"), (2, 1, "dec"), (3, 1, "dec"),
             (4, 1, "full"), (5, 1, "full"), (6, 1, "full"),
             (7, 1, "refs"), (8, 2, "refs"),
             (12, 1, "dec"), (bad, 1, "dec"), (13, 1, "dec"), (10, 1, "dec"),
             (15, 8, "dec")]
    with MipEngine(w, h, max_batch=8, filter=filt, kernel_idx=k) as eng:
        tickets = []
        for f0, nf, kind in calls:
            r = pr[f0 - 7:f0 - 7 + nf] if kind == "refs" else None
            tickets.append(eng.search_async(pf[f0:f0 + nf], refs=r, costs=kind != "dec", best=True,
                                            out=outs(nf, kind != "dec")))
        results = []
        for t in tickets:
            try:
                results.append(eng.wait(t))
            except MipError as exc:
                results.append(exc)
        stats = eng.host_stats()
    assert stats["merged_launches"] == 4 and stats["merged_calls"] == 13, stats
    assert stats["calls"] == len(calls) and stats["launches"] >= 5, stats
    for (f0, nf, kind), res in zip(calls, results):
        if f0 == bad:
            assert isinstance(res, MipError) and "above 10 bits" in str(res), res
            continue
        assert not isinstance(res, MipError), (f0, kind, res)
        for i in range(nf):
            f = f0 + i
            if kind == "refs":
                oc = O.search(frames[f], refs[f - 7])
            else:
                oc = O.engine_search(frames[f], filt, k)
            bm, bc = layout.best_modes(oc, nct)
            assert np.array_equal(res["best_mode"][i], bm), (f0, kind, i)
            assert np.array_equal(res["best_cost"][i], bc), (f0, kind, i)
            if kind != "dec":
                assert np.array_equal(res["cost"][i], oc), (f0, kind, i)


def test_merged_launches_1080p_default_policy(gpu_available, monkeypatch):
    """Default merge policy at the bench size: 24 one-frame 1080p calls queued back to back
    (page-locked, decisions only and full tables in runs) merge while the pipeline is busy;
    every output equals a synchronous search of the same frame.  Then a one-frame call queued
    behind a 4-frame call stays open after that search has completed, until mip_flush -- or
    the next call, which finds the GPU idle -- launches it.  The reference search runs the
    six-wave kernel throughout (MIPGPU_PIPE_KERNEL=0), the queued calls the four-wave twin
    (default for small alternating and decisions-only chunks): the two kernels agree."""
    import time
    from mipgpu import pinned_empty
    W, H = 1920, 1080
    pool = synth_frames(W, H, 4, 0x6E7, 0)
    monkeypatch.setenv("MIPGPU_PIPE_KERNEL", "0")
    with MipEngine(W, H, max_batch=4) as ref_eng:
        want = ref_eng.search(pool, best=True)
    monkeypatch.delenv("MIPGPU_PIPE_KERNEL")
    with MipEngine(W, H, max_batch=8) as eng:
        pf = pinned_empty(pool.shape, np.uint16)
        pf[:] = pool

        def outs(nf, full):
            o = {"best_mode": pinned_empty((nf, eng.cus_per_frame), np.uint8),
                 "best_cost": pinned_empty((nf, eng.cus_per_frame), np.int32)}
            if full:
                o["cost"] = pinned_empty((nf, eng.costs_per_frame), np.int32)
            return o
        kinds = [(i // 6) % 2 == 1 for i in range(24)]
        bufs = [outs(1, full) for full in kinds]  # (allocated before: the calls queue back to back)
        tickets = [eng.search_async(pf[i % 4:i % 4 + 1], costs=full, best=True, out=bufs[i])
                   for i, full in enumerate(kinds)]
        outs_ = [eng.wait(t) for t in tickets]
        s0 = eng.host_stats()
        assert s0["merged_calls"] >= 2 and s0["launches"] < s0["calls"], s0
        for i, (full, o) in enumerate(zip(kinds, outs_)):
            j = i % 4
            assert np.array_equal(o["best_mode"][0], want["best_mode"][j]), (i, full)
            assert np.array_equal(o["best_cost"][0], want["best_cost"][j]), (i, full)
            if full:
                assert np.array_equal(o["cost"][0], want["cost"][j]), i
        # an open chunk with the GPU idle: launched by mip_flush, or by the next call
        b4, b1, b1b, b1c = outs(4, False), outs(1, False), outs(1, False), outs(1, False)
        t4 = eng.search_async(pf, costs=False, best=True, out=b4)  # 4 frames of an 8-frame slot: launched
        t1 = eng.search_async(pf[2:3], costs=False, best=True, out=b1)  # busy: opens a chunk
        s_open = eng.host_stats()
        time.sleep(0.2)  # (the 4-frame search completes; the chunk stays open)
        assert eng.host_stats()["merged_launches"] == s_open["merged_launches"] == s0["merged_launches"]
        eng.flush()
        assert eng.host_stats()["merged_launches"] == s0["merged_launches"] + 1
        o4, o1 = eng.wait(t4), eng.wait(t1)
        assert np.array_equal(o4["best_mode"], want["best_mode"]) and np.array_equal(o1["best_cost"][0], want["best_cost"][2])
        t4 = eng.search_async(pf, costs=False, best=True, out=b4)
        t1 = eng.search_async(pf[1:2], costs=False, best=True, out=b1b)  # opens
        time.sleep(0.2)
        t2 = eng.search_async(pf[3:4], costs=False, best=True, out=b1c)  # finds the GPU idle: t1's chunk goes
        assert eng.host_stats()["merged_launches"] == s0["merged_launches"] + 2
        o4, o1, o2 = eng.wait(t4), eng.wait(t1), eng.wait(t2)
        assert np.array_equal(o4["best_cost"], want["best_cost"])
        assert np.array_equal(o1["best_mode"][0], want["best_mode"][1]) and np.array_equal(o2["best_mode"][0], want["best_mode"][3])


def test_engine_churn_reuses_parked_device_blocks(gpu_available):
    """Device block cache (mipgpu.cpp dev_malloc / dev_free): a destroyed engine's large buffers
    are parked, not freed (a large hipFree halves the process's later transfer rate,
    profiles/r06_free_repro.txt), and the next engine on the device takes them -- whose
    results stay exact although its buffers hold the previous engine's data (every output is
    written, the split accumulator re-initialised)."""
    from mipgpu import device_cache, pinned_empty
    W, H = 1920, 1080
    frames = synth_frames(W, H, 2, 0xC4C, 0)
    with MipEngine(W, H, max_batch=16) as big:
        want = big.search(frames, best=True)
        dec0 = big.search(frames, costs=False, best=True)
    assert np.array_equal(dec0["best_cost"], want["best_cost"])
    c0 = device_cache(0)
    assert c0["idle_bytes"] >= 16 * 135 * 97840 * 4 // 4, c0  # (at least the cost table's slots)
    pf = pinned_empty(frames.shape, np.uint16)
    pf[:] = frames
    with MipEngine(W, H, max_batch=2) as eng:
        c1 = device_cache(0)
        assert c1["reused_blocks"] > c0["reused_blocks"] and c1["idle_bytes"] < c0["idle_bytes"], (c0, c1)
        full = eng.search(pf, best=True)
        dec = eng.search(pf, costs=False, best=True)
    for k in ("cost", "best_mode", "best_cost"):
        assert np.array_equal(full[k], want[k]), k
    assert np.array_equal(dec["best_mode"], want["best_mode"]) and np.array_equal(dec["best_cost"], want["best_cost"])
    assert np.array_equal(want["cost"][1], O.search(frames[1]))
