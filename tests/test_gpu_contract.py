"""Input contract of the engine (include/mipgpu.h): samples are 10-bit.  The search kernel's
packed 16-bit / f16 arithmetic is exact for samples <= 1023 only, so a
staged sample above 1023 must fail the search loudly -- never come back as plausible-looking
costs.  The reference reads its CSV into unsigned short and its kernels take short*
(main.cpp:364-384, intra.cl:17, 545) with 10-bit constants (constants.cl:22-23)."""
import numpy as np
import pytest

import oracle_lib as O
from mipgpu import MipEngine, MipError
from mipgpu.synth import synth_frame, synth_frames

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("value", [1024, 4095, 65535])
def test_host_api_refuses_samples_above_10_bits(gpu_available, value):
    w, h = 264, 136
    frames = synth_frames(w, h, 3, 0xE10, 0)
    bad = frames.copy()
    bad[2, 100, 200] = value
    with MipEngine(w, h, max_batch=3) as eng:
        with pytest.raises(MipError, match="above 10 bits"):
            eng.search(bad)
        # reported once, then cleared: the engine goes on with valid frames
        out = eng.search(frames)
        assert np.array_equal(out["cost"][0], O.search(frames[0]))
        # decisions-only path (fused argmin, no table) checks too
        with pytest.raises(MipError, match="above 10 bits"):
            eng.search(bad, costs=False, best=True)
        # the last sample of the frame and the first one (window corners)
        for y, x in ((h - 1, w - 1), (0, 0)):
            b2 = frames[:1].copy()
            b2[0, y, x] = 2000
            with pytest.raises(MipError, match="above 10 bits"):
                eng.search(b2)
        # 1023 is in range
        ok = frames[:1].copy()
        ok[0, 5, 5] = 1023
        eng.search(ok)


def test_device_api_reports_at_check_or_next_call(gpu_available):
    import torch
    w, h = 256, 128
    frame = synth_frame(w, h, 0xE11, 1)
    bad = frame.copy()
    bad[64, 64] = 4095
    with MipEngine(w, h) as eng:
        d = torch.from_numpy(bad[None].astype(np.int16)).cuda()
        eng.search_device(d)
        with pytest.raises(MipError, match="above 10 bits"):
            eng.check_input()
        eng.check_input()  # cleared
        eng.search_device(d)
        torch.cuda.synchronize()
        with pytest.raises(MipError, match="above 10 bits"):  # the next search call reports it
            eng.search_device(torch.from_numpy(frame[None].astype(np.int16)).cuda())
        good = torch.from_numpy(frame[None].astype(np.int16)).cuda()
        c = eng.search_device(good)
        eng.check_input()
        assert np.array_equal(c.cpu().numpy()[0], O.search(frame))


def test_caller_references_are_checked(gpu_available):
    w, h = 256, 136
    frame = synth_frame(w, h, 0xE12, 0)
    refs = synth_frame(w, h, 0xE13, 1)
    refs[63, 100] = 3000  # a reference row (y = 4i - 1) the lattice stages
    with MipEngine(w, h) as eng:
        with pytest.raises(MipError, match="reference samples above 10 bits"):
            eng.search(frame, refs=refs)
        refs[63, 100] = 1000
        assert np.array_equal(eng.search(frame, refs=refs)["cost"][0], O.search(frame, refs))


def test_prefetching_launch_checks_the_prefetched_windows(gpu_available):
    """A launch large enough to prefetch windows (>= 32 items per workgroup: the staging wave
    of the previous item loads them): the bad sample is in a late frame."""
    import torch
    w, h, n = 1920, 1080, 34
    frames = torch.from_numpy(synth_frames(w, h, 2, 0xE14, 0).astype(np.int16)).cuda()
    batch = frames[torch.arange(n) % 2].clone()
    batch[29, 500, 700] = 1500
    with MipEngine(w, h, max_batch=n) as eng:
        costs = torch.empty((n, eng.costs_per_frame), dtype=torch.int32, device="cuda")
        eng.search_device(batch, costs=costs)
        with pytest.raises(MipError, match="above 10 bits"):
            eng.check_input()
        batch[29, 500, 700] = 15
        eng.search_device(batch, costs=costs)
        eng.check_input()


def test_contract_error_belongs_to_the_call_that_searched_it(gpu_available):
    """Per-call status (mip_wait reads only its own call's status set): three calls in flight,
    only the second holds a sample above 1023.  Its ticket fails -- whichever ticket is waited
    for first -- and the good calls' tickets succeed with the oracle's tables."""
    w, h = 256, 136
    frames = synth_frames(w, h, 3, 0xE15, 0)
    bad = frames[1:2].copy()
    bad[0, 70, 30] = 2047
    with MipEngine(w, h, max_batch=1) as eng:
        for order in ((2, 0, 1), (0, 1, 2), (1, 2, 0)):
            t = [eng.search_async(frames[0:1]), eng.search_async(bad), eng.search_async(frames[2:3])]
            for i in order:
                if i == 1:
                    with pytest.raises(MipError, match="above 10 bits"):
                        eng.wait(t[i])
                else:
                    out = eng.wait(t[i])
                    assert np.array_equal(out["cost"][0], O.search(frames[i])), (order, i)


def test_caller_reference_check_at_the_last_columns(gpu_available):
    """Caller-supplied references: frame columns W-2, W-1 are exempt from the 10-bit check only
    at widths that are not multiples of 128 (their CUs go to the exact 32-bit fixup kernel);
    at W = 256 a bad sample there is refused like anywhere else, at W = 264 it is searched
    exactly (oracle)."""
    frame256 = synth_frame(256, 136, 0xE16, 0)
    with MipEngine(256, 136) as eng:
        for y, x in ((63, 255), (63, 254), (63, 253)):  # row 63: the top row of CUs at y = 64
            refs = synth_frame(256, 136, 0xE17, 1)
            refs[y, x] = 1500
            with pytest.raises(MipError, match="reference samples above 10 bits"):
                eng.search(frame256, refs=refs)
    # (row 100 is no reference row, but column 263 = 4 * 66 - 1 is a left reference column)
    frame264 = synth_frame(264, 136, 0xE18, 0)
    with MipEngine(264, 136) as eng:
        for y, x in ((63, 263), (63, 262), (100, 263)):
            refs = synth_frame(264, 136, 0xE19, 1)
            refs[y, x] = 1500
            assert np.array_equal(eng.search(frame264, refs=refs)["cost"][0], O.search(frame264, refs)), (y, x)
        refs = synth_frame(264, 136, 0xE19, 1)
        refs[63, 261] = 1500  # column W-3: checked at every width
        with pytest.raises(MipError, match="reference samples above 10 bits"):
            eng.search(frame264, refs=refs)
