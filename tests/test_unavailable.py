"""mip_unavailable_cus (host only, no GPU): the CUs an engine reports as MIP_COST_UNAVAILABLE,
restated in the product (mipgpu.cpp filter_poison) from the reference's tile addressing,
against the oracle's model of the same (mipo_filter_frame_ex poison bit + mipo_ref_undefined_cus,
itself pinned by the fill experiment of tools/ref_golden.py)."""
import numpy as np
import pytest

import oracle_lib as O
from mipgpu import FILTERS, layout, unavailable_cus
from mipgpu.synth import synth_frame

SIZES = [(416, 240), (264, 136), (292, 36), (300, 68), (128, 4), (1280, 720), (256, 136), (832, 480), (4, 4), (132, 4), (4, 132), (8, 36)]


@pytest.mark.parametrize("w,h", SIZES)
@pytest.mark.parametrize("filt", [None] + list(FILTERS))
def test_unavailable_cus_match_the_oracle_model(w, h, filt):
    frame = synth_frame(w, h, 0x0A + w, 1)
    n = layout.num_ctus(w, h)
    got = layout.expand_cu_mask(unavailable_cus(w, h, filt), n)
    assert np.array_equal(got, O.engine_unavailable_mask(frame, filt, 0)), (w, h, filt)
    # never more than the reference leaves undefined (poison + race + geometry)
    if filt is not None:
        _, und = O.filter_frame(frame, filt, 0, with_undefined=True)
        assert not (got & O.defined_mask(w, h, und)).any()


def test_full_size_separable_bottom_row():
    """1080p, separable 3-tap filter: the reference reads the rows below the frame unguarded
    (intra.cl:3330-3332), so the last frame row of its filtered frame is undefined and the CUs
    reading it are unavailable; the 5-tap separable and the 2-D filters at 1080p are not."""
    w, h = 1920, 1080
    base = unavailable_cus(w, h, None)
    sep3 = unavailable_cus(w, h, "filterFrame_1d_int")
    assert (sep3 >= base).all() and sep3.sum() > base.sum()
    for f in ("filterFrame_1d_int_5x5", "filterFrame_2d_int_quarterCtu", "filterFrame_2d_float_5x5_quarterCtu"):
        assert np.array_equal(unavailable_cus(w, h, f), base), f
    frame = synth_frame(w, h, 0x1080, 0)
    assert np.array_equal(layout.expand_cu_mask(sep3, layout.num_ctus(w, h)),
                          O.engine_unavailable_mask(frame, "filterFrame_1d_int", 0))
