"""CTU-row bands of one frame over several GPUs (mipgpu.split): host logic on CPU, the
banded search against the whole-frame search on the GPU."""
import numpy as np
import pytest

from mipgpu import layout
from mipgpu.split import band_slices, ctu_row_bands


@pytest.mark.parametrize("w,h,parts", [(1920, 1080, 8), (7680, 4320, 8), (264, 392, 3), (256, 136, 4), (128, 128, 1)])
def test_bands_tile_the_frame(w, h, parts):
    bands = ctu_row_bands(w, h, parts)
    n = layout.num_ctus(w, h)
    cols = (w + 127) // 128
    assert len(bands) == parts
    assert bands[0][0] == 0 and bands[-1][1] == n
    for (b0, e0), (b1, e1) in zip(bands, bands[1:]):
        assert e0 == b1
    for b, e in bands:
        assert b % cols == 0 and e % cols == 0 and e >= b
    rows = [(e - b) // cols for b, e in bands]
    assert max(rows) - min(rows) <= 1
    sl = band_slices(w, h, parts, layout.COSTS_PER_CTU)
    assert sl[0].start == 0 and sl[-1].stop == n * layout.COSTS_PER_CTU


@pytest.mark.gpu
@pytest.mark.parametrize("filt,k,parts", [(None, 0, 3), ("filterFrame_2d_int_5x5_quarterCtu", 1, 3),
                                          ("filterFrame_1d_int_5x5", 2, 6)])
def test_banded_search_equals_whole_frame(gpu_available, filt, k, parts):
    """Bands of a 3x4-CTU frame (partial right column and bottom row) equal the whole-frame
    search; 6 parts > 4 CTU rows: the empty bands are no-ops; the separable filter gives the
    last columns samples above 10 bits (the exact per-CU kernel honours the band too)."""
    import torch

    import oracle_lib as O
    from mipgpu import MipEngine
    from mipgpu.synth import synth_frames
    w, h, n = 264, 392, 2  # 3 x 4 CTUs, partial right column and bottom row
    frames = synth_frames(w, h, n, 0xB4D, 0)
    d = torch.from_numpy(frames.astype(np.int16)).cuda()
    with MipEngine(w, h, max_batch=n, filter=filt, kernel_idx=k) as eng:
        whole = eng.search_device(d).cpu().numpy()
        banded = torch.full((n, eng.costs_per_frame), -5, dtype=torch.int32, device="cuda")
        bands = ctu_row_bands(w, h, parts)
        assert sum(b == e for b, e in bands) == max(0, parts - 4)
        for b, e in bands:
            eng.search_device_range(d, b, e, banded)
            torch.cuda.synchronize()
            got = banded.cpu().numpy()
            # the band's CTU blocks are written, nothing after them yet
            assert (got[:, e * layout.COSTS_PER_CTU:] == -5).all()
        got = banded.cpu().numpy()
    assert np.array_equal(got, whole)
    for f in range(n):
        assert np.array_equal(whole[f], O.engine_search(frames[f], filt, k))


def _gather_worker(rank, world, port, q):
    import os

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mipgpu.split import band_slices, gather_bands
    w, h = 384, 392
    full = np.zeros((2, layout.num_ctus(w, h) * layout.COSTS_PER_CTU), np.int32)
    mine = full.copy()
    for r, sl in enumerate(band_slices(w, h, world, layout.COSTS_PER_CTU)):
        full[:, sl] = 1000 + r
    sl = band_slices(w, h, world, layout.COSTS_PER_CTU)[rank]
    mine[:, sl] = full[:, sl]
    got = gather_bands(mine, w, h, rank, world)
    q.put((rank, bool(np.array_equal(got, full))))
    dist.destroy_process_group()


def test_gather_bands_two_ranks_gloo():
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
