"""One large frame over several GPUs: every GPU holds the whole frame
(its reference samples and the filter need rows / columns outside its band) and searches one
band of CTU rows with mip_search_device_range; the bands tile the frame, so the assembled
cost table equals a single-GPU search.  Frames are independent, so throughput runs shard
whole frames instead (bench.py); the band split cuts the latency of one 8K frame."""
from .layout import num_ctus


def ctu_row_bands(width: int, height: int, parts: int):
    """[ctu_begin, ctu_end) per part: contiguous whole CTU rows, balanced by the number of
    CTU rows (the last, possibly partial, row counts as one); parts beyond the row count
    get empty bands (begin == end)."""
    if parts < 1:
        raise ValueError("parts must be >= 1")
    cols = (width + 127) // 128
    rows = num_ctus(width, height) // cols
    bands = []
    for p in range(parts):
        r0, r1 = rows * p // parts, rows * (p + 1) // parts
        bands.append((r0 * cols, r1 * cols))
    return bands


def band_slices(width: int, height: int, parts: int, costs_per_ctu: int):
    """Per part: the slice of one frame's flat cost table that its band writes."""
    return [slice(b * costs_per_ctu, e * costs_per_ctu) for b, e in ctu_row_bands(width, height, parts)]


def gather_bands(costs, width, height, rank, world, group=None):
    """All ranks' bands of one cost table -> the full table on every rank.  `costs`: this
    rank's full-size table ([F, nCTUs*97840], numpy int32) with only its own band written;
    exchanged with torch.distributed (gloo or nccl via CPU objects).  Returns numpy."""
    import numpy as np
    import torch.distributed as dist

    from .layout import COSTS_PER_CTU
    sl = band_slices(width, height, world, COSTS_PER_CTU)[rank]
    mine = np.ascontiguousarray(costs[:, sl])
    parts = [None] * world
    dist.all_gather_object(parts, mine, group=group)
    return np.concatenate(parts, axis=1)
