"""H2O with L2-norm heavy hitters (reference: kvcompress/methods/h2o_l2.py:25-153).

sinks ++ lowest-norm heavy hitters of the middle ++ recent window; the middle's norm / argsort /
sort / gather and the three-way cat run in one batched HIP engine launch.
"""
from typing import List, Tuple

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import layer_offset, normalize_kv_cache


@E.memoized
def h2o_l2_compress(
    past_key_values,
    start_size: int = 4,
    heavy_hitter_size: int = 64,
    recent_size: int = 444,
    skip_layers: List[int] = [],
    **kwargs
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    past_key_values = list(normalize_kv_cache(past_key_values))
    offset = layer_offset(kwargs)  # global index of layer 0 (layer-sharded callers)
    if not past_key_values:                                           # :79
        return past_key_values
    total_cache_size = start_size + heavy_hitter_size + recent_size
    jobs = []
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if seq_len <= total_cache_size:                               # :89
            continue
        if layer_idx + offset in skip_layers:
            continue
        sink = E.py_slice(seq_len, None, start_size)[1]
        t0, tl = E.py_slice(seq_len, -recent_size)
        middle_start = start_size
        middle_end = seq_len - recent_size
        if middle_end <= middle_start:                                # :99-109
            jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, tail_start=t0,
                                   tail_len=tl))
            continue
        z0, zl = E.py_slice(seq_len, middle_start, middle_end)
        num_to_keep = min(heavy_hitter_size, zl)                      # :125
        jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, zone_start=z0,
                               zone_len=zl, n_select=len(range(zl)[:num_to_keep]),
                               tail_start=t0, tail_len=tl))
    E.execute(jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


__all__ = ["h2o_l2_compress"]
