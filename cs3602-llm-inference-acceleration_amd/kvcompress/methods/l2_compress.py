"""KnormPress ratio compression (reference: kvcompress/methods/l2_compress.py:18-92).

Keeps ceil(keep_ratio * S) lowest-norm tokens per (b, h); one batched HIP engine launch per call.
"""
from math import ceil
from typing import List, Tuple

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import layer_offset, normalize_kv_cache


@E.memoized
def l2_compress(
    past_key_values,
    keep_ratio: float = 1.0,
    prune_after: int = 1000,
    skip_layers: List[int] = [0, 1],
    **kwargs
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    past_key_values = list(normalize_kv_cache(past_key_values))
    offset = layer_offset(kwargs)  # global index of layer 0 (layer-sharded callers)
    if keep_ratio >= 1.0:                                              # :48-49
        return past_key_values
    jobs = []
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if seq_len <= prune_after:                                    # :55
            continue
        if layer_idx + offset in skip_layers:                         # :59
            continue
        tokens_to_keep = ceil(keep_ratio * seq_len)                   # :62
        if tokens_to_keep >= seq_len:
            continue
        if tokens_to_keep < -1:
            # the reference's expand(..., tokens_to_keep, ...) rejects sizes below -1
            raise RuntimeError(
                f"The expanded size of the tensor ({tokens_to_keep}) isn't allowed")
        n_sel = len(range(seq_len)[:tokens_to_keep])  # argsort(...)[:, :, :k] (k = -1 quirk)
        jobs.append(E.Segments(layer_idx, keys, values, zone_start=0, zone_len=seq_len,
                               n_select=n_sel))
    E.execute(jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


__all__ = ["l2_compress"]
