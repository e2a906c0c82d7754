"""SnapKV-lite observation-window voting (reference: kvcompress/methods/snapkv_lite.py:24-154).

Importance = (max(norm) + 1e-6) - norm, avg_pool1d-smoothed, torch.topk-selected; the whole
chain (norms, bf16/fp32 score arithmetic, pooling, introselect / heap-select tie order, gather,
cat with the observation window) runs in one batched HIP engine launch.
"""
from typing import List, Tuple

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import layer_offset, normalize_kv_cache


@E.memoized
def snapkv_lite_compress(
    past_key_values,
    observation_window: int = 32,
    keep_size: int = 512,
    pooling_kernel: int = 5,
    skip_layers: List[int] = [],
    **kwargs
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    past_key_values = list(normalize_kv_cache(past_key_values))
    offset = layer_offset(kwargs)  # global index of layer 0 (layer-sharded callers)
    if not past_key_values:
        return past_key_values
    jobs = []
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if seq_len <= keep_size:                                      # :70
            continue
        if layer_idx + offset in skip_layers:
            continue
        prefix_len = seq_len - observation_window                     # :83
        if prefix_len <= 0:
            continue
        o0, ol = E.py_slice(seq_len, -observation_window)
        num_prefix_to_keep = min(keep_size - observation_window, prefix_len)   # :125-126
        if num_prefix_to_keep <= 0:                                   # :128-131 (views)
            past_key_values[layer_idx] = (keys[:, :, -observation_window:, :],
                                          values[:, :, -observation_window:, :])
            continue
        pool = pooling_kernel if (pooling_kernel > 1 and prefix_len >= pooling_kernel) else 0
        jobs.append(E.Segments(layer_idx, keys, values, zone_start=0, zone_len=prefix_len,
                               n_select=num_prefix_to_keep, tail_start=o0, tail_len=ol,
                               score_mode=N.KVC_SCORE_SNAPKV, pool_kernel=pool))
    E.execute(jobs, past_key_values, N.KVC_DESC, N.KVC_ALGO_TOPK)
    return past_key_values


__all__ = ["snapkv_lite_compress"]
