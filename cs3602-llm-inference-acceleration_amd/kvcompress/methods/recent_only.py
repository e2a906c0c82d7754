"""Sliding window (reference: kvcompress/methods/recent_only.py:16-70).

Returns views K[:, :, -window:] exactly like the reference; no kernel is needed.
"""
from typing import List, Tuple

import torch

from .. import _engine as E
from ..utils import layer_offset, normalize_kv_cache


@E.memoized
def recent_only_compress(
    past_key_values,
    window_size: int = 512,
    skip_layers: List[int] = [0, 1],
    **kwargs
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    past_key_values = list(normalize_kv_cache(past_key_values))
    offset = layer_offset(kwargs)  # global index of layer 0 (layer-sharded callers)
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if seq_len <= window_size:
            continue
        if layer_idx + offset in skip_layers:
            continue
        past_key_values[layer_idx] = (keys[:, :, -window_size:, :],
                                      values[:, :, -window_size:, :])
    return past_key_values


__all__ = ["recent_only_compress"]
