"""Sequence-length-adaptive L2 compression (reference: kvcompress/methods/adaptive_l2.py:20-201).

Both branches (hard-limit sinks/middle/recent and gradual keep-ratio with protected recent
tokens) map onto the engine's segment model; one batched HIP launch per call.
"""
from typing import List, Tuple

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import layer_offset, normalize_kv_cache


@E.memoized
def adaptive_l2_compress(
    past_key_values,
    target_size: int = 512,
    soft_limit: int = 256,
    hard_limit: int = 1024,
    keep_ratio_min: float = 0.3,
    keep_ratio_max: float = 0.9,
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
        if layer_idx + offset in skip_layers:                         # :71 (before length test)
            continue
        if seq_len <= soft_limit:
            continue
        if seq_len > hard_limit:                                      # :81-145
            if seq_len <= target_size:
                continue
            start_size = 4
            recent_size = target_size // 2
            middle_to_keep = target_size - start_size - recent_size
            if middle_to_keep <= 0:
                past_key_values[layer_idx] = (keys[:, :, -target_size:, :],
                                              values[:, :, -target_size:, :])
                continue
            sink = E.py_slice(seq_len, None, start_size)[1]
            middle_start, middle_end = start_size, seq_len - recent_size
            if middle_end <= middle_start:
                t0, tl = E.py_slice(seq_len, -(target_size - start_size))
                jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, tail_start=t0,
                                       tail_len=tl))
                continue
            z0, zl = E.py_slice(seq_len, middle_start, middle_end)
            num_to_keep = min(middle_to_keep, zl)
            t0, tl = E.py_slice(seq_len, -recent_size)
            jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, zone_start=z0,
                                   zone_len=zl, n_select=len(range(zl)[:num_to_keep]),
                                   tail_start=t0, tail_len=tl))
        else:                                                         # :147-199
            progress = (seq_len - soft_limit) / (hard_limit - soft_limit)
            keep_ratio = keep_ratio_max - progress * (keep_ratio_max - keep_ratio_min)
            tokens_to_keep = int(seq_len * keep_ratio)
            tokens_to_keep = max(tokens_to_keep, soft_limit)
            if tokens_to_keep >= seq_len:
                continue
            protected_recent = int(tokens_to_keep * 0.2)
            tokens_from_history = tokens_to_keep - protected_recent
            if tokens_from_history <= 0:
                past_key_values[layer_idx] = (keys[:, :, -tokens_to_keep:, :],
                                              values[:, :, -tokens_to_keep:, :])
                continue
            selection_end = seq_len - protected_recent
            if selection_end <= tokens_from_history:
                continue
            z0, zl = E.py_slice(seq_len, None, selection_end)
            t0, tl = E.py_slice(seq_len, -protected_recent)
            jobs.append(E.Segments(layer_idx, keys, values, zone_start=z0, zone_len=zl,
                                   n_select=len(range(zl)[:tokens_from_history]),
                                   tail_start=t0, tail_len=tl))
    E.execute(jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


__all__ = ["adaptive_l2_compress"]
