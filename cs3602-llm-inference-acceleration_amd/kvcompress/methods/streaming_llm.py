"""StreamingLLM sinks + recent window (reference: kvcompress/methods/streaming_llm.py:19-170).

cat(K[:, :, :start], K[:, :, -recent:]) per layer runs as the engine's gather kernel (no
selection), all layers in one launch.  `recent_size=0` keeps the reference's `-0:` quirk
(the whole sequence is appended after the sinks).
"""
from typing import List, Tuple

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import layer_offset, normalize_kv_cache


def _sink_recent_jobs(past_key_values, start_size, recent_size, skip_layers, fits, offset=0):
    jobs = []
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if fits(seq_len):
            continue
        if layer_idx + offset in skip_layers:
            continue
        s0, sl = E.py_slice(seq_len, None, start_size)
        t0, tl = E.py_slice(seq_len, -recent_size)
        jobs.append(E.Segments(layer_idx, keys, values, sink_len=sl, tail_start=t0,
                               tail_len=tl))
    return jobs


@E.memoized
def streaming_llm_compress(
    past_key_values,
    start_size: int = 4,
    recent_size: int = 508,
    skip_layers: List[int] = [],
    **kwargs
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    past_key_values = list(normalize_kv_cache(past_key_values))
    if not past_key_values:                                           # :79
        return past_key_values
    cache_size = start_size + recent_size
    jobs = _sink_recent_jobs(past_key_values, start_size, recent_size, skip_layers,
                             lambda S: S <= cache_size, layer_offset(kwargs))  # :88
    E.execute(jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


@E.memoized
def evict_for_space(
    past_key_values,
    num_coming: int,
    start_size: int = 4,
    recent_size: int = 508,
    skip_layers: List[int] = [],
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """streaming_llm.py:114-170 (exported, not registered)."""
    past_key_values = list(normalize_kv_cache(past_key_values))
    if not past_key_values:
        return past_key_values
    cache_size = start_size + recent_size
    effective_recent = recent_size - num_coming
    if effective_recent <= 0:
        effective_recent = recent_size
    jobs = _sink_recent_jobs(past_key_values, start_size, effective_recent, skip_layers,
                             lambda S: S + num_coming <= cache_size)
    E.execute(jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


__all__ = ["streaming_llm_compress", "evict_for_space"]
