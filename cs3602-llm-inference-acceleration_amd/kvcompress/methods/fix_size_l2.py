"""Fixed-size L2-norm eviction (reference: kvcompress/methods/fix_size_l2.py:15-154).

Same signature, defaults, branch order and size arithmetic as the reference; the norm ->
argsort -> [:keep] -> sort -> gather -> cat pipeline of every compressed layer runs as one
batched HIP engine launch (score, select, gather kernels) across all layers of the call.
"""
from typing import List, Literal, Tuple, Union

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import layer_offset, normalize_kv_cache


@E.memoized
def fix_size_l2_compress(
    past_key_values,
    fix_kv_size: int = 1024,
    keep_ratio: float = 0.0,
    strategy: Literal["keep_low", "keep_high", "random"] = "keep_low",
    skip_layers: List[int] = [0, 1],
    **kwargs
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    past_key_values = list(normalize_kv_cache(past_key_values))
    offset = layer_offset(kwargs)  # global index of layer 0 (layer-sharded callers)
    jobs = []
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if seq_len <= fix_kv_size:                                    # :69
            continue
        if layer_idx + offset in skip_layers:                         # :73
            continue
        batch_size, num_heads, seq_len, head_dim = keys.shape
        protected_length = int(fix_kv_size * keep_ratio)              # :79
        protected_length = min(protected_length, seq_len)
        eviction_zone_end = seq_len - protected_length
        tokens_to_keep = fix_kv_size - protected_length
        if tokens_to_keep <= 0:                                       # :88-93 (views)
            past_key_values[layer_idx] = (keys[:, :, -protected_length:, :],
                                          values[:, :, -protected_length:, :])
            continue
        if eviction_zone_end <= tokens_to_keep:                       # :95
            continue
        ext = None
        if strategy == "random":                                      # :116-124
            ext = torch.stack([
                torch.stack([
                    torch.randperm(eviction_zone_end, device=keys.device)[:tokens_to_keep]
                    for _ in range(num_heads)
                ])
                for _ in range(batch_size)
            ])
            ext, _ = torch.sort(ext, dim=-1)
        elif strategy not in ("keep_low", "keep_high"):
            raise ValueError(f"Unknown strategy: {strategy}")         # :125-126
        tail_start, tail_len = (E.py_slice(seq_len, -protected_length) if protected_length > 0
                                else (0, 0))
        jobs.append(E.Segments(layer_idx, keys, values, zone_start=0,
                               zone_len=eviction_zone_end, n_select=tokens_to_keep,
                               tail_start=tail_start, tail_len=tail_len, ext_index=ext))
    order = N.KVC_DESC if strategy == "keep_high" else N.KVC_ASC
    E.execute(jobs, past_key_values, order, N.KVC_ALGO_SORT)
    return past_key_values


__all__ = ["fix_size_l2_compress"]
