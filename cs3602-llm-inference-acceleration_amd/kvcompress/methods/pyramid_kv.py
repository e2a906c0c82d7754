"""Layer-wise pyramid budgets (reference: kvcompress/methods/pyramid_kv.py:26-185).

Per-layer target sizes come from the layer's index in the list and len(list) exactly as in the
reference.  For a layer-sharded run (one shard of a deeper stack per GPU) pass the extension
kwargs `layer_offset` / `num_layers_total` so every shard uses the global index and depth (and
`skip_layers` holds global indices, as for every method); without them the behaviour is the
reference's.
"""
from typing import List, Literal, Tuple

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import layer_offset, normalize_kv_cache


def pyramid_layer_sizes(num_layers, base_size=512, layer_decay=0.9, min_size=64,
                        profile="exponential", layer_offset=0, count=None):
    """pyramid_kv.py:82-97, for global layers [layer_offset, layer_offset + count)."""
    sizes = []
    count = num_layers if count is None else count
    for layer_idx in range(layer_offset, layer_offset + count):
        if profile == "exponential":
            size = int(base_size * (layer_decay ** layer_idx))
        elif profile == "linear":
            decay_per_layer = (base_size - min_size) / max(num_layers - 1, 1)
            size = int(base_size - layer_idx * decay_per_layer)
        else:
            size = base_size
        sizes.append(max(size, min_size))
    return sizes


@E.memoized
def pyramid_kv_compress(
    past_key_values,
    base_size: int = 512,
    layer_decay: float = 0.9,
    min_size: int = 64,
    profile: Literal["linear", "exponential", "constant"] = "exponential",
    skip_layers: List[int] = [],
    **kwargs
) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    past_key_values = list(normalize_kv_cache(past_key_values))
    if not past_key_values:
        return past_key_values
    offset = layer_offset(kwargs)
    num_layers = int(kwargs.get("num_layers_total", len(past_key_values)))
    layer_sizes = pyramid_layer_sizes(num_layers, base_size, layer_decay, min_size, profile,
                                      offset, len(past_key_values))
    jobs = []
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        target_size = layer_sizes[layer_idx]
        if seq_len <= target_size:                                    # :111
            continue
        if layer_idx + offset in skip_layers:
            continue
        start_size = min(4, target_size // 8)                         # :115-117
        recent_size = target_size // 2
        middle_to_keep = target_size - start_size - recent_size
        if middle_to_keep <= 0:                                       # :119-123 (views)
            past_key_values[layer_idx] = (keys[:, :, -target_size:, :],
                                          values[:, :, -target_size:, :])
            continue
        sink = E.py_slice(seq_len, None, start_size)[1]
        middle_start, middle_end = start_size, seq_len - recent_size
        if middle_end <= middle_start:                                # :128-140
            t0, tl = E.py_slice(seq_len, -(target_size - start_size))
            jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, tail_start=t0,
                                   tail_len=tl))
            continue
        z0, zl = E.py_slice(seq_len, middle_start, middle_end)
        num_to_keep = min(middle_to_keep, zl)
        n_sel = num_to_keep if (num_to_keep > 0 and zl > 0) else 0  # :153 / empty branch
        t0, tl = E.py_slice(seq_len, -recent_size)
        jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, zone_start=z0,
                               zone_len=zl, n_select=n_sel, tail_start=t0, tail_len=tl))
    E.execute(jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


__all__ = ["pyramid_kv_compress", "pyramid_layer_sizes"]
