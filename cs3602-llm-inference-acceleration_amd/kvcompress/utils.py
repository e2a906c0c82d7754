"""Cache-format helpers with the API of the reference's kvcompress/utils.py:12-116.

`normalize_kv_cache` also unpacks transformers >= 5 caches, whose iteration yields 3-tuples the
reference cannot unpack; for tuple lists and legacy caches it returns what
the reference returns.
"""
from typing import List, Tuple

import torch

KVList = List[Tuple[torch.Tensor, torch.Tensor]]


def to_dynamic_cache(past_key_values: KVList):
    """A transformers DynamicCache filled layer by layer with update(k, v, i) (utils.py:12-27)."""
    from transformers import DynamicCache
    cache = DynamicCache()
    for i, kv in enumerate(past_key_values):
        cache.update(kv[0], kv[1], i)
    return cache


def normalize_kv_cache(past_key_values) -> KVList:
    """(K, V) list view of a cache object (utils.py:30-44): legacy caches through
    to_legacy_cache(), transformers-5 caches through their per-layer keys / values."""
    legacy = getattr(past_key_values, "to_legacy_cache", None)
    if legacy is not None:
        return legacy()
    layers = getattr(past_key_values, "layers", None)
    if layers is not None and all(hasattr(l, "keys") and hasattr(l, "values") for l in layers):
        return [(l.keys, l.values) for l in layers]
    return list(past_key_values)


def layer_offset(kwargs) -> int:
    """Global index of the first layer of the list (extension kwarg `layer_offset`, default 0).

    Layer-sharded callers (one contiguous block of a deeper stack per GPU) pass
    it so that every method tests `skip_layers` -- and pyramid_kv sizes its layers -- by GLOBAL
    layer index, exactly as the unsharded reference call would; 0 reproduces the reference."""
    return int(kwargs.get("layer_offset", 0))


def _nbytes(t: torch.Tensor) -> int:
    return t.element_size() * t.nelement()


def get_cache_size_mb(past_key_values) -> float:
    """K and V bytes of every layer, in MiB (utils.py:47-65)."""
    return sum(_nbytes(k) + _nbytes(v) for k, v in normalize_kv_cache(past_key_values)) / 2 ** 20


def get_cache_info(past_key_values) -> dict:
    """Layer count, per-layer sequence lengths and their min / max / mean, total MiB
    (utils.py:68-94; an empty cache reports zeros)."""
    layers = normalize_kv_cache(past_key_values)
    if not layers:
        return {"num_layers": 0, "seq_lengths": [], "total_size_mb": 0}
    lens = [k.size(2) for k, _ in layers]
    return {"num_layers": len(layers), "seq_lengths": lens, "min_seq_len": min(lens),
            "max_seq_len": max(lens), "avg_seq_len": sum(lens) / len(lens),
            "total_size_mb": get_cache_size_mb(layers)}


def get_seq_len(past_key_values, layer_idx: int = 0) -> int:
    """Sequence length of one layer, 0 when the cache has no such layer (utils.py:97-116)."""
    layers = normalize_kv_cache(past_key_values)
    if len(layers) == 0 or layer_idx >= len(layers):
        return 0
    return layers[layer_idx][0].size(2)  # negative indices count from the end, as there


__all__ = ["to_dynamic_cache", "normalize_kv_cache", "get_cache_size_mb", "get_cache_info",
           "get_seq_len"]
