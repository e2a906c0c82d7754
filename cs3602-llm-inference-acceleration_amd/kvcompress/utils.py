"""KV cache format helpers -- same API as the reference's kvcompress/utils.py:12-116.

normalize_kv_cache additionally accepts transformers-5 caches (whose iteration the reference
cannot unpack); for lists and legacy caches it behaves identically.
"""
from typing import List, Tuple, Union

import torch


def _dynamic_cache_cls():
    from transformers import DynamicCache
    return DynamicCache


def to_dynamic_cache(past_key_values: List[Tuple[torch.Tensor, torch.Tensor]]):
    """utils.py:12-27: DynamicCache rebuilt with update(k, v, layer_idx) per layer."""
    cache = _dynamic_cache_cls()()
    for layer_idx, (keys, values) in enumerate(past_key_values):
        cache.update(keys, values, layer_idx)
    return cache


def normalize_kv_cache(past_key_values) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """utils.py:30-44: legacy tuple list out of any supported cache object."""
    if hasattr(past_key_values, "to_legacy_cache"):
        return past_key_values.to_legacy_cache()
    layers = getattr(past_key_values, "layers", None)
    if layers is not None and all(hasattr(l, "keys") and hasattr(l, "values") for l in layers):
        return [(l.keys, l.values) for l in layers]  # transformers >= 5 DynamicCache
    return list(past_key_values)


def get_cache_size_mb(past_key_values) -> float:
    """utils.py:47-65"""
    past_key_values = normalize_kv_cache(past_key_values)
    total = 0
    for keys, values in past_key_values:
        total += keys.element_size() * keys.nelement()
        total += values.element_size() * values.nelement()
    return total / (1024 ** 2)


def get_cache_info(past_key_values) -> dict:
    """utils.py:68-94"""
    past_key_values = normalize_kv_cache(past_key_values)
    if not past_key_values:
        return {"num_layers": 0, "seq_lengths": [], "total_size_mb": 0}
    seq_lengths = [keys.size(2) for keys, values in past_key_values]
    return {
        "num_layers": len(past_key_values),
        "seq_lengths": seq_lengths,
        "min_seq_len": min(seq_lengths),
        "max_seq_len": max(seq_lengths),
        "avg_seq_len": sum(seq_lengths) / len(seq_lengths),
        "total_size_mb": get_cache_size_mb(past_key_values),
    }


def get_seq_len(past_key_values, layer_idx: int = 0) -> int:
    """utils.py:97-116"""
    past_key_values = normalize_kv_cache(past_key_values)
    if not past_key_values or layer_idx >= len(past_key_values):
        return 0
    return past_key_values[layer_idx][0].size(2)


__all__ = ["to_dynamic_cache", "normalize_kv_cache", "get_cache_size_mb", "get_cache_info",
           "get_seq_len"]
