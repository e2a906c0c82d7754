"""Cache-format helpers with the API of the reference's kvcompress/utils.py:12-116.

`normalize_kv_cache` also unpacks transformers >= 5 caches, whose iteration yields 3-tuples the
reference cannot unpack; for tuple lists and legacy caches it returns what
the reference returns.
"""
import sys
from contextlib import contextmanager
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



# ---------------------------------------------------------------------------------------------
# Attention with per-layer key lengths under transformers >= 5.  Compressed caches give layers
# different lengths (skip_layers keep everything).  transformers 4.x -- which the reference ran
# on -- cut the causal mask to each layer's keys in its eager kernels
# (attention_mask[:, :, :, :key_len]); 5.x eager adds the mask built for the longest layer as is
# and raises, and 5.x sdpa / flash return no attention weights.  "kvc_eager" is the model's own
# eager attention with the 4.x cut.
# ---------------------------------------------------------------------------------------------
KEY_LENGTH_EAGER = "kvc_eager"


def _eager_forward(module, query, key, value, attention_mask, **kwargs):
    """The attention module's own eager_attention_forward (llama's for a model file without
    one), the mask cut to this layer's key length."""
    fn = getattr(sys.modules.get(type(module).__module__), "eager_attention_forward", None)
    if fn is None:
        from transformers.models.llama.modeling_llama import eager_attention_forward as fn
    if attention_mask is not None and attention_mask.shape[-1] != key.shape[-2]:
        attention_mask = attention_mask[..., :key.shape[-2]]
    return fn(module, query, key, value, attention_mask, **kwargs)


def _register_eager():
    from transformers import AttentionInterface
    from transformers.masking_utils import ALL_MASK_ATTENTION_FUNCTIONS, AttentionMaskInterface
    if KEY_LENGTH_EAGER not in ALL_MASK_ATTENTION_FUNCTIONS:
        AttentionInterface.register(KEY_LENGTH_EAGER, _eager_forward)
        AttentionMaskInterface.register(KEY_LENGTH_EAGER, ALL_MASK_ATTENTION_FUNCTIONS["eager"])


@contextmanager
def key_length_attention(model, need_weights: bool = False):
    """Inside the block the model runs kvc_eager when it is configured for eager attention, or
    for any implementation when `need_weights` (output_attentions); its previous implementation
    is restored on exit.  Models without set_attn_implementation (transformers 4.x) are left
    alone: their eager kernels already cut the mask."""
    impl = getattr(getattr(model, "config", None), "_attn_implementation", None)
    switch = (hasattr(model, "set_attn_implementation") and impl is not None and
              impl != KEY_LENGTH_EAGER and (need_weights or impl == "eager"))
    if switch:
        _register_eager()
        try:
            model.set_attn_implementation(KEY_LENGTH_EAGER)
        except (ValueError, TypeError, KeyError, NotImplementedError):
            # a model class that refuses registered attention functions: its own eager kernel
            # for the weights (ragged layer lengths then fail as they would without this)
            if need_weights and impl != "eager":
                model.set_attn_implementation("eager")
            else:
                switch = False
    try:
        yield
    finally:
        if switch:
            model.set_attn_implementation(impl)


__all__ = ["to_dynamic_cache", "normalize_kv_cache", "get_cache_size_mb", "get_cache_info",
           "get_seq_len"]
