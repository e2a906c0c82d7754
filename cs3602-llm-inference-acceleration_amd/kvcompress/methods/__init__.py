"""Method registry of the MI355X engine (API of the reference's kvcompress/methods/__init__.py:21-101).

Lookup by name works as in the reference -- the nine names in its order (the README lists eight:
`h2o_attention` is registered too), `get_compress_fn` raising the same ValueError text, and
`register_method` for user additions.  Every method that compresses runs on the HIP engine
(libkvc.so); `recent_only` only slices.
"""
from typing import Callable, Dict, List

from .adaptive_l2 import adaptive_l2_compress
from .fix_size_l2 import fix_size_l2_compress
from .h2o_attention import H2OAttentionManager, create_h2o_manager_from_model, h2o_attention_compress
from .h2o_l2 import h2o_l2_compress
from .l2_compress import l2_compress
from .pyramid_kv import pyramid_kv_compress
from .recent_only import recent_only_compress
from .snapkv_lite import snapkv_lite_compress
from .streaming_llm import streaming_llm_compress

# (registry name, function) in the reference's registration order -- list_methods() order
_BUILTIN = (
    ("l2_compress", l2_compress),
    ("fix_size_l2", fix_size_l2_compress),
    ("streaming_llm", streaming_llm_compress),
    ("recent_only", recent_only_compress),
    ("h2o_l2", h2o_l2_compress),
    ("h2o_attention", h2o_attention_compress),
    ("snapkv_lite", snapkv_lite_compress),
    ("pyramid_kv", pyramid_kv_compress),
    ("adaptive_l2", adaptive_l2_compress),
)
COMPRESS_METHODS: Dict[str, Callable] = dict(_BUILTIN)


def get_compress_fn(method: str) -> Callable:
    """The compress function registered under `method` (ValueError naming the choices if none)."""
    fn = COMPRESS_METHODS.get(method)
    if fn is None:
        raise ValueError(f"Unknown method: {method}. Available: {list(COMPRESS_METHODS)}")
    return fn


def list_methods() -> List[str]:
    """Registered names, in registration order."""
    return [name for name in COMPRESS_METHODS]


def register_method(name: str, fn: Callable) -> None:
    """Add (or replace) a method: fn(past_key_values, **kwargs) -> list of (K, V)."""
    COMPRESS_METHODS[name] = fn


__all__ = [fn.__name__ for _, fn in _BUILTIN] + [
    "H2OAttentionManager", "create_h2o_manager_from_model",
    "get_compress_fn", "list_methods", "register_method", "COMPRESS_METHODS",
]
