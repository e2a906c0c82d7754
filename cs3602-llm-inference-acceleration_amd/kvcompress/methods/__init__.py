"""Compression-method registry (reference: kvcompress/methods/__init__.py:21-101).

Same names, same order, same lookup errors.  Every compressing method runs on the MI355X HIP
engine (libkvc.so); see DESIGN.md.
"""
from typing import Callable, Dict, List

from .l2_compress import l2_compress
from .fix_size_l2 import fix_size_l2_compress
from .streaming_llm import streaming_llm_compress
from .recent_only import recent_only_compress
from .h2o_l2 import h2o_l2_compress
from .h2o_attention import (h2o_attention_compress, H2OAttentionManager,
                            create_h2o_manager_from_model)
from .snapkv_lite import snapkv_lite_compress
from .pyramid_kv import pyramid_kv_compress
from .adaptive_l2 import adaptive_l2_compress

COMPRESS_METHODS: Dict[str, Callable] = {
    "l2_compress": l2_compress,
    "fix_size_l2": fix_size_l2_compress,
    "streaming_llm": streaming_llm_compress,
    "recent_only": recent_only_compress,
    "h2o_l2": h2o_l2_compress,
    "h2o_attention": h2o_attention_compress,
    "snapkv_lite": snapkv_lite_compress,
    "pyramid_kv": pyramid_kv_compress,
    "adaptive_l2": adaptive_l2_compress,
}


def get_compress_fn(method: str) -> Callable:
    """methods/__init__.py:36-61"""
    if method not in COMPRESS_METHODS:
        available = list(COMPRESS_METHODS.keys())
        raise ValueError(f"Unknown method: {method}. Available: {available}")
    return COMPRESS_METHODS[method]


def list_methods() -> List[str]:
    return list(COMPRESS_METHODS.keys())


def register_method(name: str, fn: Callable) -> None:
    COMPRESS_METHODS[name] = fn


__all__ = [
    "l2_compress", "fix_size_l2_compress", "streaming_llm_compress", "recent_only_compress",
    "h2o_l2_compress", "h2o_attention_compress", "H2OAttentionManager",
    "create_h2o_manager_from_model", "snapkv_lite_compress", "pyramid_kv_compress",
    "adaptive_l2_compress", "get_compress_fn", "list_methods", "register_method",
    "COMPRESS_METHODS",
]
