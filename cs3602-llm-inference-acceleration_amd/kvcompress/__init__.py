"""kvcompress -- MI355X-native drop-in for od-liu/CS3602-LLM-Inference-Acceleration's
kvcompress package (reference: kvcompress/__init__.py:1-97).

The compress functions keep the reference's signatures, registry and results (bit-exact
indices, byte-identical K/V); their norm / top-k / gather work runs in hand-written HIP kernels
for gfx950 (libkvc.so, C ABI in include/kvc.h).
"""
from .methods import (
    l2_compress,
    fix_size_l2_compress,
    streaming_llm_compress,
    get_compress_fn,
    list_methods,
    register_method,
    COMPRESS_METHODS,
)
from .evaluate import (
    evaluate_with_compression,
    evaluate_baseline,
    compare_methods,
)
from .benchmark import (
    benchmark,
    measure_generation_metrics,
    run_benchmark_suite,
    print_benchmark_summary,
)
from .utils import (
    to_dynamic_cache,
    normalize_kv_cache,
    get_cache_size_mb,
    get_cache_info,
    get_seq_len,
)

__all__ = [
    "l2_compress", "fix_size_l2_compress", "streaming_llm_compress",
    "get_compress_fn", "list_methods", "register_method", "COMPRESS_METHODS",
    "evaluate_with_compression", "evaluate_baseline", "compare_methods",
    "benchmark", "measure_generation_metrics", "run_benchmark_suite", "print_benchmark_summary",
    "to_dynamic_cache", "normalize_kv_cache", "get_cache_size_mb", "get_cache_info",
    "get_seq_len",
]

__version__ = "2.0.0"
