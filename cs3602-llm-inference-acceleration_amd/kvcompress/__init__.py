"""kvcompress -- MI355X-native drop-in for od-liu/CS3602-LLM-Inference-Acceleration's
kvcompress package (reference: kvcompress/__init__.py:1-97).

The compress functions keep the reference's signatures, registry and results (bit-exact
indices, byte-identical K/V); their norm / top-k / gather work runs in hand-written HIP kernels
for gfx950 (libkvc.so, C ABI in include/kvc.h).  Top-level names: the reference's exports.
"""
from .benchmark import (benchmark, measure_generation_metrics, print_benchmark_summary,
                        run_benchmark_suite)
from .evaluate import compare_methods, evaluate_baseline, evaluate_with_compression
from .methods import (COMPRESS_METHODS, fix_size_l2_compress, get_compress_fn, l2_compress,
                      list_methods, register_method, streaming_llm_compress)
from .utils import (get_cache_info, get_cache_size_mb, get_seq_len, normalize_kv_cache,
                    to_dynamic_cache)

__version__ = "2.0.0"  # the reference package version this mirrors

__all__ = sorted(name for name in dir() if not name.startswith("_") and name not in (
    "benchmark_module", "methods", "evaluate", "utils"))
