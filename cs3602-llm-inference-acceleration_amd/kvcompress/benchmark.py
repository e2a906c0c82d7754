"""Generation timing + quality benchmark drivers (reference: kvcompress/benchmark.py:23-351).
Same functions, arguments and result keys; transformers-5 compatible."""
import time
from typing import Callable, Dict, List, Optional

import torch

from .evaluate import evaluate_with_compression
from .utils import key_length_attention, normalize_kv_cache, to_dynamic_cache


def measure_generation_metrics(model, tokenizer, text: str, compress_fn: Optional[Callable] = None,
                               compress_kwargs: Optional[Dict] = None, max_new_tokens: int = 1000,
                               max_input_tokens: int = 3000, skip_layers: List[int] = [0, 1],
                               device: Optional[torch.device] = None) -> Dict[str, float]:
    """benchmark.py:23-142: prefill (TTFT), compress once, then greedy decode compressing every
    step."""
    device = device if device is not None else next(model.parameters()).device
    compress_kwargs = compress_kwargs or {}
    ids = tokenizer.encode(text, return_tensors="pt")[:, :max_input_tokens].to(device)
    if getattr(tokenizer, "pad_token_id", None) is None:
        tokenizer.pad_token_id = getattr(tokenizer, "eos_token_id", None)
    model.eval()
    generated = []

    def compress(cache):
        if compress_fn is None or cache is None:
            return cache
        return to_dynamic_cache(compress_fn(list(normalize_kv_cache(cache)),
                                            skip_layers=skip_layers, **compress_kwargs))

    t_start = time.perf_counter()
    with torch.inference_mode(), key_length_attention(model):
        t0 = time.perf_counter()
        out = model(ids, use_cache=True, return_dict=True)
        tok = torch.argmax(out.logits[:, -1, :], dim=-1, keepdim=True)
        generated.append(tok)
        ttft = time.perf_counter() - t0
        cache = compress(out.past_key_values)
        for _ in range(max_new_tokens - 1):
            out = model(tok, past_key_values=cache, use_cache=True, return_dict=True)
            tok = torch.argmax(out.logits[:, -1, :], dim=-1, keepdim=True)
            generated.append(tok)
            if tok.item() == getattr(tokenizer, "eos_token_id", None):
                break
            cache = compress(out.past_key_values)
    total = time.perf_counter() - t_start
    n = len(generated)
    return {"ttft": ttft, "tpot": (total - ttft) / max(n - 1, 1),
            "throughput": n / total if total > 0 else 0, "total_time": total, "num_tokens": n,
            "input_length": ids.shape[1]}


def benchmark(model, tokenizer, text: str, compress_fn: Optional[Callable] = None,
              compress_kwargs: Optional[Dict] = None, max_new_tokens: int = 1000,
              eval_tokens: int = 3000, skip_layers: List[int] = [0, 1],
              device: Optional[torch.device] = None) -> Dict[str, float]:
    """benchmark.py:145-209: one teacher-forced pass gives timing and quality metrics."""
    m = evaluate_with_compression(model, tokenizer, text, compress_fn=compress_fn,
                                  compress_kwargs=compress_kwargs or {}, max_tokens=eval_tokens,
                                  skip_layers=skip_layers, device=device, show_progress=True)
    return {"ttft": m["ttft"], "tpot": m["tpot"], "throughput": m["throughput"],
            "total_time": m["total_time"], "perplexity": m["perplexity"],
            "accuracy": m["accuracy"], "eval_tokens": m["num_tokens"],
            "final_cache_size": m["final_cache_size"]}


def run_benchmark_suite(model, tokenizer, text: str, methods_config: List[Dict],
                        max_new_tokens: int = 1000, eval_tokens: int = 3000,
                        skip_layers: List[int] = [0, 1],
                        device: Optional[torch.device] = None) -> List[Dict[str, float]]:
    """benchmark.py:212-290"""
    results = []
    for cfg in methods_config:
        name, kwargs = cfg.get("name", "unknown"), cfg.get("kwargs", {})
        print(f"\n{'=' * 60}\nTesting: {name}\n{'=' * 60}")
        r = benchmark(model, tokenizer, text, compress_fn=cfg.get("compress_fn", None),
                      compress_kwargs=kwargs, max_new_tokens=max_new_tokens,
                      eval_tokens=eval_tokens, skip_layers=skip_layers, device=device)
        r["method"], r["config"] = name, kwargs
        results.append(r)
        print(f"\nTiming Metrics (across {r['eval_tokens']} tokens):")
        print(f"  TTFT:       {r['ttft']:.4f} seconds")
        print(f"  TPOT:       {r['tpot']:.4f} seconds")
        print(f"  Throughput: {r['throughput']:.2f} tokens/sec")
        print(f"  Total time: {r['total_time']:.2f} seconds")
        print("\nQuality Metrics:")
        print(f"  PPL:        {r['perplexity']:.2f}")
        print(f"  Accuracy:   {r['accuracy']:.2%}")
        print(f"  Cache size: {r['final_cache_size']} tokens")
    return results


def print_benchmark_summary(results: List[Dict[str, float]]) -> None:
    """benchmark.py:293-351"""
    bar = "=" * 90
    print(f"\n{bar}\nBENCHMARK SUMMARY\n{bar}")
    print(f"{'Method':<20} {'TTFT(s)':>10} {'TPOT(s)':>10} {'Thruput':>10} {'PPL':>10} "
          f"{'Acc':>10} {'Cache':>8}")
    print("-" * 90)
    base = next((r for r in results if r.get("method") == "baseline" or
                 r.get("compress_fn") is None), results[0] if results else None)
    for r in results:
        print(f"{r.get('method', 'unknown')[:20]:<20} {r['ttft']:>10.4f} {r['tpot']:>10.4f} "
              f"{r['throughput']:>10.2f} {r['perplexity']:>10.2f} {r['accuracy']:>10.2%} "
              f"{r['final_cache_size']:>8}")
    print(bar)
    if base and len(results) > 1:
        print("\nComparison with baseline (Throughput ↑ better, TPOT ↓ better, PPL ↓ better):")
        for r in results:
            if r.get("method") == base.get("method"):
                continue

            def rel(a, b, inv=False):
                if b <= 0:
                    return 0.0
                return (1 - a / b) * 100 if inv else (a / b - 1) * 100
            print(f"  {r.get('method', 'unknown')}: "
                  f"Throughput {rel(r['throughput'], base['throughput']):+.1f}%, "
                  f"TPOT {rel(r['tpot'], base['tpot'], True):+.1f}%, "
                  f"PPL {rel(r['perplexity'], base['perplexity']):+.1f}%, "
                  f"Acc {rel(r['accuracy'], base['accuracy']):+.1f}%")


__all__ = ["measure_generation_metrics", "benchmark", "run_benchmark_suite",
           "print_benchmark_summary"]
