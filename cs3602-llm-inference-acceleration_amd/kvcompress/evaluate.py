"""Teacher-forced PPL / accuracy evaluation with per-token compression.

Same functions, arguments and result keys as the reference's kvcompress/evaluate.py:26-327;
works with transformers >= 5 caches (the reference's loop cannot unpack them).
One token per forward; after every forward the cache is normalised to a (K, V) list, compressed
by `compress_fn(kv_list, skip_layers=..., **compress_kwargs)` (the MI355X engine when it is one of
this package's methods) and rebuilt as a DynamicCache.  A model configured for eager attention
runs utils.key_length_attention's kvc_eager meanwhile (transformers 5's eager kernel cannot take
layers of different lengths).
"""
import time
from typing import Callable, Dict, List, Optional

import torch
from torch.nn import CrossEntropyLoss

from .utils import key_length_attention, normalize_kv_cache, to_dynamic_cache


def _progress(it, show):
    if not show:
        return it
    try:
        from tqdm import tqdm
        return tqdm(it, desc="Evaluating")
    except ImportError:  # pragma: no cover
        return it


def evaluate_with_compression(model, tokenizer, text: str, compress_fn: Optional[Callable] = None,
                              compress_kwargs: Optional[Dict] = None, max_tokens: int = 3000,
                              skip_layers: List[int] = [0, 1],
                              device: Optional[torch.device] = None,
                              show_progress: bool = True) -> Dict[str, float]:
    """evaluate.py:26-226"""
    device = device if device is not None else next(model.parameters()).device
    compress_kwargs = compress_kwargs or {}
    ids = tokenizer.encode(text, return_tensors="pt")[:, :max_tokens].to(device)
    n = ids.shape[1]
    if n < 2:
        return {"perplexity": float("inf"), "accuracy": 0.0, "num_tokens": 0,
                "final_cache_size": 0, "ttft": 0.0, "tpot": 0.0, "throughput": 0.0,
                "total_time": 0.0}
    loss_fn = CrossEntropyLoss(reduction="none")
    cache, nlls, correct, times = None, [], [], []
    model.eval()
    steps = _progress(range(n - 1), show_progress)
    t_start = time.perf_counter()
    with torch.inference_mode(), key_length_attention(model):
        for i in steps:
            t0 = time.perf_counter()
            out = model(ids[:, i:i + 1], past_key_values=cache, use_cache=True)
            logits = out.logits[:, -1, :].view(-1, model.config.vocab_size)
            target = ids[:, i + 1:i + 2].view(-1)
            nlls.append(loss_fn(logits, target).item())
            correct.append((torch.argmax(logits, dim=-1) == target).int().item())
            cache = out.past_key_values
            if compress_fn is not None and cache is not None:
                kv = list(normalize_kv_cache(cache))
                cache = to_dynamic_cache(compress_fn(kv, skip_layers=skip_layers,
                                                     **compress_kwargs))
            times.append(time.perf_counter() - t0)
    total = time.perf_counter() - t_start
    num = len(nlls)
    final = 0
    if cache is not None:
        kv = list(normalize_kv_cache(cache))
        for li, (k, _) in enumerate(kv):
            if li not in skip_layers:
                final = k.size(2)
                break
        if final == 0 and kv:
            final = kv[0][0].size(2)
    return {
        "perplexity": torch.exp(torch.tensor(nlls).mean()).item(),
        "accuracy": sum(correct) / len(correct),
        "num_tokens": num,
        "final_cache_size": final,
        "ttft": times[0],
        "tpot": sum(times[1:]) / (num - 1) if num > 1 else times[0],
        "throughput": num / total if total > 0 else 0.0,
        "total_time": total,
    }


def evaluate_baseline(model, tokenizer, text: str, max_tokens: int = 3000,
                      device: Optional[torch.device] = None,
                      show_progress: bool = False) -> Dict[str, float]:
    """evaluate.py:229-259"""
    return evaluate_with_compression(model, tokenizer, text, compress_fn=None,
                                     max_tokens=max_tokens, device=device,
                                     show_progress=show_progress)


def compare_methods(model, tokenizer, text: str, methods_config: List[Dict],
                    max_tokens: int = 3000, skip_layers: List[int] = [0, 1],
                    device: Optional[torch.device] = None) -> List[Dict[str, float]]:
    """evaluate.py:262-327"""
    results = []
    for cfg in methods_config:
        name, kwargs = cfg.get("name", "unknown"), cfg.get("kwargs", {})
        print(f"\nEvaluating {name}...")
        r = evaluate_with_compression(model, tokenizer, text,
                                      compress_fn=cfg.get("compress_fn", None),
                                      compress_kwargs=kwargs, max_tokens=max_tokens,
                                      skip_layers=skip_layers, device=device, show_progress=True)
        r["method"], r["config"] = name, kwargs
        results.append(r)
        print(f"  PPL: {r['perplexity']:.2f}")
        print(f"  Accuracy: {r['accuracy']:.2%}")
        print(f"  Final cache size: {r['final_cache_size']}")
    return results


__all__ = ["evaluate_with_compression", "evaluate_baseline", "compare_methods"]
