"""Teacher-forced evaluation with attention-score H2O (reference: kvcompress/evaluate_attention.py).

Same functions, arguments and result keys as the reference (evaluate_attention.py:24-332).  Per
token: one forward with output_attentions=True, the NLL / argmax accuracy of the next token, the
manager's accumulation updated with the step's attentions, and -- once the first layer's cache
exceeds start + heavy + recent -- h2o_attention_compress (the MI355X engine: accumulate, heavy
hitters and gather on the GPU, replayed natively for repeated decode shapes) followed by a manager
reset, exactly the reference's call sequence (:153-180, including its second accumulation inside
the compress call).

transformers >= 5 returns no attention weights from the sdpa / flash kernels (the 4.x releases
the reference ran on fell back to eager attention by themselves), and its eager attention adds the
causal mask without cutting it to the layer's key length -- a mask built for the uncompressed
skip layers no longer fits the compressed ones.  For the duration of the call the model runs
"kvc_eager" (utils.key_length_attention): the model's own eager attention with the mask cut to
the keys, as the 4.x eager kernels did; the previous implementation is restored after.
"""
import time
from typing import Dict, List, Optional

import torch
from torch.nn import CrossEntropyLoss

from .evaluate import _progress
from .methods.h2o_attention import H2OAttentionManager, h2o_attention_compress
from .utils import key_length_attention, normalize_kv_cache, to_dynamic_cache

_EMPTY = {"perplexity": float("inf"), "accuracy": 0.0, "num_tokens": 0, "final_cache_size": 0,
          "ttft": 0.0, "tpot": 0.0, "throughput": 0.0, "total_time": 0.0}


def evaluate_with_attention_compression(model, tokenizer, text: str,
                                        h2o_manager: Optional[H2OAttentionManager] = None,
                                        start_size: int = 4, heavy_hitter_size: int = 64,
                                        recent_size: int = 444, max_tokens: int = 3000,
                                        skip_layers: List[int] = [0, 1],
                                        device: Optional[torch.device] = None,
                                        show_progress: bool = True) -> Dict[str, float]:
    """evaluate_attention.py:24-228"""
    device = device if device is not None else next(model.parameters()).device
    if h2o_manager is None:  # (:73-83)
        h2o_manager = H2OAttentionManager(
            start_size=start_size, heavy_hitter_size=heavy_hitter_size, recent_size=recent_size,
            num_layers=getattr(model.config, "num_hidden_layers", 32),
            num_heads=getattr(model.config, "num_attention_heads", 32), device=device)
    else:
        h2o_manager.reset()
    ids = tokenizer.encode(text, return_tensors="pt")[:, :max_tokens].to(device)
    n = ids.shape[1]
    if n < 2:
        return dict(_EMPTY)
    loss_fn = CrossEntropyLoss(reduction="none")
    cache, nlls, correct, times = None, [], [], []
    limit = start_size + heavy_hitter_size + recent_size
    model.eval()
    steps = _progress(range(n - 1), show_progress)
    t_start = time.perf_counter()
    with torch.inference_mode(), key_length_attention(model, need_weights=True):
        for i in steps:
            t0 = time.perf_counter()
            out = model(ids[:, i:i + 1], past_key_values=cache, use_cache=True,
                        output_attentions=True)
            logits = out.logits[:, -1, :].view(-1, model.config.vocab_size)
            target = ids[:, i + 1:i + 2].view(-1)
            nlls.append(loss_fn(logits, target).item())
            correct.append((torch.argmax(logits, dim=-1) == target).int().item())
            cache, attentions = out.past_key_values, out.attentions
            h2o_manager.update_attention_scores(attentions, skip_layers)  # (:158)
            if cache is not None:
                kv = list(normalize_kv_cache(cache))
                if kv and kv[0][0].size(2) > limit:  # (:161-180)
                    cache = to_dynamic_cache(h2o_attention_compress(
                        kv, attention_scores=attentions, h2o_manager=h2o_manager,
                        start_size=start_size, heavy_hitter_size=heavy_hitter_size,
                        recent_size=recent_size, skip_layers=skip_layers))
                    h2o_manager.reset()  # positions moved
            times.append(time.perf_counter() - t0)
            if show_progress and hasattr(steps, "set_description"):
                steps.set_description(
                    f"H2O-Attn | PPL: {torch.exp(torch.tensor(nlls).mean()).item():.2f}, "
                    f"Acc: {sum(correct) / len(correct):.2%}")
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
        "ttft": times[0] if times[0] else 0.0,
        "tpot": sum(times[1:]) / (num - 1) if num > 1 else times[0],
        "throughput": num / total if total > 0 else 0.0,
        "total_time": total,
    }


def compare_h2o_methods(model, tokenizer, text: str, max_tokens: int = 2000,
                        heavy_hitter_sizes: List[int] = [32, 64, 128],
                        skip_layers: List[int] = [0, 1],
                        device: Optional[torch.device] = None) -> List[Dict]:
    """evaluate_attention.py:231-332: baseline, then per heavy-hitter size H2O-L2 and
    H2O-attention, each with a 512-token budget (4 sinks + hh + 508 - hh recent)."""
    from .evaluate import evaluate_with_compression
    from .methods import h2o_l2_compress
    device = device if device is not None else next(model.parameters()).device
    bar = "=" * 60
    print(f"\n{bar}\nTesting: Baseline (no compression)\n{bar}")
    base = evaluate_with_compression(model, tokenizer, text, compress_fn=None,
                                     max_tokens=max_tokens, device=device)
    base["method"] = "baseline"
    results = [base]
    print(f"  PPL: {base['perplexity']:.2f}, Acc: {base['accuracy']:.2%}")
    for hh in heavy_hitter_sizes:
        recent = 512 - 4 - hh
        print(f"\n{bar}\nTesting: H2O-L2 (hh={hh}, total=512)\n{bar}")
        r = evaluate_with_compression(
            model, tokenizer, text, compress_fn=h2o_l2_compress,
            compress_kwargs={"start_size": 4, "heavy_hitter_size": hh, "recent_size": recent},
            max_tokens=max_tokens, skip_layers=skip_layers, device=device)
        r["method"] = f"h2o_l2_hh{hh}"
        results.append(r)
        print(f"  PPL: {r['perplexity']:.2f}, Acc: {r['accuracy']:.2%}")
        print(f"\n{bar}\nTesting: H2O-Attention (hh={hh}, total=512)\n{bar}")
        r = evaluate_with_attention_compression(
            model, tokenizer, text, start_size=4, heavy_hitter_size=hh, recent_size=recent,
            max_tokens=max_tokens, skip_layers=skip_layers, device=device)
        r["method"] = f"h2o_attention_hh{hh}"
        results.append(r)
        print(f"  PPL: {r['perplexity']:.2f}, Acc: {r['accuracy']:.2%}")
    wide = "=" * 80
    print(f"\n{wide}\nCOMPARISON SUMMARY\n{wide}")
    print(f"{'Method':<25} {'PPL':>10} {'Acc':>10} {'Throughput':>12} {'Cache':>8}")
    print("-" * 80)
    for r in results:
        print(f"{r['method']:<25} {r['perplexity']:>10.2f} {r['accuracy']:>10.2%} "
              f"{r['throughput']:>12.2f} {r['final_cache_size']:>8}")
    return results


__all__ = ["evaluate_with_attention_compression", "compare_h2o_methods"]
