#!/usr/bin/env python3
"""Unified benchmark CLI for KV-cache compression -- the reference's scripts/benchmark.py
surface (same arguments, defaults, method configurations and report; reference
scripts/benchmark.py:232-757) over this package, whose compress functions run on the MI355X HIP
engine.

Offline extensions (the reference has none; everything else is unchanged):
  --random_model {pythia-2.8b,pythia-6.9b,pythia-tiny}
      random-weight GPT-NeoX of that geometry (hand-written config, seeded) instead of
      downloading --model_id; the PPL numbers then measure compression parity, not language
      quality.
  --text_file PATH   samples from a local text file (split on blank-line-separated chapters)
  --synthetic_text   deterministic pseudo-English samples
When neither is given, PG-19 is loaded exactly like the reference (data/pg19.parquet, then HF).
"""
import argparse
import os
import sys

import numpy as np
import torch

# like the reference: the project root (the directory holding the kvcompress package) on path
project_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, project_root)

from kvcompress.methods import (  # noqa: E402
    get_compress_fn, list_methods,
    l2_compress, fix_size_l2_compress, streaming_llm_compress, recent_only_compress,
    h2o_l2_compress, snapkv_lite_compress, pyramid_kv_compress, adaptive_l2_compress
)
from kvcompress.benchmark import benchmark, run_benchmark_suite, print_benchmark_summary  # noqa
from kvcompress.evaluate import evaluate_with_compression  # noqa: E402,F401

LOCAL_PG19_PATH = os.path.join(project_root, "data", "pg19.parquet")

# pythia geometries (pythia-2.8b H=32 D=80 L=32; pythia-6.9b H=32 D=128 L=32)
RANDOM_MODELS = {
    "pythia-2.8b": dict(hidden_size=2560, num_hidden_layers=32, num_attention_heads=32,
                        intermediate_size=10240, vocab_size=50304),
    "pythia-6.9b": dict(hidden_size=4096, num_hidden_layers=32, num_attention_heads=32,
                        intermediate_size=16384, vocab_size=50432),
    "pythia-tiny": dict(hidden_size=256, num_hidden_layers=4, num_attention_heads=4,
                        intermediate_size=1024, vocab_size=512),
}


def get_device():
    """Get the best available device."""
    if torch.cuda.is_available():
        return torch.device("cuda")
    if getattr(torch.backends, "mps", None) is not None and torch.backends.mps.is_available():
        return torch.device("mps")
    return torch.device("cpu")


class ByteTokenizer:
    """Offline tokenizer for --random_model: UTF-8 bytes folded into the vocabulary."""

    def __init__(self, vocab):
        self.vocab = vocab
        self.eos_token_id = None
        self.pad_token_id = None
        self.eos_token = None
        self.pad_token = None

    def encode(self, text, return_tensors="pt"):
        ids = [(b * 7 + i) % self.vocab for i, b in enumerate(text.encode("utf-8"))]
        return torch.tensor([ids], dtype=torch.long)


def load_random_model(name, device):
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM
    torch.manual_seed(0)
    g = RANDOM_MODELS[name]
    cfg = GPTNeoXConfig(rotary_pct=0.25, max_position_embeddings=20480, **g)
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    model = GPTNeoXForCausalLM(cfg).to(dtype).to(device).eval()
    print(f"Random-weight {name} ({g['num_hidden_layers']} layers, "
          f"{g['num_attention_heads']} heads, head_dim "
          f"{g['hidden_size'] // g['num_attention_heads']}, {dtype}) on {device}")
    return model, ByteTokenizer(g["vocab_size"]), device


def load_model_and_tokenizer(model_id: str = "EleutherAI/pythia-2.8b"):
    """Reference scripts/benchmark.py:78-143: cache first, then the Hub."""
    from transformers import AutoModelForCausalLM, AutoTokenizer
    print(f"Loading model: {model_id}")
    device = get_device()
    print(f"Using device: {device}")
    try:
        model = AutoModelForCausalLM.from_pretrained(model_id, low_cpu_mem_usage=True,
                                                     local_files_only=True)
        print("Model loaded from cache")
    except (OSError, ValueError):
        print("Model not in cache, downloading from HuggingFace Hub...")
        model = AutoModelForCausalLM.from_pretrained(model_id, low_cpu_mem_usage=True,
                                                     local_files_only=False)
        print("Model downloaded and loaded")
    model.to(device)
    model.eval()
    try:
        tokenizer = AutoTokenizer.from_pretrained(model_id, local_files_only=True)
    except (OSError, ValueError):
        tokenizer = AutoTokenizer.from_pretrained(model_id, local_files_only=False)
    if tokenizer.pad_token is None:
        tokenizer.pad_token = tokenizer.eos_token
    return model, tokenizer, device


def warmup_model(model, tokenizer, device, num_warmup: int = 3):
    """Reference scripts/benchmark.py:146-190."""
    print(f"\nPerforming {num_warmup} warmup iterations...")
    input_ids = tokenizer.encode("The quick brown fox jumps over the lazy dog. " * 10,
                                 return_tensors="pt").to(device)
    with torch.inference_mode():
        for i in range(num_warmup):
            outputs = model(input_ids, use_cache=True)
            past = outputs.past_key_values
            nxt = torch.argmax(outputs.logits[:, -1, :], dim=-1, keepdim=True)
            for _ in range(10):
                outputs = model(nxt, past_key_values=past, use_cache=True)
                past = outputs.past_key_values
                nxt = torch.argmax(outputs.logits[:, -1, :], dim=-1, keepdim=True)
            print(f"  Warmup {i+1}/{num_warmup} completed")
    if device.type == "cuda":
        torch.cuda.empty_cache()
    print("  Warmup finished!\n")


def load_pg19_samples(num_samples: int = 3):
    """Reference scripts/benchmark.py:193-229 (samples longer than 10 000 characters)."""
    from datasets import load_dataset
    print("\nLoading PG-19 dataset...")
    dataset = None
    if os.path.exists(LOCAL_PG19_PATH):
        print(f"  Found local file: {LOCAL_PG19_PATH}")
        try:
            dataset = load_dataset("parquet", data_files={"test": LOCAL_PG19_PATH}, split="test")
            print(f"  Loaded {len(dataset)} samples from local file")
        except Exception as e:  # noqa: BLE001 (reference behaviour)
            print(f"  Failed to load local file: {e}")
            dataset = None
    if dataset is None:
        try:
            print("  Loading from HuggingFace...")
            dataset = load_dataset("pg19", split="test")
        except Exception as e:  # noqa: BLE001
            print(f"  Failed to load from HuggingFace: {e}")
            return []
    samples = []
    for i, sample in enumerate(dataset):
        if i >= num_samples:
            break
        text = sample.get("text", "")
        if len(text) > 10000:
            samples.append(text)
            print(f"  Sample {i+1}: {len(text)} characters")
    print(f"  Total: {len(samples)} samples loaded")
    return samples


def load_text_file_samples(path, num_samples):
    text = open(path, encoding="utf-8", errors="replace").read()
    chunks = [c for c in text.split("\n\n\n") if c.strip()] or [text]
    return chunks[:num_samples]


def synthetic_samples(num_samples, chars=12000):
    words = ("the of and to a in that was he it his with as had for on you her not but at "
             "which be they this from by she were all one have said an are so him there").split()
    rng = np.random.default_rng(19)
    out = []
    for _ in range(num_samples):
        w = rng.choice(words, size=chars // 4)
        out.append(" ".join(w)[:chars])
    return out


def build_methods_config(args) -> list:
    """Reference scripts/benchmark.py:232-513 (incl. its quirk: --compare_new adds no method)."""
    methods = []
    if not args.no_baseline:
        methods.append({"name": "baseline", "compress_fn": None, "kwargs": {}})

    def recent(size):
        return {"name": f"recent_only_{size}", "compress_fn": recent_only_compress,
                "kwargs": {"window_size": size}}

    if args.method == "l2_compress":
        for kr in [float(x) for x in args.keep_ratios.split(",")]:
            if kr >= 1.0 and not args.no_baseline:
                continue
            methods.append({"name": f"l2_kr={kr:.1f}", "compress_fn": l2_compress,
                            "kwargs": {"keep_ratio": kr, "prune_after": args.prune_after}})
    elif args.method == "fix_size_l2":
        fix_kv_sizes = [int(x) for x in args.fix_kv_sizes.split(",")]
        strategies = [x.strip() for x in args.strategies.split(",")]
        keep_ratios = [float(x) for x in args.keep_ratios.split(",")]
        if not args.no_recent_only:
            methods.extend(recent(fs) for fs in fix_kv_sizes)
        for fs in fix_kv_sizes:
            for st in strategies:
                for kr in keep_ratios:
                    methods.append({"name": f"fix{fs}_{st}_kr={kr:.1f}",
                                    "compress_fn": fix_size_l2_compress,
                                    "kwargs": {"fix_kv_size": fs, "strategy": st,
                                               "keep_ratio": kr}})
    elif args.method == "streaming_llm":
        recent_sizes = [int(x) for x in args.recent_sizes.split(",")]
        if not args.no_recent_only:
            methods.extend(recent(args.start_size + r) for r in recent_sizes)
        for r in recent_sizes:
            methods.append({"name": f"streaming_{args.start_size + r}",
                            "compress_fn": streaming_llm_compress,
                            "kwargs": {"start_size": args.start_size, "recent_size": r}})
    elif args.method == "h2o_l2":
        hh_sizes = [int(x) for x in args.heavy_hitter_sizes.split(",")]
        if not args.no_recent_only:
            methods.extend(recent(args.start_size + hh + args.h2o_recent_size) for hh in hh_sizes)
        for hh in hh_sizes:
            methods.append({"name": f"h2o_l2_{args.start_size + hh + args.h2o_recent_size}",
                            "compress_fn": h2o_l2_compress,
                            "kwargs": {"start_size": args.start_size, "heavy_hitter_size": hh,
                                       "recent_size": args.h2o_recent_size}})
    elif args.method == "snapkv_lite":
        obs_windows = [int(x) for x in args.observation_windows.split(",")]
        for keep in [int(x) for x in args.snapkv_keep_sizes.split(",")]:
            if not args.no_recent_only:
                methods.append(recent(keep))
            for obs in obs_windows:
                methods.append({"name": f"snapkv_{keep}_obs{obs}",
                                "compress_fn": snapkv_lite_compress,
                                "kwargs": {"observation_window": obs, "keep_size": keep}})
    elif args.method == "pyramid_kv":
        for base in [int(x) for x in args.base_sizes.split(",")]:
            if not args.no_recent_only:
                methods.append(recent(base))
            methods.append({"name": f"pyramid_{base}", "compress_fn": pyramid_kv_compress,
                            "kwargs": {"base_size": base, "layer_decay": args.layer_decay,
                                       "min_size": args.min_size,
                                       "profile": args.pyramid_profile}})
    elif args.method == "adaptive_l2":
        for target in [int(x) for x in args.target_sizes.split(",")]:
            if not args.no_recent_only:
                methods.append(recent(target))
            methods.append({"name": f"adaptive_{target}", "compress_fn": adaptive_l2_compress,
                            "kwargs": {"target_size": target, "soft_limit": args.soft_limit,
                                       "hard_limit": args.hard_limit}})
    elif args.compare_all:
        for size, hh, h2o_recent, obs, pmin, soft, hard in ((512, 64, 444, 32, 64, 256, 1024),
                                                             (1024, 128, 892, 64, 128, 512, 2048)):
            methods.extend([
                recent(size),
                {"name": f"streaming_{size}", "compress_fn": streaming_llm_compress,
                 "kwargs": {"start_size": 4, "recent_size": size - 4}},
                {"name": f"h2o_l2_{size}", "compress_fn": h2o_l2_compress,
                 "kwargs": {"start_size": 4, "heavy_hitter_size": hh, "recent_size": h2o_recent}},
                {"name": f"snapkv_{size}", "compress_fn": snapkv_lite_compress,
                 "kwargs": {"observation_window": obs, "keep_size": size}},
                {"name": f"pyramid_{size}", "compress_fn": pyramid_kv_compress,
                 "kwargs": {"base_size": size, "layer_decay": 0.9, "min_size": pmin}},
                {"name": f"adaptive_{size}", "compress_fn": adaptive_l2_compress,
                 "kwargs": {"target_size": size, "soft_limit": soft, "hard_limit": hard}},
                {"name": f"fix_l2_{size}", "compress_fn": fix_size_l2_compress,
                 "kwargs": {"fix_kv_size": size, "strategy": "keep_low", "keep_ratio": 0.5}},
            ])
    return methods


# (flag, type, default, help) -- the reference's argument surface (scripts/benchmark.py:551-626):
# same flags, types, defaults and choices; store_true flags have type None
_METHOD_CHOICES = ["l2_compress", "fix_size_l2", "streaming_llm", "h2o_l2", "snapkv_lite",
                   "pyramid_kv", "adaptive_l2"]
_ARGS = (
    ("--model_id", str, "EleutherAI/pythia-2.8b", "HF model id (cache first, then the Hub)"),
    ("--num_samples", int, 2, "PG-19 samples"),
    ("--max_tokens", int, 2000, "tokens of the teacher-forced PPL pass"),
    ("--max_new_tokens", int, 500, "generated tokens (TTFT / TPOT)"),
    ("--skip_layers", str, "0,1", "layers never compressed, comma-separated"),
    ("--no_baseline", None, False, "do not run the uncompressed baseline"),
    ("--no_recent_only", None, False, "no recent_only control group for fixed-size methods"),
    ("--num_warmup", int, 3, "warmup iterations"),
    ("--method", str, None, "method to sweep"),
    ("--compare_all", None, False, "every method at the 512 / 1024 defaults"),
    ("--compare_new", None, False, "the newer methods (selects none, as in the reference)"),
    ("--keep_ratios", str, "0.8,0.5,0.3", "keep_ratio list (l2_compress, fix_size_l2)"),
    ("--prune_after", int, 100, "l2_compress: compress only beyond this length"),
    ("--fix_kv_sizes", str, "256,512", "fix_size_l2: cache sizes"),
    ("--strategies", str, "keep_low", "fix_size_l2: keep_low / keep_high / random"),
    ("--start_size", int, 4, "attention-sink tokens"),
    ("--recent_sizes", str, "252,508,1020", "streaming_llm: recent windows"),
    ("--heavy_hitter_sizes", str, "32,64,128", "h2o_l2: heavy hitters"),
    ("--h2o_recent_size", int, 444, "h2o_l2: recent window"),
    ("--observation_windows", str, "16,32,64", "snapkv_lite: observation windows"),
    ("--snapkv_keep_sizes", str, "512", "snapkv_lite: kept tokens"),
    ("--base_sizes", str, "256,512", "pyramid_kv: first-layer budgets"),
    ("--layer_decay", float, 0.9, "pyramid_kv: per-layer decay"),
    ("--min_size", int, 64, "pyramid_kv: smallest per-layer budget"),
    ("--pyramid_profile", str, "exponential", "pyramid_kv: budget profile"),
    ("--target_sizes", str, "256,512", "adaptive_l2: target sizes"),
    ("--soft_limit", int, 256, "adaptive_l2: no compression up to this length"),
    ("--hard_limit", int, 1024, "adaptive_l2: full compression beyond this length"),
    # offline extensions (not in the reference)
    ("--random_model", str, None, "[offline] random-weight GPT-NeoX of this geometry"),
    ("--text_file", str, None, "[offline] samples from a local text file"),
    ("--synthetic_text", None, False, "[offline] deterministic pseudo-text samples"),
    ("--tie_policy", str, "reference", "[extension] tie order of the selections: the "
                                       "reference's (default) or stable (faster, not bit-exact)"),
)
_CHOICES = {"--method": _METHOD_CHOICES, "--pyramid_profile": ["exponential", "linear", "constant"],
            "--random_model": sorted(RANDOM_MODELS), "--tie_policy": ["reference", "stable"]}


def build_parser():
    p = argparse.ArgumentParser(description="Unified Benchmark for KV Cache Compression",
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    for flag, typ, default, help_text in _ARGS:
        if typ is None:
            p.add_argument(flag, action="store_true", help=help_text)
        else:
            p.add_argument(flag, type=typ, default=default, choices=_CHOICES.get(flag),
                           help=help_text)
    return p


def main(argv=None):
    parser = build_parser()
    args = parser.parse_args(argv)
    if not args.method and not args.compare_all and not args.compare_new:
        parser.error("Must specify --method, --compare_all, or --compare_new")
    from kvcompress import _engine
    prev = _engine.set_tie_policy(args.tie_policy)
    try:
        return _run(args)
    finally:
        _engine.set_tie_policy(prev)


def _run(args):
    skip_layers = [int(x) for x in args.skip_layers.split(",")]

    print("=" * 70)
    print("KV Cache Compression Benchmark")
    print("=" * 70)
    print("\nConfiguration:")
    print(f"  Model: {args.random_model + ' (random weights)' if args.random_model else args.model_id}")
    print(f"  Method: {args.method or ('compare_all' if args.compare_all else 'compare_new')}")
    print(f"  Skip layers: {skip_layers}")
    if args.tie_policy != "reference":
        print(f"  Tie policy: {args.tie_policy} (not the reference's tie order)")
    print(f"  Number of samples: {args.num_samples}")
    print(f"  Max eval tokens: {args.max_tokens}")
    print(f"  Max new tokens: {args.max_new_tokens}")
    print(f"  Warmup iterations: {args.num_warmup}")

    if args.random_model:
        model, tokenizer, device = load_random_model(args.random_model, get_device())
    else:
        model, tokenizer, device = load_model_and_tokenizer(args.model_id)
    if args.num_warmup > 0:
        warmup_model(model, tokenizer, device, num_warmup=args.num_warmup)

    if args.text_file:
        samples = load_text_file_samples(args.text_file, args.num_samples)
    elif args.synthetic_text:
        samples = synthetic_samples(args.num_samples)
    else:
        samples = load_pg19_samples(args.num_samples)
    if not samples:
        print("No samples loaded. Exiting.")
        return []

    methods_config = build_methods_config(args)
    print("\nMethods to test:")
    for m in methods_config:
        print(f"  - {m['name']}: {m['kwargs']}")

    all_results = []
    for i, text in enumerate(samples):
        print(f"\n{'=' * 70}\nSample {i+1}/{len(samples)} ({len(text)} characters)\n{'=' * 70}")
        all_results.extend(run_benchmark_suite(
            model=model, tokenizer=tokenizer, text=text, methods_config=methods_config,
            max_new_tokens=args.max_new_tokens, eval_tokens=args.max_tokens,
            skip_layers=skip_layers, device=device))

    print("\n" + "=" * 80)
    print("AGGREGATED RESULTS (averaged across samples)")
    print("=" * 80)
    grouped = {}
    for r in all_results:
        grouped.setdefault(r.get("method", "unknown"), []).append(r)
    print(f"\n{'Method':<25} {'TTFT(s)':>10} {'TPOT(s)':>10} "
          f"{'Thruput':>10} {'PPL':>10} {'Acc':>10} {'Cache':>8}")
    print("-" * 90)

    def avg(rs, key):
        return float(np.mean([r[key] for r in rs]))

    base = grouped.get("baseline")
    for method, rs in grouped.items():
        print(f"{method:<25} {avg(rs, 'ttft'):>10.4f} {avg(rs, 'tpot'):>10.4f} "
              f"{avg(rs, 'throughput'):>10.2f} {avg(rs, 'perplexity'):>10.2f} "
              f"{avg(rs, 'accuracy'):>10.2%} {avg(rs, 'final_cache_size'):>8.0f}")
    print("=" * 90)
    if base is not None and len(grouped) > 1:
        bppl, bacc = avg(base, "perplexity"), avg(base, "accuracy")
        bthr, btpot = avg(base, "throughput"), avg(base, "tpot")
        print("\nComparison with baseline (Throughput ↑ better, TPOT ↓ better, PPL ↓ better):")
        for method, rs in grouped.items():
            if method == "baseline":
                continue
            thr = (avg(rs, "throughput") / bthr - 1) * 100 if bthr > 0 else 0
            tpot = (1 - avg(rs, "tpot") / btpot) * 100 if btpot > 0 else 0
            ppl = (avg(rs, "perplexity") / bppl - 1) * 100 if bppl > 0 else 0
            acc = (avg(rs, "accuracy") / bacc - 1) * 100 if bacc > 0 else 0
            print(f"  {method}: Throughput {thr:+.1f}%, TPOT {tpot:+.1f}%, PPL {ppl:+.1f}%, "
                  f"Acc {acc:+.1f}%")
    print("\nBenchmark completed!")
    return all_results


if __name__ == "__main__":
    main()
