"""The PPL half of the metric: teacher-forced evaluation (evaluate_with_compression, per-token
compression) on a small random-weight GPT-NeoX (pythia architecture, weights unavailable
offline).  GPU: the HIP engine and the CPU oracle produce identical caches at every step, so
every per-token NLL and the PPL match exactly (PPL delta vs reference = 0)."""
import numpy as np
import pytest
import torch

from gpu_util import to_dev, to_np
from oracle import oracle


class ToyTokenizer:
    eos_token_id = None
    pad_token_id = None

    def __init__(self, vocab):
        self.vocab = vocab

    def encode(self, text, return_tensors="pt"):
        ids = [(b * 7 + i) % self.vocab for i, b in enumerate(text.encode())]
        return torch.tensor([ids], dtype=torch.long)


def toy_model(dtype, device, layers=4, heads=4, head_dim=64, vocab=512):
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM
    torch.manual_seed(0)
    cfg = GPTNeoXConfig(vocab_size=vocab, hidden_size=heads * head_dim, num_hidden_layers=layers,
                        num_attention_heads=heads, intermediate_size=4 * heads * head_dim,
                        rotary_pct=0.25, max_position_embeddings=4096)
    return GPTNeoXForCausalLM(cfg).to(dtype).to(device).eval()


def gqa_model(dtype, device, layers=3):
    """A tiny random-weight Llama with grouped-query attention: 4 query heads over 2 K/V heads
    (head_dim 64), the other cache geometry transformers models hand the methods."""
    from transformers import LlamaConfig, LlamaForCausalLM
    torch.manual_seed(0)
    cfg = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512,
                      num_hidden_layers=layers, num_attention_heads=4, num_key_value_heads=2,
                      max_position_embeddings=4096)
    return LlamaForCausalLM(cfg).to(dtype).to(device).eval()


def oracle_compress(name):
    """compress_fn backed by the CPU oracle (test infrastructure)."""
    def fn(kv_list, **kw):
        dev = kv_list[0][0].device
        out = oracle.METHODS[name]([(to_np(k), to_np(v)) for k, v in kv_list], **kw)
        res = []
        for (k, v), (ko, vo, kind) in zip(kv_list, out):
            res.append((k, v) if kind == "same" else (to_dev(ko, dev), to_dev(vo, dev)))
        return res
    return fn


TEXT = "The quick brown fox jumps over the lazy dog. " * 12

CASES = [("fix_size_l2", dict(fix_kv_size=64, keep_ratio=0.5)),
         ("fix_size_l2", dict(fix_kv_size=48, keep_ratio=0.0)),
         ("h2o_l2", dict(start_size=4, heavy_hitter_size=16, recent_size=40)),
         ("snapkv_lite", dict(observation_window=8, keep_size=64)),
         ("streaming_llm", dict(start_size=4, recent_size=60)),
         ("l2_compress", dict(keep_ratio=0.8, prune_after=50)),
         ("pyramid_kv", dict(base_size=80)),
         ("adaptive_l2", dict(target_size=64, soft_limit=32, hard_limit=128))]


def test_harness_runs_with_oracle_on_cpu():
    from kvcompress.evaluate import evaluate_with_compression
    model = toy_model(torch.float32, "cpu", layers=2)
    tok = ToyTokenizer(512)
    r = evaluate_with_compression(model, tok, TEXT[:200], compress_fn=oracle_compress("fix_size_l2"),
                                  compress_kwargs=dict(fix_kv_size=32), max_tokens=120,
                                  skip_layers=[0], show_progress=False)
    assert r["num_tokens"] == 119 and r["final_cache_size"] == 32
    assert np.isfinite(r["perplexity"])
    base = evaluate_with_compression(model, tok, TEXT[:200], max_tokens=120, show_progress=False)
    assert base["final_cache_size"] == 119


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("name,kw", CASES)
def test_ppl_delta_zero_engine_vs_oracle(dtype, name, kw):
    from kvcompress.evaluate import evaluate_with_compression
    from kvcompress.methods import get_compress_fn
    model = toy_model(dtype, "cuda:0")
    tok = ToyTokenizer(512)
    runs = []
    for fn in (get_compress_fn(name), oracle_compress(name)):
        r = evaluate_with_compression(model, tok, TEXT, compress_fn=fn, compress_kwargs=kw,
                                      max_tokens=300, skip_layers=[0], show_progress=False)
        runs.append(r)
    a, b = runs
    assert a["final_cache_size"] == b["final_cache_size"]
    assert a["perplexity"] == b["perplexity"], (a["perplexity"], b["perplexity"])
    assert a["accuracy"] == b["accuracy"]


def test_eager_model_with_compressed_layers_runs_on_cpu():
    """transformers 5's eager attention adds a mask sized for the longest layer; the harness
    runs such a model through utils.key_length_attention (the 4.x mask cut) and restores its
    implementation.  Its PPL agrees with the sdpa run of the same model (fp32, 1e-4)."""
    from kvcompress.benchmark import measure_generation_metrics
    from kvcompress.evaluate import evaluate_with_compression
    model = toy_model(torch.float32, "cpu", layers=2)
    tok = ToyTokenizer(512)
    kw = dict(compress_fn=oracle_compress("fix_size_l2"), compress_kwargs=dict(fix_kv_size=32),
              skip_layers=[0])
    sdpa = evaluate_with_compression(model, tok, TEXT[:200], max_tokens=120, show_progress=False,
                                     **kw)
    model.set_attn_implementation("eager")
    eager = evaluate_with_compression(model, tok, TEXT[:200], max_tokens=120, show_progress=False,
                                      **kw)
    assert model.config._attn_implementation == "eager"
    assert eager["final_cache_size"] == sdpa["final_cache_size"] == 32
    assert abs(eager["perplexity"] / sdpa["perplexity"] - 1) < 1e-4
    g = measure_generation_metrics(model, tok, TEXT[:200], max_new_tokens=40, max_input_tokens=60,
                                   **kw)
    assert g["num_tokens"] == 40 and model.config._attn_implementation == "eager"


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw", [c for c in CASES if c[0] in
                                     ("fix_size_l2", "snapkv_lite", "pyramid_kv", "h2o_l2")])
def test_gqa_ppl_delta_zero_engine_vs_oracle(name, kw):
    from kvcompress.evaluate import evaluate_with_compression
    from kvcompress.methods import get_compress_fn
    model = gqa_model(torch.bfloat16, "cuda:0")
    tok = ToyTokenizer(512)
    a, b = (evaluate_with_compression(model, tok, TEXT, compress_fn=fn, compress_kwargs=kw,
                                      max_tokens=240, skip_layers=[0], show_progress=False)
            for fn in (get_compress_fn(name), oracle_compress(name)))
    assert a["final_cache_size"] == b["final_cache_size"]
    assert a["perplexity"] == b["perplexity"], (a["perplexity"], b["perplexity"])
    assert a["accuracy"] == b["accuracy"]
