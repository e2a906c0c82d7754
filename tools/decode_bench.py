"""Per-token decode-step latency of the drop-in compress functions:
32 layers of [1,32,S,128] bf16 where S = the method's steady-state cache + 1 (one new token),
one compress call per step, as evaluate_with_compression makes it.  Reports the engine's
wall time per call (synchronised) and, for comparison, the reference's torch op sequence run on
the same GPU tensors (written inline here: norm -> argsort -> [:k] -> sort -> gather -> cat).
GPU box only (tuning / evidence)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress.methods import get_compress_fn  # noqa: E402

dev = torch.device("cuda:0")
L, H, D = 32, 32, 128
g = torch.Generator(device=dev).manual_seed(0)


def layers_of(S):
    return [(torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16),
             torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16))
            for _ in range(L)]


def ref_fix_size_torch(kv, fix):
    """The reference's fix_size_l2 keep_low op sequence (fix_size_l2.py:99-150) on GPU tensors."""
    out = []
    for k, v in kv:
        S = k.size(2)
        if S <= fix:
            out.append((k, v))
            continue
        n = torch.norm(k, p=2, dim=-1)
        idx = torch.argsort(n, dim=-1)[:, :, :fix]
        idx, _ = torch.sort(idx, dim=-1)
        e = idx.unsqueeze(-1).expand(-1, -1, -1, D)
        out.append((torch.gather(k, 2, e), torch.gather(v, 2, e)))
    return out


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


cases = [
    ("fix_size_l2", dict(fix_kv_size=512, keep_ratio=0.0, skip_layers=[]), 513),
    ("streaming_llm", dict(start_size=4, recent_size=1020, skip_layers=[]), 1025),
    ("h2o_l2", dict(start_size=4, heavy_hitter_size=64, recent_size=444, skip_layers=[]), 513),
    ("snapkv_lite", dict(observation_window=32, keep_size=512, skip_layers=[]), 513),
    ("pyramid_kv", dict(base_size=512, skip_layers=[]), 513),
    ("adaptive_l2", dict(skip_layers=[]), 257),
]
res = {}
for name, kw, S in cases:
    kv = layers_of(S)
    fn = get_compress_fn(name)
    res[name] = {"S": S, "engine_ms_per_step": round(timeit(lambda: fn(list(kv), **kw)), 4)}
# h2o_attention: per step the manager accumulates one query row of attention per layer, then the
# heavy hitters (head sum + topk) and the compaction -- S = 513, heavy_hitter_size 64 / recent 444
from kvcompress.methods.h2o_attention import H2OAttentionManager, h2o_attention_compress  # noqa
kv = layers_of(513)
att = tuple(torch.softmax(torch.randn(1, H, 1, 513, device=dev, generator=g), -1).to(torch.bfloat16)
            for _ in range(L))
mgr = H2OAttentionManager(start_size=4, heavy_hitter_size=64, recent_size=444)
res["h2o_attention"] = {"S": 513, "engine_ms_per_step": round(timeit(
    lambda: h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr,
                                   skip_layers=[])), 4)}
# a long-context call: heavy hitters over a 15 936-position middle (std::partial_sort path)
kv = layers_of(16384)
att = tuple(torch.softmax(torch.randn(1, H, 1, 16384, device=dev, generator=g), -1).to(torch.bfloat16)
            for _ in range(L))
mgr = H2OAttentionManager(start_size=4, heavy_hitter_size=64, recent_size=444)
res["h2o_attention_s16384"] = {"S": 16384, "engine_ms_per_call": round(timeit(
    lambda: h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr,
                                   skip_layers=[]), reps=10), 4)}
kv = layers_of(513)
res["fix_size_l2"]["reference_ops_on_gpu_ms_per_step"] = round(
    timeit(lambda: ref_fix_size_torch(kv, 512)), 4)
print(json.dumps(res))
