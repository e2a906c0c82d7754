"""Golden fixture for h2o_attention at the long-context geometry (build container only):

    cd /tmp && PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_h2o_attention_long.py

BASELINE cfg4's sizes -- start 4, heavy 64, recent 444 over S = 16 384 positions (a middle of
15 936: the heap select of std::partial_sort, and the engine's side-stream copy of the fixed rows
for middles >= OVERLAP_MIN_ZONE) -- run through the UNMODIFIED reference H2OAttentionManager /
h2o_attention_compress on CPU (torch.set_num_threads(THREADS)), three q = 1 decode steps of the
same shape (the engine replays the third natively), in bf16 and fp32.  Writes data only
(h2o_attention_long.json): per step, SHA-256 of every layer's accumulated-attention tensor, the
heavy-hitter indices and SHA-256 / shape of every compressed K / V.  Inputs are regenerated from
recipes: attention from tests/golden/h2o_inputs.py (tie-heavy, non-dyadic), K / V from
tests/golden/prng.py (one K/V per layer, reused by every step).
Reference: kvcompress/methods/h2o_attention.py:84-213 (manager), :216-361 (compress).
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import h2o_inputs  # noqa: E402
import prng  # noqa: E402

THREADS = 8
H, D, S = 32, 80, 16384
LAYERS = 2
STEPS = 3
KW = dict(start_size=4, heavy_hitter_size=64, recent_size=444)
DECAY = 0.9
DTYPES = ("bf16", "fp32")


def att_seed(step, layer):
    return 500000 + 100 * step + layer


def kv_seed(layer):
    return 81000 + layer


def sha(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(str(a.shape).encode() + a.tobytes()).hexdigest()


def to_torch(a, dtype):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.view(torch.bfloat16) if dtype == "bf16" else t


def to_np(t, dtype):
    t = t.contiguous()
    return t.view(torch.int16).numpy().view(np.uint16) if dtype == "bf16" else t.numpy()


def main():
    assert os.path.abspath(os.environ.get("PYTHONPATH", "").split(":")[0]) == "/root/reference"
    from kvcompress.methods.h2o_attention import (  # the reference
        H2OAttentionManager, h2o_attention_compress)
    torch.set_num_threads(THREADS)
    out = dict(threads=THREADS, capability=torch.backends.cpu.get_cpu_capability(), H=H, D=D,
               S=S, layers=LAYERS, steps=STEPS, kw=KW, decay=DECAY, results={})
    for dt in DTYPES:
        kv = [(to_torch(prng.gen_keys(kv_seed(li), (1, H, S, D), dt), dt),
               to_torch(prng.gen_values(kv_seed(li), (1, H, S, D), dt), dt))
              for li in range(LAYERS)]
        mgr = H2OAttentionManager(decay_factor=DECAY, num_layers=LAYERS, num_heads=H, **KW)
        recs = []
        for st in range(STEPS):
            atts = tuple(to_torch(h2o_inputs.attention(att_seed(st, li), H, 1, S, dt), dt)
                         for li in range(LAYERS))
            res = h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                         skip_layers=[], **KW)
            recs.append(dict(
                k=[sha(to_np(r[0], dt)) for r in res],
                v=[sha(to_np(r[1], dt)) for r in res],
                n_out=[int(r[0].shape[2]) for r in res],
                acc=[sha(to_np(mgr.accumulated_attention[li], dt)) for li in range(LAYERS)],
                idx=[mgr.get_heavy_hitter_indices(li, S).tolist() for li in range(LAYERS)]))
        out["results"][dt] = recs
        print(dt, [r["n_out"] for r in recs], [len(r["idx"][0]) for r in recs])
    with open(os.path.join(HERE, "h2o_attention_long.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
