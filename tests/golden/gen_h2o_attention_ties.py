"""Golden fixtures for h2o_attention on tie-heavy, non-dyadic attention (build container only):

    cd /tmp && PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_h2o_attention_ties.py

Replays SCENARIOS (below) through the UNMODIFIED reference H2OAttentionManager /
h2o_attention_compress on CPU (torch.set_num_threads(THREADS)) and writes data only:
  h2o_attention_ties.json - per scenario and step: SHA-256 of every layer's accumulated-attention
                            tensor (bytes + shape), heavy-hitter indices, and the SHA-256 / shape of
                            every compressed K / V
Inputs are regenerated from recipes: attention from tests/golden/h2o_inputs.py, K / V from
tests/golden/prng.py.  Every branch of update_attention_scores runs (first call, zero-extension,
equal length, reset after the cache shrank), q > 1 (prefill, 3-token steps) and q == 1, skipped
layers and None attentions, topk's partial_sort (k * 64 <= m) and nth_element paths, and middle
regions long enough that torch splits the head sum over threads.
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
H, D = 32, 64


def _s(op, **kw):
    return dict(op=op, **kw)


# step: ("update", k, q) or ("compress", S, q); att[layer] = True/False (None attention),
# skip = skip_layers of the call
SCENARIOS = [
    dict(name="hh64", kw=dict(start_size=4, heavy_hitter_size=64, recent_size=444), decay=0.9,
         steps=[_s("compress", S=1500, q=1500, att=[1, 1, 1], skip=[]),      # first call, prefill
                _s("update", k=1501, q=1, att=[1, 1, 0], skip=[]),           # zero-extend
                _s("compress", S=1502, q=1, att=[1, 1, 1], skip=[1]),        # extend / skip
                _s("compress", S=513, q=1, att=[1, 1, 1], skip=[]),          # reset (shrunk)
                _s("compress", S=513, q=1, att=[1, 0, 1], skip=[]),          # equal length
                _s("compress", S=2100, q=3, att=[1, 1, 1], skip=[2])]),      # extend, q = 3
    dict(name="hh16", kw=dict(start_size=4, heavy_hitter_size=16, recent_size=100), decay=0.85,
         steps=[_s("compress", S=1200, q=37, att=[1, 1, 1], skip=[]),
                _s("compress", S=1201, q=1, att=[1, 1, 1], skip=[]),
                _s("compress", S=1201, q=1, att=[1, 1, 1], skip=[0]),
                _s("compress", S=3000, q=2, att=[1, 1, 1], skip=[])]),
]
DTYPES = ("fp32", "bf16", "fp16")
LAYERS = 3


def att_seed(si, step, layer):
    return 100000 * si + 100 * step + layer


def kv_seed(si, step, layer):
    return 7000 + 1000 * si + 10 * step + layer


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
               layers=LAYERS, scenarios=SCENARIOS, results={})
    for si, sc in enumerate(SCENARIOS):
        for dt in DTYPES:
            mgr = H2OAttentionManager(decay_factor=sc["decay"], num_layers=LAYERS, num_heads=H,
                                      **sc["kw"])
            recs = []
            for st, step in enumerate(sc["steps"]):
                k = step["k"] if step["op"] == "update" else step["S"]
                atts = tuple(to_torch(h2o_inputs.attention(att_seed(si, st, li), H, step["q"], k,
                                                           dt), dt) if step["att"][li] else None
                             for li in range(LAYERS))
                rec = {}
                if step["op"] == "update":
                    mgr.update_attention_scores(atts, skip_layers=step["skip"])
                    S = k
                else:
                    S = step["S"]
                    kv = [(to_torch(prng.gen_keys(kv_seed(si, st, li), (1, H, S, D), dt), dt),
                           to_torch(prng.gen_values(kv_seed(si, st, li), (1, H, S, D), dt), dt))
                          for li in range(LAYERS)]
                    res = h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                                 skip_layers=step["skip"], **sc["kw"])
                    rec["k"] = [sha(to_np(r[0], dt)) for r in res]
                    rec["v"] = [sha(to_np(r[1], dt)) for r in res]
                    rec["n_out"] = [int(r[0].shape[2]) for r in res]
                rec["acc"] = [sha(to_np(mgr.accumulated_attention[li], dt))
                              if li in mgr.accumulated_attention else None
                              for li in range(LAYERS)]
                rec["idx"] = [mgr.get_heavy_hitter_indices(li, S).tolist()
                              for li in range(LAYERS)]
                recs.append(rec)
            out["results"][f"{sc['name']}/{dt}"] = recs
            print(sc["name"], dt, [r["n_out"] if "n_out" in r else None for r in recs])
    with open(os.path.join(HERE, "h2o_attention_ties.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
