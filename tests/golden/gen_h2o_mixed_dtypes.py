"""Golden fixtures for h2o_attention when the carried accumulation and a new step's attention
differ in dtype (build container only):

    cd /tmp && PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_h2o_mixed_dtypes.py

The reference type-promotes through `existing * decay_factor`, `torch.cat` and `+`
(kvcompress/methods/h2o_attention.py:129-151): an accumulation of one 16/32-bit float dtype
combined with attention of another becomes float32; a reset (the cache shrank) starts over in the
attention's dtype.  SCENARIOS (below) drive the UNMODIFIED reference H2OAttentionManager /
h2o_attention_compress through such steps on CPU (torch.set_num_threads(THREADS)); stored, data
only (h2o_attention_mixed.json): per step, every layer's accumulated-attention dtype and SHA-256
(bytes + shape), the heavy-hitter indices, and the SHA-256 / shape of every compressed K / V.
Attention comes from tests/golden/h2o_inputs.py (tie-heavy, non-dyadic), K / V (bf16) from
tests/golden/prng.py.
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
H, D, LAYERS = 32, 64, 3
KV_DTYPE = "bf16"


def _s(op, dt, **kw):
    return dict(op=op, dt=dt, **kw)


# step: op "update" (k keys) or "compress" (S positions); dt = the attention's dtype;
# att[layer] = False: None attention; skip = skip_layers of the call
SCENARIOS = [
    dict(name="fp32_then_bf16", kw=dict(start_size=4, heavy_hitter_size=64, recent_size=444),
         decay=0.9,
         steps=[_s("compress", "fp32", S=1500, q=1500, att=[1, 1, 1], skip=[]),
                _s("update", "bf16", k=1501, q=1, att=[1, 1, 0], skip=[]),   # extend -> fp32
                _s("compress", "bf16", S=1501, q=1, att=[1, 1, 1], skip=[]),  # equal -> fp32
                _s("compress", "bf16", S=1502, q=3, att=[1, 1, 1], skip=[1]),  # extend, skip
                _s("compress", "bf16", S=800, q=1, att=[1, 1, 1], skip=[]),   # reset -> bf16
                _s("compress", "fp16", S=801, q=1, att=[1, 1, 1], skip=[])]),  # bf16+fp16 -> fp32
    dict(name="bf16_then_fp32", kw=dict(start_size=4, heavy_hitter_size=16, recent_size=100),
         decay=0.85,
         steps=[_s("compress", "bf16", S=1200, q=37, att=[1, 1, 1], skip=[]),
                _s("compress", "fp32", S=1201, q=1, att=[1, 1, 1], skip=[]),   # extend -> fp32
                _s("compress", "bf16", S=1201, q=1, att=[1, 1, 1], skip=[0]),  # equal -> fp32
                _s("compress", "fp32", S=3000, q=2, att=[1, 1, 1], skip=[])]),
    dict(name="fp16_then_bf16", kw=dict(start_size=4, heavy_hitter_size=32, recent_size=60),
         decay=0.7,
         steps=[_s("compress", "fp16", S=600, q=5, att=[1, 1, 1], skip=[]),
                _s("compress", "bf16", S=600, q=1, att=[1, 0, 1], skip=[]),    # equal -> fp32
                _s("update", "fp16", k=601, q=1, att=[1, 1, 1], skip=[]),
                _s("compress", "fp16", S=602, q=1, att=[1, 1, 1], skip=[])]),
]


def att_seed(si, step, layer):
    return 500000 + 100000 * si + 100 * step + layer


def kv_seed(si, step, layer):
    return 90000 + 1000 * si + 10 * step + layer


def sha(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(str(a.shape).encode() + a.tobytes()).hexdigest()


def to_torch(a, dtype):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.view(torch.bfloat16) if dtype == "bf16" else t


def t2np(t):
    """Bytes of a tensor of any of the three dtypes (bf16 as uint16 bit patterns)."""
    t = t.contiguous()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


DTNAME = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "fp16"}


def main():
    assert os.path.abspath(os.environ.get("PYTHONPATH", "").split(":")[0]) == "/root/reference"
    from kvcompress.methods.h2o_attention import (  # the reference
        H2OAttentionManager, h2o_attention_compress)
    torch.set_num_threads(THREADS)
    out = dict(threads=THREADS, capability=torch.backends.cpu.get_cpu_capability(), H=H, D=D,
               layers=LAYERS, kv_dtype=KV_DTYPE, scenarios=SCENARIOS, results={})
    for si, sc in enumerate(SCENARIOS):
        mgr = H2OAttentionManager(decay_factor=sc["decay"], num_layers=LAYERS, num_heads=H,
                                  **sc["kw"])
        recs = []
        for st, step in enumerate(sc["steps"]):
            k = step["k"] if step["op"] == "update" else step["S"]
            atts = tuple(to_torch(h2o_inputs.attention(att_seed(si, st, li), H, step["q"], k,
                                                       step["dt"]), step["dt"])
                         if step["att"][li] else None for li in range(LAYERS))
            rec = {}
            if step["op"] == "update":
                mgr.update_attention_scores(atts, skip_layers=step["skip"])
                S = k
            else:
                S = step["S"]
                kv = [(to_torch(prng.gen_keys(kv_seed(si, st, li), (1, H, S, D), KV_DTYPE),
                                KV_DTYPE),
                       to_torch(prng.gen_values(kv_seed(si, st, li), (1, H, S, D), KV_DTYPE),
                                KV_DTYPE)) for li in range(LAYERS)]
                res = h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                             skip_layers=step["skip"], **sc["kw"])
                rec["k"] = [sha(t2np(r[0])) for r in res]
                rec["v"] = [sha(t2np(r[1])) for r in res]
                rec["n_out"] = [int(r[0].shape[2]) for r in res]
            accs = [mgr.accumulated_attention.get(li) for li in range(LAYERS)]
            rec["acc"] = [None if a is None else sha(t2np(a)) for a in accs]
            rec["acc_dtype"] = [None if a is None else DTNAME[a.dtype] for a in accs]
            rec["idx"] = [mgr.get_heavy_hitter_indices(li, S).tolist() for li in range(LAYERS)]
            recs.append(rec)
        out["results"][sc["name"]] = recs
        print(sc["name"], [r["acc_dtype"] for r in recs])
    with open(os.path.join(HERE, "h2o_attention_mixed.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
