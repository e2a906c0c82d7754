"""Golden fixtures for h2o_attention (build container only):

    cd /tmp && PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_h2o_attention.py

Runs the UNMODIFIED reference H2OAttentionManager / h2o_attention_compress on CPU on
deterministic inputs from tests/golden/prng.py and writes tests/golden/h2o_attention.npz:
accumulated attention after each update and heavy-hitter indices (npz), SHA-256 of the
compressed K/V of every layer (h2o_attention.json).  Attention values are small dyadic rationals and decay_factor = 0.5, so every sum is exact
(summation order cannot matter) and all accumulated scores are distinct (no top-k ties): the
fixture pins the algorithm, not one device's reduction order.
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import prng  # noqa: E402


L, H, D = 3, 4, 64
LENS = [600, 601, 602]
KW = dict(start_size=4, heavy_hitter_size=32, recent_size=100)


def attention(step, layer, key_len):
    """[1,H,1,key_len] fp32, values j/1024 with j a per-(step,layer,head) permutation: exact
    sums, distinct head-sums."""
    rng = np.random.default_rng(1000 * step + layer)
    a = np.stack([rng.permutation(key_len) for _ in range(H)]).astype(np.float32) / 1024.0
    a[1:] *= 0.0  # only head 0 varies: head sums stay distinct after decay
    a[1:] += (np.arange(key_len, dtype=np.float32) % 7) / 1024.0
    return torch.from_numpy(a[None, :, None, :].copy())


def sha(t):
    """SHA-256 of a K/V output's bytes (shape is part of the digest input)."""
    a = np.ascontiguousarray(t.numpy())
    return hashlib.sha256(str(a.shape).encode() + a.tobytes()).hexdigest()


def main():
    assert os.path.abspath(os.environ.get("PYTHONPATH", "").split(":")[0]) == "/root/reference"
    from kvcompress.methods.h2o_attention import (  # the reference
        H2OAttentionManager, h2o_attention_compress)
    out = {}
    S = LENS[-1]
    kv = [(torch.from_numpy(prng.gen_keys(50 + i, (1, H, S, D), "fp32")),
           torch.from_numpy(prng.gen_values(50 + i, (1, H, S, D), "fp32"))) for i in range(L)]
    mgr = H2OAttentionManager(decay_factor=0.5, num_layers=L, num_heads=H, **KW)
    for step, key_len in enumerate(LENS[:-1]):
        atts = tuple(None if li == 2 else attention(step, li, key_len) for li in range(L))
        mgr.update_attention_scores(atts, skip_layers=[])
    atts = tuple(None if li == 2 else attention(9, li, S) for li in range(L))
    res = h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                 skip_layers=[], **KW)
    for li in range(L):
        if li in mgr.accumulated_attention:
            out[f"acc_{li}"] = mgr.accumulated_attention[li].numpy()
        out[f"idx_{li}"] = mgr.get_heavy_hitter_indices(li, S).numpy()
        out[f"k_{li}"], out[f"v_{li}"] = sha(res[li][0]), sha(res[li][1])
    # no manager: the L2-norm fallback
    res = h2o_attention_compress(list(kv), skip_layers=[1], **KW)
    for li in range(L):
        out[f"fk_{li}"], out[f"fv_{li}"] = sha(res[li][0]), sha(res[li][1])
    arrays = {k: v for k, v in out.items() if not isinstance(v, str)}
    np.savez_compressed(os.path.join(HERE, "h2o_attention.npz"), **arrays)
    json.dump({k: v for k, v in out.items() if isinstance(v, str)},
              open(os.path.join(HERE, "h2o_attention.json"), "w"), indent=1)
    print(sorted(out))


if __name__ == "__main__":
    main()
