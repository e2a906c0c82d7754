"""h2o_attention: the accumulated-attention manager reproduces the
reference's state and heavy hitters (CPU), and the engine's compaction with those indices -- and
the L2-norm fallback without a manager -- reproduces the reference's K/V bytes (GPU).  Golden
data from the unmodified reference: tests/golden/gen_h2o_attention.py."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import gen_h2o_attention as G  # noqa: E402  (input recipe only; runs nothing at import)
import prng  # noqa: E402

GOLD = np.load(os.path.join(HERE, "golden", "h2o_attention.npz"))
SHA = json.load(open(os.path.join(HERE, "golden", "h2o_attention.json")))


def _sha(t):
    a = np.ascontiguousarray(t.detach().cpu().numpy())
    return hashlib.sha256(str(a.shape).encode() + a.tobytes()).hexdigest()


def _drive(device):
    from kvcompress.methods.h2o_attention import H2OAttentionManager, h2o_attention_compress
    S = G.LENS[-1]
    kv = [(torch.from_numpy(prng.gen_keys(50 + i, (1, G.H, S, G.D), "fp32")).to(device),
           torch.from_numpy(prng.gen_values(50 + i, (1, G.H, S, G.D), "fp32")).to(device))
          for i in range(G.L)]
    mgr = H2OAttentionManager(decay_factor=0.5, num_layers=G.L, num_heads=G.H, **G.KW)
    for step, key_len in enumerate(G.LENS[:-1]):
        mgr.update_attention_scores(
            tuple(None if li == 2 else G.attention(step, li, key_len).to(device)
                  for li in range(G.L)), skip_layers=[])
    atts = tuple(None if li == 2 else G.attention(9, li, S).to(device) for li in range(G.L))
    return kv, mgr, atts


def test_oracle_manager_matches_reference_dyadic_golden():
    """The CPU restatement (oracle/h2o_oracle.py) on the round-1 dyadic fixture."""
    from oracle import h2o_oracle as HO
    S = G.LENS[-1]
    mgr = HO.H2OManager(decay_factor=0.5, **G.KW)
    for step, key_len in enumerate(G.LENS[:-1]):
        mgr.update_attention_scores(tuple(None if li == 2 else G.attention(step, li, key_len).numpy()
                                          for li in range(G.L)))
    mgr.update_attention_scores(tuple(None if li == 2 else G.attention(9, li, S).numpy()
                                      for li in range(G.L)))
    for li in range(G.L):
        if f"acc_{li}" in GOLD:
            np.testing.assert_array_equal(mgr.acc[li], GOLD[f"acc_{li}"])
        else:
            assert li not in mgr.acc
        np.testing.assert_array_equal(mgr.get_heavy_hitter_indices(li, S), GOLD[f"idx_{li}"])


@pytest.mark.gpu
def test_manager_state_and_heavy_hitters_match_reference():
    kv, mgr, atts = _drive("cuda:0")
    mgr.update_attention_scores(atts, skip_layers=[])
    S = G.LENS[-1]
    for li in range(G.L):
        if f"acc_{li}" in GOLD:
            np.testing.assert_array_equal(mgr.accumulated_attention[li].cpu().numpy(),
                                          GOLD[f"acc_{li}"])
        else:
            assert li not in mgr.accumulated_attention
        np.testing.assert_array_equal(mgr.get_heavy_hitter_indices(li, S).cpu().numpy(),
                                      GOLD[f"idx_{li}"])


def test_registry_and_exports():
    from kvcompress.methods import get_compress_fn, list_methods
    from kvcompress.methods.h2o_attention import (H2OAttentionManager,  # noqa: F401
                                                  create_h2o_manager_from_model,
                                                  h2o_attention_compress)
    assert "h2o_attention" in list_methods()
    assert get_compress_fn("h2o_attention") is h2o_attention_compress


def test_cpu_tensors_raise():
    """No CPU path: CPU attention (the manager's sums) and CPU K/V (the compaction) raise."""
    from kvcompress.methods.h2o_attention import H2OAttentionManager, h2o_attention_compress
    mgr = H2OAttentionManager(decay_factor=0.5, num_layers=G.L, num_heads=G.H, **G.KW)
    with pytest.raises(RuntimeError, match="ROCm GPU tensors only"):
        mgr.update_attention_scores((G.attention(0, 0, 600),))
    S = G.LENS[-1]
    kv = [(torch.zeros(1, G.H, S, G.D), torch.zeros(1, G.H, S, G.D))]
    with pytest.raises(RuntimeError, match="ROCm GPU tensors only"):
        h2o_attention_compress(kv, **G.KW)


@pytest.mark.gpu
def test_engine_compaction_matches_reference():
    from kvcompress.methods.h2o_attention import h2o_attention_compress
    kv, mgr, atts = _drive("cuda:0")
    out = h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                 skip_layers=[], **G.KW)
    for li in range(G.L):
        assert _sha(out[li][0]) == SHA[f"k_{li}"], li
        assert _sha(out[li][1]) == SHA[f"v_{li}"], li
    out = h2o_attention_compress(list(kv), skip_layers=[1], **G.KW)  # L2-norm fallback
    for li in range(G.L):
        assert _sha(out[li][0]) == SHA[f"fk_{li}"], li
        assert _sha(out[li][1]) == SHA[f"fv_{li}"], li
