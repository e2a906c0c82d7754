"""Per-step digests of an evaluation loop's compress calls (test infrastructure, data only).

Recorder(fn) wraps a compress_fn: every call records
  kd -- a digest of the call's INPUT keys (every layer's K bytes and shape), and
  pd -- a digest of the positions the call kept (every layer's output rows), recovered by
        calling fn a second time with position-encoding values (prng.encode_positions, as
        gen_goldens.py does) in place of V,
and returns fn's result on the real values.  Comparing two loops' records step by step says
where their inputs first differ (kd) and, up to there, whether the two compress functions kept
the same positions from the same keys (pd).  tests/golden/gen_eval_attention.py records the
unmodified reference's loops; tests/test_eval_attention.py replays them.
"""
import hashlib

import numpy as np
import torch

import prng

DIGEST_HEX = 12  # 48 bits per digest


def _h(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()[:DIGEST_HEX]


def _np32(t):
    return t.detach().to("cpu", torch.float32).contiguous().numpy()


def k_digest(kv_list):
    return _h(*[_np32(k) for k, _ in kv_list])


def pos_digest(out_enc):
    pos = []
    for _, v in out_enc:
        p, ok = prng.decode_positions(_np32(v), "fp32")
        assert ok, "position-encoded values came back altered"
        pos.append(p.astype(np.int32))
    return _h(*pos)


class Recorder:
    def __init__(self, fn):
        self.fn = fn
        self.steps = []  # [(kd, pd)] per call

    def __call__(self, kv_list, **kw):
        kv_list = list(kv_list)
        kd = k_digest(kv_list)
        enc = [(k, torch.from_numpy(prng.encode_positions(tuple(v.shape), "fp32")).to(v.dtype))
               for k, v in kv_list]
        pd = pos_digest(self.fn(enc, **kw))
        self.steps.append((kd, pd))
        return self.fn(kv_list, **kw)

    def packed(self):
        """The record as one string, 'kd:pd' per call, comma-separated."""
        return ",".join(f"{a}:{b}" for a, b in self.steps)


def unpack(s):
    return [tuple(x.split(":")) for x in s.split(",")] if s else []


def first_divergence(got, ref):
    """Compare two records: (n_compared, first step whose input keys differ or None,
    [steps before it whose kept positions differ])."""
    n = min(len(got), len(ref))
    bad = []
    for i in range(n):
        if got[i][0] != ref[i][0]:
            return i, i, bad
        if got[i][1] != ref[i][1]:
            bad.append(i)
    return n, None, bad
