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
        if getattr(self, "rows", None) is not None:
            self.rows.append(np.stack([_np32(kv_list[l][0][:, :, -1:, :])
                                       for l in self.row_layers]))
        enc = [(k, torch.from_numpy(prng.encode_positions(tuple(v.shape), "fp32")).to(v.dtype))
               for k, v in kv_list]
        pd = pos_digest(self.fn(enc, **kw))
        self.steps.append((kd, pd))
        return self.fn(kv_list, **kw)

    def new_rows(self, layers):
        """Keep, from every call, the last K row of each of `layers` (the token the model
        appended since the previous call): with the first call's cache, enough to replay every
        call's input without the model (replay)."""
        self.row_layers = list(layers)
        self.rows = []
        return self

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


def replay(fn, rows, n_layers, row_layers, kwargs, steps=None):
    """Re-run a recorded loop's compress calls without its model: the cache starts empty and
    every call appends one row per layer -- the recorded K row for `row_layers` (`rows`:
    [calls, len(row_layers), B, H, 1, D] float32), zeros for the others, which must be layers
    the calls pass through untouched (skip_layers) -- then compresses with fn, values encoding
    positions.  The next call continues from fn's output, as the loop did.  Returns the
    position digests per call (the `pd` of a Recorder record)."""
    B, H, D = rows.shape[2], rows.shape[3], rows.shape[5]
    ks = [torch.zeros(B, H, 0, D) for _ in range(n_layers)]
    out = []
    for t in range(rows.shape[0] if steps is None else steps):
        kv = []
        for l in range(n_layers):
            new = (torch.from_numpy(rows[t, row_layers.index(l)]) if l in row_layers
                   else torch.zeros(B, H, 1, D))
            k = torch.cat([ks[l], new], dim=2)
            v = torch.from_numpy(prng.encode_positions(tuple(k.shape), "fp32"))
            kv.append((k, v))
        res = fn(kv, **kwargs)
        out.append(pos_digest(res))
        ks = [r[0].detach().to("cpu", torch.float32) for r in res]
    return out
