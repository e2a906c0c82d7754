"""Deterministic attention-probability inputs for the h2o_attention fixtures (test data recipe).

attention(seed, H, q, k, dtype) -> [1, H, q, k] in storage representation (bf16 = uint16 bits).
Row i of a q-query block attends causally to keys [0, k - q + i]; each weight is one of the
integers {1, 2, 3, 5} and the row is normalised by its integer sum in float64 (one correctly
rounded division, then RNE to fp32 and to the storage dtype): non-dyadic probabilities with
heavy ties, computed without any transcendental function so the recipe gives the same bits on
every host.  Keys j % 3 != 0 carry the same weight in every head, so head sums tie exactly
across many positions.
"""
import numpy as np

import prng

LEVELS = np.array([1, 2, 3, 5], dtype=np.int64)
_M = np.uint64(0x9E3779B97F4A7C15)


def attention(seed, H, q, k, dtype):
    j = np.arange(k, dtype=np.uint64)[None, :]
    i = np.arange(q, dtype=np.uint64)[:, None]
    out = np.empty((H, q, k), dtype=np.float32)
    with np.errstate(over="ignore"):
        for h in range(H):
            hh = np.where(j % np.uint64(3) == np.uint64(0), np.uint64(h + 1), np.uint64(0))
            key = (np.uint64(seed) * np.uint64(1000003) + i * np.uint64(7919)) ^ \
                  (j * np.uint64(2654435761) + hh * np.uint64(97))
            mix = (key * _M) >> np.uint64(60)
            w = LEVELS[(mix % np.uint64(4)).astype(np.int64)]
            w = np.where(j.astype(np.int64) <= k - q + i.astype(np.int64), w, 0)
            out[h] = (w.astype(np.float64) / w.sum(axis=1, keepdims=True)).astype(np.float32)
    return prng.to_dtype(out.reshape(-1), dtype).reshape(1, H, q, k)
