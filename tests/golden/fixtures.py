"""Loader for the golden fixtures produced by gen_goldens.py (data only; no reference code)."""
import functools
import hashlib
import json
import os

import numpy as np

import prng

HERE = os.path.dirname(os.path.abspath(__file__))


@functools.lru_cache(maxsize=None)
def cases():
    with open(os.path.join(HERE, "cases.json")) as f:
        return json.load(f)


@functools.lru_cache(maxsize=None)
def positions():
    return dict(np.load(os.path.join(HERE, "positions.npz")))


@functools.lru_cache(maxsize=None)
def prims():
    with open(os.path.join(HERE, "prims.json")) as f:
        meta = json.load(f)
    return meta, dict(np.load(os.path.join(HERE, "prims.npz")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def case_ids(max_elems=None, big=None):
    out = []
    for c in cases()["cases"]:
        n = max(int(np.prod(L["shape"])) for L in c["layers"])
        is_big = n > 8_000_000
        if big is not None and is_big != big:
            continue
        if max_elems is not None and n > max_elems:
            continue
        out.append(c["id"])
    return out


def get_case(cid):
    for c in cases()["cases"]:
        if c["id"] == cid:
            return c
    raise KeyError(cid)


def make_inputs(case, values="data"):
    """Regenerate a case's per-layer (K, V) numpy arrays; checks the stored input hashes."""
    out = []
    for li, L in enumerate(case["layers"]):
        shape = tuple(L["shape"])
        K = prng.gen_keys(L["kseed"], shape, case["dtype"], L.get("variant", "normal"))
        assert sha(K) == case["input_sha"][li], "PRNG drift: regenerated K differs from fixture"
        V = (prng.gen_values(L["kseed"], shape, case["dtype"]) if values == "data"
             else prng.encode_positions(shape, case["dtype"]))
        out.append((K, V))
    return out
