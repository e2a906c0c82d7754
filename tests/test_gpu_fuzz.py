"""Randomised GPU parity: seeded random method / kwargs / geometry / dtype / key distribution,
engine vs the CPU oracle, bit-exact K/V and identical output kinds.  Each case mixes several
layers (ragged lengths, skip lists) in one call, so batching and per-layer branches are
exercised together; the three launch paths take turns.  Seeds are fixed: a failure names its case."""
import os

import numpy as np
import pytest

import prng
from gpu_util import kind_of, to_dev, to_np
from oracle import oracle

pytestmark = pytest.mark.gpu

N_CASES = int(os.environ.get("KVC_FUZZ_CASES", "300"))  # more for a soak run


def _kwargs(rng, method, S):
    r = lambda lo, hi: int(rng.integers(lo, hi + 1))  # noqa: E731
    if method == "fix_size_l2":
        return dict(fix_kv_size=r(1, S), keep_ratio=float(rng.choice([0.0, 0.25, 0.5, 0.9])),
                    strategy=str(rng.choice(["keep_low", "keep_high"])))
    if method == "l2_compress":
        return dict(keep_ratio=float(rng.choice([0.1, 0.5, 0.8, 0.95])), prune_after=r(0, S))
    if method == "streaming_llm":
        return dict(start_size=r(0, 8), recent_size=r(0, S))
    if method == "h2o_l2":
        return dict(start_size=r(0, 8), heavy_hitter_size=r(1, 200), recent_size=r(0, S // 2))
    if method == "snapkv_lite":
        return dict(observation_window=r(0, 64), keep_size=r(1, S),
                    pooling_kernel=int(rng.choice([1, 2, 3, 5, 7])))
    if method == "pyramid_kv":
        return dict(base_size=r(8, S), layer_decay=float(rng.choice([0.5, 0.9, 1.0])),
                    min_size=r(1, 64), profile=str(rng.choice(["exponential", "linear",
                                                               "constant"])))
    if method == "adaptive_l2":
        soft = r(2, S)
        return dict(target_size=r(1, S), soft_limit=soft, hard_limit=r(soft + 1, 2 * S))
    return dict(window_size=r(1, S))  # recent_only


def _gen_case(case, max_len=None):
    """Seeded (method, layers, kwargs) of one fuzz case (layer lengths clipped to max_len)."""
    rng = np.random.default_rng(90000 + case)
    method = str(rng.choice(["fix_size_l2", "l2_compress", "streaming_llm", "h2o_l2",
                             "snapkv_lite", "pyramid_kv", "adaptive_l2", "recent_only"]))
    dtype = str(rng.choice(["bf16", "fp16", "fp32"]))
    D = int(rng.choice([32, 64, 80, 128, 256]))
    B, H = int(rng.integers(1, 3)), int(rng.integers(1, 5))
    S0 = int(rng.choice([20, 100, 700, 2000, 5000, 16384]))
    n_layers = int(rng.integers(1, 5))
    variants = ["normal", "scaled", "few", "equal", "special", "tiny"]
    layers = []
    for li in range(n_layers):
        S = max(1, S0 + int(rng.integers(-S0 // 4, S0 // 4 + 1)))
        if max_len:
            S = min(S, max_len)
        shape = (B, H, S, D)
        seed = 100000 + 100 * case + li
        layers.append((prng.gen_keys(seed, shape, dtype, str(rng.choice(variants))),
                       prng.gen_values(seed, shape, dtype)))
    kw = _kwargs(rng, method, S0)
    kw["skip_layers"] = [int(x) for x in rng.choice(n_layers, size=int(rng.integers(0, 2)),
                                                      replace=False)]
    return method, layers, kw, dtype, D


def _check(case, method, layers, kw, dtype, D):
    from kvcompress.methods import get_compress_fn
    try:
        ref = oracle.METHODS[method](layers, **kw)
    except Exception as e:  # the reference raises here too (same shape rules)
        with pytest.raises(type(e)):
            get_compress_fn(method)([(to_dev(k), to_dev(v)) for k, v in layers], **kw)
        return
    tin = [(to_dev(k), to_dev(v)) for k, v in layers]
    out = get_compress_fn(method)(list(tin), **kw)
    assert len(out) == len(ref)
    for li, ((ki, vi), (ko, vo), (rk, rv, kind)) in enumerate(zip(tin, out, ref)):
        ctx = (case, method, dtype, D, kw, li)
        assert kind_of(ki, ko) == kind, ctx
        assert np.array_equal(to_np(ko).view(np.uint8), np.ascontiguousarray(rk).view(np.uint8)), ctx
        assert np.array_equal(to_np(vo).view(np.uint8), np.ascontiguousarray(rv).view(np.uint8)), ctx


@pytest.mark.parametrize("case", range(N_CASES))
def test_random_configs_match_oracle(case, monkeypatch):
    # launch paths in rotation: SCORE + SELECT_GATHER, and SCORE / SELECT / GATHER
    from kvcompress import _engine
    monkeypatch.setattr(_engine, "split_select_gather", case % 2 == 1)
    _check(case, *_gen_case(case))


@pytest.mark.parametrize("case", range(N_CASES // 3))
def test_random_configs_stable_policy_match_oracle(case, monkeypatch):
    """The same generator under the opt-in stable tie policy (engine and oracle alike; layers of
    up to 20 480 positions: zones past 16 384 take the global-scratch kernel)."""
    from kvcompress import _engine
    monkeypatch.setattr(_engine, "split_select_gather", case % 2 == 0)
    monkeypatch.setattr(_engine, "tie_policy", "stable")
    monkeypatch.setattr(oracle, "TIE", "stable")
    _engine.call_memo.clear()
    _check(case, *_gen_case(case))
