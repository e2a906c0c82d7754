"""Repeated call shapes replayed by the native host path (GPU): every method, called again and
again with the same shapes and new K/V, gives the oracle's bytes on the first (Python path),
second (recorded) and later (replayed by kvc_host.run) calls; passthrough layers stay the same
objects and slices stay views; changing kwargs or shapes never reuses a recording."""
import numpy as np
import pytest
import torch

import prng
from gpu_util import kind_of, to_dev, to_np
from oracle import oracle

pytestmark = pytest.mark.gpu

CASES = [
    ("fix_size_l2", dict(fix_kv_size=128, skip_layers=[0])),
    ("fix_size_l2", dict(fix_kv_size=128, keep_ratio=0.5, strategy="keep_high", skip_layers=[])),
    ("fix_size_l2", dict(fix_kv_size=100, keep_ratio=1.0, skip_layers=[])),  # views (-P:)
    ("l2_compress", dict(keep_ratio=0.5, prune_after=100, skip_layers=[])),
    ("streaming_llm", dict(start_size=4, recent_size=100)),
    ("streaming_llm", dict(start_size=4, recent_size=0)),                  # the -0: quirk
    ("recent_only", dict(window_size=100, skip_layers=[1])),               # views only
    ("h2o_l2", dict(start_size=4, heavy_hitter_size=32, recent_size=60)),
    ("snapkv_lite", dict(observation_window=16, keep_size=120)),
    ("pyramid_kv", dict(base_size=160, min_size=8, skip_layers=[2])),      # ragged n_out
    ("pyramid_kv", dict(base_size=12, min_size=4)),                         # views + copies
    ("adaptive_l2", dict(target_size=128, soft_limit=64, hard_limit=200)),
]
ORACLE = dict(oracle.METHODS)
ORACLE["fix_size_l2"] = oracle.fix_size_l2_compress


def _layers(seed, lens, dt="bf16", D=64):
    return [(prng.gen_keys(seed + i, (1, 4, S, D), dt, "few"), prng.gen_values(seed + i, (1, 4, S, D), dt))
            for i, S in enumerate(lens)]


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_replayed_calls_match_oracle(ci):
    from kvcompress import _engine
    from kvcompress.methods import get_compress_fn
    name, kw = CASES[ci]
    fn = get_compress_fn(name)
    _engine.call_memo.clear()
    r0 = _engine.memo_stats["replayed"]
    for step in range(5):
        lens = [300, 301, 170, 300] if step < 4 else [300, 301, 171, 300]  # last: new shape
        layers_np = _layers(1000 + 17 * step + ci, lens)
        tin = [(to_dev(k), to_dev(v)) for k, v in layers_np]
        out = fn(list(tin), **kw)
        ref = ORACLE[name](layers_np, **kw)
        assert len(out) == len(ref)
        for (ki, vi), (ko, vo), (rk, rv, kind) in zip(tin, out, ref):
            assert kind_of(ki, ko) == kind and kind_of(vi, vo) == kind, (step, kind)
            assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv), step
    # calls 3 and 4 (same shape as 1 and 2) were replays; call 5 (new shape) was not
    assert _engine.memo_stats["replayed"] - r0 == 2


def test_kwargs_and_streams_key_the_recording():
    from kvcompress import _engine
    from kvcompress.methods import fix_size_l2_compress
    _engine.call_memo.clear()
    side = torch.cuda.Stream()
    kept = []
    for step in range(8):
        layers_np = _layers(5000 + step, [400, 400])
        tin = [(to_dev(k), to_dev(v)) for k, v in layers_np]
        fix = 100 if step % 4 < 2 else 90
        with torch.cuda.stream(side if step % 2 else torch.cuda.current_stream()):
            out = fix_size_l2_compress(list(tin), fix_kv_size=fix, skip_layers=[])
        kept.append((layers_np, fix, out))
    torch.cuda.synchronize()
    for layers_np, fix, out in kept:
        ref = oracle.fix_size_l2_compress(layers_np, fix_kv_size=fix, skip_layers=[])
        for (ko, vo), (rk, rv, _) in zip(out, ref):
            assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv)


def test_dynamic_cache_and_fp32_replay():
    """transformers-5 DynamicCache input and fp32 K/V through the replay path."""
    from transformers import DynamicCache
    from kvcompress import _engine
    from kvcompress.methods import snapkv_lite_compress
    _engine.call_memo.clear()
    for step in range(4):
        layers_np = _layers(7000 + step, [260, 260, 260], dt="fp32", D=32)
        cache = DynamicCache()
        for i, (k, v) in enumerate(layers_np):
            cache.update(to_dev(k), to_dev(v), i)
        out = snapkv_lite_compress(cache, observation_window=8, keep_size=64)
        ref = oracle.snapkv_lite_compress(layers_np, observation_window=8, keep_size=64)
        for (ko, vo), (rk, rv, _) in zip(out, ref):
            assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv)
