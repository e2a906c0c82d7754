"""World-size-2 gloo tests (CPU) of the multi-GPU path: layer sharding with global layer ids
(no data-path collective), and bench.py's barrier + MAX-over-ranks timing harness."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _capture_plans(fn, layers, **kw):
    """Run a compress function with the engine replaced by a recorder (host plans only)."""
    from kvcompress import _engine
    rec = []
    real = _engine.execute

    def fake(jobs, out_list, order, algo):
        for j in jobs:
            rec.append((j.layer_idx, j.sink_len, j.zone_start, j.zone_len, j.n_select,
                        j.tail_start, j.tail_len, order, algo))
    _engine.execute = fake
    try:
        out = fn(layers, **kw)
    finally:
        _engine.execute = real
    return rec, out


def _layers(n, S=1000):
    g = torch.Generator().manual_seed(0)
    return [(torch.randn(1, 2, S + 37 * i, 64, generator=g), torch.randn(1, 2, S + 37 * i, 64,
                                                                         generator=g))
            for i in range(n)]


# every registered method with a layer-sharding-sensitive configuration: skip_layers (global ids,
# the reference's defaults where it has them) and, for pyramid_kv, the depth-dependent sizes
SHARD_CASES = (
    ("pyramid_kv", dict(base_size=512, layer_decay=0.8, skip_layers=[3]), True),
    ("fix_size_l2", dict(fix_kv_size=256, keep_ratio=0.5), False),        # default skip [0, 1]
    ("l2_compress", dict(keep_ratio=0.8, prune_after=100), False),         # default skip [0, 1]
    ("h2o_l2", dict(start_size=4, heavy_hitter_size=64, recent_size=444, skip_layers=[5]), False),
    ("snapkv_lite", dict(observation_window=32, keep_size=512, skip_layers=[0, 9]), False),
    ("adaptive_l2", dict(target_size=256, skip_layers=[2, 7]), False),
    ("streaming_llm", dict(start_size=4, recent_size=300, skip_layers=[4]), False),
    ("recent_only", dict(window_size=512), False),                        # default skip [0, 1]
)


def _worker_shard(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bench import shard_layers
    from kvcompress.methods import get_compress_fn
    L = 10
    allL = _layers(L)
    a, b = shard_layers(L, world, rank)
    mine = allL[a:b]
    plans = {}
    for name, kw, depth in SHARD_CASES:
        extra = dict(layer_offset=a, num_layers_total=L) if depth else dict(layer_offset=a)
        rec, out = _capture_plans(get_compress_fn(name), list(mine), **kw, **extra)
        shapes = [(a + i, tuple(k.shape)) for i, (k, _) in enumerate(out)]
        plans[name] = ([(r[0] + a,) + r[1:] for r in rec], shapes)  # to global layer ids
    gathered = [None] * world
    dist.all_gather_object(gathered, plans)
    if rank == 0:
        res = {}
        for name, kw, _ in SHARD_CASES:
            got = (sorted(sum((g[name][0] for g in gathered), [])),
                   sorted(sum((g[name][1] for g in gathered), [])))
            ref, out = _capture_plans(get_compress_fn(name), list(allL), **kw)
            want = (sorted(ref), sorted((i, tuple(k.shape)) for i, (k, _) in enumerate(out)))
            res[name] = (got == want, got, want)
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


def _worker_timing(rank, world, port, q):
    import sys
    import time
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bench import timed_steps
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.02 * (rank + 1))  # rank 1 is the slow one
    el = timed_steps(step, steps=5, warmup=2, dist=dist, sync=lambda: None, device="cpu")
    q.put((rank, el, len(calls)))
    dist.destroy_process_group()


def _run(worker, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    return [q.get(timeout=10) for _ in range(q.qsize())]


def test_sharded_plans_equal_unsharded():
    """Every method, sharded over 2 ranks with layer_offset, plans exactly the engine jobs (and
    returns the layer shapes) of the unsharded reference call."""
    res, = _run(_worker_shard)
    assert set(res) == {c[0] for c in SHARD_CASES}
    for name, (ok, got, want) in res.items():
        assert ok, (name, got, want)
        assert got[0] or name == "recent_only", name  # the case exercises the engine


def test_timing_is_max_over_ranks():
    res = sorted(_run(_worker_timing))
    assert all(r[2] == 7 for r in res)            # 2 warmup + 5 timed steps on every rank
    assert res[0][1] == res[1][1]                   # every rank reports the reduced value
    assert res[0][1] >= 5 * 0.04 * 0.95             # ... which is the slow rank's time


def test_shard_layers_partition():
    from bench import shard_layers
    for L in (1, 7, 32, 33):
        for W in (1, 2, 4, 8):
            spans = [shard_layers(L, W, r) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == L
            assert all(spans[i][1] == spans[i + 1][0] for i in range(W - 1))
