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


def _worker_shard(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bench import shard_layers
    from kvcompress.methods import pyramid_kv_compress, fix_size_l2_compress
    L = 10
    allL = _layers(L)
    a, b = shard_layers(L, world, rank)
    mine = allL[a:b]
    plans = {}
    for name, fn, kw in (("pyramid", pyramid_kv_compress,
                          dict(base_size=512, layer_decay=0.8, skip_layers=[3],
                               layer_offset=a, num_layers_total=L)),
                         ("fix", fix_size_l2_compress, dict(fix_kv_size=256, keep_ratio=0.5))):
        rec, _ = _capture_plans(fn, list(mine), **kw)
        plans[name] = [(r[0] + a,) + r[1:] for r in rec]  # to global layer ids
    gathered = [None] * world
    dist.all_gather_object(gathered, plans)
    if rank == 0:
        merged = {k: sorted(sum((g[k] for g in gathered), [])) for k in plans}
        ref_p, _ = _capture_plans(pyramid_kv_compress, list(allL), base_size=512,
                                  layer_decay=0.8, skip_layers=[3])
        q.put((merged["pyramid"] == sorted(ref_p), merged["pyramid"], sorted(ref_p)))
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
    (ok, got, ref), = _run(_worker_shard)
    assert ok, (got, ref)


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
