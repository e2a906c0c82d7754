"""The real engine in two ranks (GPU): `bench.py --gpus 2` on BASELINE cfg4 (h2o_l2 4/64/444,
ONE 32-layer pythia-2.8b model sharded over the ranks, S = 16384) with both ranks on cuda:0
(--same-device: a 1-GPU box), then each rank's first layer checked against the oracle.  The
ranks share no data; the harness's only cross-rank traffic is gloo on host scalars."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_two_rank_bench_runs_the_engine(tmp_path):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--workload", "cfg4-h2o-l32", "--steps", "2", "--warmup", "1",
                          "--same-device", "--dump-layer", str(tmp_path)],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    r = lines[0]
    assert r["n_gpus"] == 2 and r["scaling"] == "strong" and r["config"]["layers_total"] == 32
    assert r["config"]["layers_per_gpu"] == 16 and r["value"] > 0
    assert "dry_run" not in r
    for rank, layer0 in ((0, 0), (1, 16)):
        d = np.load(tmp_path / f"rank{rank}.npz")
        assert int(d["layer"]) == layer0
        k, v = d["k"].view(np.uint16), d["v"].view(np.uint16)  # bf16 bits, heads 0-1
        rk, rv, kind = oracle.h2o_l2_compress([(k, v)], start_size=4, heavy_hitter_size=64,
                                              recent_size=444, skip_layers=[])[0]
        assert kind == "new" and rk.shape == (1, 2, 512, 80)
        assert np.array_equal(d["k_out"].view(np.uint16), rk)
        assert np.array_equal(d["v_out"].view(np.uint16), rv)
