"""bench.py's multi-GPU launch contract, checked on CPU with its --dry-run harness (gloo, a
stand-in step whose last rank is the slow one, no engine and no GPU):
  * `python bench.py --gpus 2` starts two ranks itself and prints ONE JSON line, n_gpus = 2;
  * under torchrun (WORLD_SIZE set) it spawns nothing and reports the same way;
  * the reported time is the MAX over ranks (the slow rank's);
  * a rank that dies after joining the process group ends the whole launch with its error code
    (the surviving ranks, waiting in a barrier, are stopped) and no JSON line is printed.
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 5


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _check(lines, n):
    assert len(lines) == 1, lines
    r = lines[0]
    assert r["n_gpus"] == n and r["steps"] == STEPS and r["dry_run"] is True
    assert r["config"]["layers_total"] == 32 * n  # weak scaling: 32 layers per rank
    # the last rank sleeps 2 ms * n per step: the max over ranks is at least that
    assert r["ms_per_step"] >= 2.0 * n * 0.95, r["ms_per_step"]
    assert r["value"] > 0


def _free_port():
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    return port


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_gpus_flag_spawns_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus",
                          "2", "--steps", str(STEPS), "--warmup", "2"], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    _check(_json_lines(out.stdout), 2)


def test_torchrun_launch_does_not_respawn():
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                          str(_free_port()), os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus", "2",
                          "--steps", str(STEPS), "--warmup", "2"], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    _check(_json_lines(out.stdout), 2)


def test_single_rank_default():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps",
                          str(STEPS), "--warmup", "1"], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    _check(_json_lines(out.stdout), 1)


def test_strong_scaling_workload_splits_32_layers():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus",
                          "2", "--workload", "cfg4-h2o-l32", "--steps", str(STEPS), "--warmup",
                          "1"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    r, = _json_lines(out.stdout)
    assert r["scaling"] == "strong" and r["config"]["layers_total"] == 32
    assert r["config"]["layers_per_gpu"] == 16


def test_eight_ranks_dry_run():
    """The driver's N=8 launch shapes (bench.py --gpus 8, and torchrun --nproc-per-node 8):
    8 gloo ranks, ONE JSON line, the max over ranks (the last rank sleeps 16 ms per step)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus",
                          "8", "--steps", str(STEPS), "--warmup", "1"], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    _check(_json_lines(out.stdout), 8)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                          "--nproc-per-node", "8", "--master-addr", "127.0.0.1", "--master-port",
                          str(_free_port()), os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus",
                          "8", "--steps", str(STEPS), "--warmup", "1"], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    _check(_json_lines(out.stdout), 8)


def test_strong_split_over_eight_ranks():
    """cfg5 over 8 ranks: 4 of the 32 layers each (pyramid_kv's min-size layers on the last)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus",
                          "8", "--workload", "cfg5-pyramid-l32", "--steps", str(STEPS),
                          "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    r, = _json_lines(out.stdout)
    assert r["scaling"] == "strong" and r["n_gpus"] == 8
    assert r["config"]["layers_total"] == 32 and r["config"]["layers_per_gpu"] == 4


def test_as_shard_runs_one_ranks_layers():
    """--as-shard 7/8: one process runs the layers rank 7 of an 8-rank strong split owns."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run",
                          "--workload", "cfg5-pyramid-l32", "--as-shard", "7/8", "--steps",
                          str(STEPS), "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    r, = _json_lines(out.stdout)
    assert r["config"]["layer_offset"] == 28 and r["config"]["layers_per_gpu"] == 4
    assert r["n_gpus"] == 1 and "rank 7 of 8" in r["config"]["as_shard"]


def test_rank_failure_after_init_stops_the_launch():
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus",
                          "2", "--steps", str(STEPS), "--warmup", "1", "--dry-run-fail-rank", "1"],
                         cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
    assert "injected failure" in out.stderr
    assert _json_lines(out.stdout) == []
    assert time.time() - t0 < 120  # rank 0 did not wait out gloo's barrier timeout
