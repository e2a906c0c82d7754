"""Headline benchmark: KV tokens scored+evicted/sec for fix_size_l2 (fix_kv_size=512,
keep_ratio=0.0, keep_low) on synthetic [1,32,16384,128] bf16 KV, 32 layers per GPU.

One step = one drop-in `fix_size_l2_compress(kv_list, ...)` call over all 32 layers (norm scoring
of 16384 positions x 32 heads per layer, reference-exact selection, gather of 512 K/V rows).
Inputs are resident in HBM before the timed region.  Multi-GPU: one process per GPU (torchrun),
each rank owns 32 layers of a 32*N-layer stack (layers sharded, no collectives on the data
path; weak scaling); a barrier + synchronize brackets the timed region and the max over ranks
is reported.  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

LAYERS, B, H, S, D = 32, 1, 32, 16384, 128
FIX = 512
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def algorithmic_bytes(es=2):
    """Per layer: K read over S + kept V rows read + K,V kept rows written."""
    R = B * H * D * es
    per_layer = R * (S + FIX + 2 * FIX)
    score = B * H * S * (D * es + es)  # score kernel: K read + one norm written per position
    return per_layer, score


PMC_FILE = "profiles/r01_v7_pmc_traffic.json"  # tools/gpu_check.sh pmc + tools/pmc_traffic.py


def pmc_traffic(kernel="kvc::score_kernel<1, 16, true>"):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes
    (PMC_FILE: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE) measured on this exact workload;
    None if absent."""
    path = os.path.join(ROOT, PMC_FILE)
    try:
        with open(path) as f:
            k = json.load(f)["kernels"][kernel]
        return k["FETCH_bytes_x2_gfx950"] + k["WRITE_SIZE_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline(seconds=12.0):
    """The reference's CPU op sequence (oracle/torch_port.py) on this host's cores, bounded."""
    from oracle.torch_port import fix_size_l2_layer
    # the GPU box exposes the whole machine's CPUs but grants one GPU a 16-core share
    # (OMP_NUM_THREADS is set to it there)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    k = torch.randn(B, H, S, D, generator=g).to(torch.bfloat16)
    v = torch.randn(B, H, S, D, generator=g).to(torch.bfloat16)
    fix_size_l2_layer(k, v, FIX)  # warm
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fix_size_l2_layer(k, v, FIX)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n * S / dt, "unit": "KV tokens/s", "cores": threads, "kind": "port",
            "sample": f"{n} layers of fix_size_l2(512) on one [1,32,16384,128] bf16 layer "
                      f"(torch CPU ops: norm->argsort->sort->gather), {dt:.1f}s, "
                      f"{torch.backends.cpu.get_cpu_capability()}"}


def timed_steps(step, steps, warmup, dist, sync, device, on_start=None):
    """W untimed warmup steps, then exactly K timed steps bracketed by barrier + sync on both
    sides; returns the MAX elapsed seconds over ranks (all ranks return the same value)."""
    for _ in range(warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    if on_start:
        on_start()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    sync()
    if dist:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    del out
    if dist:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def shard_layers(num_layers_total, world, rank):
    """Contiguous layer block [start, end) owned by `rank` (layers sharded, no collectives)."""
    per = num_layers_total // world
    extra = num_layers_total % world
    start = rank * per + min(rank, extra)
    return start, start + per + (1 if rank < extra else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from kvcompress import _engine
    from kvcompress.methods import fix_size_l2_compress

    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    layers = []
    for _ in range(LAYERS):
        k = torch.randn(B, H, S, D, device=dev, generator=g, dtype=torch.float32).to(torch.bfloat16)
        v = torch.randn(B, H, S, D, device=dev, generator=g, dtype=torch.float32).to(torch.bfloat16)
        layers.append((k, v))

    def step():
        return fix_size_l2_compress(layers, fix_kv_size=FIX, keep_ratio=0.0, strategy="keep_low",
                                    skip_layers=[])

    # per-kernel durations: the engine splits each launch into its three kernels with HIP
    # events (recorded on the stream they run on) for the whole timed region
    timer = _engine.PhaseTimer()
    elapsed = timed_steps(step, args.steps, args.warmup, dist, torch.cuda.synchronize, dev,
                          on_start=lambda: _engine.set_phase_timer(timer))
    _engine.set_phase_timer(None)
    dur = timer.durations_ms()

    if rank == 0:
        per_layer, score_bytes_layer = algorithmic_bytes()
        ms_step = elapsed / args.steps * 1e3
        tokens = LAYERS * S * args.steps * world
        score_ms = sum(dur["score"]) / len(dur["score"])
        score_gbps = score_bytes_layer * LAYERS / (score_ms * 1e-3) / 1e9
        traffic = pmc_traffic()
        path_gbps = per_layer * LAYERS / (ms_step * 1e-3) / 1e9
        res = {
            "metric": "KV tokens scored+evicted/sec at S=16384, fix_size=512; PPL delta vs ref",
            "value": tokens / elapsed,
            "unit": "KV tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (torch.randn, HBM-resident)",
            "config": {"workload": "fix_size_l2_compress(fix_kv_size=512, keep_ratio=0.0, "
                                   "strategy='keep_low', skip_layers=[]) over 32 layers of "
                                   "K,V [1,32,16384,128] per GPU, one call per step",
                       "layers_per_gpu": LAYERS, "seq_len": S, "heads": H, "head_dim": D,
                       "fix_kv_size": FIX, "parallelism": f"layers sharded x{world}, no collectives"},
            "roofline": {"bound": "hbm", "kernel": "score_kernel (key L2 norms)",
                         "achieved": score_gbps, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": score_gbps / PEAK_HBM_GBPS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": score_bytes_layer * LAYERS,
                         "traffic_source": PMC_FILE + " (rocprofv3 --pmc)"},
            "path_roofline": {"achieved": path_gbps, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                              "frac": path_gbps / PEAK_HBM_GBPS,
                              "bytes_per_layer": per_layer},
            "kernel_ms_per_step": {k: sum(v) / len(v) for k, v in dur.items()},
            "tokens_evicted_per_sec": (S - FIX) * LAYERS * args.steps * world / elapsed,
        }
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline()
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
