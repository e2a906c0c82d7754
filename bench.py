"""Headline benchmark: KV tokens scored+evicted/sec for fix_size_l2 (fix_kv_size=512,
keep_ratio=0.0, keep_low) on synthetic [1,32,16384,128] bf16 KV, 32 layers per GPU.

One step = one drop-in `fix_size_l2_compress(kv_list, ...)` call over all 32 layers (norm scoring
of 16384 positions x 32 heads per layer, reference-exact selection, gather of 512 K/V rows).
Inputs are resident in HBM before the timed region.  Multi-GPU: one process per GPU, each rank
owns 32 layers of a 32*N-layer stack (layers sharded, no collectives on the data path; weak
scaling); a barrier + synchronize brackets the timed region and the max over ranks is reported.
Prints ONE JSON line on rank 0.  Ranks come from torchrun (RANK / LOCAL_RANK / WORLD_SIZE in the
environment) or, for `--gpus N` without them, from N child processes this script starts before
anything touches the GPU (the parent only waits for them).

`--workload` selects one of the other BASELINE / SURVEY §8(d) configurations (same contract, same
JSON line; the default is the headline).  `--layers-total L` shards an L-layer model over the
ranks instead (strong scaling, global layer indices; e.g. cfg4: h2o_l2, 32 layers over 8 GPUs);
the `cfg4-*` / `cfg5-*` workloads default to that 32-layer split.  `--dry-run` runs the launch,
timing and reporting harness on CPU with gloo and a stand-in step (tests/test_bench_launch.py).
"""
import argparse
import json
import os
import socket
import subprocess
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

# name -> (method, kwargs, seq_len, head_dim, what).  The headline is BASELINE.json's metric
# config; the others are its configs[1..4] at the §8(d) geometries (pythia-2.8b: D=80,
# pythia-6.9b: D=128; 32 heads, 32 layers).
WORKLOADS = {
    "fix512-s16384": ("fix_size_l2", dict(fix_kv_size=512, keep_ratio=0.0, strategy="keep_low"),
                      16384, 128, "headline"),
    "fix512-s4096": ("fix_size_l2", dict(fix_kv_size=512, keep_ratio=0.0, strategy="keep_low"),
                     4096, 128, "cfg2 geometry of the north star ([1,32,S,128])"),
    "fix512-s8192": ("fix_size_l2", dict(fix_kv_size=512, keep_ratio=0.0, strategy="keep_low"),
                     8192, 128, "between the north star's two lengths"),
    "fix512-s4096-d80": ("fix_size_l2", dict(fix_kv_size=512, keep_ratio=0.0,
                                             strategy="keep_low"), 4096, 80, "cfg2, pythia-2.8b"),
    "streaming-s16384": ("streaming_llm", dict(start_size=4, recent_size=1020), 16384, 80,
                         "cfg3, pythia-2.8b"),
    "h2o-s16384": ("h2o_l2", dict(start_size=4, heavy_hitter_size=64, recent_size=444), 16384, 80,
                   "cfg4, pythia-2.8b"),
    "snapkv-s16384": ("snapkv_lite", dict(observation_window=32, keep_size=512), 16384, 128,
                      "cfg5, pythia-6.9b"),
    "snapkv-s4096": ("snapkv_lite", dict(observation_window=32, keep_size=512), 4096, 128,
                     "cfg5 at the north star's short length"),
    "pyramid-s16384": ("pyramid_kv", dict(base_size=512), 16384, 128, "cfg5, pythia-6.9b"),
    "l2-s16384": ("l2_compress", dict(keep_ratio=0.8, prune_after=100), 16384, 80,
                  "cfg1 method (one-shot), pythia-2.8b"),
    "adaptive-s16384": ("adaptive_l2", dict(), 16384, 128, "adaptive_l2 defaults"),
    # BASELINE configs[3] / [4] as named: ONE 32-layer model sharded over the ranks (strong
    # scaling; 4 layers per GPU at N=8), global layer ids (skip_layers, pyramid depth)
    "cfg4-h2o-l32": ("h2o_l2", dict(start_size=4, heavy_hitter_size=64, recent_size=444), 16384,
                     80, "cfg4, pythia-2.8b, 32 layers sharded over the GPUs"),
    "cfg5-snapkv-l32": ("snapkv_lite", dict(observation_window=32, keep_size=512), 16384, 128,
                        "cfg5, pythia-6.9b, 32 layers sharded over the GPUs"),
    "cfg5-pyramid-l32": ("pyramid_kv", dict(base_size=512), 16384, 128,
                         "cfg5, pythia-6.9b, 32 layers sharded over the GPUs"),
}
STRONG_DEFAULT = {"cfg4-h2o-l32": 32, "cfg5-snapkv-l32": 32, "cfg5-pyramid-l32": 32}
HEADLINE = "fix512-s16384"


def algorithmic_bytes(es=2):
    """Per layer: K read over S + kept V rows read + K,V kept rows written."""
    R = B * H * D * es
    per_layer = R * (S + FIX + 2 * FIX)
    score = B * H * S * (D * es + es)  # score kernel: K read + one norm written per position
    return per_layer, score


def job_bytes(jobs, es):
    """Algorithmic bytes of one call from its engine jobs (generalised): per layer
    R = B*H*D*e and out = sink + selected + tail rows:
      path   = R * (zone + sink + tail + 3*out)   K scored over the zone, K rows copied from the
               sink/tail, V kept rows read, K and V out written (selected K rows not re-counted)
      score  = B*H*zone*(D*e + e)                 K read + one norm written per scored position
      select+gather = 4 * R * out                 K,V kept rows read + written (the selection's
                                                  norm reads / index traffic stay on chip)
    """
    path = score = gather = 0
    for j in jobs:
        b, h, _, d = j.keys.shape
        R = b * h * d * es
        out = j.sink_len + j.n_select + j.tail_len
        zone = j.zone_len if j.n_select else 0
        path += R * (zone + j.sink_len + j.tail_len + 3 * out)
        score += b * h * zone * (d * es + es)
        gather += 4 * R * out
    return {"path": path, "score": score, "select+gather": gather}


PMC_FILE = "profiles/r06_z_pmc_traffic.json"  # tools/pmc_round.sh (tools/gpu.sh pmc) + tools/pmc_traffic.py


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


DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def cpu_baseline(seq_len=S, head_dim=D, seconds=12.0, dtype="bf16"):
    """The reference's CPU op sequence (oracle/torch_port.py) on this host's cores, bounded."""
    from oracle.torch_port import fix_size_l2_layer
    # the GPU box exposes the whole machine's CPUs but grants one GPU a 16-core share
    # (OMP_NUM_THREADS is set to it there)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    k = torch.randn(B, H, seq_len, head_dim, generator=g).to(DTYPES[dtype])
    v = torch.randn(B, H, seq_len, head_dim, generator=g).to(DTYPES[dtype])
    fix_size_l2_layer(k, v, FIX)  # warm

    def rate(secs):
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < secs:
            fix_size_l2_layer(k, v, FIX)
            n += 1
        return n, time.perf_counter() - t0

    print(f"[bench] cpu_baseline: {seconds:.0f} s on {threads} threads + 1 thread",
          file=sys.stderr, flush=True)
    n, dt = rate(seconds)
    torch.set_num_threads(1)  # also a 1-thread run
    n1, dt1 = rate(seconds / 3)
    torch.set_num_threads(threads)
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return {"value": n * seq_len / dt, "unit": "KV tokens/s", "cores": threads, "kind": "port",
            "value_1_thread": n1 * seq_len / dt1, "cpu_model": model,
            "cpu_capability": torch.backends.cpu.get_cpu_capability(),
            "sample": f"{n} layers of fix_size_l2(512) on one [1,32,{seq_len},{head_dim}] {dtype} "
                      f"layer (torch CPU ops: norm->argsort->sort->gather) in {dt:.1f}s on "
                      f"{threads} threads, {n1} layers in {dt1:.1f}s on 1 thread"}


PPL_MODELS = {  # GPT-NeoX geometries (pythia configs; weights are random: none offline)
    "pythia-2.8b": dict(vocab_size=50304, hidden_size=2560, num_hidden_layers=32,
                        num_attention_heads=32, intermediate_size=10240),
    "tiny": dict(vocab_size=512, hidden_size=256, num_hidden_layers=4, num_attention_heads=4,
                 intermediate_size=1024),
}


def ppl_delta(device, arch="pythia-2.8b", tokens=2000, fix=512, keep_ratio=0.5):
    """The metric's "PPL delta vs ref" half on BASELINE's config: teacher-forced
    evaluate_with_compression (one compress call per token, skip_layers=[0, 1] as the
    reference's default) of a random-init GPT-NeoX with pythia-2.8b's geometry (32 layers, 32
    heads, D = 80; weights unavailable offline) in bf16 on `device`, once with the engine's
    fix_size_l2_compress and once with the reference's CPU op sequence (oracle/torch_port.py: norm -> argsort -> sort ->
    gather -> cat, every branch of fix_size_l2.py:76-150, pinned to the unmodified reference's
    golden outputs by tests/test_torch_port.py; K/V copied to the host and back) as compress_fn;
    same model, same synthetic token stream.
    fix_kv_size=512 / keep_ratio=0.5 is the reference's README configuration; `tokens` > fix so
    that ~tokens - fix steps compress (2000: the length of the reference's PG-19 samples)."""
    from transformers import GPTNeoXConfig, GPTNeoXForCausalLM
    from kvcompress.evaluate import evaluate_with_compression
    from kvcompress.methods import fix_size_l2_compress
    from oracle.torch_port import fix_size_l2_layer

    geo = PPL_MODELS[arch]

    class Tok:  # deterministic synthetic token stream over the vocabulary
        def encode(self, text, return_tensors="pt"):
            v = geo["vocab_size"]
            return torch.tensor([[(b * 7919 + i * 104729) % v for i, b in enumerate(text.encode())]])

    def reference(kv, skip_layers=(), fix_kv_size=fix, keep_ratio=keep_ratio):
        out = []
        for i, (k, v) in enumerate(kv):  # fix_size_l2.py:69-74 skip tests, then :76-150
            if k.size(2) <= fix_kv_size or i in skip_layers:
                out.append((k, v))
                continue
            kk, vv = fix_size_l2_layer(k.cpu(), v.cpu(), fix_kv_size, keep_ratio)
            out.append((kk.to(k.device), vv.to(v.device)))
        return out

    torch.manual_seed(0)
    cfg = GPTNeoXConfig(rotary_pct=0.25, max_position_embeddings=2048, **geo)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            model = GPTNeoXForCausalLM(cfg).eval()
    finally:
        torch.set_default_dtype(prev)
    text = "The quick brown fox jumps over the lazy dog. " * (tokens // 40 + 1)
    kw = dict(fix_kv_size=fix, keep_ratio=keep_ratio)
    print(f"[bench] PPL-delta leg: {tokens} tokens x 2 runs", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    r = []
    for name, fn in (("engine", fix_size_l2_compress), ("reference", reference)):
        r.append(evaluate_with_compression(model, Tok(), text, compress_fn=fn, compress_kwargs=kw,
                                           max_tokens=tokens, skip_layers=[0, 1],
                                           show_progress=False))
        print(f"[bench] PPL-delta leg: {name} run done ({time.perf_counter() - t0:.0f} s)",
              file=sys.stderr, flush=True)
    dt = time.perf_counter() - t0
    del model
    torch.cuda.empty_cache()
    return {"value": r[0]["perplexity"] - r[1]["perplexity"], "ppl": r[0]["perplexity"],
            "ppl_ref": r[1]["perplexity"], "accuracy_delta": r[0]["accuracy"] - r[1]["accuracy"],
            "tokens": r[0]["num_tokens"], "final_cache_size": r[0]["final_cache_size"],
            "tpot_engine_s": r[0]["tpot"], "tpot_ref_cpu_compress_s": r[1]["tpot"],
            "sample": f"fix_size_l2(fix_kv_size={fix}, keep_ratio={keep_ratio}), "
                      f"skip_layers=[0, 1], random-init {arch} architecture (GPT-NeoX) bf16, "
                      f"{r[0]['num_tokens']} synthetic tokens teacher-forced; engine vs the "
                      f"reference's CPU op sequence (golden-pinned port) as compress_fn "
                      f"({dt:.0f} s)"}


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
    if dist:  # gloo on a host tensor: the harness needs no device collective
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def shard_layers(num_layers_total, world, rank):
    """Contiguous layer block [start, end) owned by `rank` (layers sharded, no collectives)."""
    per = num_layers_total // world
    extra = num_layers_total % world
    start = rank * per + min(rank, extra)
    return start, start + per + (1 if rank < extra else 0)


def capture_jobs(step):
    """Run one call with the engine's execute() wrapped, returning the jobs it was given."""
    from kvcompress import _engine
    seen, real = [], _engine.execute

    def spy(jobs, *a, **kw):
        seen.extend(jobs)
        return real(jobs, *a, **kw)
    _engine.execute = spy
    try:
        step()
    finally:
        _engine.execute = real
    return seen


def dump_first_layer(dirname, rank, layer0, layers, out):
    """Test hook (--dump-layer): heads 0-1 of this rank's first layer -- inputs and the engine's
    outputs -- as bit patterns in DIR/rank<r>.npz, for tests/test_bench_multirank.py to check
    against the oracle.  Nothing here runs in the timed region."""
    import numpy as np

    def bits(t):
        t = t[:, :2].contiguous().cpu()
        return t.view(torch.int16).numpy() if t.element_size() == 2 else t.numpy()
    os.makedirs(dirname, exist_ok=True)
    (k, v), (ko, vo) = layers[0], out[0]
    np.savez(os.path.join(dirname, f"rank{rank}.npz"), k=bits(k), v=bits(v), k_out=bits(ko),
             v_out=bits(vo), layer=layer0, dtype=str(k.dtype))


def _free_port():
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    return port


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N copies of this script as ranks 0..N-1 (one GPU
    each, LOCAL_RANK = rank) and wait for them.  This process never touches the GPU (importing
    torch initialises nothing) and never re-execs itself; rank 0 prints the JSON line.  Returns
    the first non-zero child exit code (the other ranks are then stopped), else 0."""
    env = dict(os.environ, WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(n)]
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:  # a failed rank would leave the others in a barrier
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            p.kill()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=HEADLINE, choices=sorted(WORKLOADS))
    ap.add_argument("--layers-total", type=int, default=0,
                    help="shard this many layers over the ranks (strong scaling); "
                         "default: 32 layers per GPU (weak scaling)")
    ap.add_argument("--dtype", default="bf16", choices=sorted(DTYPES),
                    help="K/V storage dtype (fp16: what transformers >= 5 loads pythia as)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ppl-model", default="pythia-2.8b", choices=sorted(PPL_MODELS),
                    help="architecture of the random-init model of the PPL-delta leg")
    ap.add_argument("--dry-run", action="store_true",
                    help="harness check on CPU: gloo, stand-in step, no engine, no GPU")
    ap.add_argument("--same-device", action="store_true",
                    help="test only: every rank uses cuda:0 (a multi-rank run on a 1-GPU box)")
    ap.add_argument("--dump-layer", default=None, metavar="DIR",
                    help="test only: after the timed region each rank writes its first layer's "
                         "K/V inputs and outputs (heads 0-1) to DIR/rank<r>.npz")
    ap.add_argument("--as-shard", default=None, metavar="R/W",
                    help="tool: a single process runs exactly the layers rank R of a W-rank "
                         "strong-scaling launch owns (--layers-total or a cfg4/cfg5 workload), "
                         "e.g. 7/8 = the last 4 of 32 layers: the per-rank cost of the N=W split")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1, metavar="R",
                    help="test only (with --dry-run): rank R exits with an error after joining "
                         "the process group, before the first barrier")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
    else:
        local = 0 if args.same_device else local
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        sync = torch.cuda.synchronize
    dist = None
    if world > 1:
        # gloo on host tensors: the only cross-rank operations are the timing barrier and two
        # MAX / SUM all-reduces of host scalars -- the data path has no exchange, so no RCCL
        import torch.distributed as dist
        dist.init_process_group("gloo")
    if args.dry_run and rank == args.dry_run_fail_rank:
        sys.exit(f"rank {rank}: injected failure (--dry-run-fail-rank)")

    from kvcompress import _engine
    from kvcompress.methods import get_compress_fn

    method, kwargs, seq_len, head_dim, what = WORKLOADS[args.workload]
    layers_total = args.layers_total or STRONG_DEFAULT.get(args.workload, 0)
    shard = None
    if args.as_shard:
        if world > 1 or not layers_total:
            sys.exit("--as-shard: one process, and a strong-scaling split (--layers-total L or "
                     "a cfg4-/cfg5- workload)")
        sr, sw = (int(x) for x in args.as_shard.split("/"))
        if not 0 <= sr < sw:
            sys.exit(f"--as-shard {args.as_shard}: need 0 <= R < W")
        shard = (sr, sw)
    if shard:
        l0, l1 = shard_layers(layers_total, shard[1], shard[0])
        total, scaling = layers_total, "strong"
    elif layers_total:
        l0, l1 = shard_layers(layers_total, world, rank)
        total, scaling = layers_total, "strong"
    else:  # rank r owns layers [32r, 32r + 32) of a 32*N-layer stack
        l0, l1 = LAYERS * rank, LAYERS * (rank + 1)
        total, scaling = LAYERS * world, "weak"
    n_layers = l1 - l0
    # global layer ids on every rank: skip_layers (and pyramid_kv's depth-dependent sizes)
    extra = dict(layer_offset=l0)
    if method == "pyramid_kv":
        extra["num_layers_total"] = total
    fn = get_compress_fn(method)

    if args.dry_run:  # stand-in data and step: the harness, not the engine, is under test
        seq_len, head_dim = 64, 8
        g = torch.Generator().manual_seed(1000 + rank)
        layers = [(torch.randn(1, 2, seq_len, head_dim, generator=g),) * 2
                  for _ in range(n_layers)]

        def step():
            time.sleep(0.002 * (rank + 1))  # the last rank is the slow one
            return [(k[:, :, :8], v[:, :, :8]) for k, v in layers]
        nbytes = {"path": 1, "score": 1, "select+gather": 1}
        timer = None
    else:
        g = torch.Generator(device=dev).manual_seed(1000 + rank)
        layers = []
        for _ in range(n_layers):
            k = torch.randn(B, H, seq_len, head_dim, device=dev, generator=g,
                            dtype=torch.float32).to(DTYPES[args.dtype])
            v = torch.randn(B, H, seq_len, head_dim, device=dev, generator=g,
                            dtype=torch.float32).to(DTYPES[args.dtype])
            layers.append((k, v))

        def step():
            return fn(layers, skip_layers=[], **kwargs, **extra)

        es = layers[0][0].element_size() if layers else 2
        nbytes = job_bytes(capture_jobs(step), es)
        # per-kernel durations come from a SECOND pass of K steps after the timed one: the engine
        # then splits each launch into its kernels with HIP events recorded on the stream they
        # run on (created with hipEventDisableSystemFence).  The timed pass itself runs exactly
        # the untimed call (no events, no split launches).
        timer = _engine.PhaseTimer(fenceless=True)
    elapsed = timed_steps(step, args.steps, args.warmup, dist, sync, dev)
    if timer:
        _engine.set_phase_timer(timer)
        timed_steps(step, args.steps, 0, dist, sync, dev)
        _engine.set_phase_timer(None)
        dur = {k: sum(v) / len(v) for k, v in timer.durations_ms().items()}
    else:
        dur = {"score": elapsed / max(args.steps, 1) * 1e3}

    # units all ranks processed: positions scored (layers x S) per step
    units = torch.tensor([n_layers * seq_len], dtype=torch.float64)
    if dist:
        dist.all_reduce(units)
    units = float(units.item())

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        kern = max(dur, key=dur.get)  # dominant kernel of the step
        kern_gbps = nbytes[kern] / (dur[kern] * 1e-3) / 1e9
        headline = args.workload == HEADLINE
        traffic = (pmc_traffic() if headline and kern == "score" and args.dtype == "bf16"
                   and not args.dry_run else None)
        path_gbps = nbytes["path"] * world / (ms_step * 1e-3) / 1e9
        desc = {"score": "score_kernel (key L2 norms)",
                "select+gather": "select_gather_kernel (selection + segment copy)"}[kern]
        cfg_kw = ", ".join(f"{k}={v!r}" for k, v in kwargs.items())
        res = {
            "metric": "KV tokens scored+evicted/sec at S=16384, fix_size=512; PPL delta vs ref",
            "value": units * args.steps / elapsed,
            "unit": "KV tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (torch.randn, HBM-resident)",
            "config": {"workload": f"{method}_compress({cfg_kw}, skip_layers=[]) over "
                                   f"{n_layers} layers of K,V [1,{H},{seq_len},{head_dim}] per "
                                   f"GPU, one call per step ({what})",
                       "name": args.workload, "layers_per_gpu": n_layers,
                       "layers_total": total, "layer_offset": l0, "seq_len": seq_len, "heads": H,
                       "head_dim": head_dim,
                       "parallelism": f"layers sharded x{world}, no collectives"},
            "roofline": {"bound": "hbm", "kernel": desc,
                         "achieved": kern_gbps, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "frac": kern_gbps / PEAK_HBM_GBPS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": nbytes[kern],
                         "traffic_source": (PMC_FILE + " (rocprofv3 --pmc)") if traffic else None},
            "path_roofline": {"achieved": path_gbps, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                              "frac": path_gbps / PEAK_HBM_GBPS,
                              "bytes_per_step_per_gpu": nbytes["path"]},
            "kernel_ms_per_step": dur,
            "tokens_evicted_per_sec": None,
        }
        ev = sum(kv[0].size(2) for kv in layers) - sum(kv[0].size(2) for kv in step())
    if args.dump_layer and not args.dry_run:
        dump_first_layer(args.dump_layer, rank, l0, layers, step())
    if rank == 0:
        res["tokens_evicted_per_sec"] = ev * world * args.steps / elapsed
        from kvcompress import _engine as _E
        if _E.tie_policy != "reference":  # KVC_TIE_POLICY=stable: not the reference's tie order
            res["config"]["tie_policy"] = _E.tie_policy
        if shard:
            res["config"]["as_shard"] = f"rank {shard[0]} of {shard[1]} (layers {l0}-{l1 - 1})"
            res["n_gpus"] = 1
        if args.dry_run:
            res["dry_run"] = True
        elif not args.no_cpu_baseline and method == "fix_size_l2" and world == 1:  # N=1 only
            res["cpu_baseline"] = cpu_baseline(seq_len, head_dim, dtype=args.dtype)
            res["ppl_delta_vs_ref"] = ppl_delta(dev, arch=args.ppl_model)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
