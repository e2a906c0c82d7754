"""Host-side cost of one drop-in compress call (GPU box, tuning aid): per-call wall time with a
sync after every call, the issue rate without syncs (host-bound if equal), and a cProfile of
the host path.  Decode-step geometry: 32 layers of [1,32,S,128] bf16, S = 513 (fix_size_l2 512)."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress.methods import get_compress_fn  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 513
method = sys.argv[2] if len(sys.argv) > 2 else "fix_size_l2"
kw = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {"fix_kv_size": 512}
dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[
    os.environ.get("HOST_PROFILE_DTYPE", "bf16")]
n = int(os.environ.get("HOST_PROFILE_CALLS", "200"))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
layers = [(torch.randn(1, 32, S, 128, device=dev, generator=g).to(dt),
           torch.randn(1, 32, S, 128, device=dev, generator=g).to(dt))
          for _ in range(32)]
fn = get_compress_fn(method)
call = lambda: fn(layers, skip_layers=[], **kw)  # noqa: E731
if method == "h2o_attention":  # one query row of attention per layer and step, a manager
    from kvcompress.methods.h2o_attention import H2OAttentionManager
    att = tuple(torch.softmax(torch.randn(1, 32, 1, S, device=dev, generator=g), -1).to(dt)
                for _ in range(32))
    mgr = H2OAttentionManager(**kw)
    call = lambda: fn(layers, attention_scores=att, h2o_manager=mgr, skip_layers=[], **kw)  # noqa
for _ in range(20):
    call()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    call()
    torch.cuda.synchronize()
synced = (time.perf_counter() - t0) / n * 1e3
t0 = time.perf_counter()
for _ in range(n):
    call()
issue = (time.perf_counter() - t0) / n * 1e3
torch.cuda.synchronize()
drained = (time.perf_counter() - t0) / n * 1e3
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    call()
e1.record()
torch.cuda.synchronize()
gpu = e0.elapsed_time(e1) / n
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    call()
pr.disable()
torch.cuda.synchronize()
buf = io.StringIO()
pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(18)
print(json.dumps({"S": S, "method": method, "dtype": str(dt), "ms_per_call_synced": synced,
                  "ms_per_call_issue_only": issue, "ms_per_call_pipelined": drained,
                  "ms_per_call_events": gpu}))
print(buf.getvalue())
