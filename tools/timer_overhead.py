"""Does the bench's live per-kernel timing (the launch split into SCORE and SELECT_GATHER with
HIP events between them) cost GPU time?  Headline step timed with and without the PhaseTimer
(GPU box, tuning aid)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _engine  # noqa: E402
from kvcompress.methods import fix_size_l2_compress  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
layers = [(torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(torch.bfloat16),
           torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(torch.bfloat16))
          for _ in range(32)]
step = lambda: fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])  # noqa: E731


def run(timer, n=30):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    _engine.set_phase_timer(timer)
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    _engine.set_phase_timer(None)
    return dt


res = {}
for rep in range(2):
    res[f"plain_{rep}"] = round(run(None), 4)
    res[f"split_events_{rep}"] = round(run(_engine.PhaseTimer()), 4)
    res[f"whole_events_{rep}"] = round(run(_engine.PhaseTimer(split=False)), 4)
    res[f"split_fenceless_{rep}"] = round(run(_engine.PhaseTimer(fenceless=True)), 4)
print(json.dumps(res))
t = _engine.PhaseTimer(fenceless=True)
run(t)
print(json.dumps({k: round(sum(v) / len(v), 4) for k, v in t.durations_ms().items()}))
