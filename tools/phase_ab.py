"""Per-phase kernel times of one library build (select KVC_LIB to A/B builds in separate
processes; GPU box, tuning aid).  32 layers of [1,32,AB_S,AB_D] in AB_DTYPE, fix_size_l2(512):
SCORE / SELECT / GATHER as three timed launches, and SCORE / SELECT_GATHER as the default two."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _engine  # noqa: E402
from kvcompress.methods import get_compress_fn  # noqa: E402

dev = torch.device("cuda:0")
dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[
    os.environ.get("AB_DTYPE", "fp32")]
S = int(os.environ.get("AB_S", "16384"))
D = int(os.environ.get("AB_D", "128"))
METHOD = os.environ.get("AB_METHOD", "fix_size_l2")
KW = json.loads(os.environ.get("AB_KW", '{"fix_kv_size": 512}'))
fn = get_compress_fn(METHOD)
g = torch.Generator(device=dev).manual_seed(0)
layers = [(torch.randn(1, 32, S, D, device=dev, generator=g).to(dt),
           torch.randn(1, 32, S, D, device=dev, generator=g).to(dt)) for _ in range(32)]
res = {"lib": os.path.basename(os.environ.get("KVC_LIB", "libkvc.so")), "dtype": str(dt),
       "method": METHOD}
for name, steps in (("three", _engine.PhaseTimer.THREE), ("two", _engine.PhaseTimer.DEFAULT)):
    _engine.split_select_gather = name == "three"
    for _ in range(3):
        fn(layers, skip_layers=[], **KW)
    t = _engine.PhaseTimer(steps=steps)
    _engine.set_phase_timer(t)
    for _ in range(10):
        fn(layers, skip_layers=[], **KW)
    _engine.set_phase_timer(None)
    res[name] = {k: round(sum(v) / len(v), 4) for k, v in t.durations_ms().items()}
print(json.dumps(res))
