"""Select-kernel tuning sweep (GPU box only): per variant (environment overrides of the engine's
tuning knobs) the SELECT phase time of one fix_size_l2 call over 32 layers of [1,32,S,128] bf16,
rounds interleaved.  Usage: select_sweep.py S "ENV=V[;ENV=V]|..." [rounds]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _engine  # noqa: E402
from kvcompress.methods import get_compress_fn  # noqa: E402

S = int(sys.argv[1])
variants = sys.argv[2].split("|")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
method = os.environ.get("SWEEP_METHOD", "fix_size_l2")
kw = json.loads(os.environ.get("SWEEP_KW", '{"fix_kv_size": 512}'))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
layers = [(torch.randn(1, 32, S, 128, device=dev, generator=g).to(torch.bfloat16),
           torch.randn(1, 32, S, 128, device=dev, generator=g).to(torch.bfloat16))
          for _ in range(32)]
fn = get_compress_fn(method)
knobs = {k for v in variants for k in (kv.split("=")[0] for kv in v.split(";") if kv)}
res = {v: [] for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        for k in knobs:
            os.environ.pop(k, None)
        for kv in v.split(";"):
            if kv:
                k, _, val = kv.partition("=")
                os.environ[k] = val
        t = _engine.PhaseTimer(split=True, steps=_engine.PhaseTimer.THREE if os.environ.get("KVC_SEL_GATHER") == "0" else None)
        _engine.set_phase_timer(t)
        for _ in range(5):
            out = fn(layers, skip_layers=[], **kw)
        _engine.set_phase_timer(None)
        d = t.durations_ms()
        res[v].append(min(d.get("select", d.get("select+gather"))))
        got = [(a.cpu(), b.cpu()) for a, b in out[:4]]
        if ref is None:
            ref = got
        else:
            assert all(torch.equal(a, c) and torch.equal(b, d) for (a, b), (c, d) in zip(got, ref)), v
print(json.dumps({"S": S, "method": method, "select_ms_min": {v: min(x) for v, x in res.items()},
                  "select_ms_median": {v: sorted(x)[len(x) // 2] for v, x in res.items()}}))
