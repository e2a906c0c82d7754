"""Interleaved A/B timing of engine kernel variants on the headline workload (one process,
rounds interleaved; cdna_hip_programming.md §5.4 rule 24).  GPU box only."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _engine  # noqa: E402
from kvcompress.methods import fix_size_l2_compress  # noqa: E402

# variant = split | unfused | fused[@W]:  split = three kernels timed per phase; unfused = three
# kernels timed as one launch (KVC_FUSED=0); fused = the persistent kernel (one launch), @W =
# W workgroups start on the row queue (KVC_SEL_WGS); suffix %T = T score tiles per wave
# (KVC_SCORE_TPW, software-pipelined score kernel)
variants = sys.argv[1].split(",") if len(sys.argv) > 1 else ["split", "unfused", "fused"]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
layers = [(torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(torch.bfloat16),
           torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(torch.bfloat16))
          for _ in range(32)]
res = {v: {} for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        v1, _, ntl = v.partition("!")  # !s / !g: temporal score loads / gather stores
        os.environ["KVC_SCORE_NT"] = "0" if "s" in ntl else "1"
        os.environ["KVC_GATHER_NT"] = "0" if "g" in ntl else "1"
        v0, _, tpw = v1.partition("%")
        os.environ["KVC_SCORE_TPW"] = tpw or "1"
        name, _, diag = v0.partition("#")
        name, _, wgs = name.partition("@")
        os.environ["KVC_FUSED_DIAG"] = diag or "0"
        os.environ["KVC_FUSED"] = "1" if name == "fused" else "0"
        if wgs:
            os.environ["KVC_SEL_WGS"] = wgs
        else:
            os.environ.pop("KVC_SEL_WGS", None)
        t = _engine.PhaseTimer(split=(name == "split"))
        _engine.set_phase_timer(t)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            out = fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])
        b.record()
        _engine.set_phase_timer(None)
        d = t.durations_ms()
        d = {ph: [sum(xs) / 5] for ph, xs in d.items()}  # per-step kernel time (all chunks)
        d["step_wall"] = [a.elapsed_time(b) / 5]
        for ph, xs in d.items():
            res[v].setdefault(ph, []).append(min(xs))
        if diag:
            pass
        elif ref is None:
            ref = [(a.clone(), b.clone()) for a, b in out]
        else:
            assert all(torch.equal(a, c) and torch.equal(b, e) for (a, b), (c, e) in zip(out, ref))
print(json.dumps({v: {ph: sorted(x)[len(x) // 2] for ph, x in d.items()} for v, d in res.items()}))
