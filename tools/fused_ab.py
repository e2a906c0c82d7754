"""Single-launch A/B of the launch paths on the headline workload (GPU box, tuning aid):
KVC_FUSED=0 (SCORE + SELECT_GATHER kernels) and 1 (persistent fused, CUs split between roles).
ms per 32-layer fix_size_l2(512) call from HIP events over 30 back-to-back calls; outputs
compared with mode 0."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress.methods import fix_size_l2_compress  # noqa: E402

dev = torch.device("cuda:0")
dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[os.environ.get("AB_DTYPE", "bf16")]
S = int(os.environ.get("AB_S", "16384"))
g = torch.Generator(device=dev).manual_seed(0)
layers = [(torch.randn(1, 32, S, 128, device=dev, generator=g).to(dt),
           torch.randn(1, 32, S, 128, device=dev, generator=g).to(dt)) for _ in range(32)]
call = lambda: fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])  # noqa: E731
res = {}
ref = None
for mode in os.environ.get("AB_MODES", "0,1,0,1").split(","):
    os.environ["KVC_FUSED"] = mode
    for _ in range(5):
        out = call()
    torch.cuda.synchronize()
    if ref is None:
        ref = out
    same = all(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) for a, b in zip(out, ref))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        call()
    e1.record()
    torch.cuda.synchronize()
    res.setdefault(f"fused={mode}", []).append((round(e0.elapsed_time(e1) / 30, 4), same))
print(json.dumps(res))
