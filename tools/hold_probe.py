"""Does keeping the previous call's outputs alive (as bench.py's `out = step()` loop does) cost
time for large fp32 outputs?  (GPU box, tuning aid.)  32 layers [1,32,16384,128], fix_size_l2(512)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress.methods import fix_size_l2_compress  # noqa: E402

res = {}
for name in sys.argv[1:] or ["fp32", "bf16"]:
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32}[name]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    layers = [(torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(dt),
               torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(dt)) for _ in range(32)]
    call = lambda: fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])  # noqa: E731
    for mode in ("drop", "hold", "drop", "hold"):
        out = None
        for _ in range(5):
            out = call() if mode == "hold" else (call(), None)[1]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            out = call() if mode == "hold" else (call(), None)[1]
        torch.cuda.synchronize()
        res.setdefault(name, {}).setdefault(mode, []).append((time.perf_counter() - t0) / 20 * 1e3)
        del out
    res[name]["reserved_GiB"] = torch.cuda.memory_reserved() / 2**30
    del layers
    torch.cuda.empty_cache()
print(json.dumps(res))
