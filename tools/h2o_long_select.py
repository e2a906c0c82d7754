"""Heavy-hitter selection of a long-context h2o_attention call on its own (A/B tool, GPU box):
32 layers of [1,32,16384] bf16 accumulated attention, k = 64 over the 15 936-position middle --
std::partial_sort's heap select, one row per layer.  Times kvc_heavy_hitters (head sum + select)
with HIP events over 50 calls; the library is the one KVC_LIB names (default libkvc.so)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress.methods.h2o_attention import H2OAttentionManager, run_heavy_hitters  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
L, H, S = 32, 32, 16384
mgr = H2OAttentionManager(start_size=4, heavy_hitter_size=64, recent_size=444)
att = tuple(torch.softmax(torch.randn(1, H, 1, S, device=dev, generator=g), -1).to(torch.bfloat16)
            for _ in range(L))
mgr.update_attention_scores(att)
rows = [mgr._hh_row(i, S) for i in range(L)]
out = torch.empty((L, 64), dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream()
for _ in range(5):
    run_heavy_hitters(mgr, rows, out.data_ptr(), 64, stream)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(50):
    run_heavy_hitters(mgr, rows, out.data_ptr(), 64, stream)
b.record()
torch.cuda.synchronize()
print(json.dumps({"lib": os.path.basename(os.environ.get("KVC_LIB", "libkvc.so")),
                  "heavy_hitters_ms": a.elapsed_time(b) / 50,
                  "checksum": int(out.long().sum().item())}))
