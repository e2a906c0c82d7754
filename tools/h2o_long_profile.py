"""The long-context h2o_attention call alone (32 layers of [1,32,16384,128] bf16, one attention
row per layer, heavy hitters over the 15 936-position middle), repeated: run it under
`rocprofv3 --kernel-trace --stats` to split its time over the accumulate, head-sum, heavy-hitter
select and gather kernels (GPU box only)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress.methods.h2o_attention import H2OAttentionManager, h2o_attention_compress  # noqa

dev = torch.device("cuda:0")
L, H, D, S = 32, 32, 128, 16384
g = torch.Generator(device=dev).manual_seed(0)
kv = [(torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16),
       torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16)) for _ in range(L)]
att = tuple(torch.softmax(torch.randn(1, H, 1, S, device=dev, generator=g), -1).to(torch.bfloat16)
            for _ in range(L))
mgr = H2OAttentionManager(start_size=4, heavy_hitter_size=64, recent_size=444)
reps = int(os.environ.get("REPS", "20"))
for _ in range(5):
    h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr, skip_layers=[])
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr, skip_layers=[])
torch.cuda.synchronize()
print(json.dumps({"h2o_attention_s16384_ms_per_call": (time.perf_counter() - t0) / reps * 1e3}))
