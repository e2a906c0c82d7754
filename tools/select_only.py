"""SELECT kernel alone on the headline rows (GPU box, profiling aid for rocprofv3 --pmc):
32 layers of [1,32,S,128] bf16, fix_size_l2-shaped rows (keep 512), one SCORE launch to fill
the norms, then REPS launches of the SELECT phase only (three-kernel path)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _native as N  # noqa: E402

dev = torch.device("cuda:0")
L, H, D, k = 32, 32, 128, 512
S = int(os.environ.get("SEL_S", "16384"))
reps = int(os.environ.get("SEL_REPS", "5"))
g = torch.Generator(device=dev).manual_seed(0)
DT = {"bf16": (torch.bfloat16, N.KVC_BF16), "fp16": (torch.float16, N.KVC_F16)}[
    os.environ.get("SEL_DTYPE", "bf16")]
SCALE = float(os.environ.get("SEL_SCALE", "1"))
Ks = [(torch.randn(1, H, S, D, device=dev, generator=g) * SCALE).to(DT[0]) for _ in range(L)]
out = torch.empty(1, H, k, D, dtype=DT[0], device=dev)
t = np.zeros(L, dtype=N.LAYER_DTYPE)
for i, K in enumerate(Ks):
    t[i]["k"] = t[i]["v"] = K.data_ptr()
    t[i]["k_out"] = t[i]["v_out"] = out.data_ptr()
    t[i]["k_stride"] = t[i]["v_stride"] = K.stride()[:3]
    t[i]["seq_len"], t[i]["zone_start"], t[i]["zone_len"], t[i]["n_select"] = S, 0, S, k
p = N.Params(dtype=DT[1], batch=1, heads=H, head_dim=D, order=0, algo=0,
             phases=N.PHASE_SCORE, external_index=0, flags=N.FLAG_SPLIT_SELECT_GATHER)
rc, info = N.plan(p, t)
assert rc == 0
ws = torch.empty(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
assert N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes), st) == 0
p.phases = N.PHASE_SELECT
if os.environ.get("SEL_SELECT_AS"):  # diagnostic: select the same norm bits as another 16-bit dtype
    p.dtype = {"bf16": N.KVC_BF16, "fp16": N.KVC_F16}[os.environ["SEL_SELECT_AS"]]
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    assert N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes), st) == 0
b.record()
torch.cuda.synchronize()
print(f"select ms/launch {a.elapsed_time(b) / reps:.4f}")
