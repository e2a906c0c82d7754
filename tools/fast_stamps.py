import os, sys, json
import numpy as np, torch
ROOT = os.environ["GRAFT_REPO_ROOT"] if "GRAFT_REPO_ROOT" in os.environ else "/root/repo"
os.environ["KVC_LIB"] = os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd/kvcompress/_lib/libkvc_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _native as N
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
L, H, S, D, k = 8, 32, 16384, 128, 512
Ks = [torch.randn(1, H, S, D, device=dev, generator=g) for _ in range(L)]
table = np.zeros(L, dtype=N.LAYER_DTYPE)
outs = []
for i, K in enumerate(Ks):
    o = torch.empty(1, H, k, D, dtype=K.dtype, device=dev); outs.append(o)
    t = table[i]; t["k"] = t["v"] = K.data_ptr(); t["k_out"] = t["v_out"] = o.data_ptr()
    t["k_stride"] = t["v_stride"] = K.stride()[:3]
    t["seq_len"], t["zone_start"], t["zone_len"], t["n_select"] = S, 0, S, k
p = N.Params(dtype=N.KVC_F32, batch=1, heads=H, head_dim=D, order=0, algo=0, phases=N.PHASE_SCORE | N.PHASE_SELECT, external_index=0)
rc, info = N.plan(p, table); assert rc == 0
ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
rc = N.launch(p, table, ws.data_ptr(), int(info.workspace_bytes), torch.cuda.current_stream().cuda_stream); assert rc == 0
torch.cuda.synchronize()
rows = int(info.rows)
st = ws[-rows * 256:].view(torch.int64).view(rows, 32).cpu().numpy().astype(np.float64)
fast = st[:, 31] > 0
print(json.dumps({"rows": rows, "fast_taken": int(fast.sum()), "load_cycles_med": float(np.median(st[:,1]-st[:,0])),
  "fast_cycles_med": float(np.median((st[fast,31]-st[fast,1]))) if fast.any() else None,
  "chain_rows_total_med": float(np.median(st[~fast,4]-st[~fast,0])) if (~fast).any() else None}))
