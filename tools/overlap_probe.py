"""Does SELECT (+GATHER) overlap with SCORE when they run on two streams?  (GPU box, tuning aid.)
Half the headline layers are scored on one stream while the other half's rows are selected
(and gathered: the select_gather kernel, unless OVERLAP_PHASES=select) on a second stream
(high priority unless OVERLAP_PRIO=0); compares with the same two launches back to back."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _native as N  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
L, H, S, D, k = 32, 32, 16384, 128, 512
Ks = [torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16) for _ in range(L)]
outs = [torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev) for _ in range(L)]


def make(layers):
    t = np.zeros(len(layers), dtype=N.LAYER_DTYPE)
    for i, li in enumerate(layers):
        K = Ks[li]
        t[i]["k"] = t[i]["v"] = K.data_ptr()
        t[i]["k_out"] = t[i]["v_out"] = outs[li].data_ptr()
        t[i]["k_stride"] = t[i]["v_stride"] = K.stride()[:3]
        t[i]["seq_len"], t[i]["zone_start"], t[i]["zone_len"], t[i]["n_select"] = S, 0, S, k
    p = N.Params(dtype=N.KVC_BF16, batch=1, heads=H, head_dim=D, order=0, algo=0,
                 phases=N.PHASE_ALL, external_index=0)
    rc, info = N.plan(p, t)
    assert rc == 0
    ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
    return p, t, info, ws


A = make(range(0, 16))
B = make(range(16, 32))


def run(tab, phases, stream):
    p, t, info, ws = tab
    p.phases = phases
    rc = N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes), stream.cuda_stream)
    assert rc == 0


SEL = N.PHASE_SELECT if os.environ.get("OVERLAP_PHASES") == "select" else (N.PHASE_SELECT | N.PHASE_GATHER)
s1 = torch.cuda.Stream(device=dev)
s2 = torch.cuda.Stream(device=dev, priority=-1 if os.environ.get("OVERLAP_PRIO", "1") == "1" else 0)
main = torch.cuda.current_stream(dev)
run(A, N.PHASE_SCORE, main)  # norms of A for its select
torch.cuda.synchronize()
res = {}
for mode in ("serial", "overlap", "serial", "overlap"):
    times = []
    for _ in range(5):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        if mode == "serial":
            run(B, N.PHASE_SCORE, main)
            run(A, SEL, main)
        else:
            s1.wait_stream(main)
            s2.wait_stream(main)
            run(B, N.PHASE_SCORE, s1)
            run(A, SEL, s2)
            main.wait_stream(s1)
            main.wait_stream(s2)
        e1.record(main)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    res.setdefault(mode, []).append(sorted(times)[2])
for nm, ph, tab in (("score_B_alone", N.PHASE_SCORE, B), ("select_A_alone", SEL, A)):
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        run(tab, ph, main)
        e1.record(main)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    res[nm] = sorted(ts)[2]
res["phases"] = int(SEL)
res["prio"] = os.environ.get("OVERLAP_PRIO", "1")
print(json.dumps(res))
