"""Can SELECT_GATHER run in the issue slots SCORE leaves idle?  (GPU box, tuning aid.)

SCORE is HBM-bound with its waves mostly parked on loads; SELECT_GATHER is LDS/issue-bound.  A
select workgroup (1024 threads, ~80 KiB LDS) can only share a CU with score workgroups if those
leave it room: here SCORE runs as a persistent grid of KVC_SCORE_GRID workgroups (256 threads,
36 KiB LDS each; 512 = two per CU = 8 waves + 72 KiB) on one stream, and the previous layer
chunk's SELECT_GATHER on a second, high-priority stream.  Reports per configuration: SCORE alone,
SELECT_GATHER alone, the chunked two-stream pipeline and the same launches back to back (ms,
32 headline layers)."""
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
Vs = [torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16) for _ in range(L)]
kouts = [torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev) for _ in range(L)]
vouts = [torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev) for _ in range(L)]


def make(layers):
    t = np.zeros(len(layers), dtype=N.LAYER_DTYPE)
    for i, li in enumerate(layers):
        t[i]["k"], t[i]["v"] = Ks[li].data_ptr(), Vs[li].data_ptr()
        t[i]["k_out"], t[i]["v_out"] = kouts[li].data_ptr(), vouts[li].data_ptr()
        t[i]["k_stride"] = t[i]["v_stride"] = Ks[li].stride()[:3]
        t[i]["seq_len"], t[i]["zone_start"], t[i]["zone_len"], t[i]["n_select"] = S, 0, S, k
    p = N.Params(dtype=N.KVC_BF16, batch=1, heads=H, head_dim=D, order=0, algo=0,
                 phases=N.PHASE_ALL, external_index=0)
    rc, info = N.plan(p, t)
    assert rc == 0
    ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
    return p, t, info, ws


def run(tab, phases, stream):
    p, t, info, ws = tab
    p.phases = phases
    rc = N.launch(p, t, 0, ws.data_ptr(), int(info.workspace_bytes), stream.cuda_stream)
    assert rc == 0


SG = N.PHASE_SELECT | N.PHASE_GATHER
main = torch.cuda.current_stream(dev)
s1 = torch.cuda.Stream(device=dev)
s2 = torch.cuda.Stream(device=dev, priority=-1)


def timed(fn, reps=7):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        fn()
        e1.record(main)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return round(sorted(ts)[len(ts) // 2], 4)


full = make(range(L))
res = {}
os.environ.pop("KVC_SCORE_GRID", None)
run(full, N.PHASE_SCORE, main)
res["default"] = {"score": timed(lambda: run(full, N.PHASE_SCORE, main)),
                  "sg": timed(lambda: run(full, SG, main)),
                  "all": timed(lambda: run(full, N.PHASE_ALL, main))}
ref_k = [x.clone() for x in kouts]
for grid in [int(x) for x in os.environ.get("PROBE_GRIDS", "256,512,768,1024").split(",")]:
    os.environ["KVC_SCORE_GRID"] = str(grid)
    r = {"score": timed(lambda: run(full, N.PHASE_SCORE, main))}
    for chunk in [int(x) for x in os.environ.get("PROBE_CHUNKS", "4,8").split(",")]:
        tabs = [make(range(c, c + chunk)) for c in range(0, L, chunk)]
        evs = [torch.cuda.Event() for _ in tabs]

        def pipe():
            s1.wait_stream(main)
            s2.wait_stream(main)
            for t, e in zip(tabs, evs):
                run(t, N.PHASE_SCORE, s1)
                e.record(s1)
                s2.wait_event(e)
                run(t, SG, s2)
            main.wait_stream(s1)
            main.wait_stream(s2)

        def serial():
            for t in tabs:
                run(t, N.PHASE_SCORE, main)
                run(t, SG, main)

        for x in kouts:
            x.zero_()
        r[f"pipe_c{chunk}"] = timed(pipe)
        torch.cuda.synchronize()
        r[f"pipe_c{chunk}_ok"] = all(torch.equal(a, b) for a, b in zip(kouts, ref_k))
        r[f"serial_c{chunk}"] = timed(serial)
    res[f"grid{grid}"] = r
print(json.dumps(res))
