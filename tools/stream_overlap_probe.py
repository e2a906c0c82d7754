"""Do SCORE and SELECT_GATHER of different layer chunks run concurrently on two plain streams?
(GPU box, tuning aid; round 6.)  With no CU mask a CU can hold one 74 KB SCORE workgroup and one
81.5 KB selection row at once, so SELECT_GATHER of chunk c could hide behind SCORE of chunk c+1.
Reports (ms, median of 7), headline geometry [1,32,16384,128] bf16, fix_size_l2 k = 512:
  * SCORE of 16 layers alone, SELECT_GATHER of 16 layers alone, both on two streams at once;
  * the 32-layer step as one SCORE + one SELECT_GATHER launch, and as a C-chunk pipeline
    (SCORE of every chunk on stream A; SELECT_GATHER of chunk c on stream B after chunk c's
    SCORE, event-ordered), C = 2, 4, 8, with stream B at default and at the highest priority."""
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
SG = N.PHASE_SELECT | N.PHASE_GATHER


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


def run(tab, phases, stream):
    p, t, info, ws = tab
    p.phases = phases
    assert N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes), stream.cuda_stream) == 0


main = torch.cuda.current_stream(dev)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
# SELECT_GATHER on a high-priority stream: the dispatcher then places its rows first as SCORE
# workgroups retire (one 81.5 KB row beside one 74 KB SCORE workgroup fits a CU's 160 KB)
lo_pri, hi_pri = torch.cuda.Stream.priority_range()
sbh = torch.cuda.Stream(dev, priority=hi_pri)


def timed(fn, reps=7):
    ts = []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        fn()
        e1.record(main)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = ts[1:]
    return round(sorted(ts)[len(ts) // 2], 4)


def fork_join(parts):
    """parts: [(stream, fn)]; both streams wait for main, main waits for both."""
    ev = torch.cuda.Event()
    ev.record(main)
    for s, fn in parts:
        s.wait_event(ev)
        with torch.cuda.stream(s):
            fn()
    for s, _ in parts:
        e = torch.cuda.Event()
        e.record(s)
        main.wait_event(e)


res = {}
lo, hi = make(range(16)), make(range(16, 32))
run(lo, N.PHASE_SCORE, main)  # norms of the low half for its SELECT_GATHER
torch.cuda.synchronize()
res["score16_alone"] = timed(lambda: run(hi, N.PHASE_SCORE, main))
res["sg16_alone"] = timed(lambda: run(lo, SG, main))
res["score16_and_sg16_two_streams"] = timed(
    lambda: fork_join([(sa, lambda: run(hi, N.PHASE_SCORE, sa)), (sb, lambda: run(lo, SG, sb))]))
whole = make(range(32))
res["step32_serial"] = timed(lambda: (run(whole, N.PHASE_SCORE, main), run(whole, SG, main)))
for C, sgs in ((2, sb), (4, sb), (8, sb), (2, sbh), (4, sbh), (8, sbh)):
    tabs = [make(range(c * L // C, (c + 1) * L // C)) for c in range(C)]

    def pipe():
        ev0 = torch.cuda.Event()
        ev0.record(main)
        sa.wait_event(ev0)
        sb.wait_event(ev0)
        for c in range(C):
            with torch.cuda.stream(sa):
                run(tabs[c], N.PHASE_SCORE, sa)
                e = torch.cuda.Event()
                e.record(sa)
            sgs.wait_event(e)
            with torch.cuda.stream(sgs):
                run(tabs[c], SG, sgs)
        for s in (sa, sgs):
            e = torch.cuda.Event()
            e.record(s)
            main.wait_event(e)
    res[f"step32_pipeline_{C}chunks" + ("_sg_high_priority" if sgs is sbh else "")] = timed(pipe)
print(json.dumps(res))
