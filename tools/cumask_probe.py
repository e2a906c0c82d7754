"""Can SELECT_GATHER hide behind SCORE if each gets its own CUs?  (GPU box, tuning aid.)

Streams created with hipExtStreamCreateWithCUMask split the chip: SCORE of a layer chunk runs on
`256 - c` CUs while the previous chunk's SELECT_GATHER runs on the other `c`.  Reports
  * SCORE alone (32 headline layers) on the full chip and on 256 - c CUs,
  * SELECT_GATHER alone on the full chip and on c CUs,
  * the pipelined step (chunks of `chunk` layers) vs the two launches back to back.
Mask bits are chosen as (i // 8) % d == 0 so either bit -> XCD mapping (i % 8 or i // 32) gives
every XCD the same share."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _native as N  # noqa: E402

dev = torch.device("cuda:0")
NCU = torch.cuda.get_device_properties(dev).multi_processor_count
g = torch.Generator(device=dev).manual_seed(0)
L, H, S, D, k = 32, 32, 16384, 128, 512
Ks = [torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16) for _ in range(L)]
outs = [torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev) for _ in range(L)]
hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]


def masked_stream(bits):
    words = (ctypes.c_uint32 * ((NCU + 31) // 32))()
    for i in bits:
        words[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(words), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device=dev)


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
    rc = N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes), stream.cuda_stream)
    assert rc == 0


SG = N.PHASE_SELECT | N.PHASE_GATHER
main = torch.cuda.current_stream(dev)


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
    return sorted(ts)[len(ts) // 2]


full = make(range(L))
run(full, N.PHASE_SCORE, main)
res = {"ncu": NCU, "score_full": timed(lambda: run(full, N.PHASE_SCORE, main)),
       "sg_full": timed(lambda: run(full, SG, main))}
for d in [int(x) for x in os.environ.get("CUMASK_D", "8,4").split(",")]:
    sel_bits = [i for i in range(NCU) if (i // 8) % d == 0]
    sc_bits = [i for i in range(NCU) if (i // 8) % d != 0]
    sA, sB = masked_stream(sc_bits), masked_stream(sel_bits)
    r = {"score_cus": len(sc_bits), "sg_cus": len(sel_bits)}

    def on(stream, fn):
        stream.wait_stream(main)
        fn(stream)
        main.wait_stream(stream)

    r["score_masked"] = timed(lambda: on(sA, lambda s: run(full, N.PHASE_SCORE, s)))
    r["sg_masked"] = timed(lambda: on(sB, lambda s: run(full, SG, s)))
    for chunk in (4, 8):
        tabs = [make(range(c, c + chunk)) for c in range(0, L, chunk)]
        evs = [torch.cuda.Event() for _ in tabs]

        def pipe():
            sA.wait_stream(main)
            sB.wait_stream(main)
            for t, e in zip(tabs, evs):
                run(t, N.PHASE_SCORE, sA)
                e.record(sA)
                sB.wait_event(e)
                run(t, SG, sB)
            main.wait_stream(sA)
            main.wait_stream(sB)

        def serial():
            for t in tabs:
                run(t, N.PHASE_SCORE, main)
                run(t, SG, main)

        r[f"pipe_chunk{chunk}"] = timed(pipe)
        r[f"serial_chunk{chunk}"] = timed(serial)
    res[f"d{d}"] = r
print(json.dumps(res))
