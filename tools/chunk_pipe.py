"""Layer-chunk pipeline probe (GPU box, tuning aid): SCORE+SELECT of chunk c+1 on one stream
beside the GATHER of chunk c on a second stream, against the default single launch
(SCORE + SELECT_GATHER) and the three-kernel launch on one stream.  32 layers of [1,32,S,D]
bf16, fix_size_l2-shaped rows (zone = whole sequence, keep k).  Each chunk is planned as its
own table with its own workspace.  One JSON line per (S, D, k)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _native as N  # noqa: E402

dev = torch.device("cuda:0")
L, H = 32, 32


def tables(Ks, Vs, outs, k, chunks, flags):
    res = []
    per = L // chunks
    for c in range(chunks):
        sl = range(c * per, (c + 1) * per)
        t = np.zeros(per, dtype=N.LAYER_DTYPE)
        for i, l in enumerate(sl):
            K, V, (ko, vo) = Ks[l], Vs[l], outs[l]
            t[i]["k"], t[i]["v"] = K.data_ptr(), V.data_ptr()
            t[i]["k_out"], t[i]["v_out"] = ko.data_ptr(), vo.data_ptr()
            t[i]["k_stride"] = K.stride()[:3]
            t[i]["v_stride"] = V.stride()[:3]
            S = K.shape[2]
            t[i]["seq_len"], t[i]["zone_start"], t[i]["zone_len"], t[i]["n_select"] = S, 0, S, k
        p = N.Params(dtype=N.KVC_BF16, batch=1, heads=H, head_dim=Ks[0].shape[3], order=0,
                     algo=0, phases=N.PHASE_ALL, external_index=0, flags=flags)
        rc, info = N.plan(p, t)
        assert rc == 0, rc
        ws = torch.empty(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
        res.append((p, t, ws, info))
    return res


def launch(entry, phases, stream):
    p, t, ws, info = entry
    p.phases = phases
    rc = N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes), stream.cuda_stream)
    assert rc == 0, rc


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps, 4)


def main():
    cases = [(16384, 128, 512), (4096, 128, 512), (4096, 80, 512), (16384, 80, 13108)]
    sA = torch.cuda.current_stream()
    sB = torch.cuda.Stream()
    for S, D, k in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        Ks = [torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16) for _ in range(L)]
        Vs = [torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16) for _ in range(L)]
        outs = [(torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev),
                 torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev)) for _ in range(L)]
        res = {"S": S, "D": D, "k": k}
        one = tables(Ks, Vs, outs, k, 1, 0)[0]
        res["fused_one_stream"] = timed(lambda: launch(one, N.PHASE_ALL, sA))
        three = tables(Ks, Vs, outs, k, 1, N.FLAG_SPLIT_SELECT_GATHER)[0]
        res["three_one_stream"] = timed(lambda: launch(three, N.PHASE_ALL, sA))
        for chunks in (2, 4, 8):
            ent = tables(Ks, Vs, outs, k, chunks, N.FLAG_SPLIT_SELECT_GATHER)

            def pipe():
                for e in ent:
                    launch(e, N.PHASE_SCORE | N.PHASE_SELECT, sA)
                    ev = torch.cuda.Event()
                    ev.record(sA)
                    sB.wait_event(ev)
                    launch(e, N.PHASE_GATHER, sB)
                ev = torch.cuda.Event()
                ev.record(sB)
                sA.wait_event(ev)
            res[f"pipe{chunks}"] = timed(pipe)
            entf = tables(Ks, Vs, outs, k, chunks, 0)

            def pipef():  # score of chunk c+1 on A beside select_gather of chunk c on B
                for e in entf:
                    launch(e, N.PHASE_SCORE, sA)
                    ev = torch.cuda.Event()
                    ev.record(sA)
                    sB.wait_event(ev)
                    launch(e, N.PHASE_SELECT | N.PHASE_GATHER, sB)
                ev = torch.cuda.Event()
                ev.record(sB)
                sA.wait_event(ev)
            res[f"pipe_sg{chunks}"] = timed(pipef)
        print(json.dumps(res), flush=True)
        del Ks, Vs, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
