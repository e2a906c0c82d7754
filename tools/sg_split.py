"""Where SELECT_GATHER's time goes at a geometry (GPU box, tuning aid): the fused kernel against
SELECT alone and GATHER alone (KVC_FLAG_SPLIT_SELECT_GATHER launches of the same plan), 32 layers
of fix_size_l2-shaped rows [1,32,S,D] bf16 (zone = the whole sequence, keep k), scores computed
once beforehand.  One JSON line per (S, D, k); times are ms per 32-layer launch (HIP events over
20 launches)."""
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


def table(Ks, Vs, outs, k, flags):
    t = np.zeros(L, dtype=N.LAYER_DTYPE)
    for i in range(L):
        K, V, (ko, vo) = Ks[i], Vs[i], outs[i]
        t[i]["k"], t[i]["v"] = K.data_ptr(), V.data_ptr()
        t[i]["k_out"], t[i]["v_out"] = ko.data_ptr(), vo.data_ptr()
        t[i]["k_stride"] = K.stride()[:3]
        t[i]["v_stride"] = V.stride()[:3]
        S = K.shape[2]
        t[i]["seq_len"], t[i]["zone_start"], t[i]["zone_len"], t[i]["n_select"] = S, 0, S, k
    p = N.Params(dtype=N.KVC_BF16, batch=1, heads=H, head_dim=Ks[0].shape[3], order=0, algo=0,
                 phases=N.PHASE_ALL, external_index=0, flags=flags)
    rc, info = N.plan(p, t)
    assert rc == 0, rc
    ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
    return p, t, ws, info


def launch(e, phases):
    p, t, ws, info = e
    p.phases = phases
    rc = N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes),
                  torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc


def timed(fn, reps=20):
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
    cases = [tuple(int(x) for x in c.split("/"))
             for c in os.environ.get("SG_CASES", "4096/80/512,4096/128/512,16384/128/512").split(",")]
    for S, D, k in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        Ks = [torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16) for _ in range(L)]
        Vs = [torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16) for _ in range(L)]
        outs = [(torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev),
                 torch.empty(1, H, k, D, dtype=torch.bfloat16, device=dev)) for _ in range(L)]
        fused = table(Ks, Vs, outs, k, 0)
        split = table(Ks, Vs, outs, k, N.FLAG_SPLIT_SELECT_GATHER)
        launch(fused, N.PHASE_SCORE)
        launch(split, N.PHASE_SCORE | N.PHASE_SELECT)
        moved = 2 * 2 * L * H * k * D * 2  # K,V rows read + written
        res = {"S": S, "D": D, "k": k,
               "select_gather_fused": timed(lambda: launch(fused, N.PHASE_SELECT | N.PHASE_GATHER)),
               "select_only": timed(lambda: launch(split, N.PHASE_SELECT)),
               "gather_only": timed(lambda: launch(split, N.PHASE_GATHER)),
               "copy_bytes": moved}
        res["gather_TBps"] = round(moved / res["gather_only"] / 1e9, 2)
        print(json.dumps(res), flush=True)
        del Ks, Vs, outs, fused, split
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
