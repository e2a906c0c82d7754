"""Phase breakdown of the select kernel from the diagnostic stamps build (libkvc_stamps.so):
median per-row cycles of key load / block chain / wave chain / emission on the headline
workload (32 layers x 32 heads, S=16384, k=512).  GPU box only; read shares, not absolutes."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["KVC_LIB"] = os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd", "kvcompress",
                                     "_lib", os.environ.get("SEL_LIB", "libkvc_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _native as N  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
L, H, D = int(os.environ.get("SEL_L", "32")), 32, 128  # SEL_L=4: the 8-way split (128 rows)
S = int(os.environ.get("SEL_S", "16384"))
k = int(os.environ.get("SEL_K", "512"))
ALGO = int(os.environ.get("SEL_ALGO", "0"))      # 1: topk (introselect)
ORDER = int(os.environ.get("SEL_ORDER", "0"))    # 1: descending
SCORE = int(os.environ.get("SEL_SCORE", "0"))    # 1: snapkv scoring (pool 5)
DT = {"bf16": (torch.bfloat16, N.KVC_BF16), "fp16": (torch.float16, N.KVC_F16),
      "fp32": (torch.float32, N.KVC_F32)}[os.environ.get("SEL_DTYPE", "bf16")]
Ks = [torch.randn(1, H, S, D, device=dev, generator=g).to(DT[0]) for _ in range(L)]
table = np.zeros(L, dtype=N.LAYER_DTYPE)
outs = []
for i, K in enumerate(Ks):
    o = torch.empty(1, H, k, D, dtype=K.dtype, device=dev)
    outs.append(o)
    t = table[i]
    t["k"] = t["v"] = K.data_ptr()
    t["k_out"] = t["v_out"] = o.data_ptr()
    t["k_stride"] = t["v_stride"] = K.stride()[:3]
    t["seq_len"], t["zone_start"], t["zone_len"], t["n_select"] = S, 0, S, k
    t["score_mode"], t["pool_kernel"] = SCORE, 5 if SCORE else 0
p = N.Params(dtype=DT[1], batch=1, heads=H, head_dim=D, order=ORDER, algo=ALGO,
             phases=N.PHASE_SCORE | N.PHASE_SELECT, external_index=0)
rc, info = N.plan(p, table)
assert rc == 0
ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
res = {"wave_seg": "compile-time kWaveSeg", "layers": L, "S": S, "k": k, "algo": ALGO, "order": ORDER,
       "score_mode": SCORE}
for rep in range(3):
    rc = N.launch(p, table, ws.data_ptr(), int(info.workspace_bytes),
                  torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
rows = int(info.rows)
allst = ws[-rows * 256:].view(torch.int64).view(rows, 32).cpu().numpy().astype(np.float64)
st = allst[:, :5]
if ALGO == 2:  # KVC_ALGO_STABLE: key load | min/max | radix (or bisection) | count + emission
    d = np.diff(st, axis=1)
    res["median_cycles"] = {n: float(np.median(d[:, i])) for i, n in enumerate(
        ("key_load", "min_max", "radix", "count_emit"))}
    res["row_total_median"] = float(np.median(st[:, 4] - st[:, 0]))
    res["span_cycles"] = float(st[:, 4].max() - st[:, 0].min())
    print(json.dumps(res))
    sys.exit(0)
for nm, off in (("block", 5), ("wave", 10)):
    acc = allst[:, off:off + 5]
    res[nm + "_levels_median"] = float(np.median(acc[:, 3]))
    res[nm + "_swaps_per_level_median"] = float(np.median(acc[:, 4] / np.maximum(acc[:, 3], 1)))
    for q, pn in enumerate(("median+P1", "P2", "P4")):
        res[f"{nm}_{pn}_cycles_per_level"] = float(np.median(acc[:, q] / np.maximum(acc[:, 3], 1)))
d = np.diff(st, axis=1)
names = ["key_load", "block_chain", "wave_chain", "emit"]
res["median_cycles"] = {n: float(np.median(d[:, i])) for i, n in enumerate(names)}
res["p90_cycles"] = {n: float(np.percentile(d[:, i], 90)) for i, n in enumerate(names)}
res["row_total_median"] = float(np.median(st[:, 4] - st[:, 0]))
res["span_cycles"] = float(st[:, 4].max() - st[:, 0].min())
starts = np.sort(st[:, 0] - st[:, 0].min())
res["start_quantiles"] = [float(x) for x in np.percentile(starts, [0, 25, 50, 75, 100])]
lv = allst[:, 16:32].reshape(rows, 8, 2)
res["block_level_cycles_median"] = [float(np.median(lv[:, i, 0])) for i in range(7)]
sp = allst[:, 16:32].reshape(rows, 8, 2)[:, :, 1].astype(np.int64)
for q, nm in enumerate(("P1", "P2", "P4")):
    res["block_level_" + nm + "_median"] = [float(np.median((sp[:, i] >> (20 * q)) & 0xFFFFF))
                                            for i in range(7)]
print(json.dumps(res))
if DT[1] == N.KVC_F32:  # untied fast path (slot 31 stamped when taken): key load, fast select
    fast = allst[:, 31] > 0
    print(json.dumps({"fp32_fast_path_rows": int(fast.sum()), "rows": rows,
                      "key_load_median": float(np.median(allst[:, 1] - allst[:, 0])),
                      "fast_select_median": float(np.median((allst[:, 31] - allst[:, 1])[fast]))
                      if fast.any() else None}))
if os.environ.get("SEL_P1_STAMPS"):  # diagnostic: level-0 P1 sub-phases (slots 26..29)
    ph = allst[:, 26:30].astype(np.float64)
    print(json.dumps({"level0_P1_phases_median": {
        n: float(np.median(ph[:, i])) for i, n in enumerate(
            ("wave_start_skew", "longest_wave_P1", "last_P1_end_after_first_start",
             "last_P2_end_after_B_a"))}}))
if os.environ.get("SEL_SNAP_STAMPS"):  # diagnostic: snapkv scoring phases (slots 26..29)
    if np.all(allst[:, 27] == 0):  # round 6: SCORE's tile maxima, no block barrier / tmp
        ph = np.stack([allst[:, 26] - allst[:, 0], allst[:, 29] - allst[:, 26],
                       allst[:, 1] - allst[:, 29], allst[:, 1] - allst[:, 0]], axis=1)
        names = ["tile max -> m", "scores+pool+keys+idx (halo loads)", "barrier",
                 "snapkv scoring total"]
    else:
        ph = np.stack([allst[:, 26] - allst[:, 0], allst[:, 27] - allst[:, 26],
                       allst[:, 28] - allst[:, 27], allst[:, 29] - allst[:, 28],
                       allst[:, 1] - allst[:, 29], allst[:, 1] - allst[:, 0]], axis=1)
        names = ["load+local max", "block max", "scores->tmp", "pool+keys", "idx init",
                 "snapkv scoring total"]
    print(json.dumps({"snapkv_phases_median": [float(np.median(ph[:, i])) for i in range(len(names))],
                      "names": names}))
