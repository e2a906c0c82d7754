"""Timeline of the fused persistent kernel on the headline workload (GPU box, tuning only).
KVC_FUSED_DIAG=2 makes the kernel stamp s_memrealtime (100 MHz) per row (dequeued, tiles
ready, selected, gathered) and per workgroup (start, score done) into the index region, which
the fused path does not otherwise use."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd"))
from kvcompress import _engine  # noqa: E402
from kvcompress.methods import fix_size_l2_compress  # noqa: E402

os.environ["KVC_FUSED"] = "1"
os.environ["KVC_FUSED_DIAG"] = "2"
dev = torch.device("cuda:0")
cus = torch.cuda.get_device_properties(dev).multi_processor_count
g = torch.Generator(device=dev).manual_seed(0)
layers = [(torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(torch.bfloat16),
           torch.randn(1, 32, 16384, 128, device=dev, generator=g).to(torch.bfloat16))
          for _ in range(32)]
out = {}
for wgs in (sys.argv[1] if len(sys.argv) > 1 else "56").split(","):
    os.environ["KVC_SEL_WGS"] = wgs
    for _ in range(3):
        fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])
    t = _engine.PhaseTimer(split=False, keep_workspace=True)
    _engine.set_phase_timer(t)
    fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])
    _engine.set_phase_timer(None)
    ms = t.durations_ms()["all"][0]
    ws, info = t.workspaces[0]
    rows = int(info.rows)
    raw = ws[info.index_offset:info.index_offset + (rows * 4 + 2 * cus) * 8].cpu().numpy()
    st = raw.view(np.uint64).astype(np.int64)
    rs = st[:rows * 4].reshape(rows, 4)
    wg = st[rows * 4:].reshape(cus, 2)
    t0 = wg[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731  (100 MHz ticks -> us)
    nsel = int(wgs)
    score_end = us(wg[:cus - nsel, 1])
    q = lambda a: [round(float(v), 1) for v in np.percentile(a, [0, 10, 50, 90, 100])]  # noqa
    wait = (rs[:, 1] - rs[:, 0]) / 100.0
    sel = (rs[:, 2] - rs[:, 1]) / 100.0
    gat = (rs[:, 3] - rs[:, 2]) / 100.0
    out[wgs] = {
        "kernel_ms": round(ms, 4),
        "wg_start_us": q(us(wg[:, 0])),
        "score_wg_done_us": q(score_end),
        "row_dequeue_us": q(us(rs[:, 0])),
        "row_wait_us": q(wait), "row_select_us": q(sel), "row_gather_us": q(gat),
        "last_row_done_us": round(float(us(rs[:, 3]).max()), 1),
        "rows_dequeued_before_score_done": int((us(rs[:, 0]) < np.median(score_end)).sum()),
    }
print(json.dumps(out))
