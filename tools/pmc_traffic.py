"""Per-launch HBM traffic of the engine kernels from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes (tools/gpu.sh pmc) -> profiles/<name>_pmc_traffic.json.

FETCH_SIZE / WRITE_SIZE are KiB.  On gfx950 FETCH_SIZE sees only half of wide coalesced read
streams (MI355X_MICROARCH.md, HBM / rocprofv3 section), so FETCH x2 is the HBM read estimate.
Usage: python tools/pmc_traffic.py gpurun_out profiles/r01_v6_pmc_traffic.json
(PMC_S / PMC_D: another fix_size_l2 workload's sequence length / head dim)"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
L, H, K = 32, 32, 512
S = int(os.environ.get("PMC_S", "16384"))  # the workload's geometry (default: the headline)
D = int(os.environ.get("PMC_D", "128"))
ALGO = {  # bytes per 32-layer launch of the headline workload
    "score_kernel": {"algorithmic_read": L * H * S * D * 2, "algorithmic_write": L * H * S * 2},
    "gather_kernel": {"algorithmic_read": 2 * L * H * K * D * 2,
                      "algorithmic_write": 2 * L * H * K * D * 2},
    # norms read + kept K,V rows read; K,V out written (the index list stays in LDS)
    "select_gather_kernel": {"algorithmic_read": L * H * S * 2 + 2 * L * H * K * D * 2,
                             "algorithmic_write": 2 * L * H * K * D * 2},
}
vals = defaultdict(lambda: defaultdict(list))
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    f = os.path.join(src, "pmc_" + ctr, "run_counter_collection.csv")
    for r in csv.DictReader(open(f)):
        m = re.search(r"kvc::(\w+)<([^>]*)>", r["Kernel_Name"])
        if not m:
            continue
        vals[f"kvc::{m.group(1)}<{m.group(2)}>"][ctr].append(float(r["Counter_Value"]))
out = {"note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 2 "
               "--warmup 1, per-dispatch averages in bytes; FETCH x2 = gfx950 HBM read estimate "
               "(tools/pmc_traffic.py)", "kernels": {}}
for k, d in vals.items():
    e = {}
    if d["FETCH_SIZE"]:
        raw = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024
        e["FETCH_SIZE_bytes_raw"] = raw
        e["FETCH_bytes_x2_gfx950"] = 2 * raw
    if d["WRITE_SIZE"]:
        e["WRITE_SIZE_bytes"] = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
    base = k.split("::")[1].split("<")[0]
    e.update(ALGO.get(base, {}))
    out["kernels"][k] = e
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
