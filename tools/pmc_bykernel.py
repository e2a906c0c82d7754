"""Per-kernel averages of every counter in the rocprofv3 --pmc passes under a directory
(pmc_*/run_counter_collection.csv), as JSON on stdout (tools/gpu.sh gatherprobe).
FETCH_SIZE is KiB (x1024 -> bytes; on gfx950 wide coalesced streams show half their bytes,
MI355X_MICROARCH.md); TCC_EA0_RDREQ* are request counts."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main(root):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(\w+)<(\d+)>", r["Kernel_Name"]) or re.search(r"(\w+)", r["Kernel_Name"])
            name = m.group(0)
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}
    for d in out.values():
        if "FETCH_SIZE" in d:
            d["FETCH_bytes_raw"] = d["FETCH_SIZE"] * 1024
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
