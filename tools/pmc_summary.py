"""Sum rocprofv3 counter_collection CSVs per (kernel, counter): python pmc_summary.py DIR..."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

tot = defaultdict(float)
n = defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "?")[:60]
            tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])].add(r.get("Dispatch_Id", ""))
out = defaultdict(dict)
for (k, c), v in tot.items():
    out[k][c] = v / max(1, len(n[(k, c)]))  # per dispatch
print(json.dumps(out, indent=1))
