"""Back-to-back check of a rocprofv3 kernel trace (python trace_gaps.py run_kernel_trace.csv):
for the engine's kernels (kvc::), the per-kernel average duration and the idle gap between the
end of one engine kernel and the start of the next, over the LAST half of the trace (warm), or
with a second argument `timed` over the second tenth to the half of it (bench.py's uninstrumented
timed pass when its K timed steps are 10x its W warmup steps: the second pass splits launches)."""
import csv
import json
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "kvc::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if len(sys.argv) > 2 and sys.argv[2] == "timed":
    rows = rows[len(rows) // 10:len(rows) // 2]
else:
    rows = rows[len(rows) // 2:]
dur, gaps = {}, []
for a, b in zip(rows, rows[1:]):
    gaps.append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    dur.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(json.dumps({"kernels": len(rows), "span_us": span,
                  "avg_us": {k: round(statistics.mean(v), 2) for k, v in dur.items()},
                  "gap_us_median": round(statistics.median(gaps), 2),
                  "gap_us_p90": round(sorted(gaps)[int(0.9 * len(gaps))], 2),
                  "busy_frac": round(sum(sum(v) for v in dur.values()) / span, 3)}))
