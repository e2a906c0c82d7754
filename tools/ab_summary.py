"""Summaries printed by tools/gpu.sh:
    ab_summary.py AB_JSONL RECIPE          one line per A/B run of the recipe (ms/step, kernels)
    ab_summary.py --kernel-stats CSV       the engine kernels of a rocprofv3 stats file (us)
"""
import csv
import json
import sys


def main(argv):
    if argv[1] == "--kernel-stats":
        for r in csv.DictReader(open(argv[2])):
            if "kvc::" in r["Name"]:
                print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
        return
    for line in open(argv[1]):
        d = json.loads(line)
        if d.get("recipe") != argv[2]:
            continue
        r = d["r"]
        print(d["rep"], d["lib"], d["workload"], round(r["ms_per_step"], 4),
              {k: round(v, 4) for k, v in r["kernel_ms_per_step"].items()})


if __name__ == "__main__":
    main(sys.argv)
