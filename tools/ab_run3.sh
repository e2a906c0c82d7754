#!/bin/bash
# dev run: full GPU suite, the long h2o_attention call profile, decode steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
bash tools/gpu.sh test || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/h2oprof -o run -- python3 $GRAFT_REPO_ROOT/tools/h2o_long_profile.py > $GRAFT_REPO_ROOT/$O/h2oprof.log 2>&1 ) || exit 1
grep ms_per_call $O/h2oprof.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/h2oprof/run_kernel_stats.csv')):
    if 'kvc::' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
rows=[r for r in csv.DictReader(open('gpurun_out/h2oprof/run_kernel_trace.csv')) if 'kvc::' in r['Kernel_Name']]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
t0=int(rows[-5]['Start_Timestamp'])
for r in rows[-5:]:
    s=int(r['Start_Timestamp'])-t0; e=int(r['End_Timestamp'])-t0
    print(f"{r['Kernel_Name'][:40]:40s} q={r['Queue_Id']} {s/1e3:8.1f} {e/1e3:8.1f}")
PY
bash tools/gpu.sh decode
