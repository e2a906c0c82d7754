#!/bin/bash
# dev run: probes, h2o GPU tests, the long h2o_attention call profile, full GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
timeout -k 10 60 tools/dpp_probe || exit 1
timeout -k 10 60 tools/heap_probe_old && timeout -k 10 60 tools/heap_probe || exit 1
timeout -k 10 600 python -u -m pytest tests/test_h2o_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/h2o_pytest.log 2>&1 || { tail -30 $O/h2o_pytest.log; exit 1; }
tail -1 $O/h2o_pytest.log
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
bash tools/gpu.sh test
