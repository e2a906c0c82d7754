#!/bin/bash
# dev run: the long h2o_attention call, three times (decode bench) + one rocprofv3 kernel-stats pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2 3; do
  timeout -k 10 300 python tools/decode_bench.py > gpurun_out/decode_$i.json 2> gpurun_out/decode.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/decode_$i.json')); print(d['h2o_attention_s16384'], d['h2o_attention'])"
done
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/h2oprof2 -o run -- python3 $GRAFT_REPO_ROOT/tools/h2o_long_profile.py > $GRAFT_REPO_ROOT/gpurun_out/h2oprof2.log 2>&1 ) || exit 1
grep ms_per_call gpurun_out/h2oprof2.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/h2oprof2/run_kernel_stats.csv')):
    if 'kvc::' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')
PY
