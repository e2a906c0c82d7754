#!/bin/bash
# Round-2 validation pass on the committed tree: GPU tests, smoke, headline bench, rocprofv3
# kernel stats of the bench, every BASELINE workload, decode step.  Each GPU step has its own
# limit; the first failure (other than pytest test failures) ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1 || exit $?
cd "$R"
bash tools/gpu_check.sh workloads > /dev/null 2>&1 || exit $?
timeout -k 10 300 python tools/decode_bench.py 2>/dev/null > gpurun_out/decode.json || exit $?
cat gpurun_out/decode.json
exit $rc
