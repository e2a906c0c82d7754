# Round-end pass on the committed tree: GPU suite, smoke, headline bench, rocprofv3 kernel stats of
# the bench, decode steps.  Each GPU step has its own limit; the first failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
grep smoke gpurun_out/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1 || exit $?
cd "$R"
timeout -k 10 300 python tools/decode_bench.py 2>/dev/null > gpurun_out/decode.json || exit $?
cat gpurun_out/decode.json
