set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python tools/decode_bench.py > gpurun_out/decode.json 2>/dev/null || exit $?
cat gpurun_out/decode.json
timeout -k 10 300 python tools/host_profile.py > gpurun_out/host_profile.txt 2>/dev/null || exit $?
head -c 400 gpurun_out/host_profile.txt; echo
cd /tmp && export TMPDIR=/tmp
HOST_PROFILE_CALLS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/dectrace" -o run -- python3 "$R/tools/host_profile.py" > "$R/gpurun_out/dectrace.log" 2>&1 || exit $?
python3 "$R/tools/trace_gaps.py" "$R/gpurun_out/dectrace/run_kernel_trace.csv"
cd "$R"
bash tools/gpu_check.sh workloads
