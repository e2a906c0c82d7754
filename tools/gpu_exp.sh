set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/decode_bench.py > gpurun_out/decode.json 2>&1 || exit $?
cat gpurun_out/decode.json
timeout -k 10 300 python tools/host_profile.py > gpurun_out/host_profile.txt 2>&1 || exit $?
head -c 600 gpurun_out/host_profile.txt
timeout -k 10 400 python tools/chunk_pipe.py > gpurun_out/chunk_pipe.jsonl 2>&1 || exit $?
cat gpurun_out/chunk_pipe.jsonl
