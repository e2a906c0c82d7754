set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for S in ${AB_S_LIST:-16384 4096 513}; do AB_S=$S AB_DTYPE=bf16 timeout -k 10 200 python tools/phase_ab.py 2>/dev/null | sed "s/^{/{\"S\": $S, /" || exit $?; done
