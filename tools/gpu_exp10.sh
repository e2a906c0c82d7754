set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
SEL_SNAP_STAMPS=1 SEL_ALGO=1 SEL_ORDER=1 SEL_SCORE=1 SEL_K=480 timeout -k 10 200 python tools/select_stamps.py | tail -1 || exit $?
AB_METHOD=snapkv_lite AB_KW="{}" AB_DTYPE=bf16 timeout -k 10 200 python tools/phase_ab.py || exit $?
AB_METHOD=snapkv_lite AB_KW="{}" AB_DTYPE=fp16 timeout -k 10 200 python tools/phase_ab.py || exit $?
