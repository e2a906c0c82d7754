set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for dt in bf16 fp32 fp16; do AB_S=4096 AB_DTYPE=$dt timeout -k 10 200 python tools/phase_ab.py 2>/dev/null | sed "s/^{/{\"S\": 4096, /" || exit $?; done
timeout -k 10 300 python tools/decode_bench.py 2>/dev/null > gpurun_out/decode.json || exit $?
cat gpurun_out/decode.json
HOST_PROFILE_CALLS=200 timeout -k 10 200 python tools/host_profile.py 2>/dev/null | head -1
bash tools/gpu_check.sh workloads "fix512-s4096 fix512-s4096-d80 fix512-s16384" > /dev/null 2>&1
cat gpurun_out/workloads.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['config']['name'], round(d['ms_per_step'],4), d['kernel_ms_per_step'], round(d['path_roofline']['frac'],3))"
