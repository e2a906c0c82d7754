set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
for v in ${PAR_LIBS:-}; do
  KVC_LIB=$L/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/par_$v.log 2>&1 || { tail -30 gpurun_out/par_$v.log; exit 1; }
  tail -1 gpurun_out/par_$v.log
done
AB_S_LIST="${AB_S_LIST:-16384 8192}" bash tools/sg_ab.sh ${AB_LIBS}
[ -n "${PMC_LIBS:-}" ] && bash tools/sel_pmc.sh ${PMC_LIBS} > gpurun_out/sel_pmc.json 2>&1
cat gpurun_out/sel_pmc.json 2>/dev/null | head -80
