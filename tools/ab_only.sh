#!/bin/bash
# dev run: an A/B of variant libraries only ($AB_LIBS on $AB_WORKLOADS), plus pytest of the
# parity files with the last variant ($AB_TEST=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
if [ -n "$AB_TEST" ]; then
  last=${AB_LIBS##* }
  KVC_LIB=$PWD/$L/$last timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
bash tools/gpu.sh ab
