#!/bin/bash
# dev run: the GPU test suite on the product library, then an A/B of the score kernel's tiles
# per wave (libkvc_tpw2/4: grids of 1/2, 1/4 the workgroups striding over the tiles)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.txt &&
AB_LIBS="libkvc.so libkvc_tpw2.so libkvc_tpw4.so" AB_WORKLOADS="fix512-s16384 snapkv-s16384" bash tools/gpu.sh ab
