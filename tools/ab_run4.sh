#!/bin/bash
# dev run: snapkv key-phase stamps and the fp32 fast-path split (diagnostic -DKVC_STAMPS
# -DKVC_SNAP_STAMPS build); parity of the fp32 radix variant; A/B of the fp32 fast path (old
# product / inlined / inlined + radix) and of the score kernel's tiles per wave
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
SEL_SNAP_STAMPS=1 SEL_SCORE=1 SEL_ALGO=1 SEL_ORDER=1 SEL_K=480 SEL_S=16352 timeout -k 10 120 python tools/select_stamps.py &&
SEL_DTYPE=fp32 timeout -k 10 120 python tools/select_stamps.py &&
KVC_LIB=$PWD/$L/libkvc_rdx.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log &&
AB_ARGS="--dtype fp32" AB_LIBS="libkvc.so libkvc_inl.so libkvc_rdx.so" AB_WORKLOADS="fix512-s16384" bash tools/gpu.sh ab &&
AB_LIBS="libkvc.so libkvc_tpw2.so libkvc_tpw4.so" AB_WORKLOADS="fix512-s16384" bash tools/gpu.sh ab
