#!/bin/bash
# One GPU call: the full GPU suite on the product library, then an A/B of variant libraries
# ($AB_LIBS, default base vs current) on $AB_WORKLOADS.  Used during development.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu.sh test || exit 1
AB_LIBS="${AB_LIBS:-libkvc_base.so libkvc_p2.so libkvc_p2p4.so}" \
  AB_WORKLOADS="${AB_WORKLOADS:-fix512-s16384 snapkv-s16384 fix512-s4096-d80 h2o-s16384}" bash tools/gpu.sh ab
