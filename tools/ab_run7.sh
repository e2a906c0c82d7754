#!/bin/bash
# dev run: heap probe, the full GPU suite, the long h2o_attention call profile and decode steps
# (tools/ab_run6.sh), then the headline / h2o / snapkv bench lines of the product library
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/ab_run6.sh && AB_LIBS="libkvc.so" AB_REPS=1 AB_WORKLOADS="fix512-s16384 h2o-s16384 snapkv-s16384 pyramid-s16384" bash tools/gpu.sh ab
