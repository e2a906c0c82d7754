#!/bin/bash
# A/B of select_gather builds (tuning aid, GPU box): every library named on the command line
# (files under kvcompress/_lib/) is timed by tools/phase_ab.py in its own process at each
# AB_S_LIST length (bf16, 32 layers x 32 heads, fix_size_l2(512)).  One JSON line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIBDIR=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
out=gpurun_out/sg_ab.jsonl
: > $out
for S in ${AB_S_LIST:-16384 4096}; do
  for lib in "$@"; do
    AB_S=$S AB_DTYPE=${AB_DTYPE:-bf16} KVC_LIB=$LIBDIR/$lib timeout -k 10 240 python tools/phase_ab.py \
        | sed "s/^{/{\"S\": $S, /" >> $out || exit $?
  done
done
cat $out
