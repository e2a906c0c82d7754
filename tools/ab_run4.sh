#!/bin/bash
# dev run: select-kernel phase stamps (diagnostic -DKVC_STAMPS build) on the headline, snapkv and
# S = 4096 rows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out
: > $O/stamps.jsonl
timeout -k 10 120 python tools/select_stamps.py >> $O/stamps.jsonl || exit 1
SEL_S=4096 timeout -k 10 120 python tools/select_stamps.py >> $O/stamps.jsonl || exit 1
SEL_SCORE=1 SEL_ALGO=1 SEL_ORDER=1 SEL_K=480 SEL_S=16352 timeout -k 10 120 python tools/select_stamps.py >> $O/stamps.jsonl || exit 1
cat $O/stamps.jsonl
