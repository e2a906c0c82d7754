#!/bin/bash
# dev run: heap probe (wave scan vs the block candidate prefilter), the full GPU suite, the long
# h2o_attention call profile and the decode steps (tools/ab_run3.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 tools/heap_probe > gpurun_out/heap_probe.jsonl 2>&1 || { cat gpurun_out/heap_probe.jsonl; exit 1; }
cat gpurun_out/heap_probe.jsonl
bash tools/ab_run3.sh
