#!/bin/bash
# SQ counters of the SELECT kernel (tools/select_only.py) for each library named on the command
# line (files under kvcompress/_lib/); one rocprofv3 --pmc pass per counter set.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
for lib in "$@"; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
    i=$((i+1))
    KVC_LIB="$R/cs3602-llm-inference-acceleration_amd/kvcompress/_lib/$lib" timeout -k 10 120 \
      rocprofv3 --pmc $set --kernel-include-regex "select_kernel" --output-format csv \
        -d "$R/gpurun_out/selpmc_${lib}_$i" -o run -- python3 "$R/tools/select_only.py" \
        > "$R/gpurun_out/selpmc_${lib}_$i.log" 2>&1 || exit $?
  done
  echo "== $lib"
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/selpmc_${lib}_1" "$R/gpurun_out/selpmc_${lib}_2"
done
