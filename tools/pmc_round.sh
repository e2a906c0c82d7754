#!/bin/bash
# PMC evidence for the current library (GPU box): FETCH_SIZE / WRITE_SIZE of every engine kernel
# on the headline bench (one pass per counter), and SQ issue / wait counters of the SELECT and
# SELECT_GATHER kernels (two passes each, <= 8 SQ counters per pass).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_$ctr" -o run \
      -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_$ctr.log" 2>&1 || exit $?
done
python3 "$R/tools/pmc_traffic.py" "$R/gpurun_out" "$R/gpurun_out/pmc_traffic.json" > /dev/null || exit $?
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "select" --output-format csv \
      -d "$R/gpurun_out/sqsel_$i" -o run -- python3 "$R/tools/select_only.py" \
      > "$R/gpurun_out/sqsel_$i.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "select_gather" --output-format csv \
      -d "$R/gpurun_out/sqsg_$i" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline \
      > "$R/gpurun_out/sqsg_$i.log" 2>&1 || exit $?
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/sqsel_1" "$R/gpurun_out/sqsel_2" "$R/gpurun_out/sqsg_1" "$R/gpurun_out/sqsg_2" > "$R/gpurun_out/sq_summary.json" || exit $?
cat "$R/gpurun_out/pmc_traffic.json" "$R/gpurun_out/sq_summary.json"
