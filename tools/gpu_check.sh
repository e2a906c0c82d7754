#!/bin/bash
# One GPU-box pass: parity tests, headline bench, rocprofv3 kernel stats.  Every GPU step has
# its own time limit and the steps are chained so the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R="${GRAFT_REPO_ROOT:-/root/repo}"
MODE="${1:-all}"
if [ "$MODE" = "all" ] || [ "$MODE" = "test" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout=300 -p no:cacheprovider \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && [ "$MODE" = "test" ] && exit $rc
  [ $rc -gt 1 ] && exit $rc
fi
if [ "$MODE" = "all" ] || [ "$MODE" = "bench" ]; then
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
  cat gpurun_out/bench.json
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
      -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1 || exit $?
  find "$R/gpurun_out/prof" -name "*stats*" | head
fi
if [ "$MODE" = "stamps" ]; then
  : > gpurun_out/stamps.json
  for ws in 1; do
    timeout -k 10 300 python tools/select_stamps.py >> gpurun_out/stamps.json 2>> gpurun_out/stamps.err || exit $?
  done
  cat gpurun_out/stamps.json
fi
if [ "$MODE" = "sqpmc" ]; then  # SQ counters of one kernel (regex $2) on the split path
  cd /tmp && export TMPDIR=/tmp
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "${2:-select}" --output-format csv \
        -d "$R/gpurun_out/sqpmc$i" -o run -- python3 "$R/tools/microbench.py" split 1 \
        > "$R/gpurun_out/sqpmc$i.log" 2>&1 || exit $?
  done
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/sqpmc1" "$R/gpurun_out/sqpmc2"
fi
if [ "$MODE" = "pmc" ]; then
  cd /tmp && export TMPDIR=/tmp
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/pmc_$ctr" -o run \
        -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmc_$ctr.log" 2>&1 || exit $?
  done
  find "$R/gpurun_out" -name "*counter_collection*" | head
fi
if [ "$MODE" = "workloads" ]; then  # every bench.py workload at N=1 (and strong-scaled cfg4 shape)
  : > gpurun_out/workloads.jsonl
  for w in ${2:-fix512-s16384 fix512-s4096 fix512-s4096-d80 streaming-s16384 h2o-s16384 snapkv-s16384 pyramid-s16384 l2-s16384 adaptive-s16384}; do
    timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 5 ${3:---no-cpu-baseline} \
        >> gpurun_out/workloads.jsonl 2>> gpurun_out/workloads.err || exit $?
  done
  cat gpurun_out/workloads.jsonl
fi
