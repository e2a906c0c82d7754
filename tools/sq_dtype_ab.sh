set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for dt in bf16 fp16; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM"; do
    i=$((i+1))
    SEL_DTYPE=$dt timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex "select_kernel" --output-format csv \
        -d "$R/gpurun_out/sq_${dt}_$i" -o run -- python3 "$R/tools/select_only.py" > "$R/gpurun_out/sq_${dt}_$i.log" 2>&1 || exit $?
  done
  echo "== $dt"; grep "select ms" "$R/gpurun_out/sq_${dt}_1.log"
  python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/sq_${dt}_1" "$R/gpurun_out/sq_${dt}_2"
done
