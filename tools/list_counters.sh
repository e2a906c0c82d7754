# List the PMC counters of the box's GPU that concern instruction fetch / the instruction cache.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/counters_all.txt" 2>&1 || exit 1
grep -i -E "icache|ifetch|inst_level|SQC_" "$R/gpurun_out/counters_all.txt" | head -80 || true
