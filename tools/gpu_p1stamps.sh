# Level-0 P1 sub-phase stamps (diagnostic build) + the box's instruction-fetch counters list.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
SEL_P1_STAMPS=1 timeout -k 10 200 python3 tools/select_stamps.py > gpurun_out/p1stamps.json 2> gpurun_out/p1stamps.err || { tail gpurun_out/p1stamps.err; exit 1; }
cat gpurun_out/p1stamps.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/counters_all.txt" 2>&1 || exit 1
grep -i -E "icache|ifetch|SQC_|INST_LEVEL" "$R/gpurun_out/counters_all.txt" | cut -c1-150 | head -60 || true
