#!/bin/bash
# PMC traffic (FETCH_SIZE / WRITE_SIZE, one pass each) of the engine kernels on the cfg2
# pythia-2.8b workload (fix512-s4096-d80: 160-byte token rows) -> gpurun_out/d80/pmc_traffic.json
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out/d80"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_$ctr" -o run \
      -- python3 "$R/bench.py" --workload fix512-s4096-d80 --steps 2 --warmup 1 --no-cpu-baseline \
      > "$O/pmc_$ctr.log" 2>&1 || exit $?
done
PMC_S=4096 PMC_D=80 python3 "$R/tools/pmc_traffic.py" "$O" "$O/pmc_traffic.json"
