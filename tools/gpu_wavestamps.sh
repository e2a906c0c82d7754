# Level-0 per-wave timing (diagnostic stamps build), two repetitions.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
for i in 1 2; do
  SEL_P1_STAMPS=1 timeout -k 10 200 python3 tools/select_stamps.py > gpurun_out/wavestamps$i.json 2> gpurun_out/wavestamps.err || { tail gpurun_out/wavestamps.err; exit 1; }
  tail -1 gpurun_out/wavestamps$i.json
done
