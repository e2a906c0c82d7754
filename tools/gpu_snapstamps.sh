# snapkv scoring phases and the plain key load (diagnostic stamps build), headline rows.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
SEL_SCORE=1 SEL_SNAP_STAMPS=1 timeout -k 10 200 python3 tools/select_stamps.py > gpurun_out/snapstamps.json 2> gpurun_out/snapstamps.err || { tail gpurun_out/snapstamps.err; exit 1; }
timeout -k 10 200 python3 tools/select_stamps.py > gpurun_out/plainstamps.json 2>> gpurun_out/snapstamps.err || { tail gpurun_out/snapstamps.err; exit 1; }
cat gpurun_out/snapstamps.json gpurun_out/plainstamps.json
