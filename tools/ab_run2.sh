set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_run.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/h2oprof -o run -- python3 $GRAFT_REPO_ROOT/tools/h2o_long_profile.py > $GRAFT_REPO_ROOT/gpurun_out/h2oprof.log 2>&1 || exit 1
cat $GRAFT_REPO_ROOT/gpurun_out/h2oprof.log | tail -2
cat $GRAFT_REPO_ROOT/gpurun_out/h2oprof/run_kernel_stats.csv | cut -d, -f1-8 | head -12
