# Headline bench in fp16 and fp32 K/V (no CPU / PPL legs), final tree.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
: > gpurun_out/dtypes.jsonl
for dt in fp16 fp32; do
  timeout -k 10 200 python bench.py --dtype $dt --steps 20 --warmup 5 --no-cpu-baseline >> gpurun_out/dtypes.jsonl 2>> gpurun_out/dtypes.err || exit $?
done
cat gpurun_out/dtypes.jsonl
