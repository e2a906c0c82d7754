set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
L=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
: > gpurun_out/exp3.jsonl
for lib in $LIBS; do
  for w in l2-s16384 fix512-s4096-d80; do
    KVC_LIB=$L/$lib timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib':'$lib','w':'$w','ms':d['ms_per_step'],'k':d['kernel_ms_per_step']}))" >> gpurun_out/exp3.jsonl || exit $?
  done
  KVC_LIB=$L/$lib HOST_PROFILE_CALLS=100 timeout -k 10 200 python tools/host_profile.py 2>/dev/null | head -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({'lib':'$lib','w':'decode513','events_ms':d['ms_per_call_events'],'issue_ms':d['ms_per_call_issue_only']}))" >> gpurun_out/exp3.jsonl || exit $?
done
cat gpurun_out/exp3.jsonl
AB_S_LIST="16384 4096" bash tools/sg_ab.sh $LIBS
