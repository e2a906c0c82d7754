# A/B of library builds on the per-token decode step (tools/decode_bench.py), after the GPU suite
# on the default build.   AB_LIBS="libkvc_base.so libkvc.so" bash tools/gpu_decode_ab.sh [notest]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/dab
mkdir -p $O
if [ "$1" != "notest" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
LIBDIR=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
: > $O/dab.jsonl
for rep in 1 2; do
  for lib in ${AB_LIBS:-libkvc_base.so libkvc.so}; do
    KVC_LIB=$LIBDIR/$lib timeout -k 10 240 python3 tools/decode_bench.py > $O/one.json 2>$O/err \
        || { tail $O/err; exit 1; }
    echo "{\"rep\": $rep, \"lib\": \"$lib\", \"r\": $(cat $O/one.json)}" >> $O/dab.jsonl
  done
done
cat $O/dab.jsonl
