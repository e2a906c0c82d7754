# A/B of library builds on one box: GPU suite on the default build (libkvc.so), then per-phase
# kernel times (tools/phase_ab.py) of every build named in AB_LIBS (separate processes), for
# fix_size_l2(512) bf16 at S=16384 / 4096 and snapkv_lite(512) bf16 at S=16384.
#   AB_LIBS="libkvc_base.so libkvc.so" bash tools/gpu_ab.sh [notest]
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/ab
mkdir -p $O
if [ "$1" != "notest" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
LIBDIR=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
: > $O/ab.jsonl
for rep in 1 2; do
  for lib in ${AB_LIBS:-libkvc_base.so libkvc.so}; do
    for s in 16384 4096; do
      KVC_LIB=$LIBDIR/$lib AB_DTYPE=bf16 AB_S=$s timeout -k 10 180 python3 tools/phase_ab.py \
          > $O/one.json 2>$O/err || { tail $O/err; exit 1; }
      echo "{\"rep\": $rep, \"case\": \"fix512 bf16 S=$s\", \"r\": $(cat $O/one.json)}" >> $O/ab.jsonl
    done
    KVC_LIB=$LIBDIR/$lib AB_DTYPE=bf16 AB_METHOD=snapkv_lite AB_KW='{"keep_size": 512}' \
        timeout -k 10 180 python3 tools/phase_ab.py > $O/one.json 2>$O/err || { tail $O/err; exit 1; }
    echo "{\"rep\": $rep, \"case\": \"snapkv512 bf16 S=16384\", \"r\": $(cat $O/one.json)}" >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
