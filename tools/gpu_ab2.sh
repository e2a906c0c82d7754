# A/B of library builds (AB_LIBS, files under kvcompress/_lib) on methods whose outputs carry
# sink / tail positions besides the selected ones, plus the headline; GPU suite first.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/ab2
mkdir -p $O
if [ "$1" != "notest" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
LIBDIR=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
: > $O/ab.jsonl
run() {  # name method kw D [S]
  KVC_LIB=$LIBDIR/$lib AB_DTYPE=bf16 AB_S=${5:-16384} AB_METHOD=$2 AB_KW="$3" AB_D=$4 \
      timeout -k 10 180 python3 tools/phase_ab.py > $O/one.json 2>$O/err || { tail $O/err; exit 1; }
  echo "{\"rep\": $rep, \"case\": \"$1\", \"r\": $(cat $O/one.json)}" >> $O/ab.jsonl
}
for rep in 1 2; do
  for lib in ${AB_LIBS:-libkvc_base.so libkvc.so}; do
    run fix512 fix_size_l2 '{"fix_kv_size": 512}' 128 || exit 1
    run h2o_d80 h2o_l2 '{}' 80 || exit 1
    run pyramid pyramid_kv '{}' 128 || exit 1
    run snapkv512 snapkv_lite '{"keep_size": 512}' 128 || exit 1
    run fix512_kr05 fix_size_l2 '{"fix_kv_size": 512, "keep_ratio": 0.5}' 128 || exit 1
    run fix512_s4096 fix_size_l2 '{"fix_kv_size": 512}' 128 4096 || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab2/ab.jsonl"):
    x = json.loads(l)
    d[(x["case"], x["r"]["lib"])].append(x["r"]["two"]["select+gather"])
for k, v in sorted(d.items()):
    print(k, v)
PY
