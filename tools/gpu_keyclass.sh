# One GPU call: the fp16 convert check, the GPU suite, and bf16-vs-fp16 selection timings of the
# shared key-class select binary (fix_size_l2 and snapkv_lite rows).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/kc
mkdir -p $O
timeout -k 10 120 tests/native/_build/cvt16_check > $O/cvt16.log 2>&1 || { cat $O/cvt16.log; exit 1; }
cat $O/cvt16.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for dt in bf16 fp16; do
  SEL_DTYPE=$dt SEL_REPS=20 timeout -k 10 120 python3 tools/select_only.py > $O/sel_$dt.log 2>&1 || exit 1
  echo "select-only $dt: $(tail -1 $O/sel_$dt.log)"
  AB_DTYPE=$dt timeout -k 10 180 python3 tools/phase_ab.py > $O/ab_$dt.json 2>$O/ab_$dt.err || exit 1
  echo "fix_size_l2 $dt: $(cat $O/ab_$dt.json)"
  AB_DTYPE=$dt AB_METHOD=snapkv_lite AB_KW='{"keep_size": 512}' \
    timeout -k 10 180 python3 tools/phase_ab.py > $O/abs_$dt.json 2>$O/abs_$dt.err || exit 1
  echo "snapkv_lite $dt: $(cat $O/abs_$dt.json)"
done
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
