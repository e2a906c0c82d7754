# Ballot-based P1/P2 partition level: GPU suite, phase timings (fix512 at S=16384/4096 bf16,
# snapkv bf16, fp32 fix512), level-0 stamps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/p12
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for s in 16384 4096; do
  AB_DTYPE=bf16 AB_S=$s timeout -k 10 180 python3 tools/phase_ab.py > $O/fix_s$s.json 2>$O/err || exit 1
  echo "fix512 bf16 S=$s: $(cat $O/fix_s$s.json)"
done
AB_DTYPE=bf16 AB_METHOD=snapkv_lite AB_KW='{"keep_size": 512}' timeout -k 10 180 python3 tools/phase_ab.py > $O/snap.json 2>$O/err || exit 1
echo "snapkv bf16: $(cat $O/snap.json)"
AB_DTYPE=fp32 timeout -k 10 180 python3 tools/phase_ab.py > $O/fp32.json 2>$O/err || exit 1
echo "fix512 fp32: $(cat $O/fp32.json)"
SEL_P1_STAMPS=1 timeout -k 10 200 python3 tools/select_stamps.py > $O/stamps.json 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
cat $O/stamps.json
