# l2_compress kr=0.8 (cfg1's method, [1,32,16384,80]): fused SELECT_GATHER vs SELECT + GATHER.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/l2c
mkdir -p $O
for d in 80 128; do
  AB_DTYPE=bf16 AB_D=$d AB_METHOD=l2_compress AB_KW='{"keep_ratio": 0.8, "prune_after": 100}' \
    timeout -k 10 180 python3 tools/phase_ab.py > $O/l2_d$d.json 2>$O/l2_d$d.err || { tail $O/l2_d$d.err; exit 1; }
  echo "l2 kr0.8 D=$d: $(cat $O/l2_d$d.json)"
done
for s in 4096 1024; do
  AB_DTYPE=bf16 AB_S=$s AB_D=128 timeout -k 10 180 python3 tools/phase_ab.py > $O/fix_s$s.json 2>$O/fix_s$s.err || exit 1
  echo "fix512 S=$s: $(cat $O/fix_s$s.json)"
done
