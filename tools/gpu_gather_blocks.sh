# Gather workgroup size A/B (KVC_GATHER_BLOCKS builds) on copy-bound calls, plus the box's copy
# ceiling: l2_compress kr=0.8 D=80/128 (three-kernel path: GATHER alone) and fix512 headline.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/gb
mkdir -p $O
L=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
timeout -k 10 120 python3 tools/copy_ceiling.py > $O/ceiling.json 2>$O/ceiling.err || { tail $O/ceiling.err; exit 1; }
echo "ceiling: $(cat $O/ceiling.json)"
for lib in libkvc.so libkvc_g4.so libkvc_g16.so; do
  for d in 80 128; do
    KVC_LIB=$R/$L/$lib AB_DTYPE=bf16 AB_D=$d AB_METHOD=l2_compress AB_KW='{"keep_ratio": 0.8, "prune_after": 100}' \
      timeout -k 10 180 python3 tools/phase_ab.py > $O/l2_${lib}_d$d.json 2>$O/err || { tail $O/err; exit 1; }
    echo "l2 D=$d: $(cat $O/l2_${lib}_d$d.json)"
  done
  KVC_LIB=$R/$L/$lib AB_DTYPE=bf16 timeout -k 10 180 python3 tools/phase_ab.py > $O/fix_${lib}.json 2>$O/err || exit 1
  echo "fix512: $(cat $O/fix_${lib}.json)"
done
