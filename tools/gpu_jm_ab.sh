# A/B of the partition-level instantiation set (instruction footprint): libkvc (JM 1/2/4/8/16),
# libkvc_jm2 (JM 4/16), libkvc_jm1 (JM 16 only); fix512 at S=16384 and S=4096, bf16.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/jm
mkdir -p $O
L=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
for rep in 1 2; do
for lib in libkvc.so libkvc_jm2.so libkvc_jm1.so; do
  for s in 16384 4096; do
    KVC_LIB=$R/$L/$lib AB_DTYPE=bf16 AB_S=$s timeout -k 10 180 python3 tools/phase_ab.py > $O/${lib}_s$s.json 2>$O/err || { tail $O/err; exit 1; }
    echo "$rep $lib S=$s: $(cat $O/${lib}_s$s.json)"
  done
done
done
