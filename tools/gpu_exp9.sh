set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=cs3602-llm-inference-acceleration_amd/kvcompress/_lib
for lib in $LIBS; do
  KVC_LIB=$L/$lib AB_METHOD=snapkv_lite AB_KW="{}" AB_DTYPE=bf16 timeout -k 10 200 python tools/phase_ab.py 2>/dev/null || exit $?
  KVC_LIB=$L/$lib AB_DTYPE=bf16 timeout -k 10 200 python tools/phase_ab.py 2>/dev/null || exit $?
  KVC_LIB=$L/$lib AB_S=4096 AB_DTYPE=bf16 timeout -k 10 200 python tools/phase_ab.py 2>/dev/null | sed 's/^{/{"S": 4096, /' || exit $?
done
