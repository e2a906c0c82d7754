#!/bin/bash
# Build an A/B variant library kvcompress/_lib/libkvc_<NAME>.so with the product's hipcc flags
# (as __graft_entry__.build_engine).  Usage:
#   bash tools/build_variant.sh NAME                 the variant NAME of tools/ab_variants.txt
#   bash tools/build_variant.sh NAME -DFOO ...       ad hoc: the working tree plus extra flags
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; shift
extra=("$@")
src="$R/cs3602-llm-inference-acceleration_amd/csrc/kvc.hip"
inc="$R/include"
if [ ${#extra[@]} -eq 0 ]; then
  line=$(grep -E "^$name[[:space:]]" "$R/tools/ab_variants.txt" || true)
  [ -n "$line" ] || { echo "variant $name not in tools/ab_variants.txt" >&2; exit 2; }
  read -r -a f <<< "$line"
  extra=("${f[@]:1}")
fi
if [[ "${extra[0]}" == rev=* ]]; then
  rev="${extra[0]#rev=}"
  extra=("${extra[@]:1}")
  tmp=$(mktemp -d)
  trap 'rm -rf "$tmp"' EXIT
  git -C "$R" archive "$rev" cs3602-llm-inference-acceleration_amd/csrc include | tar -x -C "$tmp"
  src="$tmp/cs3602-llm-inference-acceleration_amd/csrc/kvc.hip"
  inc="$tmp/include"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt -I "$inc" "${extra[@]}" "$src" \
    -o "$R/cs3602-llm-inference-acceleration_amd/kvcompress/_lib/libkvc_$name.so" 2>&1 \
    | grep -v "warning\|note:\|^ *[0-9]* |\|^ *|" || true
ls -la "$R/cs3602-llm-inference-acceleration_amd/kvcompress/_lib/libkvc_$name.so"
