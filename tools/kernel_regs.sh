#!/bin/bash
# VGPR / SGPR / scratch / LDS of every kernel in a built libkvc*.so (CPU; ROCm LLVM tools).
# usage: bash tools/kernel_regs.sh path/to/lib.so [grep-pattern]
set -e
LIB=$(readlink -f "$1"); PAT="${2:-.}"
T=$(mktemp -d); cd "$T"; cp "$LIB" lib.so
/opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so >/dev/null
CO=$(ls | grep gfx950 | head -1)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$CO" | awk '
  /^    \.name:/ {n=$2} /^    \.vgpr_count:/ {v=$2} /^    \.sgpr_count:/ {s=$2}
  /^    \.private_segment_fixed_size:/ {p=$2} /^    \.group_segment_fixed_size:/ {g=$2}
  /^    \.vgpr_spill_count:/ {sp=$2; print "vgpr=" v, "sgpr=" s, "scratch=" p, "lds=" g, "spill=" sp, n}' \
  | grep -E "$PAT" | c++filt | sed 's/(kvc::LayerChunk.*//' 
rm -rf "$T"
