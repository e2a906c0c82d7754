#!/bin/bash
# Build the current csrc/kvc.hip as an A/B variant library kvcompress/_lib/libkvc_<NAME>.so (same
# flags as __graft_entry__.build_engine; extra hipcc flags after the name), for tools/gpu.sh ab.
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt -I "$R/include" "$@" \
    "$R/cs3602-llm-inference-acceleration_amd/csrc/kvc.hip" \
    -o "$R/cs3602-llm-inference-acceleration_amd/kvcompress/_lib/libkvc_$name.so" 2>&1 | grep -v "warning\|note:\|^ *[0-9]* |\|^ *|" || true
ls -la "$R/cs3602-llm-inference-acceleration_amd/kvcompress/_lib/libkvc_$name.so"
