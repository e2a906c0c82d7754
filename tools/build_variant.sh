#!/bin/bash
# Experimental engine build for A/B runs (tools/gpu.sh ab): build_variant.sh NAME [-DDEFS...]
# -> kvcompress/_lib/libkvc_NAME.so.  Variants are scratch: delete them before committing.
cd "$(dirname "$0")/.." && name="$1" && shift && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 \
  -std=c++17 -fPIC -shared -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt "$@" \
  -I include cs3602-llm-inference-acceleration_amd/csrc/kvc.hip \
  -o "cs3602-llm-inference-acceleration_amd/kvcompress/_lib/libkvc_$name.so" 2>&1 | grep -v "occupancy\|warnings generated\|^ \|^$" || true
