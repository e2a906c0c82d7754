#!/bin/bash
# KVC_STAMP_DEFS=-DKVC_SNAP_STAMPS: snapkv scoring stamps in slots 26..29 instead of the level-0 ones.
# Diagnostic build of the engine with s_memtime stamps in the select kernel (tools/select_stamps.py).
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared \
  -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -DKVC_STAMPS ${KVC_STAMP_DEFS} -I include \
  cs3602-llm-inference-acceleration_amd/csrc/kvc.hip \
  -o cs3602-llm-inference-acceleration_amd/kvcompress/_lib/libkvc_stamps.so
