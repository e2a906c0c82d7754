"""Register / scratch budgets of the built engine kernels (CPU: reads the gfx950 code object's
AMDGPU metadata out of libkvc.so with the ROCm LLVM tools; no GPU).

The 16-bit-key select kernels run two 1 024-thread rows per CU (and four 512-thread rows), i.e.
8 waves per SIMD, which leaves each wave 512 / 8 = 64 VGPRs: one more and the CU holds one row,
which measured the headline SELECT_GATHER 0.147 -> 0.208 ms (the
heap prefilter that now lives only in the heavy-hitter instance).  The hot kernels also must not
spill to scratch."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd", "kvcompress", "_lib", "libkvc.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(tmp_path):
    objdump, readelf = os.path.join(LLVM, "llvm-objdump"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(LIB) and os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("libkvc.so or the ROCm LLVM tools are missing")
    lib = tmp_path / "libkvc.so"
    shutil.copy(LIB, lib)
    subprocess.run([objdump, "--offloading", str(lib)], cwd=tmp_path, check=True,
                   capture_output=True, timeout=120)
    (co,) = [p for p in tmp_path.iterdir() if p.name.endswith("gfx950")]
    notes = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True,
                           text=True, timeout=120).stdout
    out, cur = {}, None
    for line in notes.splitlines():  # kernel-level keys sit at four spaces of indentation
        m = re.match(r"^    \.(name|vgpr_count|private_segment_fixed_size|vgpr_spill_count):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1) == "name":
            cur = m.group(2)
            out[cur] = {}
        elif cur:
            out[cur][m.group(1)] = int(m.group(2))
    return out


def test_select_kernels_fit_two_rows_per_cu(tmp_path):
    ks = _kernels(tmp_path)
    # KC = 1: 16-bit keys (bf16 / fp16 rows); select_kernel<1, NT, false> and every
    # select_gather_kernel<1, NT, NC>
    hot = {n: v for n, v in ks.items()
           if re.match(r"_ZN3kvc(13select_kernelILi1ELi(512|1024)ELb0E|20select_gather_kernelILi1E)", n)}
    assert len(hot) >= 9, sorted(ks)
    for n, v in hot.items():
        assert v["vgpr_count"] <= 64, (n, v)
        assert v["private_segment_fixed_size"] == 0 and v.get("vgpr_spill_count", 0) == 0, (n, v)


def test_stream_kernels_do_not_spill(tmp_path):
    """score / gather kernels for rows of up to 512 bytes (NC <= 32 chunks of 16 B: every
    BASELINE geometry; the NC = 64 score kernels -- fp32 D = 256, 16-bit D = 512 -- hold a
    whole 1 KiB row per lane group and do spill)."""
    ks = _kernels(tmp_path)
    hot = {n: v for n, v in ks.items()
           if re.match(r"_ZN3kvc(12score_kernel|13gather_kernel)ILi\dELi(4|8|10|16|20|32)E", n)}
    assert hot, sorted(ks)
    for n, v in hot.items():
        assert v["private_segment_fixed_size"] == 0 and v.get("vgpr_spill_count", 0) == 0, (n, v)
