"""The C ABI from a plain C caller (tests/native/abi_smoke.c: include/kvc.h + libkvc.so + the HIP
runtime API, no Python or torch in the process): host-side kvc_plan checks on CPU, and on the GPU
one fix_size_l2 layer through kvc_plan + kvc_launch compared bit-exactly with the oracle."""
import os
import subprocess

import numpy as np
import pytest

import prng
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "_build", "abi_smoke")


def _exe():
    if not os.path.exists(EXE):
        import sys
        sys.path.insert(0, ROOT)
        import __graft_entry__
        __graft_entry__.build_abi_smoke()
    return EXE


def test_c_caller_plan_checks():
    r = subprocess.run([_exe(), "plan"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "abi_smoke plan: ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["sort", "stable"])
@pytest.mark.parametrize("desc", [0, 1])
def test_c_caller_fix_size_l2_matches_oracle(tmp_path, desc, algo, monkeypatch):
    H, S, D, K = 4, 1000, 128, 100
    k = prng.gen_keys(321 + desc, (1, H, S, D), "bf16", "few")
    v = prng.gen_values(321 + desc, (1, H, S, D), "bf16")
    k.tofile(tmp_path / "k.bin")
    v.tofile(tmp_path / "v.bin")
    if algo == "stable":  # KVC_ALGO_STABLE = 2; the oracle under the same policy
        monkeypatch.setattr(oracle, "TIE", "stable")
    r = subprocess.run([_exe(), "run", str(tmp_path), str(H), str(S), str(D), str(K), str(desc),
                        "2" if algo == "stable" else "0"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ko = np.fromfile(tmp_path / "k_out.bin", dtype=np.uint16).reshape(1, H, K, D)
    vo = np.fromfile(tmp_path / "v_out.bin", dtype=np.uint16).reshape(1, H, K, D)
    strategy = "keep_high" if desc else "keep_low"
    rk, rv, _ = oracle.fix_size_l2_compress([(k, v)], fix_kv_size=K, keep_ratio=0.0,
                                            strategy=strategy, skip_layers=[])[0]
    assert np.array_equal(ko, rk.view(np.uint16)) and np.array_equal(vo, rv.view(np.uint16))


def test_div5_matches_ieee_division():
    """The snapkv pooling's x / 5 (csrc/kvc.hip div5_rn) equals IEEE x / 5.0f: every 61st of the
    2^32 fp32 patterns here (all of them: `div5_check 1`, ~1 min)."""
    src = os.path.join(ROOT, "tests", "native", "div5_check.c")
    exe = os.path.join(ROOT, "tests", "native", "_build", "div5_check")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", src, "-o", exe, "-lm"])
    r = subprocess.run([exe, "61"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and " 0 mismatches" in r.stdout, r.stdout


@pytest.mark.gpu
def test_hw_fp16_converts_match_c10():
    """The hardware fp16 converts of the snapkv scoring (kvc_common.h f16_to_f32_hw /
    f32_to_f16_hw) against the c10-exact conversions for all 2^16 and all 2^32 inputs
    (tests/native/cvt16_check.hip, built by __graft_entry__.build())."""
    exe = os.path.join(ROOT, "tests", "native", "_build", "cvt16_check")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "\n0 mismatches" in "\n" + r.stdout.splitlines()[-1], r.stdout
