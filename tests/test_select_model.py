"""CPU checks of the selection algorithm and numerics helpers the HIP select kernel is built from.

tests/native/select_model.cpp runs the kernel's partition-chain algorithm serially with the
kernel's own serial helpers (csrc/kvc_serial.h) and key mapping (csrc/kvc_common.h).  Compared
here against real libstdc++ (through the oracle): heavy ties, every boundary, the partial_sort
heap-select path and McIlroy-adversary inputs that force introsort's depth-limit heapsort."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "select_model.cpp")
OUT = os.path.join(ROOT, "tests", "native", "_build", "libselect_model.so")


@pytest.fixture(scope="module")
def model():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if not os.path.exists(OUT) or os.path.getmtime(OUT) < max(
            os.path.getmtime(SRC),
            os.path.getmtime(os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd/csrc/kvc_serial.h")),
            os.path.getmtime(os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd/csrc/kvc_common.h"))):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-I",
                               os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd", "csrc"),
                               SRC, "-o", OUT])
    L = ctypes.CDLL(OUT)
    L.model_select.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    for f in ("model_key_bf16", "model_key_f32", "model_canon_nan"):
        getattr(L, f).restype = ctypes.c_uint32
        getattr(L, f).argtypes = [ctypes.c_uint32, ctypes.c_int] if "key" in f else [ctypes.c_uint32]
    L.model_f32_to_bf16.restype = ctypes.c_uint32
    L.model_f32_to_bf16.argtypes = [ctypes.c_float]
    L.model_key_f16.restype = ctypes.c_uint32
    L.model_key_f16.argtypes = [ctypes.c_uint32, ctypes.c_int]
    L.model_f32_to_f16.restype = ctypes.c_uint32
    L.model_f32_to_f16.argtypes = [ctypes.c_float]
    L.model_f16_to_f32.restype = ctypes.c_float
    L.model_f16_to_f32.argtypes = [ctypes.c_uint32]
    L.model_canon_nan_f16.restype = ctypes.c_uint32
    L.model_canon_nan_f16.argtypes = [ctypes.c_uint32]
    return L


def run_model(L, keys_u32, k, topk):
    keys_u32 = np.ascontiguousarray(keys_u32, dtype=np.uint32)
    out = np.empty(max(k, 1), dtype=np.int32)
    path = ctypes.c_int(0)
    L.model_select(keys_u32.ctypes.data, len(keys_u32), k, topk, out.ctypes.data, ctypes.byref(path))
    return out[:k], path.value


def ref_set(keys_u32, k, topk):
    vals = keys_u32.astype(np.float32)[None, None, :]  # small ints: float order == int order
    if topk:  # the model works on ascending keys; topk(largest) on -key is the same set
        idx = oracle.topk_indices(-vals, k)
    else:
        idx = oracle.argsort_prefix(vals, k)
    return np.sort(idx[0, 0])


def test_model_matches_libstdcxx_heavy_ties(model):
    rng = np.random.default_rng(0)
    for trial in range(1500):
        n = int(rng.integers(2, 3000)) if trial % 10 else int(rng.integers(3000, 16385))
        keys = rng.integers(0, int(rng.choice([1, 2, 3, 7, 80, 1 << 20])), n).astype(np.uint32)
        k = int(rng.integers(1, n))
        for topk in (0, 1):
            got, _ = run_model(model, keys, k, topk)
            np.testing.assert_array_equal(got, ref_set(keys, k, topk), err_msg=f"n={n} k={k}")


def test_model_partial_sort_path(model):
    rng = np.random.default_rng(1)
    for trial in range(200):
        n = int(rng.integers(64, 20000))
        k = int(rng.integers(1, max(2, n // 64 + 1)))
        keys = rng.integers(0, 50, n).astype(np.uint32)
        got, path = run_model(model, keys, k, 1)
        assert path == 1
        np.testing.assert_array_equal(got, ref_set(keys, k, 1))


@pytest.mark.parametrize("n", [100, 1000, 4096, 16384])
def test_model_depth_limit_heap_fallback(model, n):
    adv = np.empty(n, dtype=np.int64)
    hit = 0
    for mode in (0, 1):
        for k in (1, n // 3, n // 2, n - 1):
            oracle.lib().orc_antiqsort(n, mode, k, adv.ctypes.data)
            keys = adv.astype(np.uint32)
            got, path = run_model(model, keys, k, mode)
            hit += path == 2
            np.testing.assert_array_equal(got, ref_set(keys, k, mode))
    assert hit > 0, "adversary never reached the depth-limit fallback"


def _torch_less(a, b, desc):
    na, nb = np.isnan(a), np.isnan(b)
    if desc:
        return (na & ~nb) | (a > b)
    return (~na & nb) | (a < b)


def test_sort_keys_induce_torch_comparator_order(model):
    allb = np.arange(65536, dtype=np.uint32)
    f = (allb << 16).view(np.float32)
    rng = np.random.default_rng(2)
    for desc in (0, 1):
        kb = np.array([model.model_key_bf16(int(b), desc) for b in allb], dtype=np.uint32)
        a, b = rng.integers(0, 65536, 200000), rng.integers(0, 65536, 200000)
        np.testing.assert_array_equal(kb[a] < kb[b], _torch_less(f[a], f[b], desc))
        np.testing.assert_array_equal(kb[a] == kb[b], ~_torch_less(f[a], f[b], desc) & ~_torch_less(f[b], f[a], desc))
        u = np.concatenate([rng.integers(0, 1 << 32, 4000, dtype=np.uint64).astype(np.uint32),
                            np.array([0, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00000, 0xFFC00001,
                                      0x7F800001, 1, 0x80000001], dtype=np.uint32)])
        kf = np.array([model.model_key_f32(int(x), desc) for x in u], dtype=np.uint64)
        ff = u.view(np.float32)
        i, j = np.meshgrid(np.arange(len(u)), np.arange(len(u)))
        i, j = i.ravel()[::37], j.ravel()[::37]
        np.testing.assert_array_equal(kf[i] < kf[j], _torch_less(ff[i], ff[j], desc))


def test_bf16_rounding_and_nan_canonicalisation(model):
    import prng
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 100,
                        np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-40, 3.3895314e38], np.float32)])
    ref = prng.f32_to_bf16_bits(x)
    got = np.array([model.model_f32_to_bf16(float(v)) for v in x], dtype=np.uint16)
    np.testing.assert_array_equal(got, ref)
    for w in (0x7FC00001, 0xFF817F80, 0x3F807F81, 0x12345678, 0xFFFF7FFF):
        lo, hi = w & 0xFFFF, w >> 16
        def c(h):
            return 0xFFFF if (h & 0x7FFF) > 0x7F80 else h
        assert model.model_canon_nan(w) == (c(lo) | (c(hi) << 16))



def test_fp16_keys_conversions_and_nan_quieting(model):
    """The kernel's fp16 helpers (csrc/kvc_common.h) vs numpy/IEEE: sort-key order equals torch's
    comparators on all 65536 patterns, f16 -> f32 exact, f32 -> f16 round-to-nearest-even at
    every fp16 midpoint (incl. subnormals and overflow), gather's NaN quieting (0x7C01 -> 0x7E01)."""
    allh = np.arange(65536, dtype=np.uint32)
    f = allh.astype(np.uint16).view(np.float16).astype(np.float32)
    got = np.array([model.model_f16_to_f32(int(h)) for h in allh], dtype=np.float32)
    same = (got.view(np.uint32) == f.view(np.uint32)) | (np.isnan(got) & np.isnan(f))
    assert same.all()
    rng = np.random.default_rng(4)
    for desc in (0, 1):
        kh = np.array([model.model_key_f16(int(b), desc) for b in allh], dtype=np.uint32)
        a, b = rng.integers(0, 65536, 200000), rng.integers(0, 65536, 200000)
        np.testing.assert_array_equal(kh[a] < kh[b], _torch_less(f[a], f[b], desc))
        np.testing.assert_array_equal(kh[a] == kh[b], ~_torch_less(f[a], f[b], desc) & ~_torch_less(f[b], f[a], desc))
    fin = allh[:0x7C00].astype(np.uint16).view(np.float16).astype(np.float64)
    mid = ((fin[:-1] + fin[1:]) / 2).astype(np.float32)  # exact midpoints (fp32 has the bits)
    x = np.concatenate([mid, -mid, np.nextafter(mid, np.float32(np.inf)), np.nextafter(mid, np.float32(0)),
                        rng.standard_normal(20000).astype(np.float32) * 1e-6,
                        np.array([np.inf, -np.inf, 0.0, -0.0, 65504, 65519.996, 65520, 1e9, 2.98e-8,
                                  2.9802322e-8, 1e-40], np.float32)])
    with np.errstate(over="ignore"):
        ref = x.astype(np.float16).view(np.uint16)
    out = np.array([model.model_f32_to_f16(float(v)) for v in x], dtype=np.uint16)
    np.testing.assert_array_equal(out, ref)
    assert model.model_f32_to_f16(float("nan")) == 0x7E00
    for w in (0x7C017C00, 0xFC01FE00, 0x7DFF3C00, 0x12345678, 0xFFFF7FFF):
        lo, hi = w & 0xFFFF, w >> 16

        def q(h):
            return h | 0x200 if (h & 0x7FFF) > 0x7C00 else h
        assert model.model_canon_nan_f16(w) == (q(lo) | (q(hi) << 16))


def test_register_heap_matches_serial_heap_select(model):
    """The select kernel's wave-parallel register heap (k <= 64: h2o_attention's heavy hitters)
    leaves exactly the heap libstdc++'s __heap_select leaves, slot by slot, on 6 000 random rows
    (a third of them with at most 4 distinct keys)."""
    model.model_regheap_check.restype = ctypes.c_int
    model.model_regheap_check.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert model.model_regheap_check(12345, 6000) == 0


def test_tiny_chain_lane_model_matches_libstdcxx(model):
    """wave_tiny_chain (csrc/kvc.hip: the chain's levels on segments of <= 64 positions from
    registers -- ballots, mbcnt ranks, forward-permute rank tables, backward-permute swaps) as a
    lane-by-lane model (select_model.cpp tiny_level) gives libstdc++'s first-k set: heavy ties,
    sort and nth_element, the k boundaries, small rows that enter the tiny levels at once, and the
    McIlroy adversary (depth-limit fallback from inside the tiny levels)."""
    model.model_set_tiny.argtypes = [ctypes.c_int]
    model.model_set_tiny(1)
    try:
        rng = np.random.default_rng(11)
        for trial in range(3000):
            n = int(rng.integers(4, 70)) if trial % 3 else int(rng.integers(70, 5000))
            keys = rng.integers(0, int(rng.choice([1, 2, 3, 5, 9, 80, 1 << 16])), n).astype(np.uint32)
            for k in {1, 2, n // 2, n - 2, n - 1, int(rng.integers(1, n))}:
                if not 0 < k < n:
                    continue
                for topk in (0, 1):
                    if topk and k * 64 <= n:
                        continue  # partial_sort: the heap path, no chain
                    got, _ = run_model(model, keys, k, topk)
                    np.testing.assert_array_equal(got, ref_set(keys, k, topk),
                                                  err_msg=f"n={n} k={k} topk={topk}")
        adv = np.empty(64, dtype=np.int64)
        for n in (20, 40, 64):
            for mode in (0, 1):
                for k in (1, n // 2, n - 1):
                    oracle.lib().orc_antiqsort(n, mode, k, adv.ctypes.data)
                    keys = adv[:n].astype(np.uint32)
                    got, _ = run_model(model, keys, k, mode)
                    np.testing.assert_array_equal(got, ref_set(keys, k, mode))
    finally:
        model.model_set_tiny(0)
