"""CPU oracle for the kvcompress/methods hot path -- TEST INFRASTRUCTURE ONLY.

This module restates, in numpy plus the small C++ library next to it (liboracle.so), what the
reference's compress functions compute.  It is the checker the HIP engine is tested against;
only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it.  The product
path (cs3602-llm-inference-acceleration_amd/kvcompress) never imports or calls anything here.

Pinning: tests/test_oracle_golden.py checks every function below against the golden fixtures in
tests/golden/, which tests/golden/gen_goldens.py produced by running the unmodified reference.

Representation: a layer is a pair (K, V) of numpy arrays [B, H, S, D]; bf16 tensors are uint16
bit patterns, fp16 tensors are float16, fp32 tensors are float32.  Every function mirrors its reference's control flow
line by line (file:line citations are to /root/reference/kvcompress/methods/).
Each returned layer is tagged with how the reference produced it:
  "same" - the input tensor objects themselves (layer untouched),
  "view" - a slice of the input (no copy),
  "new"  - a freshly gathered / concatenated tensor.
"""
import ctypes
import math
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

DT_F32, DT_BF16, DT_F16 = 0, 1, 2

# Tie policy of argsort_prefix / topk_indices: "reference" (libstdc++ std::sort / nth_element /
# partial_sort, the reference's order) or "stable" (the engine's opt-in KVC_ALGO_STABLE: the
# first k of torch.argsort(stable=True), ties in position order; pinned against torch by
# tests/test_stable_ties.py).
TIE = "reference"


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _LIB = ctypes.CDLL(path)
        i64, vp = ctypes.c_int64, ctypes.c_void_p
        _LIB.orc_row_norms.argtypes = [ctypes.c_int, vp, i64, i64, i64, vp]
        _LIB.orc_sort_prefix.argtypes = [ctypes.c_int, vp, i64, i64, ctypes.c_int, vp]
        _LIB.orc_topk.argtypes = [ctypes.c_int, vp, i64, i64, ctypes.c_int, vp]
        _LIB.orc_snapkv_scores.argtypes = [ctypes.c_int, vp, i64, i64, vp]
        _LIB.orc_antiqsort.argtypes = [i64, ctypes.c_int, i64, vp]
        _LIB.orc_to_dtype_bits.argtypes = [ctypes.c_int, vp, i64, vp]
    return _LIB


def _dt(arr):
    if arr.dtype == np.uint16:
        return DT_BF16
    if arr.dtype == np.float32:
        return DT_F32
    if arr.dtype == np.float16:
        return DT_F16
    raise TypeError(f"oracle supports bf16 (uint16 bits), float16 and float32, got {arr.dtype}")


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


# ----------------------------------------------------------------------------------------------
# torch primitives restated
# ----------------------------------------------------------------------------------------------
def norms(K):
    """torch.norm(K, p=2, dim=-1) -> [B, H, Z] in K's dtype."""
    K = np.ascontiguousarray(K)
    B, H, Z, D = K.shape
    out = np.empty((B, H, Z), dtype=K.dtype)
    if Z:
        rc = lib().orc_row_norms(_dt(K), _ptr(K), B * H * Z, D, D, _ptr(out))
        assert rc == 0
    return out


def as_float(vals):
    """Values of a bf16 (uint16 bits) / fp16 / fp32 array as float32 (exact)."""
    if vals.dtype == np.uint16:
        return (vals.astype(np.uint32) << 16).view(np.float32)
    return vals.astype(np.float32)


def stable_prefix(vals, k, descending=False):
    """The first k of a stable sort along the last axis (NaN last ascending, first descending,
    as torch.sort orders them), in sort order."""
    v = as_float(np.ascontiguousarray(vals))
    nan = np.isnan(v)
    B, H, n = v.shape
    out = np.empty((B, H, k), dtype=np.int64)
    for b in range(B):
        for h in range(H):
            keys = (-v[b, h], ~nan[b, h]) if descending else (v[b, h], nan[b, h])
            out[b, h] = np.lexsort(keys)[:k]
    return out


def argsort_prefix(vals, k, descending=False):
    """vals.argsort(dim=-1, descending)[..., :k] (k >= 0) in sort order."""
    if TIE == "stable":
        return stable_prefix(vals, k, descending)
    vals = np.ascontiguousarray(vals)
    B, H, n = vals.shape
    out = np.empty((B, H, k), dtype=np.int64)
    for b in range(B):
        for h in range(H):
            row = np.ascontiguousarray(vals[b, h])
            o = np.empty(k, dtype=np.int64)
            assert lib().orc_sort_prefix(_dt(vals), _ptr(row), n, k, int(descending), _ptr(o)) == 0
            out[b, h] = o
    return out


def topk_indices(vals, k):
    """torch.topk(vals, k, dim=-1)[1] (largest=True, sorted=True)."""
    if TIE == "stable":
        return stable_prefix(vals, k, descending=True)
    vals = np.ascontiguousarray(vals)
    B, H, n = vals.shape
    out = np.empty((B, H, k), dtype=np.int64)
    for b in range(B):
        for h in range(H):
            row = np.ascontiguousarray(vals[b, h])
            o = np.empty(k, dtype=np.int64)
            assert lib().orc_topk(_dt(vals), _ptr(row), n, k, 1, _ptr(o)) == 0
            out[b, h] = o
    return out


def snapkv_scores(prefix_norms, pool_k):
    """snapkv_lite.py:99-121 importance scores (max+1e-6 - norms, optional avg_pool1d)."""
    prefix_norms = np.ascontiguousarray(prefix_norms)
    B, H, n = prefix_norms.shape
    out = np.empty_like(prefix_norms)
    for b in range(B):
        for h in range(H):
            row = np.ascontiguousarray(prefix_norms[b, h])
            o = np.empty(n, dtype=prefix_norms.dtype)
            assert lib().orc_snapkv_scores(_dt(row), _ptr(row), n, pool_k, _ptr(o)) == 0
            out[b, h] = o
    return out


def gather(X, idx):
    """torch.gather(X, 2, idx[..., None].expand(..., D)).

    torch's CPU gather rewrites every bf16 NaN bit pattern to 0xFFFF and quiets every fp16 NaN
    (sets bit 9: 0x7C01 -> 0x7E01), measured over all 65536 patterns of each; fp32 payloads and
    torch.cat copies are untouched.  The gathered segment of an output carries the rewritten
    patterns wherever the source held a NaN.
    """
    B, H = idx.shape[:2]
    out = X[np.arange(B)[:, None, None], np.arange(H)[None, :, None], idx, :]
    if out.dtype == np.uint16:
        out = np.where((out & 0x7FFF) > 0x7F80, np.uint16(0xFFFF), out).astype(np.uint16)
    elif out.dtype == np.float16:
        b = out.view(np.uint16)
        out = np.where((b & 0x7FFF) > 0x7C00, b | np.uint16(0x200), b).astype(np.uint16).view(np.float16)
    return out


def cat(parts):
    return np.ascontiguousarray(np.concatenate(parts, axis=2))


def select_low(K_zone, k):
    """norm -> argsort -> [:k] -> sort  (the shared Select primitive)."""
    idx = argsort_prefix(norms(K_zone), k)
    return np.sort(idx, axis=-1)


# ----------------------------------------------------------------------------------------------
# methods (mirror /root/reference/kvcompress/methods/*.py)
# ----------------------------------------------------------------------------------------------
def _tag(kv, kind):
    return (kv[0], kv[1], kind)


def l2_compress(layers, keep_ratio=1.0, prune_after=1000, skip_layers=(0, 1), **kw):
    """l2_compress.py:18-92"""
    out = [(k, v, "same") for k, v in layers]
    if keep_ratio >= 1.0:
        return out
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S <= prune_after or i in skip_layers:
            continue
        k = math.ceil(keep_ratio * S)
        if k >= S:
            continue
        if k < -1:
            raise RuntimeError("expand with negative size (reference l2_compress.py:82)")
        order = argsort_prefix(norms(keys), S)[:, :, :k]
        idx = np.sort(order, axis=-1)
        out[i] = (np.ascontiguousarray(gather(keys, idx)),
                  np.ascontiguousarray(gather(values, idx)), "new")
    return out


def fix_size_l2_compress(layers, fix_kv_size=1024, keep_ratio=0.0, strategy="keep_low",
                         skip_layers=(0, 1), **kw):
    """fix_size_l2.py:15-154 (strategy 'random' is not restated: it consumes torch's RNG)."""
    out = [(k, v, "same") for k, v in layers]
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S <= fix_kv_size or i in skip_layers:
            continue
        P = min(int(fix_kv_size * keep_ratio), S)
        Z = S - P
        keep = fix_kv_size - P
        if keep <= 0:
            out[i] = (keys[:, :, -P:, :], values[:, :, -P:, :], "view")
            continue
        if Z <= keep:
            continue
        zk, zv = keys[:, :, :Z, :], values[:, :, :Z, :]
        if strategy == "keep_low":
            order = argsort_prefix(norms(zk), keep)
        elif strategy == "keep_high":
            order = argsort_prefix(norms(zk), keep, descending=True)
        else:
            raise ValueError(f"Unknown strategy: {strategy}")
        idx = np.sort(order, axis=-1)
        kk, kv = gather(zk, idx), gather(zv, idx)
        if P > 0:
            out[i] = (cat([kk, keys[:, :, -P:, :]]), cat([kv, values[:, :, -P:, :]]), "new")
        else:
            out[i] = (np.ascontiguousarray(kk), np.ascontiguousarray(kv), "new")
    return out


def streaming_llm_compress(layers, start_size=4, recent_size=508, skip_layers=(), **kw):
    """streaming_llm.py:19-111"""
    out = [(k, v, "same") for k, v in layers]
    if not layers:
        return out
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S <= start_size + recent_size or i in skip_layers:
            continue
        out[i] = (cat([keys[:, :, :start_size], keys[:, :, -recent_size:]]),
                  cat([values[:, :, :start_size], values[:, :, -recent_size:]]), "new")
    return out


def evict_for_space(layers, num_coming, start_size=4, recent_size=508, skip_layers=()):
    """streaming_llm.py:114-170 (exported, not registered): the length test includes the
    incoming tokens, and the recent window shrinks by them unless that empties it."""
    out = [(k, v, "same") for k, v in layers]
    if not layers:
        return out
    cache_size = start_size + recent_size
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S + num_coming <= cache_size:                               # :149
            continue
        if i in skip_layers:                                           # :152
            continue
        eff = recent_size - num_coming                                 # :156-158
        if eff <= 0:
            eff = recent_size
        out[i] = (cat([keys[:, :, :start_size], keys[:, :, -eff:]]),
                  cat([values[:, :, :start_size], values[:, :, -eff:]]), "new")
    return out


def recent_only_compress(layers, window_size=512, skip_layers=(0, 1), **kw):
    """recent_only.py:16-70 (returns views)"""
    out = [(k, v, "same") for k, v in layers]
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S <= window_size or i in skip_layers:
            continue
        out[i] = (keys[:, :, -window_size:, :], values[:, :, -window_size:, :], "view")
    return out


def h2o_l2_compress(layers, start_size=4, heavy_hitter_size=64, recent_size=444,
                    skip_layers=(), **kw):
    """h2o_l2.py:25-153"""
    out = [(k, v, "same") for k, v in layers]
    if not layers:
        return out
    total = start_size + heavy_hitter_size + recent_size
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S <= total or i in skip_layers:
            continue
        ms, me = start_size, S - recent_size
        if me <= ms:
            out[i] = (cat([keys[:, :, :start_size], keys[:, :, -recent_size:]]),
                      cat([values[:, :, :start_size], values[:, :, -recent_size:]]), "new")
            continue
        mk, mv = keys[:, :, ms:me], values[:, :, ms:me]
        k = min(heavy_hitter_size, mk.shape[2])
        idx = select_low(mk, k)
        out[i] = (cat([keys[:, :, :start_size], gather(mk, idx), keys[:, :, -recent_size:]]),
                  cat([values[:, :, :start_size], gather(mv, idx), values[:, :, -recent_size:]]),
                  "new")
    return out


def snapkv_lite_compress(layers, observation_window=32, keep_size=512, pooling_kernel=5,
                         skip_layers=(), **kw):
    """snapkv_lite.py:24-154"""
    out = [(k, v, "same") for k, v in layers]
    if not layers:
        return out
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S <= keep_size or i in skip_layers:
            continue
        P = S - observation_window
        if P <= 0:
            continue
        pk, pv = keys[:, :, :P], values[:, :, :P]
        ok, ov = keys[:, :, -observation_window:], values[:, :, -observation_window:]
        scores = snapkv_scores(norms(pk), pooling_kernel if pooling_kernel > 1 and P >= pooling_kernel else 0)
        k = min(keep_size - observation_window, P)
        if k <= 0:
            out[i] = (ok, ov, "view")
            continue
        idx = np.sort(topk_indices(scores, k), axis=-1)
        out[i] = (cat([gather(pk, idx), ok]), cat([gather(pv, idx), ov]), "new")
    return out


def pyramid_layer_sizes(num_layers, base_size=512, layer_decay=0.9, min_size=64,
                        profile="exponential"):
    """pyramid_kv.py:82-97"""
    sizes = []
    for i in range(num_layers):
        if profile == "exponential":
            s = int(base_size * (layer_decay ** i))
        elif profile == "linear":
            s = int(base_size - i * ((base_size - min_size) / max(num_layers - 1, 1)))
        else:
            s = base_size
        sizes.append(max(s, min_size))
    return sizes


def pyramid_kv_compress(layers, base_size=512, layer_decay=0.9, min_size=64,
                        profile="exponential", skip_layers=(), **kw):
    """pyramid_kv.py:26-185"""
    out = [(k, v, "same") for k, v in layers]
    if not layers:
        return out
    sizes = pyramid_layer_sizes(len(layers), base_size, layer_decay, min_size, profile)
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        t = sizes[i]
        if S <= t or i in skip_layers:
            continue
        start = min(4, t // 8)
        recent = t // 2
        mid_keep = t - start - recent
        if mid_keep <= 0:
            out[i] = (keys[:, :, -t:, :], values[:, :, -t:, :], "view")
            continue
        ms, me = start, S - recent
        if me <= ms:
            out[i] = (cat([keys[:, :, :start], keys[:, :, -(t - start):]]),
                      cat([values[:, :, :start], values[:, :, -(t - start):]]), "new")
            continue
        mk, mv = keys[:, :, ms:me], values[:, :, ms:me]
        k = min(mid_keep, mk.shape[2])
        if k > 0 and mk.shape[2] > 0:
            idx = select_low(mk, k)
            sk, sv = gather(mk, idx), gather(mv, idx)
        else:
            sk, sv = mk[:, :, :0], mv[:, :, :0]
        out[i] = (cat([keys[:, :, :start], sk, keys[:, :, -recent:]]),
                  cat([values[:, :, :start], sv, values[:, :, -recent:]]), "new")
    return out


def adaptive_l2_compress(layers, target_size=512, soft_limit=256, hard_limit=1024,
                         keep_ratio_min=0.3, keep_ratio_max=0.9, skip_layers=(), **kw):
    """adaptive_l2.py:20-201"""
    out = [(k, v, "same") for k, v in layers]
    if not layers:
        return out
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if i in skip_layers or S <= soft_limit:
            continue
        if S > hard_limit:
            if S <= target_size:
                continue
            start, recent = 4, target_size // 2
            mid_keep = target_size - start - recent
            if mid_keep <= 0:
                out[i] = (keys[:, :, -target_size:, :], values[:, :, -target_size:, :], "view")
                continue
            ms, me = start, S - recent
            if me <= ms:
                out[i] = (cat([keys[:, :, :start], keys[:, :, -(target_size - start):]]),
                          cat([values[:, :, :start], values[:, :, -(target_size - start):]]),
                          "new")
                continue
            mk, mv = keys[:, :, ms:me], values[:, :, ms:me]
            k = min(mid_keep, mk.shape[2])
            idx = select_low(mk, k)
            out[i] = (cat([keys[:, :, :start], gather(mk, idx), keys[:, :, -recent:]]),
                      cat([values[:, :, :start], gather(mv, idx), values[:, :, -recent:]]),
                      "new")
        else:
            progress = (S - soft_limit) / (hard_limit - soft_limit)
            kr = keep_ratio_max - progress * (keep_ratio_max - keep_ratio_min)
            t = max(int(S * kr), soft_limit)
            if t >= S:
                continue
            prot = int(t * 0.2)
            hist = t - prot
            if hist <= 0:
                out[i] = (keys[:, :, -t:, :], values[:, :, -t:, :], "view")
                continue
            se = S - prot
            if se <= hist:
                continue
            sk, sv = keys[:, :, :se], values[:, :, :se]
            idx = select_low(sk, hist)
            out[i] = (cat([gather(sk, idx), keys[:, :, -prot:]]),
                      cat([gather(sv, idx), values[:, :, -prot:]]), "new")
    return out


METHODS = {
    "l2_compress": l2_compress,
    "fix_size_l2": fix_size_l2_compress,
    "streaming_llm": streaming_llm_compress,
    "recent_only": recent_only_compress,
    "h2o_l2": h2o_l2_compress,
    "snapkv_lite": snapkv_lite_compress,
    "pyramid_kv": pyramid_kv_compress,
    "adaptive_l2": adaptive_l2_compress,
    "evict_for_space": evict_for_space,  # not in the reference's registry; goldens only
}
