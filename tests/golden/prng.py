"""Deterministic synthetic KV inputs for golden fixtures and parity tests.

Fixtures store only a recipe (seed, shape, dtype, variant) plus expected outputs, so the
inputs must be reproducible bit-for-bit on any IEEE machine: splitmix64 counter stream ->
53-bit uniforms -> (u0+u1+u2+u3-2)*sqrt(3) in float64 (plain IEEE adds/multiplies, no libm)
-> RNE to float32 -> RNE to bfloat16 (c10::BFloat16 rounding) or float16 (IEEE RNE, as numpy's
and c10::Half's conversions both do).

bf16 tensors are represented as numpy uint16 bit patterns, fp16 tensors as numpy float16.
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_SQRT3 = 1.7320508075688772


def splitmix64(seed, n, offset=0):
    i = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def uniform(seed, n):
    return (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


_C = None


def _clib():
    """oracle/liboracle.so's restatement of normal_f32 (same operations; ~50x faster), if built."""
    global _C
    if _C is None:
        import ctypes
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "oracle",
                            "liboracle.so")
        try:
            lib = ctypes.CDLL(path)
            lib.orc_normal_f32.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p]
            _C = lib
        except (OSError, AttributeError):
            _C = False
    return _C


def normal_f32(seed, n):
    lib = _clib()
    if lib:
        out = np.empty(n, dtype=np.float32)
        assert lib.orc_normal_f32(seed & 0xFFFFFFFFFFFFFFFF, n, out.ctypes.data) == 0
        return out
    return normal_f32_numpy(seed, n)


def normal_f32_numpy(seed, n):
    out = np.empty(n, dtype=np.float32)
    step = 1 << 22
    for s in range(0, n, step):
        m = min(step, n - s)
        u = (splitmix64(seed, 4 * m, offset=4 * s) >> np.uint64(11)).astype(np.float64)
        u = (u * (2.0 ** -53)).reshape(m, 4)
        x = ((((u[:, 0] + u[:, 1]) + u[:, 2]) + u[:, 3]) - 2.0) * _SQRT3
        out[s:s + m] = x.astype(np.float32)
    return out


def f32_to_bf16_bits(x):
    """c10::BFloat16 round_to_nearest_even, NaN -> 0x7FC0."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + ((u >> np.uint64(16)) & np.uint64(1)) + np.uint64(0x7FFF)) >> np.uint64(16))
    r = r.astype(np.uint16)
    r[np.isnan(x)] = 0x7FC0
    return r


def bf16_bits_to_f32(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def to_dtype(x_f32, dtype):
    if dtype == "bf16":
        return f32_to_bf16_bits(x_f32)
    if dtype == "fp32":
        return np.ascontiguousarray(x_f32, dtype=np.float32)
    if dtype == "fp16":
        with np.errstate(over="ignore"):
            return np.ascontiguousarray(x_f32, dtype=np.float32).astype(np.float16)
    raise ValueError(dtype)


def gen_keys(seed, shape, dtype, variant="normal"):
    """K[B,H,S,D] in storage representation (uint16 bits for bf16, float16 / float32 otherwise)."""
    B, H, S, D = shape
    n = B * H * S * D
    if variant == "normal":
        x = normal_f32(seed, n)
    elif variant == "scaled":  # per-token scale in [0.5, 2): spread norms, fewer ties
        x = normal_f32(seed, n).reshape(B * H * S, D)
        sc = (0.5 + 1.5 * uniform(seed ^ 0x5A5A, B * H * S)).astype(np.float32)
        x = (x * sc[:, None]).astype(np.float32).reshape(-1)
    elif variant == "equal":  # every token row identical: all norms tie
        row = normal_f32(seed, D)
        x = np.tile(row, B * H * S)
    elif variant == "few":  # three distinct rows: three distinct norms, heavy ties
        rows = normal_f32(seed, 3 * D).reshape(3, D)
        pick = (splitmix64(seed ^ 0x77, B * H * S) % np.uint64(3)).astype(np.int64)
        x = rows[pick].reshape(-1)
    elif variant == "special":  # NaN / +-Inf / zero rows sprinkled in
        x = normal_f32(seed, n).reshape(B * H * S, D)
        sel = (splitmix64(seed ^ 0x99, B * H * S) % np.uint64(23)).astype(np.int64)
        x[sel == 1, 3] = np.nan
        x[sel == 2, 5] = np.inf
        x[sel == 3, 0] = -np.inf
        x[sel == 4, :] = 0.0
        x[sel == 5, :] = -0.0
        x = x.reshape(-1)
    elif variant == "tiny":  # norms ~1e-3: the +1e-6 in snapkv_lite becomes visible
        x = (normal_f32(seed, n) * np.float32(1e-4)).astype(np.float32)
    elif variant == "micro":  # norms at the bottom of the dtype's range, where snapkv_lite's
        # `max + 1e-6` rounds differently for a dtype-cast and an fp32 epsilon
        scale = {"bf16": 2.3e-10, "fp32": 2.3e-10, "fp16": 1.1e-5}[dtype]
        x = (normal_f32(seed, n) * np.float32(scale)).astype(np.float32)
    elif variant == "zero":
        x = np.zeros(n, dtype=np.float32)
    else:
        raise ValueError(variant)
    return to_dtype(x, dtype).reshape(B, H, S, D)


def gen_values(seed, shape, dtype):
    B, H, S, D = shape
    return to_dtype(normal_f32(seed ^ 0xABCDEF, B * H * S * D), dtype).reshape(B, H, S, D)


def encode_positions(shape, dtype):
    """V whose rows encode their own (b, h, s): exact in bf16 (ints <= 255), fp16 and fp32."""
    B, H, S, D = shape
    assert D >= 4
    v = np.zeros((B, H, S, D), dtype=np.float32)
    s = np.arange(S, dtype=np.float32)
    v[..., 0] = (np.arange(S) // 256).astype(np.float32)[None, None, :]
    v[..., 1] = (np.arange(S) % 256).astype(np.float32)[None, None, :]
    v[..., 2] = np.arange(H, dtype=np.float32)[None, :, None]
    v[..., 3] = np.arange(B, dtype=np.float32)[:, None, None]
    del s
    return to_dtype(v.reshape(-1), dtype).reshape(B, H, S, D)


def decode_positions(v_out, dtype):
    """Inverse of encode_positions on a [B,H,n,D] array; returns (pos[B,H,n], ok)."""
    v = bf16_bits_to_f32(v_out) if dtype == "bf16" else np.asarray(v_out).astype(np.float32)
    pos = (v[..., 0].astype(np.int64) * 256 + v[..., 1].astype(np.int64))
    B, H = v.shape[0], v.shape[1]
    ok = bool(np.all(v[..., 2] == np.arange(H)[None, :, None]) and
              np.all(v[..., 3] == np.arange(B)[:, None, None]))
    return pos, ok
