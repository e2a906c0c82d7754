"""CPU oracle for h2o_attention's heavy-hitter scoring -- TEST INFRASTRUCTURE ONLY.

Restates, in numpy, the torch CPU arithmetic that the reference's H2OAttentionManager runs
(/root/reference/kvcompress/methods/h2o_attention.py):

  update_attention_scores (:84-153)
      importance = attn.sum(dim=2)                      (:116)   [B,H,q,k] -> [B,H,k]
      acc = zeros | acc*decay (zero-extended) | zeros   (:118-146)
      acc = acc + importance                            (:149-151)
  get_heavy_hitter_indices (:156-213)
      head = acc[:, :, m0:m1].sum(dim=1)                (:194-198)
      top  = torch.topk(head, k); sort(top)             (:208-211)

`Tensor.sum` over a non-innermost dimension is aten's cascade_sum (SumKernel.cpp) reached through
TensorIterator's parallel_reduce.  Per output column the additions happen in one of two orders:

  cascade : multi_row_sum -- four fp32 accumulator levels; rows are added one by one into level 0
            and every 2^p rows (p = max(4, CeilLog2(n) // 4)) level j-1 is folded into level j
            while the row counter's j-th p-bit digit is zero; at the end
            acc0 + acc1 + acc2 + acc3.
  ilp4    : row_sum -- rows split into four interleaved lanes (row i -> lane i % 4) of n // 4
            rows, each lane a cascade over its rows, the n % 4 leftover rows added to lane 0,
            then lane0 + lane1 + lane2 + lane3.

The vectorised outer-sum loop (an inner-loop call of L >= one Vectorized<scalar_t> columns: 8
fp32 / 16 bf16-fp16; sum_stub has no AVX512 kernel, AVX512 hosts run the AVX2 one) runs
multi_row_sum on groups of four SIMD vectors (Vectorized<float>: 8 lanes) and row_sum on the single
vectors and scalar columns after the last whole group; a shorter call takes the scalar loop,
which runs multi_row_sum on groups of four columns and row_sum on the rest.  L is the whole
column count, except when parallel_reduce splits the column dimension over threads: chunks of
ceil(cols / threads) columns with bounds rounded down to 128 bytes, each chunk one call.  A reduced dimension of size
1 is no reduction at all: out = 0 + x elementwise.  bf16 / fp16 inputs are widened to fp32,
accumulated in fp32 and rounded once (RNE) into the output.

`acc * decay` on reduced-precision tensors multiplies by the fp32 value of the Python float
(TensorIterator's original_scalar_value<opmath_t>) and rounds; fp32 likewise.  `acc + imp` is one
fp32 add, rounded to the dtype.

Pinned by tests/test_h2o_oracle.py against torch's own CPU ops (sums across shapes and thread
counts, AVX512 and AVX2 capabilities) and against the unmodified reference's outputs in
tests/golden/h2o_attention_ties.json (tests/golden/gen_h2o_attention_ties.py).
"""
import numpy as np

from . import oracle as O

GRAIN_SIZE = 32768  # at::internal::GRAIN_SIZE


def _ceil_log2(x):
    """c10::utils::CeilLog2."""
    return 1 if x <= 2 else int(x - 1).bit_length()


def cascade_rows(X):
    """multi_row_sum over the rows of X [n, C] (fp32), all C columns at once."""
    n = X.shape[0]
    lp = max(4, _ceil_log2(n) // 4)
    step, mask = 1 << lp, (1 << lp) - 1
    zero = np.zeros(X.shape[1:], np.float32)
    acc = [zero.copy() for _ in range(4)]
    i = 0
    while i + step <= n:
        for _ in range(step):
            acc[0] = acc[0] + X[i]
            i += 1
        for j in range(1, 4):
            acc[j] = acc[j] + acc[j - 1]
            acc[j - 1] = zero.copy()
            if i & (mask << (j * lp)):
                break
    while i < n:
        acc[0] = acc[0] + X[i]
        i += 1
    for j in range(1, 4):
        acc[0] = acc[0] + acc[j]
    return acc[0]


def ilp4_rows(X):
    """row_sum (ilp_factor 4) over the rows of X [n, C] (fp32)."""
    n = X.shape[0]
    n4 = n // 4
    lanes = [cascade_rows(X[l:4 * n4:4]) for l in range(4)]
    for i in range(4 * n4, n):
        lanes[0] = lanes[0] + X[i]
    for l in range(1, 4):
        lanes[0] = lanes[0] + lanes[l]
    return lanes[0]


def vec_bytes(capability):
    """Bytes of one Vectorized<T> in the kernel that runs sum_stub for an ATen CPU capability.
    SumKernel.cpp registers sum_stub with REGISTER_DISPATCH only (no AVX512 variant: "these
    kernels are slower with AVX512 than with AVX2"), so an AVX512 host runs the AVX2 kernel:
    256-bit vectors on every x86 capability (DEFAULT's generic Vectorized is 32 bytes too)."""
    return 32


def column_chunks(cols, outer, red, esz, threads):
    """[(start, end)] of the inner-loop calls that cover the `cols` contiguous output columns.

    `outer`: sizes of the other non-reduced dims (innermost first, after TensorIterator's
    coalescing; size-1 dims dropped), `red`: size of the reduced dim (>= 2), esz: input element
    bytes, threads: at::get_num_threads() of the reducing process.  One call [0, cols) unless
    parallel_reduce splits the column dimension (parallel_dim_reduction / find_split_dim)."""
    numel = red * cols
    for s in outer:
        numel *= s
    if numel < GRAIN_SIZE or threads <= 1:
        return [(0, cols)]
    dims = [cols] + list(outer)  # innermost first; the reduced dim sits below them
    best, split = len(dims) - 1, None
    for d in range(len(dims) - 1, -1, -1):  # from the outermost dim
        if dims[d] >= threads:
            split = d
            break
        if dims[d] > dims[best]:
            best = d
    if (best if split is None else split) != 0:
        return [(0, cols)]
    nthr = min(threads, cols)
    chunk = -(-cols // nthr)
    mult = 128 // esz  # chunk bounds rounded down to 128 bytes (the final end stays)
    out = []
    for t in range(nthr):
        b, e = t * chunk, min(cols, (t + 1) * chunk)
        if b >= cols:
            break
        b -= b % mult
        if e != cols:
            e -= e % mult
        if b < e:
            out.append((b, e))
    return out


def ilp_mask(cols, outer, red, esz, threads, capability):
    """Boolean per output column: True where cascade_sum adds with row_sum (ilp4).

    Per inner-loop call [s, e) of L columns: the vectorised outer sum (L >= one
    Vectorized<scalar_t>) runs multi_row_sum on groups of four SIMD vectors and row_sum on the
    remaining single vectors and the scalar tail; the scalar loop (shorter L) runs multi_row_sum
    on groups of four columns and row_sum on the rest."""
    vb = vec_bytes(capability)
    vec_scalar = vb // esz      # Vectorized<scalar_t>::size()
    group = 4 * (vb // 4)       # four Vectorized<float>
    mask = np.zeros(cols, bool)
    for s, e in column_chunks(cols, outer, red, esz, threads):
        L = e - s
        g = group if L >= vec_scalar else 4
        mask[s + (L // g) * g:e] = True
    return mask


def sum_reduce_first(X, ilp):
    """Sum over axis 0 of X [n, C] (fp32 values): cascade where ilp is False, row_sum where it is
    True; n == 1 is the elementwise 0 + x."""
    n = X.shape[0]
    if n == 1:
        return np.float32(0) + X[0]
    out = np.empty(X.shape[1], np.float32)
    if (~ilp).any():
        out[~ilp] = cascade_rows(X[:, ~ilp])
    if ilp.any():
        out[ilp] = ilp4_rows(X[:, ilp])
    return out


# ---- dtype helpers (bf16 = uint16 bits, fp16 = float16, fp32 = float32) ----------------------
def to_f32(a):
    if a.dtype == np.uint16:
        return (a.astype(np.uint32) << np.uint32(16)).view(np.float32)
    return a.astype(np.float32)


def from_f32(x, like_dtype):
    x = np.ascontiguousarray(x, dtype=np.float32)
    if like_dtype == np.uint16:
        u = x.view(np.uint32).astype(np.uint64)
        r = ((u + ((u >> np.uint64(16)) & np.uint64(1)) + np.uint64(0x7FFF)) >> np.uint64(16))
        r = r.astype(np.uint16)
        r[np.isnan(x)] = 0x7FC0
        return r
    if like_dtype == np.float16:
        with np.errstate(over="ignore"):
            return x.astype(np.float16)
    return x


def _esz(dtype):
    return 4 if dtype == np.float32 else 2


def attn_importance(attn, threads, capability):
    """attn.sum(dim=2) of [B,H,q,k] (h2o_attention.py:116), in attn's dtype."""
    B, H, q, k = attn.shape
    x = to_f32(attn)
    out = np.empty((B, H, k), np.float32)
    outer = [s for s in (B * H,) if s > 1]  # B and H coalesce (contiguous in and out)
    ilp = ilp_mask(k, outer, q, _esz(attn.dtype), threads, capability)
    for b in range(B):
        for h in range(H):
            out[b, h] = sum_reduce_first(x[b, h], ilp)
    return from_f32(out, attn.dtype)


def head_sum(mid, threads, capability):
    """acc[:, :, m0:m1].sum(dim=1) of a [B,H,m] slice (h2o_attention.py:198), in its dtype."""
    B, H, m = mid.shape
    x = to_f32(mid)
    out = np.empty((B, m), np.float32)
    outer = [B] if B > 1 else []
    ilp = ilp_mask(m, outer, H, _esz(mid.dtype), threads, capability)
    for b in range(B):
        out[b] = sum_reduce_first(x[b], ilp)
    return from_f32(out, mid.dtype)


class H2OManager:
    """numpy restatement of H2OAttentionManager's state (h2o_attention.py:28-213)."""

    def __init__(self, start_size=4, heavy_hitter_size=64, recent_size=444, decay_factor=0.9,
                 threads=8, capability="AVX512"):
        self.start_size, self.heavy_hitter_size = start_size, heavy_hitter_size
        self.recent_size, self.decay_factor = recent_size, decay_factor
        self.threads, self.capability = threads, capability
        self.acc = {}
        self.current_seq_len = 0

    def update_attention_scores(self, attentions, skip_layers=()):
        """h2o_attention.py:84-153"""
        if attentions is None:
            return
        for li, attn in enumerate(attentions):
            if li in skip_layers or attn is None:
                continue
            B, H, q, k = attn.shape
            imp = to_f32(attn_importance(attn, self.threads, self.capability))
            old = self.acc.get(li)
            base = np.zeros((B, H, k), np.float32)
            out_dtype = attn.dtype
            if old is not None and old.shape[-1] <= k:
                L = old.shape[-1]
                dec = to_f32(old) * np.float32(self.decay_factor)  # (:136, :146), in old's dtype
                base[:, :, :L] = to_f32(from_f32(dec, old.dtype))
                # torch.cat / + type promotion (:129-151): two different float dtypes of
                # {bf16, fp16, fp32} promote to fp32 (exact widening of both operands)
                if old.dtype != attn.dtype:
                    out_dtype = np.float32
            self.acc[li] = from_f32(base + imp, out_dtype)       # (:149-151)
            self.current_seq_len = k

    def get_heavy_hitter_indices(self, li, seq_len):
        """h2o_attention.py:156-213 -> int64 indices ([k] for B == 1, else [B, k])."""
        if li not in self.acc:
            m0, m1 = self.start_size, seq_len - self.recent_size
            if m1 <= m0:
                return np.zeros(0, np.int64)
            step = max(1, (m1 - m0) // self.heavy_hitter_size)
            return np.arange(0, m1 - m0, step)[:self.heavy_hitter_size]
        acc = self.acc[li]
        B, H, L = acc.shape
        m0, m1 = self.start_size, min(seq_len, L) - self.recent_size
        if m1 <= m0:
            return np.zeros(0, np.int64)
        agg = head_sum(acc[:, :, m0:m1], self.threads, self.capability)  # [B, m]
        k = min(self.heavy_hitter_size, m1 - m0)
        top = O.topk_indices(agg[:, None, :], k)[:, 0, :]
        top = np.sort(top, axis=-1)
        return top[0] if B == 1 else top


def h2o_attention_compress(layers, attention_scores=None, h2o_manager=None, start_size=4,
                           heavy_hitter_size=64, recent_size=444, skip_layers=(), **kw):
    """h2o_attention.py:216-363 (manager path and the L2-norm fallback)."""
    out = [(k, v, "same") for k, v in layers]
    if not layers:
        return out
    total = start_size + heavy_hitter_size + recent_size
    if h2o_manager is not None and attention_scores is not None:
        h2o_manager.update_attention_scores(attention_scores, skip_layers)
    for i, (keys, values) in enumerate(layers):
        S = keys.shape[2]
        if S <= total or i in skip_layers:
            continue
        B, H, _, D = keys.shape
        ms, me = start_size, S - recent_size
        if me <= ms:
            out[i] = (O.cat([keys[:, :, :start_size], keys[:, :, -recent_size:]]),
                      O.cat([values[:, :, :start_size], values[:, :, -recent_size:]]), "new")
            continue
        mk, mv = keys[:, :, ms:me], values[:, :, ms:me]
        mlen = mk.shape[2]
        if h2o_manager is not None:
            hi = h2o_manager.get_heavy_hitter_indices(i, S)
            num = min(len(hi), heavy_hitter_size, mlen)
            if num > 0 and len(hi) > 0:
                if hi.ndim != 1:
                    raise RuntimeError("expand: index rank (reference h2o_attention.py:327-330)")
                idx = np.clip(hi[:num], 0, mlen - 1)
                idx = np.broadcast_to(idx, (B, H, num))
                hk, hv = O.gather(mk, idx), O.gather(mv, idx)
            else:
                hk, hv = mk[:, :, :0], mv[:, :, :0]
        else:
            k = min(heavy_hitter_size, mlen)
            idx = O.select_low(mk, k)
            hk, hv = O.gather(mk, idx), O.gather(mv, idx)
        out[i] = (O.cat([keys[:, :, :start_size], hk, keys[:, :, -recent_size:]]),
                  O.cat([values[:, :, :start_size], hv, values[:, :, -recent_size:]]), "new")
    return out
