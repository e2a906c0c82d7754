"""Which addition order torch's CPU `Tensor.sum` over a non-innermost dim gives each column.

h2o_attention's reference arithmetic (h2o_attention.py:116, :198) is two such sums.  aten's
cascade_sum (SumKernel.cpp) adds each output column's rows either as a four-level cascade
(multi_row_sum) or as four interleaved lanes (row_sum), depending on where the column falls in
the inner-loop calls TensorIterator makes: one call over all columns, or -- when parallel_reduce
splits the column dimension over threads (parallel_dim_reduction / find_split_dim) -- one call
per thread chunk of ceil(cols / threads) columns with bounds rounded down to 128 bytes.  The HIP
kernels (csrc/kvc.hip, col_ilp) take that chunk size per layer and derive the rest; this module
computes it from the reference process's thread count (torch.get_num_threads()).
"""
import torch

GRAIN_SIZE = 32768  # at::internal::GRAIN_SIZE
# sum_stub is registered without an AVX512 variant, so x86 hosts of every capability run a
# 256-bit kernel (Vectorized<float> = 8 lanes)
SUM_VEC_BYTES = 32


def threads():
    return torch.get_num_threads()


def column_chunk(cols, outer, red, esz, nthreads):
    """Columns per thread chunk of the reduction's contiguous output dim, or 0 when one loop call
    covers every column.  `outer`: the other non-reduced dims' sizes, innermost first, after
    TensorIterator's coalescing (size-1 dims dropped); `red` >= 2: the reduced size."""
    numel = red * cols
    for s in outer:
        numel *= s
    if numel < GRAIN_SIZE or nthreads <= 1:
        return 0
    dims = [cols] + list(outer)
    best = len(dims) - 1
    for d in range(len(dims) - 1, -1, -1):  # find_split_dim: from the outermost non-reduced dim
        if dims[d] >= nthreads:
            best = d
            break
        if dims[d] > dims[best]:
            best = d
    if best != 0:
        return 0  # split over another dim: every call spans all columns
    return -(-cols // min(nthreads, cols))


def attn_sum_chunk(attn, nthreads):
    """Chunk of attn.sum(dim=2) for attn [B,H,q,k] (last dim contiguous)."""
    B, H, q, k = attn.shape
    if q < 2:
        return 0
    st = attn.stride()
    # B and H coalesce when attn's strides allow it (the output [B,H,k] is contiguous)
    if B > 1 and H > 1 and st[0] == H * st[1]:
        outer = [B * H]
    else:
        outer = [s for s in (H, B) if s > 1]
    return column_chunk(k, outer, q, attn.element_size(), nthreads)


def head_sum_chunk(B, H, m, esz, nthreads):
    """Chunk of acc[:, :, m0:m1].sum(dim=1) for acc [B,H,*] (m = m1 - m0 columns)."""
    if H < 2:
        return 0
    return column_chunk(m, [B] if B > 1 else [], H, esz, nthreads)
