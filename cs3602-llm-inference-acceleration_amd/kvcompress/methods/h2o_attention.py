"""H2O with attention-score heavy hitters (reference: kvcompress/methods/h2o_attention.py).

The manager keeps the reference's per-layer accumulated attention (h2o_attention.py:84-213) and
every piece of its arithmetic runs on the HIP engine with the CPU reference's exact results:

  update_attention_scores   kvc_attn_accumulate: acc = dt((acc*decay | 0) + dt(attn.sum(dim=2)))
                            for all layers of the call in one kernel, each column's q-sum in
                            torch CPU's addition order (cascade_sum; _cpu_order.py)
  get_heavy_hitter_indices  kvc_heavy_hitters: the head sum acc[:, :, m0:m1].sum(dim=1) in the
                            same order, then the reference-exact top-k set (std::nth_element /
                            std::partial_sort tie order, KVC_ALGO_TOPK) as ascending indices
  h2o_attention_compress    heavy hitters of every layer written straight into the index region
                            of one gather launch (KVC_FLAG_SHARED_INDEX: one list per layer,
                            shared by all heads), which copies sinks ++ heavy ++ recent of K/V

Without a manager the reference falls back to L2-norm heavy hitters, which is exactly h2o_l2's
selection: the engine's score / select / gather path.  Tensors must be on a ROCm device (bf16,
fp16 or fp32); there is no CPU path.
"""
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _cpu_order as CO
from .. import _engine as E
from .. import _native as N
from ..utils import normalize_kv_cache

_DT = {torch.bfloat16: N.KVC_BF16, torch.float16: N.KVC_F16, torch.float32: N.KVC_F32}


def _attn_params(dtype, B, H, decay, device, old_dtype=None):
    """old_dtype: the carried accumulations' dtype when it differs from the attention's (torch
    then promotes to float32, h2o_attention.py:129-151; kvc_attn_accumulate's
    KVC_ATTN_OLD_DTYPE flag)."""
    flags = N.ATTN_OLD_DTYPE(_DT[old_dtype]) if old_dtype not in (None, dtype) else 0
    if E.tie_policy == "stable":  # the heavy hitters' selection (kvc_heavy_hitters) only
        flags |= N.ATTN_HH_STABLE
    return N.AttnParams(dtype=_DT[dtype], batch=B, heads=H, vec_bytes=CO.SUM_VEC_BYTES,
                        decay=float(np.float32(decay)), flags=flags,
                        device_status=E.status_word(device).data_ptr())


def _check_gpu(t, what):
    if not t.is_cuda:
        raise RuntimeError(f"kvcompress (MI355X HIP engine): {what} is on {t.device}; the "
                           "h2o_attention scoring runs on ROCm GPU tensors only (no CPU fallback).")
    if t.dtype not in _DT:
        raise TypeError(f"kvcompress (MI355X HIP engine): {what} must be bfloat16, float16 or "
                        f"float32, got {t.dtype}")


class H2OAttentionManager:
    """Accumulated attention per layer (h2o_attention.py:28-213): same constructor, state and
    methods as the reference.  `reduction_threads` (extension, default None = the process's
    torch.get_num_threads()) is the thread count whose CPU reduction order the sums reproduce."""

    def __init__(self, start_size: int = 4, heavy_hitter_size: int = 64, recent_size: int = 444,
                 num_layers: int = 32, num_heads: int = 32, decay_factor: float = 0.9,
                 device: torch.device = None):
        self.start_size = start_size
        self.heavy_hitter_size = heavy_hitter_size
        self.recent_size = recent_size
        self.total_cache_size = start_size + heavy_hitter_size + recent_size
        self.num_layers = num_layers
        self.num_heads = num_heads
        self.decay_factor = decay_factor
        self.device = device
        self.accumulated_attention: Dict[int, torch.Tensor] = {}
        self.token_positions: Dict[int, torch.Tensor] = {}
        self.current_seq_len = 0
        self.reduction_threads: Optional[int] = None

    def reset(self):
        self.accumulated_attention = {}
        self.token_positions = {}
        self.current_seq_len = 0

    def _threads(self):
        return self.reduction_threads or CO.threads()

    @E.status_checked
    def update_attention_scores(self, attentions, skip_layers: List[int] = []):
        """h2o_attention.py:84-153 for every given layer in one engine launch per
        (device, dtype, B, H, carried dtype) group: acc <- acc*decay (zero-extended to the new key
        length; reset to zeros if the cache shrank) + attention summed over queries.  A carried
        accumulation of another float dtype than the new attention is promoted as torch does
        (`acc * decay` rounded in its own dtype, the sum in float32, a float32 result: :129-151)."""
        if attentions is None:
            return
        groups = {}
        threads = self._threads()
        for layer_idx, attn in enumerate(attentions):
            if layer_idx in skip_layers or attn is None:
                continue
            b, h, q, key_len = attn.shape
            _check_gpu(attn, f"attention of layer {layer_idx}")
            if attn.stride(3) != 1 or attn.data_ptr() % attn.element_size():
                attn = attn.contiguous()
            # the q-sum's thread chunks follow the attention the reference sums (:116), before
            # any broadcast below
            chunk = CO.attn_sum_chunk(attn, threads)
            acc = self.accumulated_attention.get(layer_idx)
            old = None
            if acc is not None and acc.size(-1) <= key_len:  # decay (and zero-extend) (:124-146)
                _check_gpu(acc, f"accumulated attention of layer {layer_idx}")
                if acc.device != attn.device:  # torch.cat / + raise the same way
                    raise RuntimeError(
                        f"layer {layer_idx}: accumulated attention on {acc.device}, new attention "
                        f"on {attn.device}: expected all tensors to be on the same device")
                if acc.shape[:2] != attn.shape[:2]:
                    if acc.size(-1) != key_len:  # torch.cat of differing batch / heads (:135)
                        raise RuntimeError(
                            f"layer {layer_idx}: Sizes of tensors must match except in dimension "
                            f"2 (accumulated attention {tuple(acc.shape)}, zero padding "
                            f"{(b, h, key_len - acc.size(-1))})")
                    # equal lengths: `acc * decay + attn.sum(dim=2)` (:146-151) broadcasts --
                    # every element's arithmetic is the same as without the broadcast
                    try:
                        shp = torch.broadcast_shapes(tuple(acc.shape), (b, h, key_len))
                    except RuntimeError as e:
                        raise RuntimeError(f"layer {layer_idx}: {e}") from None
                    b, h = shp[0], shp[1]
                    acc = acc.expand(b, h, key_len)
                    attn = attn.expand(b, h, q, key_len)
                old = acc.contiguous()
            # acc.size(-1) > key_len: reset to zeros (:138-144) -- old stays None
            key = (attn.get_device(), attn.dtype, b, h, attn.dtype if old is None else old.dtype)
            groups.setdefault(key, []).append((layer_idx, attn, old, chunk))
            self.current_seq_len = key_len
        for (device, dtype, b, h, odt), jobs in groups.items():
            with torch.cuda.device(device):
                sizes = [b * h * a.size(3) for _, a, _, _ in jobs]
                ndt = dtype if odt == dtype else torch.float32  # torch's promotion (:129-151)
                buf = torch.empty(sum(sizes), dtype=ndt, device=torch.device("cuda", device))
                accs = [t.view(b, h, a.size(3)) for t, (_, a, _, _) in zip(buf.split(sizes), jobs)]
                table = np.zeros(len(jobs), dtype=N.ATTN_LAYER_DTYPE)
                for i, ((li, a, old, chunk), acc) in enumerate(zip(jobs, accs)):
                    table[i] = (a.data_ptr(), a.stride()[:3],
                                old.data_ptr() if old is not None else 0, acc.data_ptr(),
                                a.size(2), a.size(3), old.size(-1) if old is not None else 0,
                                chunk)
                p = _attn_params(dtype, b, h, self.decay_factor, device, odt)
                rc = N.attn_accumulate(p, table, torch.cuda.current_stream(device).cuda_stream)
                N.check(rc, "kvc_attn_accumulate")
                for (li, _, _, _), acc in zip(jobs, accs):
                    self.accumulated_attention[li] = acc

    def _hh_row(self, layer_idx, seq_len):
        """(acc, m0, m, k) of a layer's heavy-hitter selection (h2o_attention.py:183-206), or
        None when the middle region is empty."""
        acc = self.accumulated_attention[layer_idx]
        attn_len = acc.shape[-1]
        m0, m1 = self.start_size, min(seq_len, attn_len) - self.recent_size
        if m1 <= m0:
            return None
        return acc, m0, m1 - m0, min(self.heavy_hitter_size, m1 - m0)

    @E.status_checked
    def get_heavy_hitter_indices(self, layer_idx: int, seq_len: int) -> torch.Tensor:
        """h2o_attention.py:156-213: ascending middle-local indices of the heavy hitters ([k], or
        [B, k] for batch > 1), computed by the engine."""
        if layer_idx not in self.accumulated_attention:  # evenly spaced middle positions
            m0, m1 = self.start_size, seq_len - self.recent_size
            if m1 <= m0:
                return torch.tensor([], dtype=torch.long)
            step = max(1, (m1 - m0) // self.heavy_hitter_size)
            return torch.arange(0, m1 - m0, step)[:self.heavy_hitter_size]
        acc = self.accumulated_attention[layer_idx]
        row = self._hh_row(layer_idx, seq_len)
        if row is None:
            return torch.tensor([], dtype=torch.long, device=acc.device)
        B = acc.shape[0]
        k = row[3]
        out = torch.empty((B, max(k, 1)), dtype=torch.int32, device=acc.device)
        run_heavy_hitters(self, [row], out.data_ptr(), out.size(1),
                          torch.cuda.current_stream(acc.device))
        top = out[:, :k].long()
        return top.squeeze(0) if B == 1 else top


def run_heavy_hitters(mgr, rows, out_ptr, out_stride, stream):
    """kvc_heavy_hitters over `rows` [(acc, m0, m, k)]: row i * B + b of the int32 array at
    out_ptr (row stride out_stride) receives the k ascending indices.  One launch when every
    accumulation shares dtype, batch, heads and device; otherwise one per run of such rows (a
    layer whose accumulation was promoted to float32, h2o_attention.py:129-151)."""
    B = rows[0][0].shape[0]
    runs, start = [], 0
    for i in range(1, len(rows) + 1):
        a, b = rows[start][0], rows[i][0] if i < len(rows) else None
        if b is None or b.dtype != a.dtype or b.shape[:2] != a.shape[:2] or b.device != a.device:
            runs.append((start, i))
            start = i
    for s0, s1 in runs:
        if rows[s0][0].shape[0] != B:
            raise RuntimeError("heavy hitters of layers with different batch sizes in one call")
        _run_hh(mgr, rows[s0:s1], out_ptr + s0 * B * out_stride * 4, out_stride, stream)


def _run_hh(mgr, rows, out_ptr, out_stride, stream):
    acc0 = rows[0][0]
    _check_gpu(acc0, "accumulated attention")
    B, H = acc0.shape[:2]
    threads = mgr._threads()
    table = np.zeros(len(rows), dtype=N.HH_LAYER_DTYPE)
    keep = []
    for i, (acc, m0, m, k) in enumerate(rows):
        acc = acc.contiguous()
        keep.append(acc)
        table[i] = (acc.data_ptr(), acc.shape[-1], m0, m, k,
                    CO.head_sum_chunk(B, H, m, acc.element_size(), threads), 0)
    device = acc0.get_device()
    p = _attn_params(acc0.dtype, B, H, mgr.decay_factor, device)
    rc, nbytes = N.hh_workspace(p, table)
    N.check(rc, "kvc_hh_workspace")
    ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=acc0.device)
    rc = N.heavy_hitters(p, table, out_ptr, out_stride, ws.data_ptr(), nbytes, stream.cuda_stream)
    N.check(rc, "kvc_heavy_hitters")


@E.status_checked
def h2o_attention_compress(past_key_values, attention_scores: Optional[Tuple] = None,
                           h2o_manager: Optional[H2OAttentionManager] = None,
                           start_size: int = 4, heavy_hitter_size: int = 64,
                           recent_size: int = 444, skip_layers: List[int] = [],
                           **kwargs) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """h2o_attention.py:216-363.  A repeated decode-step shape with a manager is replayed by the
    native host path (_replay_step); everything else runs the per-layer logic below."""
    past_key_values = list(normalize_kv_cache(past_key_values))
    if not past_key_values:
        return past_key_values
    if h2o_manager is not None and attention_scores is not None:
        out = _replay_step(past_key_values, attention_scores, h2o_manager, start_size,
                           heavy_hitter_size, recent_size, skip_layers)
        if out is not None:
            return out
    total_cache_size = start_size + heavy_hitter_size + recent_size
    if h2o_manager is not None and attention_scores is not None:
        h2o_manager.update_attention_scores(attention_scores, skip_layers)
    hh_jobs, host_jobs, norm_jobs = [], [], []  # (Segments, hh row | host indices)
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if seq_len <= total_cache_size or layer_idx in skip_layers:
            continue
        b, h, _, d = keys.shape
        sink = E.py_slice(seq_len, None, start_size)[1]
        t0, tl = E.py_slice(seq_len, -recent_size)
        middle_start, middle_end = start_size, seq_len - recent_size
        if middle_end <= middle_start:  # sinks ++ recent (StreamingLLM fallback)
            seg = E.Segments(layer_idx, keys, values, sink_len=sink, tail_start=t0, tail_len=tl)
            (host_jobs if h2o_manager is not None else norm_jobs).append((seg, None))
            continue
        z0, zl = E.py_slice(seq_len, middle_start, middle_end)
        if h2o_manager is None:  # L2-norm heavy hitters (= h2o_l2's selection)
            norm_jobs.append((E.Segments(layer_idx, keys, values, sink_len=sink, zone_start=z0,
                                         zone_len=zl,
                                         n_select=len(range(zl)[:min(heavy_hitter_size, zl)]),
                                         tail_start=t0, tail_len=tl), None))
            continue
        seg = E.Segments(layer_idx, keys, values, sink_len=sink, zone_start=z0, zone_len=zl,
                         tail_start=t0, tail_len=tl)
        if layer_idx in h2o_manager.accumulated_attention:
            acc = h2o_manager.accumulated_attention[layer_idx]
            row = h2o_manager._hh_row(layer_idx, seq_len)
            if row is not None and acc.shape[0] == 1 and b == 1:
                # heavy_indices[:num] (:318-321): the first num of the k ascending indices; the
                # clamp to the middle (:324) never binds when the manager's middle fits in it.
                # (K/V batch > 1 with a batch-1 accumulation: the reference broadcasts its 1-D
                # index list over the K/V batch (:327-330) -- the host-index path below does.)
                seg.n_select = min(row[3], heavy_hitter_size, zl)
                hh_jobs.append((seg, row))
                continue
            idx = h2o_manager.get_heavy_hitter_indices(layer_idx, seq_len)
        else:
            idx = h2o_manager.get_heavy_hitter_indices(layer_idx, seq_len)
        num = min(len(idx), heavy_hitter_size, zl)
        if num > 0 and len(idx) > 0:
            idx = idx[:num].clamp(0, zl - 1).to(keys.device)
            # the reference's index expansion (same shape rules / errors), shared by all heads
            idx.unsqueeze(0).unsqueeze(0).unsqueeze(-1).expand(b, h, num, d)
            seg.n_select = num
            host_jobs.append((seg, idx))
        else:
            host_jobs.append((seg, None))
    if hh_jobs or host_jobs:
        _compact_shared(h2o_manager, hh_jobs + host_jobs, len(hh_jobs), past_key_values)
    E.execute([s for s, _ in norm_jobs], past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


# heavy-hitter middles at least this long copy their fixed rows beside the selection (a side
# stream, throttled so that the selection keeps its CUs).  Under the stable policy too: the long
# call is then bound by the copy, and the side copy still measured ahead of one copy after the
# selection (0.144 vs 0.148-0.154 ms; unthrottled side copies: reference 0.155 -> 0.216 ms)
OVERLAP_MIN_ZONE = 4096


def _overlap(max_zone):
    return max_zone >= OVERLAP_MIN_ZONE


def _compact_shared(mgr, jobs, n_hh, out_list):
    """One shared-index gather for the manager path: the index rows of the first n_hh jobs come
    from kvc_heavy_hitters (written in place when every row fits), the rest from host indices.
    Within each engine group the heavy-hitter jobs keep their leading positions."""
    idx_of = {s.layer_idx: extra for s, extra in jobs}
    hh_layers = {s.layer_idx for s, _ in jobs[:n_hh]}

    def fill(js, region, stride, stream):
        B = js[0].keys.shape[0]
        hh = [(i, idx_of[s.layer_idx]) for i, s in enumerate(js) if s.layer_idx in hh_layers]
        if hh:
            rows = [r for _, r in hh]
            zl = [js[i].zone_len for i, _ in hh]
            direct = all(r[3] <= stride and r[3] == js[i].n_select and r[2] <= zl_i
                         for (i, r), zl_i in zip(hh, zl))
            if direct:  # rows 0 .. n_hh*B - 1 of the region, in table order
                run_heavy_hitters(mgr, rows, region, stride, stream)
            else:  # manager k > compress heavy_hitter_size, or a middle longer than the zone
                kmax = max(r[3] for r in rows)
                tmp = torch.empty((len(rows) * B, kmax), dtype=torch.int32,
                                  device=js[0].keys.device)
                run_heavy_hitters(mgr, rows, tmp.data_ptr(), kmax, stream)
                reg = _region_view(region, len(js) * B, stride, js[0].keys.device)
                for (i, r), zl_i in zip(hh, zl):
                    n = js[i].n_select
                    if n:
                        reg[i * B:(i + 1) * B, :n] = tmp[i * B:(i + 1) * B, :n].clamp(0, zl_i - 1)
        host = [(i, idx_of[s.layer_idx]) for i, s in enumerate(js)
                if s.layer_idx not in hh_layers]
        if any(x is not None for _, x in host):
            reg = _region_view(region, len(js) * B, stride, js[0].keys.device)
            for i, x in host:
                if x is not None:
                    reg[i * B:(i + 1) * B, :x.numel()] = x.to(torch.int32)
    # long middles: the heavy-hitter selection takes a while, so the sink / recent rows copy
    # beside it on a side stream
    overlap = _overlap(max((s.zone_len for s, _ in jobs[:n_hh]), default=0))
    E.execute_shared([s for s, _ in jobs], out_list, fill, overlap=overlap)


# ---------------------------------------------------------------------------------------------
# Decode steps replayed natively: a repeated (shapes, kwargs, manager settings) step is three
# engine calls whose tables are fixed up to their pointers (kvc_host.run_h2o)
# ---------------------------------------------------------------------------------------------
step_memo = E._PlanCache(capacity=8)
step_stats = {"replayed": 0, "planned": 0}
replay_steps = True  # False: every step takes the Python path (tests compare the two)
_NO_PLAN = object()  # step_memo entry of a shape that stays on the Python path


class _StepPlan:
    __slots__ = ("a_layers", "a_table", "a_params", "hh_rows", "hh_table", "hh_ws", "idx",
                 "idx_stride", "actions", "table", "n_outs", "params", "ws", "info", "seq_len",
                 "p_fixed", "p_sel")


def _replay_step(kvl, attention_scores, mgr, start_size, heavy_hitter_size, recent_size,
                 skip_layers):
    """The step's outputs from kvc_host.run_h2o, with the manager's state updated as
    update_attention_scores would, or None when the step takes the Python path (no host module,
    a timer or recording active, a first sighting, or a shape outside _plan_step's case)."""
    hm = E.host_module() if replay_steps else None
    if hm is None or E._timer is not None or E._recording is not None:
        return None
    if not isinstance(attention_scores, (tuple, list)):
        return None
    accs = [mgr.accumulated_attention.get(i) for i in range(len(attention_scores))]
    sig = hm.scan_h2o(kvl, attention_scores, accs)
    if sig is None:
        return None
    try:
        key = (sig, start_size, heavy_hitter_size, recent_size, E._freeze(skip_layers),
               mgr.start_size, mgr.heavy_hitter_size, mgr.recent_size,
               float(np.float32(mgr.decay_factor)), mgr._threads(), E.split_select_gather,
               E.tie_policy, torch.cuda.current_stream(sig[4]).cuda_stream)
    except TypeError:
        return None
    plan = step_memo.get(key)
    if plan is _NO_PLAN:  # a shape _plan_step does not cover: the Python path, unplanned
        return None
    if plan is None:
        if not step_memo.admit(key):
            return None
        with torch.cuda.device(sig[4]):
            plan = _plan_step(kvl, attention_scores, accs, mgr, start_size, heavy_hitter_size,
                              recent_size, skip_layers)
        if plan is None:
            step_memo.put(key, _NO_PLAN, 0)
            return None
        step_memo.put(key, plan, int(plan.ws.numel()) + int(plan.hh_ws.numel()))
        step_stats["planned"] += 1
    step_stats["replayed"] += 1
    with torch.cuda.device(sig[4]):
        out, acc = hm.run_h2o(
            kvl, attention_scores, accs, plan.a_layers, plan.a_table.ctypes.data,
            E.ctypes_addr(plan.a_params), plan.hh_rows, plan.hh_table.ctypes.data,
            plan.hh_ws.data_ptr(), int(plan.hh_ws.numel()), plan.idx, plan.idx_stride,
            plan.actions, plan.table.ctypes.data, len(plan.table), plan.n_outs,
            E.ctypes_addr(plan.params), plan.ws.data_ptr(), int(plan.info.workspace_bytes),
            key[-1], E.ctypes_addr(plan.p_fixed) if plan.p_fixed is not None else 0,
            E.ctypes_addr(plan.p_sel) if plan.p_sel is not None else 0)
    for li, a in zip(plan.a_layers, acc):
        mgr.accumulated_attention[li] = a
    mgr.current_seq_len = plan.seq_len
    return out


def _plan_step(kvl, attns, accs, mgr, start_size, heavy_hitter_size, recent_size, skip_layers):
    """Tables of one step -- the same branch logic and arithmetic as update_attention_scores +
    h2o_attention_compress above, pointer columns left to run_h2o -- for the case where every
    compressed layer takes its heavy hitters straight from this step's accumulation (batch 1,
    one attention group, the manager's k equal to the kept count); else None."""
    L = len(kvl)
    if len(attns) != L:
        return None
    threads = mgr._threads()
    a_layers, a_rows, acc_len, grp = [], [], {}, None
    seq_len = mgr.current_seq_len
    for li, attn in enumerate(attns):  # update_attention_scores (:84-153)
        if li in skip_layers or attn is None:
            continue
        b, h, q, key_len = attn.shape
        g = (attn.dtype, b, h, attn.get_device())
        if grp is None:
            grp = g
        elif g != grp:
            return None
        acc = accs[li]
        old_len = 0
        if acc is not None and acc.size(-1) <= key_len:
            if acc.dtype != attn.dtype or acc.device != attn.device or \
                    acc.shape[:2] != attn.shape[:2]:
                return None  # mixed dtypes (promotion) / other devices: the Python path
            old_len = acc.size(-1)
        a_layers.append(li)
        a_rows.append((0, attn.stride()[:3], 0, 0, q, key_len, old_len,
                       CO.attn_sum_chunk(attn, threads)))
        acc_len[li] = key_len
        seq_len = key_len
    if (not a_layers or grp[1] != 1 or grp[3] != kvl[0][0].get_device() or
            kvl[0][0].shape[0] != 1):
        return None
    adt, _, AH, device = grp
    total_cache_size = start_size + heavy_hitter_size + recent_size
    actions = np.zeros((L, 3), dtype=np.int64)
    segs, hh = [], []
    for layer_idx, (keys, values) in enumerate(kvl):  # h2o_attention_compress (:262-361)
        S = keys.size(2)
        if S <= total_cache_size or layer_idx in skip_layers:
            continue
        if start_size >= S - recent_size or layer_idx not in acc_len:
            return None
        attn_len = acc_len[layer_idx]  # _hh_row
        m0, m1 = mgr.start_size, min(S, attn_len) - mgr.recent_size
        if m1 <= m0:
            return None
        k = min(mgr.heavy_hitter_size, m1 - m0)
        sink = E.py_slice(S, None, start_size)[1]
        t0, tl = E.py_slice(S, -recent_size)
        z0, zl = E.py_slice(S, start_size, S - recent_size)
        n_sel = min(k, heavy_hitter_size, zl)
        if n_sel != k or m1 - m0 > zl:  # not the direct case of _compact_shared
            return None
        actions[layer_idx] = (2, len(segs), 0)
        segs.append((S, z0, zl, n_sel, sink, t0, tl))
        hh.append((a_layers.index(layer_idx), attn_len, m0, m1 - m0, k,
                   CO.head_sum_chunk(1, AH, m1 - m0, _esize(adt), threads)))
    if not segs:
        return None
    B, H, _, D = kvl[0][0].shape
    plan = _StepPlan()
    plan.a_layers = a_layers
    plan.a_table = np.array(a_rows, dtype=N.ATTN_LAYER_DTYPE)
    plan.a_params = _attn_params(adt, 1, AH, mgr.decay_factor, device)
    plan.hh_rows = [r[0] for r in hh]
    plan.hh_table = np.zeros(len(hh), dtype=N.HH_LAYER_DTYPE)
    for i, (_, alen, m0, m, k, chunk) in enumerate(hh):
        plan.hh_table[i] = (256, alen, m0, m, k, chunk, 0)  # stand-in acc pointer
    rc, nbytes = N.hh_workspace(plan.a_params, plan.hh_table)
    N.check(rc, "kvc_hh_workspace")
    plan.hh_table["acc"] = 0
    plan.hh_ws = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=keys.device)
    table = np.zeros(len(segs), dtype=N.LAYER_DTYPE)
    arr = np.array(segs, dtype=np.int64)
    S_ = arr[:, 0]
    st = np.stack([H * S_ * D, S_ * D, np.full_like(S_, D)], axis=1)
    table["k_stride"] = st
    table["v_stride"] = st
    for c, name in enumerate(("seq_len", "zone_start", "zone_len", "n_select", "sink_len",
                              "tail_start", "tail_len")):
        table[name] = arr[:, c]
    for name in ("k", "v", "k_out", "v_out"):
        table[name] = 256
    p = E._params(keys.dtype, B, H, D, N.KVC_ASC, N.KVC_ALGO_SORT, True, shared=True)
    rc, info = N.plan(p, table)
    N.check(rc, "kvc_plan")
    if max(r[4] for r in hh) > int(info.index_row_stride):
        return None
    for name in ("k", "v", "k_out", "v_out"):
        table[name] = 0
    plan.table, plan.params, plan.info = table, p, info
    plan.p_fixed = plan.p_sel = None
    if _overlap(max(r[3] for r in hh)):  # as _compact_shared: fixed rows beside
        plan.p_fixed = E._params(keys.dtype, B, H, D, N.KVC_ASC, N.KVC_ALGO_SORT, True, shared=True)
        plan.p_fixed.flags |= N.FLAG_GATHER_FIXED
        plan.p_sel = E._params(keys.dtype, B, H, D, N.KVC_ASC, N.KVC_ALGO_SORT, True, shared=True)
        plan.p_sel.flags |= N.FLAG_GATHER_SELECTED
    plan.n_outs = [int(x) for x in arr[:, 4] + arr[:, 3] + arr[:, 6]]
    plan.ws = torch.empty(max(int(info.workspace_bytes), 256), dtype=torch.uint8,
                          device=keys.device)
    plan.idx = plan.ws.data_ptr() + int(info.index_offset)
    plan.idx_stride = int(info.index_row_stride)
    plan.actions = actions
    plan.seq_len = seq_len
    return plan


def _esize(dtype):
    return torch.empty(0, dtype=dtype).element_size()


def _region_view(ptr, rows, stride, device):
    """The int32 index region at device address `ptr` as a [rows, stride] tensor (it lives in a
    workspace the caller keeps alive until the launch)."""
    class _Mem:  # minimal __cuda_array_interface__ provider
        __cuda_array_interface__ = dict(shape=(rows, stride), typestr="<i4", data=(ptr, False),
                                        version=3, strides=None)
    with torch.cuda.device(device):
        return torch.as_tensor(_Mem(), device=device)


def create_h2o_manager_from_model(model, **kwargs) -> H2OAttentionManager:
    """h2o_attention.py:366-391"""
    config = model.config
    return H2OAttentionManager(
        start_size=kwargs.get("start_size", 4),
        heavy_hitter_size=kwargs.get("heavy_hitter_size", 64),
        recent_size=kwargs.get("recent_size", 444),
        num_layers=getattr(config, "num_hidden_layers", 32),
        num_heads=getattr(config, "num_attention_heads", 32),
        decay_factor=kwargs.get("decay_factor", 0.9),
        device=next(model.parameters()).device,
    )


__all__ = ["H2OAttentionManager", "h2o_attention_compress", "create_h2o_manager_from_model"]
