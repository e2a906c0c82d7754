"""H2O with attention-score heavy hitters (reference: kvcompress/methods/h2o_attention.py).

The manager keeps the reference's per-layer accumulated attention (sum over queries, exponential
decay, zero-extension, reset when the cache shrank) and picks heavy hitters as the top-k of the
head-summed middle region (h2o_attention.py:84-213).  That bookkeeping is a few small torch ops
on the attention tensors' own device -- the same ops as the reference, so the same results on the
same device.  The compaction -- sinks ++ K/V rows of the heavy hitters (one index list shared by
every head) ++ recent window, for every layer of the call -- runs as one HIP engine launch
(external-index GATHER).  Without a manager the reference falls back to L2-norm heavy hitters,
which is exactly h2o_l2's selection: the engine's score / select / gather path.
"""
from typing import Dict, List, Optional, Tuple

import torch

from .. import _engine as E
from .. import _native as N
from ..utils import normalize_kv_cache


class H2OAttentionManager:
    """Accumulated attention per layer (h2o_attention.py:27-213): same constructor, state and
    methods as the reference."""

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

    def reset(self):
        self.accumulated_attention = {}
        self.token_positions = {}
        self.current_seq_len = 0

    def update_attention_scores(self, attentions, skip_layers: List[int] = []):
        """h2o_attention.py:84-153: acc <- acc*decay (zero-extended to the new key length, or
        reset if the cache shrank) + attention summed over queries."""
        if attentions is None:
            return
        for layer_idx, attn in enumerate(attentions):
            if layer_idx in skip_layers or attn is None:
                continue
            b, h, _, key_len = attn.shape
            importance = attn.sum(dim=2)
            acc = self.accumulated_attention.get(layer_idx)
            if acc is None:
                acc = torch.zeros(b, h, key_len, device=attn.device, dtype=attn.dtype)
            elif acc.size(-1) < key_len:
                pad = torch.zeros(b, h, key_len - acc.size(-1), device=attn.device,
                                  dtype=attn.dtype)
                acc = torch.cat([acc * self.decay_factor, pad], dim=-1)
            elif acc.size(-1) > key_len:
                acc = torch.zeros(b, h, key_len, device=attn.device, dtype=attn.dtype)
            else:
                acc = acc * self.decay_factor
            self.accumulated_attention[layer_idx] = acc + importance
            self.current_seq_len = key_len

    def get_heavy_hitter_indices(self, layer_idx: int, seq_len: int) -> torch.Tensor:
        """h2o_attention.py:155-213: ascending middle-local indices of the heavy hitters."""
        acc = self.accumulated_attention.get(layer_idx)
        if acc is None:  # no attention yet: evenly spaced middle positions
            m0, m1 = self.start_size, seq_len - self.recent_size
            if m1 <= m0:
                return torch.tensor([], dtype=torch.long)
            step = max(1, (m1 - m0) // self.heavy_hitter_size)
            return torch.arange(0, m1 - m0, step)[:self.heavy_hitter_size]
        b, _, attn_len = acc.shape
        m0, m1 = self.start_size, min(seq_len, attn_len) - self.recent_size
        if m1 <= m0:
            return torch.tensor([], dtype=torch.long, device=acc.device)
        agg = acc[:, :, m0:m1].sum(dim=1)
        if b == 1:
            agg = agg.squeeze(0)
        _, top = torch.topk(agg, min(self.heavy_hitter_size, m1 - m0), dim=-1)
        top, _ = torch.sort(top, dim=-1)
        return top


def h2o_attention_compress(past_key_values, attention_scores: Optional[Tuple] = None,
                           h2o_manager: Optional[H2OAttentionManager] = None,
                           start_size: int = 4, heavy_hitter_size: int = 64,
                           recent_size: int = 444, skip_layers: List[int] = [],
                           **kwargs) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """h2o_attention.py:216-376."""
    past_key_values = list(normalize_kv_cache(past_key_values))
    if not past_key_values:
        return past_key_values
    total_cache_size = start_size + heavy_hitter_size + recent_size
    if h2o_manager is not None and attention_scores is not None:
        h2o_manager.update_attention_scores(attention_scores, skip_layers)
    ext_jobs, norm_jobs = [], []
    for layer_idx, (keys, values) in enumerate(past_key_values):
        seq_len = keys.size(2)
        if seq_len <= total_cache_size or layer_idx in skip_layers:
            continue
        b, h, _, d = keys.shape
        sink = E.py_slice(seq_len, None, start_size)[1]
        t0, tl = E.py_slice(seq_len, -recent_size)
        middle_start, middle_end = start_size, seq_len - recent_size
        jobs = ext_jobs if h2o_manager is not None else norm_jobs
        if middle_end <= middle_start:  # sinks ++ recent (StreamingLLM fallback)
            jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, tail_start=t0,
                                   tail_len=tl))
            continue
        z0, zl = E.py_slice(seq_len, middle_start, middle_end)
        if h2o_manager is None:  # L2-norm heavy hitters (= h2o_l2's selection)
            norm_jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, zone_start=z0,
                                        zone_len=zl,
                                        n_select=len(range(zl)[:min(heavy_hitter_size, zl)]),
                                        tail_start=t0, tail_len=tl))
            continue
        idx = h2o_manager.get_heavy_hitter_indices(layer_idx, seq_len)
        num = min(len(idx), heavy_hitter_size, zl)
        ext = None
        if num > 0 and len(idx) > 0:
            idx = idx[:num].clamp(0, zl - 1).to(keys.device)
            # the reference's index expansion (same shape rules / errors), shared by all heads
            ext = idx.unsqueeze(0).unsqueeze(0).unsqueeze(-1).expand(b, h, num, d)[..., 0]
        else:
            num = 0
        ext_jobs.append(E.Segments(layer_idx, keys, values, sink_len=sink, zone_start=z0,
                                   zone_len=zl, n_select=num, tail_start=t0, tail_len=tl,
                                   ext_index=ext))
    E.execute(ext_jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    E.execute(norm_jobs, past_key_values, N.KVC_ASC, N.KVC_ALGO_SORT)
    return past_key_values


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
