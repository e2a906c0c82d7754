"""h2o_attention's heavy-hitter scoring on the HIP engine vs the CPU reference (GPU tests).

* the unmodified reference's outputs on tie-heavy, non-dyadic attention
  (tests/golden/h2o_attention_ties.json): every layer's accumulated-attention bytes after every
  step, the heavy-hitter indices and the compressed K/V, in fp32 / bf16 / fp16;
* torch's own CPU ops (the reference's arithmetic) on random attention, across shapes and
  thread counts: the engine's q-sum / decay / head-sum / top-k against torch CPU.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import h2o_inputs  # noqa: E402
import prng  # noqa: E402
from gen_h2o_attention_ties import att_seed, kv_seed  # noqa: E402
from gpu_util import to_dev, to_np  # noqa: E402

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(HERE, "golden", "h2o_attention_ties.json")))


def sha(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(str(a.shape).encode() + a.tobytes()).hexdigest()


@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("si", [0, 1])
def test_engine_replays_reference_tie_goldens(si, dt):
    from kvcompress.methods.h2o_attention import H2OAttentionManager, h2o_attention_compress
    sc = GOLD["scenarios"][si]
    H, D, L = GOLD["H"], GOLD["D"], GOLD["layers"]
    mgr = H2OAttentionManager(decay_factor=sc["decay"], num_layers=L, num_heads=H, **sc["kw"])
    mgr.reduction_threads = GOLD["threads"]  # the generating process's torch threads
    recs = GOLD["results"][f"{sc['name']}/{dt}"]
    for st, step in enumerate(sc["steps"]):
        k = step["k"] if step["op"] == "update" else step["S"]
        atts = tuple(to_dev(h2o_inputs.attention(att_seed(si, st, li), H, step["q"], k, dt))
                     if step["att"][li] else None for li in range(L))
        rec = recs[st]
        if step["op"] == "update":
            mgr.update_attention_scores(atts, skip_layers=step["skip"])
            S = k
        else:
            S = step["S"]
            kv = [(to_dev(prng.gen_keys(kv_seed(si, st, li), (1, H, S, D), dt)),
                   to_dev(prng.gen_values(kv_seed(si, st, li), (1, H, S, D), dt)))
                  for li in range(L)]
            out = h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                         skip_layers=step["skip"], **sc["kw"])
            for li in range(L):
                assert out[li][0].shape[2] == rec["n_out"][li], (st, li)
                assert sha(to_np(out[li][0])) == rec["k"][li], ("K", st, li)
                assert sha(to_np(out[li][1])) == rec["v"][li], ("V", st, li)
        for li in range(L):
            acc = mgr.accumulated_attention.get(li)
            assert (None if acc is None else sha(to_np(acc))) == rec["acc"][li], ("acc", st, li)
            got = mgr.get_heavy_hitter_indices(li, S)
            assert got.cpu().tolist() == rec["idx"][li], ("idx", st, li)
            if acc is not None and len(rec["idx"][li]):
                assert got.device == acc.device and got.dtype == torch.int64
    from kvcompress import _engine
    assert _engine.device_status(0) == 0


TORCH_DT = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}


def _tie_attention(rng, shape, levels=4):
    """Softmax rows over a few distinct logits (ties within and across heads), fp32."""
    logits = rng.integers(0, levels, size=shape).astype(np.float32) * np.float32(0.7)
    x = torch.from_numpy(logits).softmax(dim=-1)
    return x


@pytest.mark.parametrize("threads", [1, 8, 16, 33])
@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp16"])
def test_engine_matches_torch_cpu_ops(threads, dt):
    """update_attention_scores over three steps (first, extend, equal, reset) and
    get_heavy_hitter_indices against the reference's arithmetic executed by torch on the CPU with
    `threads` threads: attn.sum(dim=2), acc * decay, cat / zeros, acc + imp, head sum, topk."""
    from kvcompress.methods.h2o_attention import H2OAttentionManager
    rng = np.random.default_rng(threads)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        for B, H, steps, hh in [(1, 32, [(37, 1500), (1, 1501), (3, 1501), (1, 700)], 64),
                                (1, 8, [(300, 2000), (1, 2001)], 16),
                                (1, 4, [(5, 100), (17, 120)], 8),
                                (1, 1, [(2, 3000), (1, 3001)], 32),
                                (2, 16, [(9, 1100), (1, 1101)], 40),
                                (1, 8, [(1, 6000)], 64),  # heap select, 512-thread rows
                                (1, 32, [(1, 16384)], 64)]:  # heap select over 16 330
            mgr = H2OAttentionManager(start_size=4, heavy_hitter_size=hh, recent_size=50,
                                      decay_factor=0.9)
            mgr.reduction_threads = threads
            acc_ref = None
            for q, k in steps:
                attn = _tie_attention(rng, (B, H, q, k)).to(TORCH_DT[dt])
                mgr.update_attention_scores((attn.to("cuda:0"),))
                imp = attn.sum(dim=2)  # the reference's ops (h2o_attention.py:116-151), CPU
                if acc_ref is None or acc_ref.size(-1) > k:
                    acc_ref = torch.zeros(B, H, k, dtype=attn.dtype)
                elif acc_ref.size(-1) < k:
                    acc_ref = torch.cat([acc_ref * 0.9, torch.zeros(B, H, k - acc_ref.size(-1),
                                                                    dtype=attn.dtype)], dim=-1)
                else:
                    acc_ref = acc_ref * 0.9
                acc_ref = acc_ref + imp
                got = mgr.accumulated_attention[0]
                assert np.array_equal(to_np(got).view(np.uint8), to_np(acc_ref).view(np.uint8)), \
                    (B, H, q, k)
                m1 = k - 50
                agg = acc_ref[:, :, 4:m1].sum(dim=1)
                if B == 1:
                    agg = agg.squeeze(0)
                _, top = torch.topk(agg, min(hh, m1 - 4), dim=-1)
                top, _ = torch.sort(top, dim=-1)
                assert mgr.get_heavy_hitter_indices(0, k).cpu().tolist() == top.tolist(), \
                    (B, H, q, k)
    finally:
        torch.set_num_threads(prev)


def test_shared_index_gather_and_index_range_status():
    """C-ABI level: a KVC_FLAG_SHARED_INDEX gather reads row (layer*B + b) for every head, and an
    external index outside its zone is clamped AND reported through params.device_status."""
    from kvcompress import _native as N
    H, S, D = 4, 256, 64
    k = torch.arange(H * S * D, dtype=torch.float32, device="cuda:0").reshape(1, H, S, D)
    v = -k
    n_sel = 3
    ko = torch.empty(1, H, n_sel, D, device="cuda:0")
    vo = torch.empty_like(ko)
    t = np.zeros(1, dtype=N.LAYER_DTYPE)
    t[0] = (k.data_ptr(), v.data_ptr(), ko.data_ptr(), vo.data_ptr(), (H * S * D, S * D, D),
            (H * S * D, S * D, D), S, 10, 100, n_sel, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    status = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    p = N.Params(dtype=N.KVC_F32, batch=1, heads=H, head_dim=D, order=0, algo=0,
                 phases=N.PHASE_GATHER, external_index=1, flags=N.FLAG_SHARED_INDEX,
                 device_status=status.data_ptr())
    rc, info = N.plan(p, t)
    assert rc == 0
    ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device="cuda:0")
    idx = ws[info.index_offset:info.index_offset + 4 * n_sel].view(torch.int32)
    idx.copy_(torch.tensor([5, 7, 99], dtype=torch.int32))
    rc = N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes),
                  torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    want = torch.tensor([15, 17, 109], device="cuda:0")
    assert torch.equal(ko, k[:, :, want]) and torch.equal(vo, v[:, :, want])
    assert int(status.item()) == 0
    idx.copy_(torch.tensor([5, 7, 100], dtype=torch.int32))  # zone_len 100: out of range
    assert N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes),
                    torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert int(status.item()) == N.DEV_INDEX_RANGE
    assert torch.equal(ko, k[:, :, want])  # clamped to the zone's last row


@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp16"])
def test_decode_steps_replayed_natively_match_python_path(dt):
    """Repeated decode-step shapes go through kvc_host.run_h2o (accumulate, heavy hitters and the
    shared-index gather from a cached plan): outputs, pass-through objects, the accumulated
    attention and current_seq_len equal the Python path's step for step, and the accumulated
    attention equals torch's CPU arithmetic; a shape change is never served by an old plan."""
    from kvcompress.methods import h2o_attention as HA
    rng = np.random.default_rng(7)
    L, H, D, start, hh, recent = 4, 8, 64, 4, 16, 40
    kw = dict(start_size=start, heavy_hitter_size=hh, recent_size=recent, skip_layers=[1])
    mk = lambda: HA.H2OAttentionManager(start_size=start, heavy_hitter_size=hh,  # noqa: E731
                                        recent_size=recent, decay_factor=0.9)
    mgr_a, mgr_b = mk(), mk()
    HA.step_memo.clear()
    r0 = HA.step_stats["replayed"]
    acc_ref = [None] * L
    n_steps = 0
    for step, S in enumerate([61] * 5 + [62] * 3 + [61] * 2):
        kv = [(to_dev(prng.gen_keys(900 + 10 * step + i, (1, H, S if i != 3 else 30, D), dt)),
               to_dev(prng.gen_values(900 + 10 * step + i, (1, H, S if i != 3 else 30, D), dt)))
              for i in range(L)]
        att_cpu = [_tie_attention(rng, (1, H, 1, S)).to(TORCH_DT[dt]) for _ in range(L)]
        att = tuple(a.to("cuda:0") for a in att_cpu)
        out_a = HA.h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr_a, **kw)
        HA.replay_steps = False
        try:
            out_b = HA.h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr_b,
                                              **kw)
        finally:
            HA.replay_steps = True
        n_steps += 1
        for li in range(L):
            assert (out_a[li] is kv[li]) == (out_b[li] is kv[li]), (step, li)
            for x, y in zip(out_a[li], out_b[li]):
                assert x.shape == y.shape, (step, li)
                assert np.array_equal(to_np(x).view(np.uint8), to_np(y).view(np.uint8)), (step, li)
            if li == 1:  # skipped: never accumulated
                assert li not in mgr_a.accumulated_attention
                continue
            a = mgr_a.accumulated_attention[li]
            b = mgr_b.accumulated_attention[li]
            assert np.array_equal(to_np(a).view(np.uint8), to_np(b).view(np.uint8)), (step, li)
            imp = att_cpu[li].sum(dim=2)
            r = acc_ref[li]
            if r is None or r.size(-1) > S:
                r = torch.zeros(1, H, S, dtype=imp.dtype)
            elif r.size(-1) < S:
                r = torch.cat([r * 0.9, torch.zeros(1, H, S - r.size(-1), dtype=imp.dtype)], -1)
            else:
                r = r * 0.9
            acc_ref[li] = r + imp
            assert np.array_equal(to_np(a).view(np.uint8), to_np(acc_ref[li]).view(np.uint8)), \
                (step, li)
        assert mgr_a.current_seq_len == mgr_b.current_seq_len == S
    # S = 61: steps 0-1 Python (first sightings of two acc shapes), 2-4 replayed; S = 62: 5-6
    # Python, 7 replayed; back at 61: the acc shape of step 8 is new once more (62 > 61: reset)
    assert HA.step_stats["replayed"] - r0 >= 5
    # a shape the plan does not cover (layer 2 compresses with the accumulation of an earlier
    # step: its attention is None now) stays on the Python path, call after call
    r1 = HA.step_stats["replayed"]
    for step in range(4):
        kv = [(to_dev(prng.gen_keys(700 + 10 * step + i, (1, H, 61, D), dt)),
               to_dev(prng.gen_values(700 + 10 * step + i, (1, H, 61, D), dt))) for i in range(L)]
        att = tuple(None if i == 2 else _tie_attention(rng, (1, H, 1, 61)).to(TORCH_DT[dt]).to("cuda:0")
                    for i in range(L))
        out_a = HA.h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr_a, **kw)
        HA.replay_steps = False
        try:
            out_b = HA.h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr_b,
                                              **kw)
        finally:
            HA.replay_steps = True
        for li in range(L):
            for x, y in zip(out_a[li], out_b[li]):
                assert np.array_equal(to_np(x).view(np.uint8), to_np(y).view(np.uint8)), (step, li)
    assert HA.step_stats["replayed"] == r1
    from kvcompress import _engine
    assert _engine.device_status(0) == 0


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_kv_batch_above_attention_batch_broadcasts_indices(dt):
    """K/V batch 2 with a batch-1 accumulation: the reference's 1-D heavy-hitter list is
    broadcast over the K/V batch (h2o_attention.py:318-333); checked against torch's CPU ops."""
    from kvcompress.methods.h2o_attention import H2OAttentionManager, h2o_attention_compress
    rng = np.random.default_rng(3)
    H, S, D, start, hh, recent = 8, 300, 64, 4, 16, 40
    mgr = H2OAttentionManager(start_size=start, heavy_hitter_size=hh, recent_size=recent)
    mgr.reduction_threads = torch.get_num_threads()
    attn = _tie_attention(rng, (1, H, 3, S)).to(TORCH_DT[dt])
    k = torch.from_numpy(rng.standard_normal((2, H, S, D)).astype(np.float32)).to(TORCH_DT[dt])
    v = torch.from_numpy(rng.standard_normal((2, H, S, D)).astype(np.float32)).to(TORCH_DT[dt])
    out = h2o_attention_compress([(k.to("cuda:0"), v.to("cuda:0"))] * 2,
                                 attention_scores=(attn.to("cuda:0"),) * 2, h2o_manager=mgr,
                                 start_size=start, heavy_hitter_size=hh, recent_size=recent)
    acc = torch.zeros(1, H, S, dtype=attn.dtype) + attn.sum(dim=2)  # CPU reference ops
    agg = acc[:, :, start:S - recent].sum(dim=1).squeeze(0)
    idx = torch.sort(torch.topk(agg, hh, dim=-1)[1])[0]
    for x, ref in zip(out[0], (k, v)):
        mid = ref[:, :, start:S - recent]
        want = torch.cat([ref[:, :, :start], mid[:, :, idx], ref[:, :, -recent:]], dim=2)
        assert np.array_equal(to_np(x).view(np.uint8), to_np(want).view(np.uint8))
    assert [x.shape for x in out[1]] == [x.shape for x in out[0]]


MIXED = json.load(open(os.path.join(HERE, "golden", "h2o_attention_mixed.json")))


@pytest.mark.parametrize("si", [0, 1, 2])
def test_engine_replays_reference_mixed_dtype_goldens(si):
    """The carried accumulation and a new step's attention differ in dtype: the engine promotes as
    the reference's `acc * decay`, torch.cat and `+` do (h2o_attention.py:129-151) -- float32
    accumulations, heavy hitters and compressed K/V identical to the unmodified reference's
    (tests/golden/gen_h2o_mixed_dtypes.py).  (A promoting step is never replayed natively: its
    scan_h2o signature carries the accumulations' dtypes and _plan_step declines it.)"""
    from gen_h2o_mixed_dtypes import att_seed as m_att, kv_seed as m_kv
    from kvcompress.methods.h2o_attention import H2OAttentionManager, h2o_attention_compress
    sc = MIXED["scenarios"][si]
    H, D, L, kdt = MIXED["H"], MIXED["D"], MIXED["layers"], MIXED["kv_dtype"]
    name = {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float16: "fp16"}
    mgr = H2OAttentionManager(decay_factor=sc["decay"], num_layers=L, num_heads=H, **sc["kw"])
    mgr.reduction_threads = MIXED["threads"]
    for st, step in enumerate(sc["steps"]):
        k = step["k"] if step["op"] == "update" else step["S"]
        atts = tuple(to_dev(h2o_inputs.attention(m_att(si, st, li), H, step["q"], k, step["dt"]))
                     if step["att"][li] else None for li in range(L))
        rec = MIXED["results"][sc["name"]][st]
        if step["op"] == "update":
            mgr.update_attention_scores(atts, skip_layers=step["skip"])
            S = k
        else:
            S = step["S"]
            kv = [(to_dev(prng.gen_keys(m_kv(si, st, li), (1, H, S, D), kdt)),
                   to_dev(prng.gen_values(m_kv(si, st, li), (1, H, S, D), kdt)))
                  for li in range(L)]
            out = h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                         skip_layers=step["skip"], **sc["kw"])
            for li in range(L):
                assert out[li][0].shape[2] == rec["n_out"][li], (st, li)
                assert sha(to_np(out[li][0])) == rec["k"][li], ("K", st, li)
                assert sha(to_np(out[li][1])) == rec["v"][li], ("V", st, li)
        for li in range(L):
            acc = mgr.accumulated_attention.get(li)
            assert (None if acc is None else name[acc.dtype]) == rec["acc_dtype"][li], (st, li)
            assert (None if acc is None else sha(to_np(acc))) == rec["acc"][li], ("acc", st, li)
            assert mgr.get_heavy_hitter_indices(li, S).cpu().tolist() == rec["idx"][li], (st, li)


def test_fixed_rows_copied_beside_the_selection_match():
    """Middles >= OVERLAP_MIN_ZONE: the sink / recent rows are copied on a side stream while the
    heavy hitters are selected (KVC_FLAG_GATHER_FIXED / _SELECTED), in the Python path and in the
    native step replay; every output equals the single-launch copy's."""
    from kvcompress.methods import h2o_attention as HA
    rng = np.random.default_rng(11)
    L, H, S, D = 3, 8, 6000, 64
    kw = dict(start_size=4, heavy_hitter_size=64, recent_size=444, skip_layers=[])
    kv = [(to_dev(prng.gen_keys(40 + i, (1, H, S, D), "bf16")),
           to_dev(prng.gen_values(40 + i, (1, H, S, D), "bf16"))) for i in range(L)]
    att = tuple(_tie_attention(rng, (1, H, 1, S)).to(torch.bfloat16).to("cuda:0")
                for _ in range(L))
    mk = lambda: HA.H2OAttentionManager(start_size=4, heavy_hitter_size=64,  # noqa: E731
                                        recent_size=444)
    saved = HA.OVERLAP_MIN_ZONE
    try:
        HA.OVERLAP_MIN_ZONE = 1 << 30  # one launch
        HA.replay_steps = False
        ref = HA.h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mk(), **kw)
        HA.OVERLAP_MIN_ZONE = saved
        got = HA.h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mk(), **kw)
        HA.replay_steps = True
        HA.step_memo.clear()
        r0 = HA.step_stats["replayed"]
        mgr = mk()
        for _ in range(4):  # the 3rd and 4th calls are native replays (fresh accumulations)
            mgr.reset()
            rep = HA.h2o_attention_compress(list(kv), attention_scores=att, h2o_manager=mgr, **kw)
        assert HA.step_stats["replayed"] - r0 >= 2
    finally:
        HA.OVERLAP_MIN_ZONE = saved
        HA.replay_steps = True
    for outs in (got, rep):
        for li in range(L):
            for x, y in zip(outs[li], ref[li]):
                assert np.array_equal(to_np(x).view(np.uint8), to_np(y).view(np.uint8)), li


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_equal_length_accumulation_broadcasts_batch_and_heads(dt):
    """`acc * decay + attn.sum(dim=2)` with equal key lengths broadcasts a batch-1 (or head-1)
    accumulation against the new attention and vice versa (h2o_attention.py:146-151), while the
    zero-extension's torch.cat (:135) raises: checked against torch's CPU ops."""
    from kvcompress.methods.h2o_attention import H2OAttentionManager
    rng = np.random.default_rng(5)
    tdt = TORCH_DT[dt]
    for first, second in [((1, 8, 3, 500), (2, 8, 1, 500)), ((2, 8, 3, 500), (1, 8, 2, 500)),
                          ((1, 1, 2, 300), (2, 4, 1, 300))]:
        mgr = H2OAttentionManager(start_size=4, heavy_hitter_size=16, recent_size=40)
        mgr.reduction_threads = torch.get_num_threads()
        a1 = _tie_attention(rng, first).to(tdt)
        a2 = _tie_attention(rng, second).to(tdt)
        mgr.update_attention_scores((a1.to("cuda:0"),))
        mgr.update_attention_scores((a2.to("cuda:0"),))
        ref = (torch.zeros(first[:2] + first[3:], dtype=tdt) + a1.sum(dim=2)) * 0.9 + a2.sum(dim=2)
        got = mgr.accumulated_attention[0]
        assert got.shape == ref.shape, (first, second)
        assert np.array_equal(to_np(got).view(np.uint8), to_np(ref).view(np.uint8)), (first, second)
    mgr = H2OAttentionManager()
    mgr.update_attention_scores((_tie_attention(rng, (1, 8, 1, 500)).to(tdt).to("cuda:0"),))
    with pytest.raises(RuntimeError):  # extension: torch.cat of [1,8,*] and zeros [2,8,*]
        mgr.update_attention_scores((_tie_attention(rng, (2, 8, 1, 501)).to(tdt).to("cuda:0"),))


LONG = json.load(open(os.path.join(HERE, "golden", "h2o_attention_long.json")))


@pytest.mark.parametrize("dt", ["bf16", "fp32"])
@pytest.mark.parametrize("native", [True, False])
def test_long_context_steps_match_reference_golden(dt, native):
    """BASELINE cfg4's geometry against the unmodified reference (tests/golden/
    h2o_attention_long.json): S = 16 384, start 4 / heavy 64 / recent 444, three q = 1 steps.  The
    middle (15 936) is >= OVERLAP_MIN_ZONE, so the sink / recent rows are copied on a side stream
    beside the heavy-hitter selection; with native=True the third step is replayed by
    kvc_host.run_h2o (its fork / join), with native=False every step takes the Python path
    (execute_shared's fork / join).  Accumulations, heavy hitters and K / V are all checked."""
    from gen_h2o_attention_long import att_seed as l_att, kv_seed as l_kv
    from kvcompress.methods import h2o_attention as HA
    H, D, S, L = LONG["H"], LONG["D"], LONG["S"], LONG["layers"]
    assert S - LONG["kw"]["start_size"] - LONG["kw"]["recent_size"] >= HA.OVERLAP_MIN_ZONE
    kv = [(to_dev(prng.gen_keys(l_kv(li), (1, H, S, D), dt)),
           to_dev(prng.gen_values(l_kv(li), (1, H, S, D), dt))) for li in range(L)]
    mgr = HA.H2OAttentionManager(decay_factor=LONG["decay"], num_layers=L, num_heads=H,
                                 **LONG["kw"])
    mgr.reduction_threads = LONG["threads"]
    HA.step_memo.clear()
    r0 = HA.step_stats["replayed"]
    HA.replay_steps = native
    try:
        for st in range(LONG["steps"]):
            atts = tuple(to_dev(h2o_inputs.attention(l_att(st, li), H, 1, S, dt))
                         for li in range(L))
            out = HA.h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                            skip_layers=[], **LONG["kw"])
            rec = LONG["results"][dt][st]
            for li in range(L):
                assert out[li][0].shape[2] == rec["n_out"][li], (st, li)
                assert sha(to_np(out[li][0])) == rec["k"][li], ("K", st, li)
                assert sha(to_np(out[li][1])) == rec["v"][li], ("V", st, li)
                assert sha(to_np(mgr.accumulated_attention[li])) == rec["acc"][li], ("acc", st, li)
                assert mgr.get_heavy_hitter_indices(li, S).cpu().tolist() == rec["idx"][li], \
                    ("idx", st, li)
    finally:
        HA.replay_steps = True
    assert (HA.step_stats["replayed"] - r0 >= 1) == native
    from kvcompress import _engine
    assert _engine.device_status(0) == 0
