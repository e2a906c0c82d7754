"""Pins oracle/h2o_oracle.py (CPU, no GPU): its restatement of torch's CPU sums against torch
itself across shapes and thread counts, and its manager / compress replay against the unmodified
reference's outputs on tie-heavy attention (tests/golden/h2o_attention_ties.json)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLD)
import h2o_inputs  # noqa: E402
import prng  # noqa: E402
from gen_h2o_attention_ties import att_seed, kv_seed, sha  # noqa: E402
from oracle import h2o_oracle as HO  # noqa: E402

TORCH_DT = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}


def t2np(t):
    t = t.contiguous()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


def np2t(a):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.view(torch.bfloat16) if a.dtype == np.uint16 else t


IMP_SHAPES = [(1, 4, 2, 17), (1, 32, 5, 100), (1, 32, 17, 513), (1, 8, 33, 1001),
              (1, 2, 300, 77), (1, 1, 40, 2000), (2, 3, 70, 129), (1, 32, 16, 15),
              (1, 32, 1, 600), (1, 4, 257, 31), (1, 16, 1100, 40), (1, 2, 64, 3000),
              (1, 1, 5000, 37), (1, 3, 20, 7)]
HS_SHAPES = [(1, 32, 600, 4, 156), (1, 32, 16384, 4, 15940), (1, 4, 5000, 4, 4000),
             (1, 32, 700, 4, 33), (2, 8, 3000, 4, 2500), (1, 32, 100, 4, 20),
             (1, 3, 40000, 10, 39000), (1, 32, 2000, 4, 1031), (1, 32, 40, 4, 9),
             (1, 1, 500, 4, 300), (1, 32, 2000, 4, 1033), (1, 32, 1100, 4, 1036)]


@pytest.mark.parametrize("threads", [1, 3, 8, 16, 33])
@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp16"])
def test_sums_match_torch_cpu(threads, dt):
    """attn.sum(dim=2) and acc[:, :, m0:m1].sum(dim=1) -- h2o_attention.py:116 / :198 -- bit for
    bit, including the thread-dependent column chunks of parallel_reduce."""
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    cap = torch.backends.cpu.get_cpu_capability()
    rng = np.random.default_rng(threads)
    try:
        for shape in IMP_SHAPES:
            x = torch.from_numpy(rng.random(shape, dtype=np.float32) ** 3).to(TORCH_DT[dt])
            assert np.array_equal(t2np(x.sum(dim=2)).view(np.uint8),
                                  HO.attn_importance(t2np(x), threads, cap).view(np.uint8)), shape
        for B, H, L, m0, m1 in HS_SHAPES:
            a = torch.from_numpy(rng.random((B, H, L), dtype=np.float32)).to(TORCH_DT[dt])
            ref = t2np(a[:, :, m0:m1].sum(dim=1))
            got = HO.head_sum(t2np(a)[:, :, m0:m1], threads, cap)
            assert np.array_equal(ref.view(np.uint8), got.view(np.uint8)), (B, H, L, m0, m1)
    finally:
        torch.set_num_threads(prev)


def test_order_model_has_power():
    """The two addition orders and the column chunking are all observable: on these inputs a
    model that sums every column in one order, or ignores the thread split, disagrees with
    torch (so the test above would catch a wrong restatement).  The split only shows when the
    final chunk is shorter than one SIMD vector: 1029 columns over 33 threads end in a 5-column
    chunk [1024, 1029), which the scalar loop sums as one group of four + one row_sum column."""
    rng = np.random.default_rng(5)
    x = rng.random((1, 32, 2000), dtype=np.float32)
    prev = torch.get_num_threads()
    torch.set_num_threads(33)
    try:
        ref = t2np(torch.from_numpy(x)[:, :, 4:1033].sum(dim=1))[0]
    finally:
        torch.set_num_threads(prev)
    mid = x[0, :, 4:1033]
    assert not np.array_equal(ref, HO.cascade_rows(mid))
    assert not np.array_equal(ref, HO.ilp4_rows(mid))
    serial = HO.sum_reduce_first(mid, HO.ilp_mask(1029, [], 32, 4, 1, "AVX512"))
    assert not np.array_equal(ref, serial)
    split = HO.sum_reduce_first(mid, HO.ilp_mask(1029, [], 32, 4, 33, "AVX512"))
    assert np.array_equal(ref, split)


def test_sums_match_torch_cpu_avx2():
    """Same restatement under ATEN_CPU_CAPABILITY=avx2 (sum_stub runs 256-bit vectors on every
    x86 capability)."""
    code = ("import sys, numpy as np, torch; sys.path.insert(0, %r); "
            "from oracle import h2o_oracle as HO; torch.set_num_threads(4); "
            "r = np.random.default_rng(0); x = r.random((1, 32, 3, 1000), dtype=np.float32); "
            "a = torch.from_numpy(x).sum(dim=2).numpy(); "
            "b = HO.attn_importance(x, 4, torch.backends.cpu.get_cpu_capability()); "
            "print(torch.backends.cpu.get_cpu_capability(), np.array_equal(a, b))") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         env=dict(os.environ, ATEN_CPU_CAPABILITY="avx2"), timeout=300)
    assert out.stdout.split() == ["AVX2", "True"], out.stdout + out.stderr


def golden():
    with open(os.path.join(GOLD, "h2o_attention_ties.json")) as f:
        return json.load(f)


def replay(gold, si, dt, mgr, compress, check):
    """Drive one scenario through a manager / compress implementation; `check(st, rec, S, out)`
    compares one step's state against the golden record."""
    sc = gold["scenarios"][si]
    H, D, L = gold["H"], gold["D"], gold["layers"]
    for st, step in enumerate(sc["steps"]):
        k = step["k"] if step["op"] == "update" else step["S"]
        atts = tuple(h2o_inputs.attention(att_seed(si, st, li), H, step["q"], k, dt)
                     if step["att"][li] else None for li in range(L))
        out = None
        if step["op"] == "update":
            mgr.update_attention_scores(atts, skip_layers=step["skip"])
            S = k
        else:
            S = step["S"]
            kv = [(prng.gen_keys(kv_seed(si, st, li), (1, H, S, D), dt),
                   prng.gen_values(kv_seed(si, st, li), (1, H, S, D), dt)) for li in range(L)]
            out = compress(kv, atts, mgr, step["skip"], sc["kw"])
        check(st, gold["results"][f"{sc['name']}/{dt}"][st], S, out)


@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("si", [0, 1])
def test_oracle_replays_reference_goldens(si, dt):
    gold = golden()
    sc = gold["scenarios"][si]
    mgr = HO.H2OManager(decay_factor=sc["decay"], threads=gold["threads"],
                        capability=gold["capability"], **sc["kw"])

    def compress(kv, atts, m, skip, kw):
        return HO.h2o_attention_compress(kv, attention_scores=atts, h2o_manager=m,
                                         skip_layers=skip, **kw)

    def check(st, rec, S, out):
        for li in range(gold["layers"]):
            acc = mgr.acc.get(li)
            assert (None if acc is None else sha(acc)) == rec["acc"][li], (st, li)
            assert mgr.get_heavy_hitter_indices(li, S).tolist() == rec["idx"][li], (st, li)
            if out is not None:
                assert sha(out[li][0]) == rec["k"][li] and sha(out[li][1]) == rec["v"][li], (st, li)
    replay(gold, si, dt, mgr, compress, check)


def test_goldens_are_tie_heavy():
    """The fixture exercises ties: at the k-th heavy-hitter boundary of most compress steps the
    head-summed score is shared by kept and dropped positions."""
    gold = golden()
    tied = total = 0
    for si, sc in enumerate(gold["scenarios"]):
        mgr = HO.H2OManager(decay_factor=sc["decay"], threads=gold["threads"],
                            capability=gold["capability"], **sc["kw"])

        def check(st, rec, S, out):
            nonlocal tied, total
            if out is None:
                return
            for li, acc in mgr.acc.items():
                m0, m1 = mgr.start_size, min(S, acc.shape[-1]) - mgr.recent_size
                if m1 - m0 <= mgr.heavy_hitter_size:
                    continue
                agg = HO.to_f32(HO.head_sum(acc[:, :, m0:m1], gold["threads"],
                                            gold["capability"]))[0]
                kept = np.zeros(m1 - m0, bool)
                kept[mgr.get_heavy_hitter_indices(li, S)] = True
                total += 1
                tied += bool(np.intersect1d(agg[kept], agg[~kept]).size)
        def update_only(kv, atts, m, skip, kw):
            m.update_attention_scores(atts, skip_layers=skip)
            return []
        replay(gold, si, "bf16", mgr, update_only, check)
    assert total >= 10 and tied >= total // 2, (tied, total)


def mixed_golden():
    with open(os.path.join(GOLD, "h2o_attention_mixed.json")) as f:
        return json.load(f)


def replay_mixed(gold, si, mgr, compress, check):
    """One scenario of h2o_attention_mixed.json: each step's attention in its own dtype, K/V in
    gold["kv_dtype"] (tests/golden/gen_h2o_mixed_dtypes.py)."""
    from gen_h2o_mixed_dtypes import att_seed as m_att_seed, kv_seed as m_kv_seed
    sc = gold["scenarios"][si]
    H, D, L, kdt = gold["H"], gold["D"], gold["layers"], gold["kv_dtype"]
    for st, step in enumerate(sc["steps"]):
        k = step["k"] if step["op"] == "update" else step["S"]
        atts = tuple(h2o_inputs.attention(m_att_seed(si, st, li), H, step["q"], k, step["dt"])
                     if step["att"][li] else None for li in range(L))
        out = None
        if step["op"] == "update":
            mgr.update_attention_scores(atts, skip_layers=step["skip"])
            S = k
        else:
            S = step["S"]
            kv = [(prng.gen_keys(m_kv_seed(si, st, li), (1, H, S, D), kdt),
                   prng.gen_values(m_kv_seed(si, st, li), (1, H, S, D), kdt)) for li in range(L)]
            out = compress(kv, atts, mgr, step["skip"], sc["kw"])
        check(st, gold["results"][sc["name"]][st], S, out)


NP_DTNAME = {np.dtype(np.float32): "fp32", np.dtype(np.uint16): "bf16",
             np.dtype(np.float16): "fp16"}


@pytest.mark.parametrize("si", [0, 1, 2])
def test_oracle_replays_mixed_dtype_goldens(si):
    """The carried accumulation and a new step's attention in different dtypes: the reference
    promotes to fp32 through the decay, torch.cat and + (h2o_attention.py:129-151); a reset
    starts over in the attention's dtype."""
    gold = mixed_golden()
    sc = gold["scenarios"][si]
    mgr = HO.H2OManager(decay_factor=sc["decay"], threads=gold["threads"],
                        capability=gold["capability"], **sc["kw"])

    def compress(kv, atts, m, skip, kw):
        return HO.h2o_attention_compress(kv, attention_scores=atts, h2o_manager=m,
                                         skip_layers=skip, **kw)

    def check(st, rec, S, out):
        for li in range(gold["layers"]):
            acc = mgr.acc.get(li)
            assert (None if acc is None else NP_DTNAME[acc.dtype]) == rec["acc_dtype"][li]
            assert (None if acc is None else sha(acc)) == rec["acc"][li], (st, li)
            assert mgr.get_heavy_hitter_indices(li, S).tolist() == rec["idx"][li], (st, li)
            if out is not None:
                assert sha(out[li][0]) == rec["k"][li] and sha(out[li][1]) == rec["v"][li], (st, li)
    replay_mixed(gold, si, mgr, compress, check)


def test_oracle_replays_long_context_golden():
    """BASELINE cfg4's geometry (tests/golden/h2o_attention_long.json, S = 16 384, middle 15 936,
    three q = 1 steps, bf16 and fp32): the oracle reproduces the unmodified reference's
    accumulations, heavy hitters and compressed K / V; the boundary is tied in most steps."""
    from gen_h2o_attention_long import att_seed as l_att, kv_seed as l_kv
    with open(os.path.join(GOLD, "h2o_attention_long.json")) as f:
        gold = json.load(f)
    H, D, S, L = gold["H"], gold["D"], gold["S"], gold["layers"]
    tied = total = 0
    for dt in ("bf16", "fp32"):
        kv = [(prng.gen_keys(l_kv(li), (1, H, S, D), dt), prng.gen_values(l_kv(li), (1, H, S, D), dt))
              for li in range(L)]
        mgr = HO.H2OManager(decay_factor=gold["decay"], threads=gold["threads"],
                            capability=gold["capability"], **gold["kw"])
        for st in range(gold["steps"]):
            atts = tuple(h2o_inputs.attention(l_att(st, li), H, 1, S, dt) for li in range(L))
            out = HO.h2o_attention_compress(list(kv), attention_scores=atts, h2o_manager=mgr,
                                            skip_layers=[], **gold["kw"])
            rec = gold["results"][dt][st]
            for li in range(L):
                assert sha(mgr.acc[li]) == rec["acc"][li], (dt, st, li)
                idx = mgr.get_heavy_hitter_indices(li, S)
                assert idx.tolist() == rec["idx"][li], (dt, st, li)
                assert sha(out[li][0]) == rec["k"][li] and sha(out[li][1]) == rec["v"][li], \
                    (dt, st, li)
                m0, m1 = mgr.start_size, S - mgr.recent_size
                agg = HO.to_f32(HO.head_sum(mgr.acc[li][:, :, m0:m1], gold["threads"],
                                            gold["capability"]))[0]
                kept = np.zeros(m1 - m0, bool)
                kept[idx] = True
                total += 1
                tied += bool(np.intersect1d(agg[kept], agg[~kept]).size)
    assert tied >= total // 2, (tied, total)
