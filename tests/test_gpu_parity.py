"""GPU parity: the HIP engine behind the drop-in compress functions vs the reference goldens and
the CPU oracle.  Bar: identical output kinds/shapes, SHA-256-identical K/V bytes, identical
source positions for every kept row (bit-exact selection incl. libstdc++ tie order)."""
import numpy as np
import pytest
import torch

import fixtures
import prng
from gpu_util import kind_of, to_dev, to_np
from oracle import oracle

pytestmark = pytest.mark.gpu


def _method(name):
    from kvcompress.methods import get_compress_fn
    if name == "evict_for_space":  # exported by streaming_llm, not in the registry
        from kvcompress.methods.streaming_llm import evict_for_space
        return evict_for_space
    return get_compress_fn(name)


def _run_case(case, values):
    layers = fixtures.make_inputs(case, values)
    tin = [(to_dev(K), to_dev(V)) for K, V in layers]
    out = _method(case["method"])(list(tin), **case["kwargs"])
    torch.cuda.synchronize()
    return tin, out


@pytest.fixture(params=["kernels", "separate"])
def launch_path(request, monkeypatch):
    """Both launch paths of kvc_launch: the default SCORE + SELECT_GATHER kernels ("kernels") and
    SCORE / SELECT / GATHER as three kernels (KVC_FLAG_SPLIT_SELECT_GATHER, "separate")."""
    from kvcompress import _engine
    monkeypatch.setattr(_engine, "split_select_gather", request.param == "separate")
    return request.param


@pytest.mark.parametrize("cid", fixtures.case_ids())
def test_engine_matches_reference_golden(cid, launch_path):
    case = fixtures.get_case(cid)
    if case["error"]:
        with pytest.raises(Exception) as ei:
            _run_case(case, "data")
        assert type(ei.value).__name__ == case["error"]
        return
    tin, out = _run_case(case, "data")
    _, out_pos = _run_case(case, "pos")
    assert len(out) == len(case["out"])
    for li, (g, (ki, vi), (ko, vo), (_, vpo)) in enumerate(zip(case["out"], tin, out, out_pos)):
        assert kind_of(ki, ko) == g["kind"] == kind_of(vi, vo), (cid, li)
        assert list(ko.shape) == g["k_shape"] and list(vo.shape) == g["v_shape"], (cid, li)
        if g["kind"] != "same":
            pos, ok = prng.decode_positions(to_np(vpo), case["dtype"])
            assert ok
            np.testing.assert_array_equal(pos, fixtures.positions()[g["pos_key"]].astype(np.int64),
                                          err_msg=f"{cid} layer {li}: selected positions")
        assert fixtures.sha(to_np(ko)) == g["k_sha"], (cid, li, "K bytes")
        assert fixtures.sha(to_np(vo)) == g["v_sha"], (cid, li, "V bytes")


# ------------------------------------------------------------------------------------------
# C-ABI level: norms and selection on random tie-heavy rows vs the oracle
# ------------------------------------------------------------------------------------------
def _abi_select(keys_np, n_select, order, algo, score_mode=0, pool=0, zone=None):
    """Run SCORE+SELECT through the C ABI on K = keys_np [1,H,S,D]; return (norms, idx)."""
    from kvcompress import _engine as E
    from kvcompress import _native as N
    K = to_dev(keys_np)
    B, H, S, D = K.shape
    z0, zl = zone if zone else (0, S)
    j = E.Segments(0, K, K, zone_start=z0, zone_len=zl, n_select=n_select,
                   score_mode=score_mode, pool_kernel=pool)
    table = np.zeros(1, dtype=N.LAYER_DTYPE)
    ko = torch.empty((B, H, n_select, D), dtype=K.dtype, device=K.device)
    t = table[0]
    t["k"] = t["v"] = K.data_ptr()
    t["k_out"] = t["v_out"] = ko.data_ptr()
    t["k_stride"] = t["v_stride"] = K.stride()[:3]
    t["seq_len"], t["zone_start"], t["zone_len"], t["n_select"] = S, z0, zl, n_select
    t["score_mode"], t["pool_kernel"] = score_mode, pool
    dts = {torch.bfloat16: N.KVC_BF16, torch.float16: N.KVC_F16, torch.float32: N.KVC_F32}
    p = N.Params(dtype=dts[K.dtype], batch=B, heads=H,
                 head_dim=D, order=order, algo=algo, phases=N.PHASE_SCORE | N.PHASE_SELECT,
                 external_index=0)
    rc, info = N.plan(p, table)
    assert rc == 0
    ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=K.device)
    rc = N.launch(p, table, ws.data_ptr(), int(info.workspace_bytes),
                  torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    del j
    es = K.element_size()
    nb = int(info.rows) * int(info.norm_row_stride) * es
    nr = ws[info.norm_offset:info.norm_offset + nb].view(K.dtype).view(B * H, -1)[:, :zl]
    ib = int(info.rows) * int(info.index_row_stride) * 4
    ir = ws[info.index_offset:info.index_offset + ib].view(torch.int32).view(B * H, -1)
    return to_np(nr).reshape(B, H, zl), ir[:, :n_select].cpu().numpy().reshape(B, H, n_select)


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("D", [32, 64, 80, 128, 256])
@pytest.mark.parametrize("variant", ["normal", "scaled", "few", "equal", "special", "tiny", "micro"])
def test_abi_norms_and_sort_select(dtype, D, variant):
    S = 3000
    K = prng.gen_keys(900 + D, (1, 4, S, D), dtype, variant)
    for desc in (0, 1):
        for k in (1, 17, 500, 2999):
            nrm, idx = _abi_select(K, k, desc, 0)
            np.testing.assert_array_equal(nrm, oracle.norms(K))
            ref = np.sort(oracle.argsort_prefix(nrm, k, descending=bool(desc)), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"sort k={k} desc={desc}")


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special"])
def test_abi_topk_select(dtype, variant):
    S = 4000
    K = prng.gen_keys(1900, (1, 4, S, 64), dtype, variant)
    for k in (1, 3, 4, 62, 63, 64, 480, 3999):  # k*64 <= n: heap select; else introselect
        nrm, idx = _abi_select(K, k, 1, 1)
        ref = np.sort(oracle.topk_indices(nrm, k), axis=-1)
        np.testing.assert_array_equal(idx, ref, err_msg=f"topk k={k}")


@pytest.mark.parametrize("S", [17, 100, 1024, 4097, 16384])
def test_abi_select_lengths(S):
    K = prng.gen_keys(77 + S, (1, 2, S, 128), "bf16", "few")
    for k in sorted({1, S // 3, S // 2, S - 1}):
        if k <= 0:
            continue
        nrm, idx = _abi_select(K, k, 0, 0)
        ref = np.sort(oracle.argsort_prefix(nrm, k), axis=-1)
        np.testing.assert_array_equal(idx, ref)
        nrm, idx = _abi_select(K, k, 1, 1)
        ref = np.sort(oracle.topk_indices(nrm, k), axis=-1)
        np.testing.assert_array_equal(idx, ref)


def _shaped_keys(seed, S, variant, dtype="bf16"):
    """Rows whose level-0 swap count m spans the range: 'ramp' / 'rramp' (norms rising / falling
    along the row), 'halves' (the large norms all in the first half: m close to n / 2), else a
    prng variant ('equal': every position ties, m = (n - 1) / 2 exactly)."""
    if variant in ("ramp", "rramp", "halves"):
        K = np.zeros((1, 2, S, 128), dtype=np.float32)
        r = np.arange(S, dtype=np.float32)
        col = {"ramp": r + 1.0, "rramp": S - r, "halves": np.where(r < S // 2, 2.0, 1.0)}[variant]
        K[0, :, :, 0] = col.astype(np.float32)[None, :]
        K[0, 1, :, 1] = 0.5  # head 1: same order, other values
        return prng.to_dtype(K, dtype)
    return prng.gen_keys(seed, (1, 2, S, 128), dtype, variant)


@pytest.mark.parametrize("S", [8193, 8194, 9000, 12000, 16383, 16384])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special", "ramp", "rramp", "halves"])
def test_abi_level0_rank_tables_in_idx_region(S, variant):
    """Level 0 of 1 024-thread plain-norm rows keeps its rank tables in the idx region and
    rebuilds the indices after its swaps (partition_level ITAB): every swap count up to the
    maximum (n - 1) / 2 ('equal', 'halves'), the J = 8 body (S = 8 193) and the J = 9..16 ones,
    ascending / descending sorts and introselect, against the oracle."""
    K = _shaped_keys(8800 + S, S, variant)
    for k in sorted({1, 512, S // 3, S // 2, S - 1}):
        for desc in (0, 1):
            nrm, idx = _abi_select(K, k, desc, 0)
            ref = np.sort(oracle.argsort_prefix(nrm, k, descending=bool(desc)), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"S={S} sort k={k} desc={desc}")
        if k * 64 > S:  # introselect (k * 64 <= n takes the heap select)
            nrm, idx = _abi_select(K, k, 1, 1)
            ref = np.sort(oracle.topk_indices(nrm, k), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"S={S} topk k={k}")


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special"])
def test_abi_decode_tail_selections(dtype, variant):
    """Per-token decode shapes (S = cache + 1, one position evicted: k = n - 1) and the other
    tail selections where 16-bit keys try the untied fast path before the chain (k or n - k
    <= 64 on rows of <= 4096 positions), on both sides of that gate; tied maxima / minima
    ('few', 'equal') must fall back to the chain."""
    for S in (65, 257, 481, 513, 1025):
        K = prng.gen_keys(4242 + S, (1, 3, S, 128), dtype, variant)
        for k in sorted({1, 2, 63, 64, 65, S - 66, S - 65, S - 64, S - 2, S - 1}):
            if not 0 < k < S:
                continue
            for desc in (0, 1):
                nrm, idx = _abi_select(K, k, desc, 0)
                ref = np.sort(oracle.argsort_prefix(nrm, k, descending=bool(desc)), axis=-1)
                np.testing.assert_array_equal(idx, ref, err_msg=f"S={S} sort k={k} desc={desc}")
            nrm, idx = _abi_select(K, k, 1, 1)
            ref = np.sort(oracle.topk_indices(nrm, k), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"S={S} topk k={k}")


@pytest.mark.parametrize("S", [900, 1024, 4097, 16384])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special", "tiny"])
def test_abi_fp32_radix_fast_path(S, variant):
    """fp32 keys: the untied fast path's radix select (from n_cap = 1024 on; rank tables hold its
    histograms) -- untied rows ('normal', 'tiny': the set from the values alone) and rows whose
    boundary ties ('few', 'equal') or whose key span covers all 32 bits ('special': NaN / inf
    keys, four 8-bit digits) so the chain must run after the histograms used its tables."""
    K = prng.gen_keys(6100 + S, (1, 2, S, 128), "fp32", variant)
    for k in sorted({1, 2, S // 7, S // 2, S - 2, S - 1}):
        for desc in (0, 1):
            nrm, idx = _abi_select(K, k, desc, 0)
            ref = np.sort(oracle.argsort_prefix(nrm, k, descending=bool(desc)), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"S={S} sort k={k} desc={desc}")
        nrm, idx = _abi_select(K, k, 1, 1)
        ref = np.sort(oracle.topk_indices(nrm, k), axis=-1)
        np.testing.assert_array_equal(idx, ref, err_msg=f"S={S} topk k={k}")


@pytest.mark.parametrize("S", [4096, 5000, 8192, 16384])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special", "ramp"])
def test_abi_heap_select_long_rows(S, variant):
    """std::partial_sort's heap select (topk with k * 64 <= n) on rows of >= 4 096 positions
    (512-thread rows up to 8 192 positions, 1 024-thread rows beyond).  'ramp': norms rising
    along the row, so every position enters the heap (a pop per position)."""
    if variant == "ramp":
        K = np.zeros((1, 2, S, 128), dtype=np.float32)
        K[0, :, :, 0] = (np.arange(S, dtype=np.float32) + 1.0)[None, :]
        K = prng.to_dtype(K, "bf16")
    else:
        K = prng.gen_keys(7300 + S, (1, 2, S, 128), "bf16", variant)
    for k in (1, 2, 17, 63, 64):
        nrm, idx = _abi_select(K, k, 1, 1)
        ref = np.sort(oracle.topk_indices(nrm, k), axis=-1)
        np.testing.assert_array_equal(idx, ref, err_msg=f"S={S} topk k={k}")


def test_random_strategy_matches_torch_restatement():
    """strategy='random' consumes torch's device RNG exactly like the reference."""
    from kvcompress.methods import fix_size_l2_compress
    K = to_dev(prng.gen_keys(5, (1, 4, 700, 64), "bf16"))
    V = to_dev(prng.gen_values(5, (1, 4, 700, 64), "bf16"))
    torch.manual_seed(123)
    out = fix_size_l2_compress([(K, V)], fix_kv_size=200, keep_ratio=0.25, strategy="random",
                               skip_layers=[])
    torch.manual_seed(123)
    P = 50
    Z, keep = 700 - P, 200 - P
    ind = torch.stack([torch.stack([torch.randperm(Z, device=K.device)[:keep] for _ in range(4)])])
    ind, _ = torch.sort(ind, dim=-1)
    e = ind.unsqueeze(-1).expand(1, 4, keep, 64)
    rk = torch.cat([torch.gather(K[:, :, :Z], 2, e), K[:, :, -P:]], dim=2)
    rv = torch.cat([torch.gather(V[:, :, :Z], 2, e), V[:, :, -P:]], dim=2)
    assert torch.equal(out[0][0].view(torch.int16), rk.view(torch.int16))
    assert torch.equal(out[0][1].view(torch.int16), rv.view(torch.int16))


def test_dynamic_cache_input():
    from transformers import DynamicCache
    from kvcompress.methods import h2o_l2_compress
    layers = [(prng.gen_keys(40 + i, (1, 4, 900, 64), "bf16"),
               prng.gen_values(40 + i, (1, 4, 900, 64), "bf16")) for i in range(3)]
    cache = DynamicCache()
    for i, (k, v) in enumerate(layers):
        cache.update(to_dev(k), to_dev(v), i)
    out = h2o_l2_compress(cache)
    ref = oracle.h2o_l2_compress(layers)
    for (ko, vo), (rk, rv, _) in zip(out, ref):
        assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv)


def test_headline_geometry_32_layers(launch_path):
    """BASELINE headline: 32 layers of [1,32,16384,128] bf16, fix_size_l2(512) in ONE call;
    two sampled layers checked bit-exactly against the oracle."""
    from kvcompress.methods import fix_size_l2_compress
    g = torch.Generator(device="cuda:0").manual_seed(0)
    layers = [(torch.randn(1, 32, 16384, 128, device="cuda:0", generator=g).to(torch.bfloat16),
               torch.randn(1, 32, 16384, 128, device="cuda:0", generator=g).to(torch.bfloat16))
              for _ in range(32)]
    out = fix_size_l2_compress(list(layers), fix_kv_size=512, keep_ratio=0.0, skip_layers=[])
    torch.cuda.synchronize()
    for li in (0, 31):
        kn, vn = to_np(layers[li][0]), to_np(layers[li][1])
        rk, rv, _ = oracle.fix_size_l2_compress([(kn, vn)], fix_kv_size=512, skip_layers=[])[0]
        assert np.array_equal(to_np(out[li][0]), rk) and np.array_equal(to_np(out[li][1]), rv)
    for ko, vo in out:
        assert ko.shape == (1, 32, 512, 128) and vo.shape == (1, 32, 512, 128)


def test_repeated_call_shapes_reuse_plan_safely():
    """Decode-step pattern: the same call shape many times (plan + workspace from the engine's
    plan cache), each call with new K/V; every call's outputs -- all kept alive -- match the
    oracle, also when calls alternate between two streams (one cached workspace per stream)."""
    from kvcompress import _engine
    from kvcompress.methods import fix_size_l2_compress, snapkv_lite_compress
    _engine.plan_cache.clear()
    side = torch.cuda.Stream()
    kept = []
    for step in range(6):
        layers_np = [(prng.gen_keys(500 + 10 * step + i, (1, 4, 300, 64), "bf16", "few"),
                      prng.gen_values(500 + 10 * step + i, (1, 4, 300, 64), "bf16"))
                     for i in range(3)]
        tin = [(to_dev(k), to_dev(v)) for k, v in layers_np]
        with torch.cuda.stream(side if step % 2 else torch.cuda.current_stream()):
            out_f = fix_size_l2_compress(list(tin), fix_kv_size=128, skip_layers=[])
            out_s = snapkv_lite_compress(list(tin), observation_window=16, keep_size=100)
        kept.append((layers_np, out_f, out_s))
    torch.cuda.synchronize()
    assert len(_engine.plan_cache.entries) == 4  # 2 shapes x 2 streams
    for layers_np, out_f, out_s in kept:
        for out, ref in ((out_f, oracle.fix_size_l2_compress(layers_np, fix_kv_size=128,
                                                             skip_layers=[])),
                         (out_s, oracle.snapkv_lite_compress(layers_np, observation_window=16,
                                                             keep_size=100))):
            for (ko, vo), (rk, rv, _) in zip(out, ref):
                assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv)


def test_variable_size_outputs_are_disjoint_views():
    """pyramid_kv gives every layer its own n_out; the engine carves all K/V outputs out of one
    allocation (INTEGRATION.md "Output tensors"): each output is contiguous with its own shape,
    no two overlap, writing one leaves the others intact, and the values match the oracle."""
    from kvcompress.methods import pyramid_kv_compress
    layers_np = [(prng.gen_keys(900 + i, (1, 4, 700, 64), "bf16"),
                  prng.gen_values(900 + i, (1, 4, 700, 64), "bf16")) for i in range(6)]
    kw = dict(base_size=400, min_size=64, profile="linear", skip_layers=[])
    out = pyramid_kv_compress([(to_dev(k), to_dev(v)) for k, v in layers_np], **kw)
    ref = oracle.pyramid_kv_compress(layers_np, **kw)
    torch.cuda.synchronize()
    spans = []
    for (ko, vo), (rk, rv, _) in zip(out, ref):
        assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv)
        for t in (ko, vo):
            assert t.is_contiguous() and t.data_ptr() % 16 == 0
            spans.append((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()))
    assert len({k.shape[2] for k, _ in out}) > 1  # the layers really differ in size
    spans.sort()
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    out[0][0].fill_(0)
    for (ko, vo), (rk, rv, _) in list(zip(out, ref))[1:]:
        assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv)
    assert np.array_equal(to_np(out[0][1]), ref[0][1])


def test_no_cpu_fallback():
    from kvcompress.methods import fix_size_l2_compress
    K = torch.zeros(1, 2, 100, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="ROCm GPU tensors only"):
        fix_size_l2_compress([(K, K)], fix_kv_size=10, skip_layers=[])


@pytest.mark.parametrize("mode", [0, 1])
def test_abi_adversarial_depth_limit(mode):
    """McIlroy-adversary keys drive libstdc++ into its depth-limit heap fallback; the device
    emulation (serial heap code in the select kernel) must land on the same set."""
    n = 4096
    adv = np.empty(n, dtype=np.int64)
    for k in (1, 100, n // 3, n // 2, n - 1):
        oracle.lib().orc_antiqsort(n, mode, k, adv.ctypes.data)
        K = np.zeros((1, 1, n, 64), dtype=np.float32)
        K[0, 0, :, 0] = (adv + 1).astype(np.float32)  # norm == adv + 1 exactly (< 2^12)
        # ascending sort keeps the smallest; topk keeps the largest -> feed -key order via desc
        nrm, idx = _abi_select(K, k, 0, mode)
        np.testing.assert_array_equal(nrm[0, 0], (adv + 1).astype(np.float32))
        if mode == 0:
            ref = np.sort(oracle.argsort_prefix(nrm, k), axis=-1)
        else:  # ascending topk == torch.topk(-x): use the oracle's topk on negated values
            ref = np.sort(oracle.topk_indices(-nrm, k), axis=-1)
        np.testing.assert_array_equal(idx, ref, err_msg=f"mode={mode} k={k}")


@pytest.mark.parametrize("launch_path", ["kernels"], indirect=True)
def test_more_layers_than_one_argument_chunk(launch_path):
    """Layer tables travel by value in chunks of 64 layers: 150 layers of mixed lengths (some
    untouched, some selecting) in one call, every layer checked against the oracle."""
    from kvcompress.methods import h2o_l2_compress
    layers = [(prng.gen_keys(300 + i, (1, 2, 100 + 7 * i, 64), "bf16", "few"),
               prng.gen_values(300 + i, (1, 2, 100 + 7 * i, 64), "bf16")) for i in range(150)]
    kw = dict(start_size=4, heavy_hitter_size=40, recent_size=60, skip_layers=[3, 77])
    out = h2o_l2_compress([(to_dev(k), to_dev(v)) for k, v in layers], **kw)
    ref = oracle.h2o_l2_compress(layers, **kw)
    for li, ((ko, vo), (rk, rv, _)) in enumerate(zip(out, ref)):
        assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv), li


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
def test_zones_longer_than_lds_limit(dtype):
    """Zones > 16384 positions select from the global-scratch variant (up to 65536; the
    cross-wave counts of segments > 32767 positions use the packed counters' top bit)."""
    from kvcompress.methods import fix_size_l2_compress, l2_compress, snapkv_lite_compress
    for S, variant in ((20000, "few"), (40000, "normal"), (65536, "equal")):
        K = prng.gen_keys(4000 + S, (1, 2, S, 64), dtype, variant)
        V = prng.gen_values(4000 + S, (1, 2, S, 64), dtype)
        kv = [(to_dev(K), to_dev(V))]
        for fn, ref, kw in (
                (fix_size_l2_compress, oracle.fix_size_l2_compress,
                 dict(fix_kv_size=700, keep_ratio=0.25, skip_layers=[])),
                (fix_size_l2_compress, oracle.fix_size_l2_compress,
                 dict(fix_kv_size=S // 2, strategy="keep_high", skip_layers=[])),
                (snapkv_lite_compress, oracle.snapkv_lite_compress,
                 dict(observation_window=32, keep_size=S // 3, skip_layers=[])),
                (l2_compress, oracle.l2_compress,
                 dict(keep_ratio=0.8, prune_after=100, skip_layers=[]))):
            out = fn(list(kv), **kw)
            rk, rv, _ = ref([(K, V)], **kw)[0]
            assert np.array_equal(to_np(out[0][0]), rk), (S, fn.__name__, kw)
            assert np.array_equal(to_np(out[0][1]), rv), (S, fn.__name__, kw)


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
def test_zones_beyond_u16_positions(dtype):
    """Zones > 65536 positions: u32-position selection from a global scratch (select_long_kernel),
    every path (introsort set asc/desc, introselect, partial-sort heap select, l2_compress's
    large k) bit-exact against the oracle; a call mixing a long and a short layer."""
    from kvcompress.methods import fix_size_l2_compress, l2_compress, snapkv_lite_compress
    for S, variant in ((65600, "few"), (100000, "normal"), (131072, "equal")):
        K = prng.gen_keys(8000 + S, (1, 2, S, 64), dtype, variant)
        V = prng.gen_values(8000 + S, (1, 2, S, 64), dtype)
        K2 = prng.gen_keys(9000 + S, (1, 2, 3000, 64), dtype, "few")
        V2 = prng.gen_values(9000 + S, (1, 2, 3000, 64), dtype)
        kv = [(to_dev(K), to_dev(V)), (to_dev(K2), to_dev(V2))]
        for fn, ref, kw in (
                (fix_size_l2_compress, oracle.fix_size_l2_compress,
                 dict(fix_kv_size=700, keep_ratio=0.25, skip_layers=[])),
                (fix_size_l2_compress, oracle.fix_size_l2_compress,
                 dict(fix_kv_size=S // 3, strategy="keep_high", skip_layers=[])),
                (snapkv_lite_compress, oracle.snapkv_lite_compress,
                 dict(observation_window=32, keep_size=512, skip_layers=[])),
                (snapkv_lite_compress, oracle.snapkv_lite_compress,
                 dict(observation_window=32, keep_size=S // 2, skip_layers=[])),
                (l2_compress, oracle.l2_compress,
                 dict(keep_ratio=0.8, prune_after=100, skip_layers=[]))):
            out = fn(list(kv), **kw)
            refs = ref([(K, V), (K2, V2)], **kw)
            for li, ((ko, vo), (rk, rv, _)) in enumerate(zip(out, refs)):
                assert np.array_equal(to_np(ko), rk), (S, fn.__name__, kw, li)
                assert np.array_equal(to_np(vo), rv), (S, fn.__name__, kw, li)


SHARDED = (
    ("pyramid_kv", dict(base_size=512, layer_decay=0.9, skip_layers=[9])),
    ("fix_size_l2", dict(fix_kv_size=256, keep_ratio=0.5)),            # default skip [0, 1]
    ("h2o_l2", dict(start_size=4, heavy_hitter_size=64, recent_size=444, skip_layers=[17])),
    ("snapkv_lite", dict(observation_window=32, keep_size=512, skip_layers=[30])),
    ("adaptive_l2", dict(target_size=512, skip_layers=[8, 24])),
    ("l2_compress", dict(keep_ratio=0.8, prune_after=100)),            # default skip [0, 1]
    ("streaming_llm", dict(start_size=4, recent_size=500, skip_layers=[31])),
)


@pytest.mark.parametrize("name,kw", SHARDED, ids=[s[0] for s in SHARDED])
def test_layer_sharded_calls_match_unsharded_oracle(name, kw):
    """a 32-layer stack split into 4 contiguous shards (the 8-GPU layout with 8
    layers per shard, here on one device), each compressed by its own call with the extension
    kwargs layer_offset (global skip_layers) / num_layers_total (pyramid_kv's depth-dependent
    sizes, pyramid_kv.py:82-97: layers >= 20 at min_size), is bit-identical to the unsharded
    reference call (the oracle) on the whole stack."""
    from bench import shard_layers
    dt = "bf16"
    L, shape = 32, (1, 8, 1200, 64)
    layers = [(prng.gen_keys(4000 + i, shape, dt, "normal"), prng.gen_values(4000 + i, shape, dt))
              for i in range(L)]
    ref = oracle.METHODS[name](layers, **kw)
    fn = _method(name)
    got = []
    for r in range(4):
        a, b = shard_layers(L, 4, r)
        extra = dict(layer_offset=a)
        if name == "pyramid_kv":
            extra["num_layers_total"] = L
        got += fn([(to_dev(k), to_dev(v)) for k, v in layers[a:b]], **kw, **extra)
    torch.cuda.synchronize()
    assert len(got) == L
    for li, ((ko, vo), (rk, rv, _)) in enumerate(zip(got, ref)):
        assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv), (name, li)


def test_misaligned_contiguous_views_take_the_general_path():
    """A contiguous K/V view at an odd element offset into a flat buffer (not 16-B aligned): the
    one-pass fast path declines it and the general path's aligned copy computes it exactly."""
    from kvcompress.methods import fix_size_l2_compress
    shape = (1, 4, 300, 64)
    kn = prng.gen_keys(4242, shape, "bf16", "few")
    vn = prng.gen_values(4242, shape, "bf16")
    n = kn.size
    flat_k = torch.empty(n + 3, dtype=torch.bfloat16, device="cuda:0")
    flat_v = torch.empty(n + 3, dtype=torch.bfloat16, device="cuda:0")
    k = flat_k[3:].view(shape)
    v = flat_v[3:].view(shape)
    k.copy_(to_dev(kn))
    v.copy_(to_dev(vn))
    assert k.is_contiguous() and k.data_ptr() % 16 != 0
    out = fix_size_l2_compress([(k, v)], fix_kv_size=100, skip_layers=[])
    rk, rv, _ = oracle.fix_size_l2_compress([(kn, vn)], fix_kv_size=100, skip_layers=[])[0]
    assert np.array_equal(to_np(out[0][0]), rk) and np.array_equal(to_np(out[0][1]), rv)


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special"])
def test_mid_length_zones_four_rows_per_cu(dtype, variant, launch_path):
    """Zones of 4 097..8 192 positions run the 512-thread rows whose LDS is budgeted for four
    rows per CU: 16-bit keys with rank windows (levels of 'equal' / 'few' rows swap more pairs
    than a window holds), fp32 keys with full tables.  Sort (fix_size_l2 keep_low / keep_high),
    topk (snapkv_lite) and segment layouts (h2o_l2) against the oracle."""
    from kvcompress.methods import fix_size_l2_compress, h2o_l2_compress, snapkv_lite_compress
    for S in (4097, 6000, 8192):
        layers_np = [(prng.gen_keys(8100 + S + i, (1, 2, S, 64), dtype, variant),
                      prng.gen_values(8100 + S + i, (1, 2, S, 64), dtype)) for i in range(2)]
        tin = [(to_dev(k), to_dev(v)) for k, v in layers_np]
        for fn, ofn, kw in (
                (fix_size_l2_compress, oracle.fix_size_l2_compress,
                 dict(fix_kv_size=512, skip_layers=[])),
                (fix_size_l2_compress, oracle.fix_size_l2_compress,
                 dict(fix_kv_size=S // 2, keep_ratio=0.25, strategy="keep_high", skip_layers=[])),
                (snapkv_lite_compress, oracle.snapkv_lite_compress,
                 dict(observation_window=32, keep_size=2000)),
                (h2o_l2_compress, oracle.h2o_l2_compress,
                 dict(start_size=4, heavy_hitter_size=S // 3, recent_size=300))):
            out = fn(list(tin), **kw)
            ref = ofn(layers_np, **kw)
            bits = {2: np.uint16, 4: np.uint32}
            for (ko, vo), (rk, rv, _) in zip(out, ref):  # bit patterns: NaN keys are kept rows
                b = bits[rk.dtype.itemsize]
                assert np.array_equal(to_np(ko).view(b), rk.view(b)) and \
                    np.array_equal(to_np(vo).view(b), rv.view(b)), (S, fn.__name__, kw)


_SPLIT_CACHE = {}


def _split_layers(dt):
    """Nine [1, 32, 9000, 80] K/V layers (generated once per dtype for the tests below)."""
    if dt not in _SPLIT_CACHE:
        shape = (1, 32, 9000, 80)
        _SPLIT_CACHE.clear()
        _SPLIT_CACHE[dt] = [(prng.gen_keys(6100 + i, shape, dt, "normal"),
                             prng.gen_values(6100 + i, shape, dt)) for i in range(9)]
    return _SPLIT_CACHE[dt]


@pytest.mark.parametrize("name,kw", [
    ("h2o_l2", dict(start_size=4, heavy_hitter_size=64, recent_size=444, skip_layers=[])),
    ("pyramid_kv", dict(base_size=512, skip_layers=[], num_layers_total=32, layer_offset=28)),
    ("snapkv_lite", dict(observation_window=32, keep_size=512, skip_layers=[])),
    ("adaptive_l2", dict(target_size=512, skip_layers=[])),
])
@pytest.mark.parametrize("dt", ["bf16", "fp16"])
def test_few_rows_split_copy_matches_oracle(name, kw, dt):
    """Calls with fewer selection rows than CUs and zones above the 512-thread path (4 layers x
    32 heads: one rank's share of an 8-way layer split) copy each row's sink / tail
    rows in a second workgroup beside the selecting one (select_gather_kernel split_rows); the
    outputs are bit-identical to the oracle's.  Nine layers (288 rows) take the one-workgroup
    copy on the same data."""
    L = 4
    layers = _split_layers(dt)
    okw = {k: v for k, v in kw.items() if k not in ("num_layers_total", "layer_offset")}
    fn = _method(name)
    for n in (L, 9):
        if name == "pyramid_kv":  # the last n layers of a 32-layer model (depth-dependent sizes)
            okw_n = dict(okw, skip_layers=list(range(32 - n)))  # stand-ins, left alone
            ref = oracle.pyramid_kv_compress([layers[0]] * (32 - n) + layers[:n], **okw_n)[32 - n:]
            extra = dict(num_layers_total=32, layer_offset=32 - n)
        else:
            ref = oracle.METHODS[name](layers[:n], **okw)
            extra = {}
        got = fn([(to_dev(k), to_dev(v)) for k, v in layers[:n]],
                 **{k: v for k, v in kw.items() if k not in ("num_layers_total", "layer_offset")},
                 **extra)
        torch.cuda.synchronize()
        for li, ((ko, vo), (rk, rv, _)) in enumerate(zip(got, ref)):
            assert ko.shape[2] == rk.shape[2], (name, n, li)
            assert np.array_equal(to_np(ko), rk) and np.array_equal(to_np(vo), rv), (name, n, li)


def _neg16(nrm):
    """-x of non-negative 16-bit norms in storage representation (bf16 bits / float16)."""
    return nrm ^ np.uint16(0x8000) if nrm.dtype == np.uint16 else -nrm


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("mode", [0, 1])
def test_abi_tiny_segments_and_adversaries(dtype, mode):
    """The chain's last levels on segments of <= 64 positions run from registers
    (wave_tiny_chain): whole rows of 5..200 positions (tie-heavy and McIlroy-adversary keys, so
    the introsort / introselect depth limit falls inside those levels and the serial heap
    fallback takes over from the registers), 16-bit keys, sort and topk (ascending: the
    oracle's topk of the negated norms), against the oracle."""
    def ref_of(nrm, k):
        if mode == 0:
            return np.sort(oracle.argsort_prefix(nrm, k), axis=-1)
        return np.sort(oracle.topk_indices(_neg16(nrm), k), axis=-1)
    for n in (5, 17, 33, 64, 65, 100, 200):
        K = prng.gen_keys(8800 + n, (1, 4, n, 64), dtype, "few")
        for k in sorted({1, 2, n // 3, n // 2, n - 2, n - 1}):
            if not 0 < k < n or (mode and k * 64 <= n):
                continue
            nrm, idx = _abi_select(K, k, 0, mode)
            np.testing.assert_array_equal(idx, ref_of(nrm, k), err_msg=f"few n={n} k={k}")
    adv = np.empty(256, dtype=np.int64)
    for n in (20, 40, 64, 100, 200):
        for k in sorted({1, n // 3, n // 2, n - 1}):
            if mode and k * 64 <= n:
                continue
            oracle.lib().orc_antiqsort(n, mode, k, adv.ctypes.data)
            K = np.zeros((1, 1, n, 64), dtype=np.float32)
            K[0, 0, :, 0] = (adv[:n] + 1).astype(np.float32)  # exact in bf16 / fp16 (<= 256)
            nrm, idx = _abi_select(prng.to_dtype(K, dtype), k, 0, mode)
            np.testing.assert_array_equal(idx, ref_of(nrm, k), err_msg=f"adversary n={n} k={k}")


@pytest.mark.parametrize("dtype", ["bf16", "fp16"])
@pytest.mark.parametrize("variant", ["special", "equal", "zero", "tiny", "few"])
def test_snapkv_scoring_from_tile_maxima(dtype, variant, launch_path):
    """snapkv_lite's row max comes from SCORE's per-64-token-tile norm maxima (bit patterns; a
    NaN's exceed +inf's) and its scores / pooling from each thread's norms plus a 4-byte halo
    (round 6, snapkv_keys16): NaN / +-inf / zero / all-equal / sub-normal rows, zones whose last
    tile is partial or a single position, on the 512-thread (<= 8 192 positions) and the
    1 024-thread rows, pooling 5 and none, against the oracle; pooling 3 keeps the two-barrier
    path on the same rows.  Both launch paths."""
    from kvcompress.methods import snapkv_lite_compress
    bits = {2: np.uint16, 4: np.uint32}
    for S, pk in ((8224, 5), (12000, 5), (16384, 5), (8257, 1), (12000, 3), (16353, 5)):
        shape = (1, 2, S, 64)
        layers_np = [(prng.gen_keys(9300 + S + i, shape, dtype, variant if i else "special"),
                      prng.gen_values(9300 + S + i, shape, dtype)) for i in range(2)]
        tin = [(to_dev(k), to_dev(v)) for k, v in layers_np]
        kw = dict(observation_window=32, keep_size=1024, pooling_kernel=pk, skip_layers=[])
        out = snapkv_lite_compress(list(tin), **kw)
        ref = oracle.snapkv_lite_compress(layers_np, **kw)
        for li, ((ko, vo), (rk, rv, _)) in enumerate(zip(out, ref)):
            b = bits[rk.dtype.itemsize]
            assert np.array_equal(to_np(ko).view(b), rk.view(b)) and \
                np.array_equal(to_np(vo).view(b), rv.view(b)), (S, pk, li)
