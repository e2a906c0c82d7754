"""The opt-in stable tie policy (KVC_ALGO_STABLE, `_engine.set_tie_policy("stable")`): the first k
of torch.argsort(stable=True) -- every key before the k-th one, then the tied keys in position
order -- instead of the reference's libstdc++ tie order.

CPU: the oracle's restatement (oracle.stable_prefix) against torch's own stable sort on tie-heavy
bf16 / fp16 / fp32 rows with NaN / inf / signed zeros, both directions; the policy switch.
GPU: the engine's radix selection through the C ABI against that oracle (every key variant, row
lengths 17 .. 16 384, k at the edges, both launch shapes, snapkv scores), every method's golden
inputs through the compress functions against the oracle's methods under the same policy, zones
past the LDS limit from the global-scratch kernel, and zones past 65 536 positions refused."""
import numpy as np
import pytest
import torch

import fixtures
import prng
from gpu_util import kind_of, to_dev, to_np
from oracle import oracle


def _torch_stable(vals, k, desc):
    t = torch.from_numpy(oracle.as_float(vals))
    return torch.argsort(t, dim=-1, stable=True, descending=desc)[..., :k].numpy()


@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special", "tiny"])
def test_oracle_stable_prefix_matches_torch(dtype, variant):
    K = prng.gen_keys(4100, (1, 3, 700, 64), dtype, variant)
    nrm = oracle.norms(K)
    rng = np.random.default_rng(5)
    vals = [nrm]
    if dtype != "bf16":  # signed zeros, infinities and NaN among the values themselves
        x = nrm.astype(np.float32).copy()
        x.reshape(-1)[rng.integers(0, x.size, 60)] = rng.choice(
            [0.0, -0.0, np.inf, -np.inf, np.nan], 60)
        vals.append(x.astype(nrm.dtype))
    for v in vals:
        for desc in (False, True):
            for k in (1, 2, 37, 350, 699, 700):
                np.testing.assert_array_equal(oracle.stable_prefix(v, k, desc),
                                              _torch_stable(v, k, desc))


def test_tie_policy_switch():
    from kvcompress import _engine as E
    assert E.tie_policy == "reference"
    with pytest.raises(ValueError):
        E.set_tie_policy("fast")
    prev = E.set_tie_policy("stable")
    try:
        assert prev == "reference" and E.tie_policy == "stable"
    finally:
        E.set_tie_policy(prev)


@pytest.fixture
def stable(monkeypatch):
    from kvcompress import _engine as E
    monkeypatch.setattr(E, "tie_policy", "stable")
    monkeypatch.setattr(oracle, "TIE", "stable")
    E.call_memo.clear()
    yield
    E.call_memo.clear()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special", "tiny", "micro"])
@pytest.mark.parametrize("S", [17, 100, 1024, 3000, 4097, 8192, 16384])
def test_abi_stable_select(dtype, variant, S):
    from kvcompress import _native as N
    from test_gpu_parity import _abi_select
    H = 2 if S > 4096 else 4
    K = prng.gen_keys(7000 + S, (1, H, S, 64), dtype, variant)
    for desc in (0, 1):
        for k in sorted({1, 2, S // 3, S // 2 + 1, S - 2, S - 1} - {0}):
            if not 0 < k < S:
                continue
            nrm, idx = _abi_select(K, k, desc, N.KVC_ALGO_STABLE)
            np.testing.assert_array_equal(nrm, oracle.norms(K))
            ref = np.sort(oracle.stable_prefix(nrm, k, bool(desc)), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"{dtype} {variant} S={S} k={k} desc={desc}")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp16", "fp32"])
def test_abi_stable_snapkv_scores(dtype):
    from kvcompress import _native as N
    from test_gpu_parity import _abi_select
    S = 5000
    K = prng.gen_keys(7301, (1, 4, S, 128), dtype, "normal")
    for pool in (1, 4, 5):
        for k in (1, 480, S - 1):
            nrm, idx = _abi_select(K, k, N.KVC_DESC, N.KVC_ALGO_STABLE, score_mode=1, pool=pool)
            scores = oracle.snapkv_scores(nrm, pool)
            ref = np.sort(oracle.stable_prefix(scores, k, True), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"pool={pool} k={k}")


def _run(case, values):
    from test_gpu_parity import _run_case
    return _run_case(case, values)


@pytest.mark.gpu
@pytest.mark.parametrize("launch", ["kernels", "separate"])
@pytest.mark.parametrize("cid", fixtures.case_ids())
def test_methods_stable_policy_match_oracle(cid, launch, stable, monkeypatch):
    """Every golden case's inputs through the compress functions with the stable policy: the
    kept rows (decoded source positions) and K / V bytes equal the oracle's methods under the
    same policy."""
    from kvcompress import _engine as E
    monkeypatch.setattr(E, "split_select_gather", launch == "separate")
    case = fixtures.get_case(cid)
    if case["error"]:
        pytest.skip("error case: no selection")
    layers = fixtures.make_inputs(case, "data")
    if max(K.shape[2] for K, _ in layers) > E.STABLE_MAX_ZONE:
        pytest.skip("zone past the stable policy's limit")
    tin, out = _run(case, "data")
    ref = oracle.METHODS[case["method"]](layers, **case["kwargs"]) if case["method"] in \
        oracle.METHODS else getattr(oracle, case["method"])(layers, **case["kwargs"])
    assert len(out) == len(ref)
    for li, ((ki, vi), (ko, vo), (rk, rv, kind)) in enumerate(zip(tin, out, ref)):
        assert kind_of(ki, ko) == kind, (cid, li)
        if kind != "same":
            np.testing.assert_array_equal(to_np(ko), rk, err_msg=f"{cid} layer {li} K")
            np.testing.assert_array_equal(to_np(vo), rv, err_msg=f"{cid} layer {li} V")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("variant", ["normal", "few", "equal", "special"])
@pytest.mark.parametrize("S", [16448, 40000, 65536])
def test_abi_stable_select_global_scratch(dtype, variant, S):
    """Zones past the LDS limit: the stable selection from the global-scratch kernel."""
    from kvcompress import _native as N
    from test_gpu_parity import _abi_select
    K = prng.gen_keys(7500 + S, (1, 1, S, 32), dtype, variant)
    for desc in (0, 1):
        for k in (1, 512, S // 2, S - 1):
            nrm, idx = _abi_select(K, k, desc, N.KVC_ALGO_STABLE)
            ref = np.sort(oracle.stable_prefix(nrm, k, bool(desc)), axis=-1)
            np.testing.assert_array_equal(idx, ref, err_msg=f"{dtype} {variant} S={S} k={k}")


@pytest.mark.gpu
def test_stable_policy_zone_limit(stable):
    """Zones up to 65 536 positions select under the stable policy (matching the oracle); longer
    ones raise."""
    from kvcompress.methods import fix_size_l2_compress
    K = prng.gen_keys(7600, (1, 2, 20000, 64), "bf16", "normal")
    V = prng.gen_values(7600, (1, 2, 20000, 64), "bf16")
    out = fix_size_l2_compress([(to_dev(K), to_dev(V))], fix_kv_size=512, skip_layers=[])
    rk, rv, _ = oracle.fix_size_l2_compress([(K, V)], fix_kv_size=512, skip_layers=[])[0]
    np.testing.assert_array_equal(to_np(out[0][0]), rk)
    np.testing.assert_array_equal(to_np(out[0][1]), rv)
    L = torch.randn(1, 1, 65600, 32, device="cuda:0").to(torch.bfloat16)
    with pytest.raises(ValueError, match="stable tie policy"):
        fix_size_l2_compress([(L, L)], fix_kv_size=512, skip_layers=[])


@pytest.mark.gpu
def test_headline_geometry_stable_vs_reference_sets():
    """At the headline geometry the stable sets differ from the reference's only among keys tied
    with the k-th one: same count, same keys below the boundary."""
    from kvcompress import _engine as E
    from kvcompress import _native as N
    from test_gpu_parity import _abi_select
    K = prng.gen_keys(7401, (1, 8, 16384, 128), "bf16", "normal")
    nrm, ref_idx = _abi_select(K, 512, 0, N.KVC_ALGO_SORT)
    _, st_idx = _abi_select(K, 512, 0, N.KVC_ALGO_STABLE)
    v = oracle.as_float(nrm)
    for h in range(8):
        T = np.sort(v[0, h])[511]
        a, b = ref_idx[0, h], st_idx[0, h]
        assert set(a[v[0, h][a] < T]) == set(b[v[0, h][b] < T])
        assert np.all(v[0, h][b] <= T) and len(set(b)) == 512
        eq = np.flatnonzero(v[0, h] == T)
        np.testing.assert_array_equal(np.sort(b[v[0, h][b] == T]), eq[:len(b[v[0, h][b] == T])])
    assert E.tie_policy == "reference"


def test_tie_policy_from_environment():
    """KVC_TIE_POLICY selects the policy at import; an unknown value refuses to import."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pkg = os.path.join(root, "cs3602-llm-inference-acceleration_amd")
    code = "import kvcompress._engine as E; print(E.tie_policy)"
    env = dict(os.environ, PYTHONPATH=pkg, KVC_TIE_POLICY="stable")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "stable", r.stderr
    env["KVC_TIE_POLICY"] = "bogus"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0 and "KVC_TIE_POLICY" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["bf16", "fp32"])
@pytest.mark.parametrize("S", [3000, 16384])
def test_h2o_attention_stable_heavy_hitters_match_oracle(dt, S, stable):
    """h2o_attention under the stable policy: accumulations, heavy hitters (the first k of a
    stable descending sort of the head sums: KVC_ATTN_HH_STABLE) and compressed K / V equal the
    oracle manager's under the same policy, over three decode-shaped steps (tie-heavy
    attention; the third step replayed natively)."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import h2o_inputs
    from oracle import h2o_oracle as HO
    from kvcompress.methods import h2o_attention as HA
    H, D, L = 4, 64, 2
    kw = dict(start_size=4, heavy_hitter_size=64, recent_size=444)
    kv = [(prng.gen_keys(8100 + li, (1, H, S, D), dt), prng.gen_values(8100 + li, (1, H, S, D), dt))
          for li in range(L)]
    kvd = [(to_dev(k), to_dev(v)) for k, v in kv]
    mgr = HA.H2OAttentionManager(num_layers=L, num_heads=H, **kw)
    mgr.reduction_threads = 8
    omgr = HO.H2OManager(threads=8, **kw)
    HA.step_memo.clear()
    for st in range(3):
        atts = [h2o_inputs.attention(9100 + 10 * st + li, H, 1, S, dt) for li in range(L)]
        out = HA.h2o_attention_compress(list(kvd), attention_scores=tuple(to_dev(a) for a in atts),
                                        h2o_manager=mgr, skip_layers=[], **kw)
        ref = HO.h2o_attention_compress(kv, atts, omgr, skip_layers=[], **kw)
        for li in range(L):
            np.testing.assert_array_equal(to_np(mgr.accumulated_attention[li]), omgr.acc[li])
            np.testing.assert_array_equal(mgr.get_heavy_hitter_indices(li, S).cpu().numpy(),
                                          omgr.get_heavy_hitter_indices(li, S))
            np.testing.assert_array_equal(to_np(out[li][0]), ref[li][0], err_msg=f"K {st} {li}")
            np.testing.assert_array_equal(to_np(out[li][1]), ref[li][1], err_msg=f"V {st} {li}")
    assert HA.step_stats["replayed"] >= 1
