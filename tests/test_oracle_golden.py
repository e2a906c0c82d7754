"""Pins the CPU oracle (oracle/) to the reference: every golden fixture generated from the
unmodified reference kvcompress must be reproduced bit-exactly (CPU only, no GPU)."""
import numpy as np
import pytest

import fixtures
import prng
from oracle import oracle


def _run(case, values):
    layers = fixtures.make_inputs(case, values)
    return oracle.METHODS[case["method"]](layers, **case["kwargs"])


def check_case_against_golden(case, out_data, out_pos):
    assert len(out_data) == len(case["out"])
    for li, (g, (ko, vo, kind), (_, veo, _)) in enumerate(zip(case["out"], out_data, out_pos)):
        assert kind == g["kind"], (case["id"], li)
        assert list(ko.shape) == g["k_shape"] and list(vo.shape) == g["v_shape"], (case["id"], li)
        assert fixtures.sha(ko) == g["k_sha"], (case["id"], li, "K bytes")
        assert fixtures.sha(vo) == g["v_sha"], (case["id"], li, "V bytes")
        if g["kind"] != "same":
            pos, ok = prng.decode_positions(veo, case["dtype"])
            assert ok
            np.testing.assert_array_equal(pos, fixtures.positions()[g["pos_key"]].astype(np.int64))


@pytest.mark.parametrize("cid", fixtures.case_ids(big=False))
def test_oracle_matches_reference_golden(cid):
    case = fixtures.get_case(cid)
    if case["error"]:
        with pytest.raises(Exception) as ei:
            _run(case, "data")
        assert type(ei.value).__name__ == case["error"]
        return
    check_case_against_golden(case, _run(case, "data"), _run(case, "pos"))


@pytest.mark.slow
@pytest.mark.parametrize("cid", fixtures.case_ids(big=True))
def test_oracle_matches_reference_golden_full_size(cid):
    case = fixtures.get_case(cid)
    check_case_against_golden(case, _run(case, "data"), _run(case, "pos"))


def _prim_inputs(p):
    K = prng.gen_keys(p["seed"], tuple(p["shape"]), p["dtype"], p["variant"])
    assert fixtures.sha(K) == p["input_sha"]
    return K


@pytest.mark.parametrize("idx", range(len(fixtures.prims()[0]["prims"])))
def test_oracle_primitives_match_torch_golden(idx):
    meta, arrs = fixtures.prims()
    p = meta["prims"][idx]
    K = _prim_inputs(p)
    n = oracle.norms(K)
    np.testing.assert_array_equal(n, arrs[p["key"]])  # torch.norm bits
    S = n.shape[-1]
    np.testing.assert_array_equal(oracle.argsort_prefix(n, S), arrs[p["key"] + "_argsort"])
    np.testing.assert_array_equal(oracle.argsort_prefix(n, S, descending=True),
                                  arrs[p["key"] + "_argsort_desc"])
    for k in p["topk_ks"]:
        np.testing.assert_array_equal(oracle.topk_indices(n, k), arrs[f"{p['key']}_topk{k}"])


@pytest.mark.parametrize("idx", range(len(fixtures.prims()[0]["snapkv"])))
def test_oracle_snapkv_scores_match_torch_golden(idx):
    """snapkv_lite scoring (snapkv_lite.py:96-121) bit-for-bit, incl. rows whose maxima sit where
    `max + 1e-6` differs between an fp32 epsilon and the dtype-cast python scalar torch uses."""
    meta, arrs = fixtures.prims()
    p = meta["snapkv"][idx]
    K = _prim_inputs(p)
    n = oracle.norms(K)

    def bits(a):
        # exact bits, except that every NaN is one value: torch's vectorised bf16 ops emit NaN
        # as 0xFFFF where a scalar conversion gives 0x7FC0, and the sort keys treat all NaNs as
        # one key, so NaN payloads never reach the selection
        f = a.astype(np.float32) if a.dtype != np.uint16 else prng.bf16_bits_to_f32(a)
        b = a.view(np.uint16).astype(np.int64) if a.dtype != np.float32 else a.view(np.uint32).astype(np.int64)
        return np.where(np.isnan(f), -1, b)
    np.testing.assert_array_equal(bits(oracle.snapkv_scores(n, 1)), bits(arrs[p["key"] + "_scores"]))
    np.testing.assert_array_equal(bits(oracle.snapkv_scores(n, p["pool"])),
                                  bits(arrs[p["key"] + "_pooled"]))


def test_prng_c_restatement_matches_numpy():
    """prng.normal_f32 uses oracle/liboracle.so's restatement when built; it must reproduce the
    numpy generator the fixtures were made with bit for bit (incl. across its 2^22 chunks)."""
    assert prng._clib(), "liboracle.so (make -C oracle) not built"
    for seed, n in ((1, 1000), (0xABCDEF ^ 1234, 123457), (2 ** 63 + 5, (4 << 20) + 17)):
        a, b = prng.normal_f32(seed, n), prng.normal_f32_numpy(seed, n)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
