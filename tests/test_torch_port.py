"""Pins oracle/torch_port.py (bench.py's CPU-baseline timing port of the reference's fix_size_l2
op sequence) to the golden fixtures of the unmodified reference: output bytes (SHA-256) and
kinds, at the BASELINE geometries (cfg2 S=4096, headline S=16384) and on the keep_ratio > 0
(protected tail), keep <= 0 (view) and tiny-cache branches.  CPU only."""
import numpy as np
import pytest
import torch

import fixtures
from oracle.torch_port import fix_size_l2_layer

# keep_low cases of every branch; the two BASELINE-size ones are marked slow-ish but run here
CASES = ["000_fix_size_l2_bf16_cfg2", "001_fix_size_l2_bf16_headline",
         "010_fix_size_l2_bf16_D128_normal", "012_fix_size_l2_bf16_D128_few",
         "015_fix_size_l2_bf16_equal_edge", "030_fix_size_l2_bf16_keep_le0_view",
         "031_fix_size_l2_bf16_fix0_quirk", "020_fix_size_l2_fp32_D80_normal"]


def _t(a):
    t = torch.from_numpy(np.ascontiguousarray(a))
    return t.view(torch.bfloat16) if a.dtype == np.uint16 else t


def _np(t):
    t = t.contiguous()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


def _kind(tin, tout):
    if tout is tin:
        return "same"
    same_storage = tout.untyped_storage().data_ptr() == tin.untyped_storage().data_ptr()
    return "view" if same_storage else "new"


def _present(cid):
    return any(c["id"] == cid for c in fixtures.cases()["cases"])


@pytest.mark.parametrize("cid", [c for c in CASES if _present(c)])
def test_torch_port_matches_reference_golden(cid):
    case = fixtures.get_case(cid)
    kw = dict(case["kwargs"])
    fix, kr = kw.get("fix_kv_size", 1024), kw.get("keep_ratio", 0.0)
    skip = kw.get("skip_layers", [0, 1])
    assert kw.get("strategy", "keep_low") == "keep_low"
    for li, ((K, V), g) in enumerate(zip(fixtures.make_inputs(case), case["out"])):
        k, v = _t(K), _t(V)
        if k.size(2) <= fix or li in skip:  # fix_size_l2.py:69-74, the caller's skip tests
            ko, vo = k, v
        else:
            ko, vo = fix_size_l2_layer(k, v, fix, kr)
        assert _kind(k, ko) == g["kind"], (cid, li)
        assert list(ko.shape) == g["k_shape"], (cid, li)
        assert fixtures.sha(_np(ko)) == g["k_sha"], (cid, li, "K bytes")
        assert fixtures.sha(_np(vo)) == g["v_sha"], (cid, li, "V bytes")
