"""The device status channel as a contract (include/kvc.h, kvc_device_status).

KVC_DEV_SELECT_BOUNDS is raised by the selection kernels when a row's zone is longer than the
kernel's capacity (csrc/kvc.hip select_body): the row then selects nothing and -- in the fused
SELECT_GATHER kernel -- writes no output row.  kvc_launch always dispatches a sufficient capacity,
so the guard is driven through kvc_debug_select_capacity, which launches the same kernels with a
caller-chosen capacity.  (tests/conftest.py also asserts after every GPU test that the engine's
own status word stayed 0.)  Reference of the selection being guarded: fix_size_l2.py:104-108."""
import numpy as np
import pytest
import torch

from kvcompress import _native as N

pytestmark = pytest.mark.gpu
KVC_E_ARG = -1


def _table(layers, H, D):
    t = np.zeros(len(layers), dtype=N.LAYER_DTYPE)
    for i, (k, v, ko, vo, S, n_sel) in enumerate(layers):
        t[i] = (k.data_ptr(), v.data_ptr(), ko.data_ptr(), vo.data_ptr(), (H * S * D, S * D, D),
                (H * S * D, S * D, D), S, 0, S, n_sel, 0, 0, 0, 0, 0, 0, 0, 0, 0)
    return t


@pytest.mark.parametrize("phases", ["select", "select_gather"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_select_bounds_reported_and_row_left_unwritten(phases, dt):
    H, D, n_sel = 4, 64, 100
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    specs = []
    for S in (1000, 3000):  # layer 1 exceeds the 1 024-position capacity given below
        k = torch.randn(1, H, S, D, device=dev, generator=g).to(dt)
        v = torch.randn(1, H, S, D, device=dev, generator=g).to(dt)
        ko = torch.full((1, H, n_sel, D), -7.0, device=dev, dtype=dt)
        vo = torch.full_like(ko, -7.0)
        specs.append((k, v, ko, vo, S, n_sel))
    t = _table(specs, H, D)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    dtype = {torch.bfloat16: N.KVC_BF16, torch.float32: N.KVC_F32}[dt]
    p = N.Params(dtype=dtype, batch=1, heads=H, head_dim=D, order=N.KVC_ASC,
                 algo=N.KVC_ALGO_SORT, phases=N.PHASE_ALL, external_index=0,
                 flags=N.FLAG_SPLIT_SELECT_GATHER, device_status=status.data_ptr())
    rc, info = N.plan(p, t)
    assert rc == 0
    stream = torch.cuda.current_stream().cuda_stream
    ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
    # the expected result through the normal launch (three kernels: the index region is
    # written), for layer 0
    assert N.launch(p, t, ws.data_ptr(), int(info.workspace_bytes), stream) == 0
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    rows = int(info.rows)
    istride = int(info.index_row_stride)
    iv = ws[info.index_offset:info.index_offset + rows * istride * 4].view(torch.int32)
    want_idx = iv[:H * istride].clone()
    want_k0, want_v0 = specs[0][2].clone(), specs[0][3].clone()
    for s in specs:  # sentinels in the outputs and the index region
        s[2].fill_(-7.0)
        s[3].fill_(-7.0)
    iv.fill_(-1)
    p.phases = N.PHASE_SELECT if phases == "select" else N.PHASE_SELECT | N.PHASE_GATHER
    assert N.debug_select_capacity(p, t, ws.data_ptr(), int(info.workspace_bytes), 1024,
                                   stream) == 0
    torch.cuda.synchronize()
    assert int(status.item()) == N.DEV_SELECT_BOUNDS
    iv2 = iv.view(rows, istride)
    if phases == "select":
        # layer 0 selected exactly as the normal launch; layer 1's rows untouched
        assert torch.equal(iv2[:H, :n_sel].flatten(),
                           want_idx.view(H, istride)[:, :n_sel].flatten())
        assert bool((iv2[H:] == -1).all())
    else:
        assert torch.equal(specs[0][2], want_k0) and torch.equal(specs[0][3], want_v0)
        assert bool((specs[1][2] == -7.0).all()) and bool((specs[1][3] == -7.0).all())
    # bad capacities are refused on the host
    for cap in (0, 100, 8256):
        assert N.debug_select_capacity(p, t, ws.data_ptr(), int(info.workspace_bytes), cap,
                                       stream) == KVC_E_ARG


def test_opt_in_status_check_raises_naming_the_bit():
    """kvcompress._engine.set_status_check(True) (or KVC_CHECK_STATUS=1 at import): a compress
    call after which the engine's device word is non-zero raises RuntimeError naming the bit and
    clears the word; clean calls pass.  The bit is set through kvc_debug_select_capacity on the
    engine's own word, as a dispatch bug inside a call would set it."""
    from kvcompress import _engine as E
    from kvcompress.methods import fix_size_l2_compress
    H, D, n_sel, S = 4, 64, 100, 3000
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(9)
    k = torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16)
    v = torch.randn(1, H, S, D, device=dev, generator=g).to(torch.bfloat16)
    ko, vo = torch.empty(1, H, n_sel, D, device=dev, dtype=k.dtype), torch.empty(
        1, H, n_sel, D, device=dev, dtype=k.dtype)
    t = _table([(k, v, ko, vo, S, n_sel)], H, D)
    word = E.status_word(0)
    p = N.Params(dtype=N.KVC_BF16, batch=1, heads=H, head_dim=D, order=N.KVC_ASC,
                 algo=N.KVC_ALGO_SORT, phases=N.PHASE_SELECT | N.PHASE_GATHER, external_index=0,
                 flags=0, device_status=word.data_ptr())
    rc, info = N.plan(p, t)
    assert rc == 0
    ws = torch.zeros(int(info.workspace_bytes), dtype=torch.uint8, device=dev)
    prev = E.set_status_check(True)
    try:
        layers = [(k, v)]
        out = fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])  # clean: no raise
        assert out[0][0].shape[2] == 512
        assert N.debug_select_capacity(p, t, ws.data_ptr(), int(info.workspace_bytes), 1024,
                                       torch.cuda.current_stream().cuda_stream) == 0
        with pytest.raises(RuntimeError, match="KVC_DEV_SELECT_BOUNDS"):
            fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])
        assert E.device_status(0) == 0  # cleared by the raise
        fix_size_l2_compress(layers, fix_kv_size=512, skip_layers=[])
    finally:
        E.set_status_check(prev)


def test_status_word_first_made_inside_inference_mode_stays_clearable():
    """The evaluation loops run under torch.inference_mode(); a status word first created there
    must still be a normal tensor, which device_status(clear=True) zeroes in place afterwards."""
    from kvcompress import _engine as E
    with torch.inference_mode():
        w = E._new_status_word(0)
    assert not w.is_inference()
    w.zero_()
    torch.cuda.synchronize()
    assert int(w.item()) == 0
