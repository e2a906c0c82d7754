"""CPU-side checks of the C ABI: the library loads, exports every symbol include/kvc.h declares,
its struct layout matches, and kvc_plan (a pure host function) validates and plans correctly."""
import ctypes
import os
import re

import numpy as np
import pytest

from kvcompress import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "kvc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kvc_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = N.lib()
    declared = _declared_functions()
    assert set(declared) == set(N.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


def test_library_built_from_these_sources():
    """The loaded libkvc.so was compiled from the sources in this tree (build provenance: a
    binary that travels to the GPU box with the tree is the one its sources describe)."""
    import __graft_entry__
    assert N.source_digest() == __graft_entry__.source_digest()


def test_struct_layout():
    L = N.lib()
    assert L.kvc_layer_struct_size() == N.LAYER_DTYPE.itemsize == 136
    assert ctypes.sizeof(N.Params) == 48
    assert ctypes.sizeof(N.PlanInfo) == 64
    assert ctypes.sizeof(N.AttnParams) == 32
    assert N.ATTN_LAYER_DTYPE.itemsize == 64 and N.HH_LAYER_DTYPE.itemsize == 32
    assert L.kvc_version() == N.ABI_VERSION == 4
    assert L.kvc_max_zone_len() == 1 << 24


def test_integration_stub_matches_abi():
    """The ctypes stub INTEGRATION.md offers a maintainer has kvc_params_t's fields, in order,
    and the layer layout of _native (which is checked against the library above)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"class Params\(ctypes\.Structure\):.*?\n(.*?)\nlib\.", doc, flags=re.S)
    names = re.findall(r'"(\w+)"', m.group(1))
    assert names == [f[0] for f in N.Params._fields_]
    layer = re.search(r"LAYER = np\.dtype\(\[(.*?)\]\)", doc, flags=re.S).group(1)
    assert re.findall(r'\("(\w+)"', layer) == list(N.LAYER_DTYPE.names)


def _layer(S, zs, zl, k, sink=0, ts=0, tl=0, ptr=4096):
    t = np.zeros(1, dtype=N.LAYER_DTYPE)[0]
    t["k"] = t["v"] = t["k_out"] = t["v_out"] = ptr
    t["k_stride"] = t["v_stride"] = (32 * S * 128, S * 128, 128)
    t["seq_len"], t["zone_start"], t["zone_len"], t["n_select"] = S, zs, zl, k
    t["sink_len"], t["tail_start"], t["tail_len"] = sink, ts, tl
    return t


def _params(**kw):
    d = dict(dtype=N.KVC_BF16, batch=1, heads=32, head_dim=128, order=0, algo=0,
             phases=N.PHASE_ALL, external_index=0)
    d.update(kw)
    return N.Params(**d)


def test_plan_fills_prefix_fields_and_layout():
    table = np.array([_layer(16384, 0, 16384, 512), _layer(4096, 4, 3648, 64, 4, 3652, 444),
                      _layer(2048, 0, 0, 0, 4, 1028, 1020)], dtype=N.LAYER_DTYPE)
    rc, info = N.plan(_params(), table)
    assert rc == 0
    assert list(table["n_out"]) == [512, 512, 1024]
    assert list(table["row0"]) == [0, 32, 64]
    assert list(table["tile0"]) == [0, 32 * 256, 32 * 256 + 32 * 57]
    assert info.score_tiles == 32 * 256 + 32 * 57
    assert list(table["unit0"]) == [0, 2 * 32 * 512 * 16, 4 * 32 * 512 * 16]
    assert info.gather_units == 2 * 32 * 16 * (512 + 512 + 1024)
    assert info.rows == 96 and info.norm_row_stride == 16384 and info.index_row_stride == 512
    assert info.norm_offset == 0 and info.index_offset >= info.norm_offset + 96 * 16384 * 2


@pytest.mark.parametrize("bad, code", [
    (dict(dtype=5), -2), (dict(dtype=3), -2), (dict(dtype=2, head_dim=96), -3),
    (dict(head_dim=96), -3), (dict(head_dim=100), -3), (dict(batch=0), -1),
    (dict(order=3), -1), (dict(algo=9), -1)])
def test_plan_rejects_bad_params(bad, code):
    """(flags, reserved and device_status are covered by test_plan_rejects_unknown_flags)"""
    table = np.array([_layer(100, 0, 100, 10)], dtype=N.LAYER_DTYPE)
    rc, _ = N.plan(_params(**bad), table)
    assert rc == code


def test_plan_accepts_fp16():
    """KVC_F16 (transformers-5 pythia caches): 2-byte elements like bf16 in every region."""
    table = np.array([_layer(16384, 0, 16384, 512)], dtype=N.LAYER_DTYPE)
    rc16, i16 = N.plan(_params(dtype=N.KVC_F16), table.copy())
    rcb, ib = N.plan(_params(dtype=N.KVC_BF16), table.copy())
    assert rc16 == 0 and rcb == 0
    assert i16.workspace_bytes == ib.workspace_bytes and i16.norm_row_stride == ib.norm_row_stride
    for hd in (32, 64, 80, 128, 160, 256):  # 64/128/160/256/320/512-byte rows
        assert N.plan(_params(dtype=N.KVC_F16, head_dim=hd), table.copy())[0] == 0


def test_plan_accepts_every_pythia_head_dim():
    """D = 32 (pythia-14m/31m), 64, 80, 128, 256 (pythia-1b) in every dtype: 64..1024-byte rows."""
    table = np.array([_layer(4096, 0, 4096, 512)], dtype=N.LAYER_DTYPE)
    for dt in (N.KVC_BF16, N.KVC_F16, N.KVC_F32):
        for hd in (32, 64, 80, 128, 256):
            assert N.plan(_params(dtype=dt, head_dim=hd), table.copy())[0] == 0, (dt, hd)
    assert N.plan(_params(dtype=N.KVC_F32, head_dim=512), table.copy())[0] == -3


def test_plan_rejects_bad_layers():
    cases = [
        (_layer(100, 0, 101, 10), -1),                 # zone past the end
        (_layer(100, 0, 100, 101), -1),                # selecting more than the zone
        (_layer(100, 0, 100, 10, ts=95, tl=10), -1),   # tail past the end
        (_layer(100, 0, 100, 10, ptr=4100), -4),       # misaligned pointer
        (_layer((1 << 24) + 64, 0, (1 << 24) + 64, 10), -5),  # zone longer than 2^24 positions
    ]
    for t, code in cases:
        rc, _ = N.plan(_params(), np.array([t], dtype=N.LAYER_DTYPE))
        assert rc == code, (t, rc)
    # select-all and pure-copy layers may be longer still (no selection runs)
    rc, _ = N.plan(_params(), np.array([_layer(70000, 0, 70000, 70000)], dtype=N.LAYER_DTYPE))
    assert rc == 0


def test_plan_long_zone_gets_global_scratch():
    """Zones longer than the LDS limit (16384) select from a per-row global scratch."""
    short = np.array([_layer(16384, 0, 16384, 512)], dtype=N.LAYER_DTYPE)
    long_ = np.array([_layer(40000, 0, 40000, 512)], dtype=N.LAYER_DTYPE)
    rc0, i0 = N.plan(_params(), short)
    rc1, i1 = N.plan(_params(), long_)
    assert rc0 == 0 and rc1 == 0
    n_cap = 40000 + (-40000 % 64)
    # key | idx | two rank tables of n_cap/2 + 1 ranks (+ 64 sinks + 8 pad each)
    row = n_cap * 2 + n_cap * 2 + 2 * (64 + n_cap // 2 + 1 + 8) * 2
    row += -row % 256
    idx_end = i1.index_offset + 32 * i1.index_row_stride * 4
    idx_end += -idx_end % 256
    tiles = 32 * (n_cap // 64) * 4  # SCORE's per-tile statistics (level-0 counts), round 6
    assert i1.workspace_bytes == idx_end + 32 * row + tiles


def test_plan_zone_beyond_u16_positions_gets_u32_scratch():
    """Zones longer than 65536 positions select with u32 positions and full rank tables:
    key | idx (u32) | two tables of n_cap/2 + 2 u32 ranks per row."""
    t = np.array([_layer(100000, 0, 100000, 512)], dtype=N.LAYER_DTYPE)
    rc, info = N.plan(_params(), t)
    assert rc == 0
    n_cap = 100000 + (-100000 % 64)
    row = n_cap * 2 + n_cap * 4 + 2 * (n_cap // 2 + 2) * 4
    row += -row % 256
    idx_end = info.index_offset + 32 * info.index_row_stride * 4
    idx_end += -idx_end % 256
    tiles = 32 * (n_cap // 64) * 4  # SCORE's per-tile statistics (level-0 counts), round 6
    assert info.workspace_bytes == idx_end + 32 * row + tiles


def test_status_strings():
    for code in range(-7, 1):
        assert N.status_string(code)


def test_launch_revalidates_against_plan():
    table = np.array([_layer(100, 0, 100, 10)], dtype=N.LAYER_DTYPE)
    rc, info = N.plan(_params(), table)
    assert rc == 0
    table["unit0"] = 7  # tampered plan fields are rejected before any HIP call
    assert N.launch(_params(), table, 0, 0, 0) == -1


def test_plan_rejects_unknown_flags():
    """Unknown flag bits and a non-zero reserved field are refused, not ignored (a future flag
    must not be silently dropped by this library); SHARED_INDEX needs external indices."""
    table = np.array([_layer(100, 0, 100, 10)], dtype=N.LAYER_DTYPE)
    assert N.plan(_params(flags=N.FLAG_SPLIT_SELECT_GATHER), table.copy())[0] == 0
    assert N.plan(_params(flags=16), table.copy())[0] == -1
    assert N.plan(_params(flags=1 << 30), table.copy())[0] == -1
    # the gather-part flags: one at a time, and only over external indices (two launches of
    # the engine's own selection would SCORE / SELECT into one workspace concurrently)
    ext = dict(external_index=1, phases=N.PHASE_GATHER)
    assert N.plan(_params(flags=N.FLAG_GATHER_FIXED, **ext), table.copy())[0] == 0
    assert N.plan(_params(flags=N.FLAG_GATHER_SELECTED, **ext), table.copy())[0] == 0
    assert N.plan(_params(flags=N.FLAG_GATHER_FIXED), table.copy())[0] == -1
    assert N.plan(_params(flags=N.FLAG_GATHER_SELECTED), table.copy())[0] == -1
    assert N.plan(_params(flags=N.FLAG_GATHER_FIXED | N.FLAG_GATHER_SELECTED, **ext),
                  table.copy())[0] == -1
    assert N.plan(_params(reserved=1), table.copy())[0] == -1
    assert N.plan(_params(flags=N.FLAG_SHARED_INDEX), table.copy())[0] == -1
    assert N.plan(_params(flags=N.FLAG_SHARED_INDEX, external_index=1,
                          phases=N.PHASE_GATHER), table.copy())[0] == 0


def _attn_params(**kw):
    d = dict(dtype=N.KVC_BF16, batch=1, heads=32, vec_bytes=32, decay=0.9, flags=0)
    d.update(kw)
    return N.AttnParams(**d)


def test_heavy_hitter_workspace_and_validation():
    """kvc_hh_workspace: head-summed rows [layers*batch, round_up(max zone, 64)] of dtype, plus
    global selection scratch for zones longer than 16384; bad tables are refused."""
    t = np.zeros(2, dtype=N.HH_LAYER_DTYPE)
    t[0] = (4096, 2100, 4, 1652, 64, 0, 0)
    t[1] = (4096, 600, 4, 152, 64, 0, 0)
    rc, n = N.hh_workspace(_attn_params(), t)
    assert rc == 0 and n == -(-(2 * 1664 * 2) // 256) * 256
    rc, n4 = N.hh_workspace(_attn_params(dtype=N.KVC_F32), t)
    assert rc == 0 and n4 == -(-(2 * 1664 * 4) // 256) * 256
    long_ = t.copy()
    long_[0]["acc_len"], long_[0]["zone_len"] = 40000, 39000
    rc, nl = N.hh_workspace(_attn_params(), long_)
    assert rc == 0 and nl > 2 * 39040 * 2 + 2 * 39040 * 4
    for field, val in (("zone_len", 2097), ("n_select", 1653), ("zone_start", -1),
                       ("reserved", 1), ("col_chunk", -2)):
        bad = t.copy()
        bad[0][field] = val
        assert N.hh_workspace(_attn_params(), bad)[0] == -1, field
    assert N.hh_workspace(_attn_params(vec_bytes=24), t)[0] == -1
    assert N.hh_workspace(_attn_params(flags=1), t)[0] == -1
    assert N.hh_workspace(_attn_params(dtype=9), t)[0] == -2


def test_attn_accumulate_validates_before_launching():
    t = np.zeros(1, dtype=N.ATTN_LAYER_DTYPE)
    t[0] = (4096, (32 * 7 * 100, 7 * 100, 100), 0, 8192, 7, 100, 0, 0)
    bad = t.copy()
    bad[0]["old_len"] = 101  # more carried columns than the new key length
    assert N.attn_accumulate(_attn_params(), bad, 0) == -1
    bad = t.copy()
    bad[0]["old_len"] = 50  # carried columns without acc_old
    assert N.attn_accumulate(_attn_params(), bad, 0) == -1
    bad = t.copy()
    bad[0]["q_len"] = 0
    assert N.attn_accumulate(_attn_params(), bad, 0) == -1
    assert N.attn_accumulate(_attn_params(batch=0), t, 0) == -1


def test_algo_enum_and_stable_zone_limit():
    """kvc_algo in the header equals the Python constants; kvc_plan accepts KVC_ALGO_STABLE for
    zones up to 65 536 positions (KVC_E_TOO_LONG beyond, unless the indices are external) and
    refuses unknown algorithms."""
    src = open(os.path.join(ROOT, "include", "kvc.h")).read()
    enum = re.search(r"enum kvc_algo \{([^}]*)\}", src).group(1)
    vals = dict((a.strip(), int(b)) for a, b in re.findall(r"(\w+)\s*=\s*(\d+)", enum))
    assert vals == {"KVC_ALGO_SORT": N.KVC_ALGO_SORT, "KVC_ALGO_TOPK": N.KVC_ALGO_TOPK,
                    "KVC_ALGO_STABLE": N.KVC_ALGO_STABLE}
    ok = np.array([_layer(16384, 0, 16384, 512)], dtype=N.LAYER_DTYPE)
    assert N.plan(_params(algo=N.KVC_ALGO_STABLE), ok)[0] == 0
    mid = np.array([_layer(65536, 0, 65536, 512)], dtype=N.LAYER_DTYPE)
    assert N.plan(_params(algo=N.KVC_ALGO_STABLE), mid)[0] == 0
    long = np.array([_layer(65600, 0, 65600, 512)], dtype=N.LAYER_DTYPE)
    assert N.plan(_params(algo=N.KVC_ALGO_STABLE), long.copy())[0] == N.KVC_E_TOO_LONG
    assert N.plan(_params(algo=N.KVC_ALGO_SORT), long.copy())[0] == 0
    assert N.plan(_params(algo=N.KVC_ALGO_STABLE, external_index=1,
                          phases=N.PHASE_GATHER), long.copy())[0] == 0
    assert N.plan(_params(algo=3), ok.copy())[0] == -1  # KVC_E_ARG


def test_heavy_hitter_stable_flag():
    """KVC_ATTN_HH_STABLE: accepted by kvc_hh_workspace (zones up to 65 536 positions), unknown
    flag bits refused."""
    def p(flags):
        return N.AttnParams(dtype=N.KVC_BF16, batch=1, heads=4, vec_bytes=32, decay=0.9,
                            flags=flags, device_status=None)

    def table(m):
        t = np.zeros(1, dtype=N.HH_LAYER_DTYPE)
        t[0] = (4096, m + 448, 4, m, 64, 0, 0)
        return t
    assert N.hh_workspace(p(N.ATTN_HH_STABLE), table(15936))[0] == 0
    assert N.hh_workspace(p(0), table(70000))[0] == 0
    assert N.hh_workspace(p(N.ATTN_HH_STABLE), table(70000))[0] == N.KVC_E_TOO_LONG
    assert N.hh_workspace(p(8), table(15936))[0] == -1  # KVC_E_ARG
    assert N.hh_workspace(p(N.ATTN_OLD_DTYPE(N.KVC_F32)), table(15936))[0] == -1  # accumulate only


def test_device_status_bits_match_header():
    """enum kvc_device_status (include/kvc.h, ABI v4) and the Python side agree, and every bit
    has a name in the opt-in status check's message table."""
    from kvcompress import _engine as E
    hdr = open(os.path.join(ROOT, "include", "kvc.h")).read()
    vals = dict(re.findall(r"(KVC_DEV_\w+) = (\d+)", hdr))
    assert vals == {"KVC_DEV_SELECT_BOUNDS": "1", "KVC_DEV_INDEX_RANGE": "2",
                    "KVC_DEV_INTERNAL": "4"}
    assert (N.DEV_SELECT_BOUNDS, N.DEV_INDEX_RANGE, N.DEV_INTERNAL) == (1, 2, 4)
    assert [b for b, _ in E._STATUS_BITS] == [1, 2, 4]
    assert all(name.split()[0] in vals for _, name in E._STATUS_BITS)


def test_scored_calls_reserve_the_tile_statistics_region():
    """kvc_plan reserves rows x norm_row_stride / 64 u32 after the index region for SCORE's
    per-tile statistics (round 6): a snapkv row's tile norm maxima, a plain-norm row's level-0
    ge / le counts -- the same size either way, and nothing for a call that selects nothing."""
    H, D = 4, 64

    def plan(mode):
        t = np.zeros(1, dtype=N.LAYER_DTYPE)
        t[0]["k"] = t[0]["v"] = t[0]["k_out"] = t[0]["v_out"] = 4096
        t[0]["k_stride"] = t[0]["v_stride"] = (H * 1000 * D, 1000 * D, D)
        t[0]["seq_len"], t[0]["zone_start"], t[0]["zone_len"], t[0]["n_select"] = 1000, 0, 968, 480
        t[0]["score_mode"], t[0]["pool_kernel"] = mode, 5 if mode else 0
        p = N.Params(dtype=N.KVC_BF16, batch=1, heads=H, head_dim=D, order=1, algo=1,
                     phases=N.PHASE_ALL, external_index=0)
        rc, info = N.plan(p, t)
        assert rc == 0
        return info
    a, b = plan(0), plan(1)
    assert a.workspace_bytes == b.workspace_bytes
    region = b.rows * (b.norm_row_stride // 64) * 4
    idx_end = b.index_offset + b.rows * b.index_row_stride * 4
    assert b.workspace_bytes == -(-idx_end // 256) * 256 + region
