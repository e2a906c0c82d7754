"""evaluate_with_attention_compression / compare_h2o_methods (reference:
kvcompress/evaluate_attention.py) on a small random-weight GPT-NeoX.

CPU: the harness runs end to end with the numpy oracle standing in for the manager and the
compress call (test infrastructure), real attention weights reach the manager although the model
is configured for sdpa, and the model's attention implementation is restored afterwards; the
loops reproduce the UNMODIFIED reference's loops on the same CPU model exactly
(tests/golden/eval_attention.json).
GPU: the engine's manager + h2o_attention_compress against the oracle's -- identical caches at
every step, so the PPL and accuracy match exactly (PPL delta 0), in fp32 / bf16 / fp16, and for a grouped-query Llama."""
import numpy as np
import pytest
import torch

from gpu_util import to_dev, to_np
from oracle import h2o_oracle as HO
from step_digest import Recorder, first_divergence, replay, unpack
from test_ppl_parity import TEXT, ToyTokenizer, gqa_model, toy_model

KW = dict(start_size=4, heavy_hitter_size=16, recent_size=40)
THREADS = 8  # reduction order of both managers' sums


class OracleManager:
    """The oracle's H2OManager behind the reference manager's interface (torch in, numpy
    state)."""

    def __init__(self, **kw):
        self.kw = kw
        self.updates = 0
        self.reset()

    def reset(self):
        self.m = HO.H2OManager(threads=THREADS, **self.kw)

    def update_attention_scores(self, attentions, skip_layers=()):
        if attentions is not None and len(attentions):
            self.updates += 1
        self.m.update_attention_scores(
            None if attentions is None else [None if a is None else to_np(a)
                                             for a in attentions], skip_layers)


def oracle_compress(kv_list, attention_scores=None, h2o_manager=None, **kw):
    dev = kv_list[0][0].device
    atts = None if attention_scores is None else [None if a is None else to_np(a)
                                                  for a in attention_scores]
    if h2o_manager is not None and atts is not None:
        h2o_manager.m.update_attention_scores(atts, kw.get("skip_layers", ()))
    out = HO.h2o_attention_compress([(to_np(k), to_np(v)) for k, v in kv_list], None,
                                    h2o_manager.m if h2o_manager is not None else None, **kw)
    return [(k, v) if kind == "same" else (to_dev(ko, dev), to_dev(vo, dev))
            for (k, v), (ko, vo, kind) in zip(kv_list, out)]


def _run_oracle(model, tok, max_tokens, monkeypatch, **kw):
    from kvcompress import evaluate_attention as EA
    monkeypatch.setattr(EA, "h2o_attention_compress", oracle_compress)
    mgr = OracleManager(**kw)
    r = EA.evaluate_with_attention_compression(model, tok, TEXT, h2o_manager=mgr,
                                               max_tokens=max_tokens, skip_layers=[0],
                                               show_progress=False, **kw)
    monkeypatch.undo()
    return r, mgr


def test_harness_runs_with_oracle_on_cpu(monkeypatch):
    model = toy_model(torch.float32, "cpu", layers=2)
    assert model.config._attn_implementation == "sdpa"
    tok = ToyTokenizer(512)
    r, mgr = _run_oracle(model, tok, 120, monkeypatch, **KW)
    assert model.config._attn_implementation == "sdpa"  # restored
    assert mgr.updates == 119  # every step's attention weights reached the manager
    assert r["num_tokens"] == 119
    assert r["final_cache_size"] == sum(KW.values())
    assert np.isfinite(r["perplexity"]) and 0.0 <= r["accuracy"] <= 1.0
    assert set(r) == {"perplexity", "accuracy", "num_tokens", "final_cache_size", "ttft",
                      "tpot", "throughput", "total_time"}


def test_gqa_model_runs_with_oracle_on_cpu(monkeypatch):
    model = gqa_model(torch.float32, "cpu", layers=2)
    r, mgr = _run_oracle(model, ToyTokenizer(512), 100, monkeypatch, **KW)
    assert mgr.updates == 99 and r["final_cache_size"] == sum(KW.values())
    assert np.isfinite(r["perplexity"])


def test_short_text_returns_reference_empty_result():
    from kvcompress.evaluate_attention import evaluate_with_attention_compression
    model = toy_model(torch.float32, "cpu", layers=1)
    r = evaluate_with_attention_compression(model, ToyTokenizer(512), "a",
                                            h2o_manager=OracleManager(**KW), show_progress=False)
    assert r["perplexity"] == float("inf") and r["num_tokens"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_ppl_delta_zero_engine_vs_oracle(dtype, monkeypatch):
    from kvcompress.evaluate_attention import evaluate_with_attention_compression
    from kvcompress.methods.h2o_attention import create_h2o_manager_from_model
    from kvcompress import _engine
    model = toy_model(dtype, "cuda:0")
    tok = ToyTokenizer(512)
    mgr = create_h2o_manager_from_model(model, **KW)
    mgr.reduction_threads = THREADS
    a = evaluate_with_attention_compression(model, tok, TEXT, h2o_manager=mgr, max_tokens=300,
                                            skip_layers=[0], show_progress=False, **KW)
    b, _ = _run_oracle(model, tok, 300, monkeypatch, **KW)
    assert a["final_cache_size"] == b["final_cache_size"] == sum(KW.values())
    assert a["perplexity"] == b["perplexity"], (a["perplexity"], b["perplexity"])
    assert a["accuracy"] == b["accuracy"]
    assert _engine.device_status(0) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gqa_ppl_delta_zero_engine_vs_oracle(dtype, monkeypatch):
    """Grouped-query attention: heavy hitters from 4-head accumulations select rows of 2-head
    K / V caches (one index list per layer, shared by the heads)."""
    from kvcompress.evaluate_attention import evaluate_with_attention_compression
    from kvcompress.methods.h2o_attention import create_h2o_manager_from_model
    from kvcompress import _engine
    model = gqa_model(dtype, "cuda:0")
    tok = ToyTokenizer(512)
    mgr = create_h2o_manager_from_model(model, **KW)
    mgr.reduction_threads = THREADS
    a = evaluate_with_attention_compression(model, tok, TEXT, h2o_manager=mgr, max_tokens=240,
                                            skip_layers=[0], show_progress=False, **KW)
    b, _ = _run_oracle(model, tok, 240, monkeypatch, **KW)
    assert a["final_cache_size"] == b["final_cache_size"] == sum(KW.values())
    assert a["perplexity"] == b["perplexity"], (a["perplexity"], b["perplexity"])
    assert a["accuracy"] == b["accuracy"]
    assert _engine.device_status(0) == 0


@pytest.mark.gpu
def test_compare_h2o_methods_runs_on_engine():
    from kvcompress.evaluate_attention import compare_h2o_methods
    model = toy_model(torch.bfloat16, "cuda:0", layers=3)
    res = compare_h2o_methods(model, ToyTokenizer(512), TEXT * 2, max_tokens=560,
                              heavy_hitter_sizes=[32], skip_layers=[0])
    assert [r["method"] for r in res] == ["baseline", "h2o_l2_hh32", "h2o_attention_hh32"]
    assert res[0]["final_cache_size"] == 559
    assert res[1]["final_cache_size"] == res[2]["final_cache_size"] == 512
    assert all(np.isfinite(r["perplexity"]) for r in res)


def _same_host(gold):
    """The golden runs' CPU forward rounding belongs to the host that made them."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from gen_eval_attention import cpu_model
    if cpu_model() != gold["cpu_model"]:
        pytest.skip(f"golden made on {gold['cpu_model']!r}; this host is {cpu_model()!r}")


def test_loops_reproduce_reference_golden(monkeypatch):
    """The unmodified reference's loops on this CPU model (tests/golden/gen_eval_attention.py ->
    eval_attention.json): the package's evaluate_with_compression (baseline, h2o_l2) and
    evaluate_with_attention_compression (h2o_attention) over the oracle's compress / manager give
    the reference's perplexity, accuracy and cache size exactly -- the same call sequence
    (update, compress with its second accumulation, reset) on the same arithmetic."""
    import json
    import os
    from kvcompress import evaluate_attention as EA
    from kvcompress.evaluate import evaluate_with_compression
    from test_ppl_parity import oracle_compress as oracle_method
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                       "eval_attention.json")))
    _same_host(gold)
    prev = torch.get_num_threads()
    torch.set_num_threads(gold["threads"])
    try:
        model = toy_model(torch.float32, "cpu", layers=gold["layers"])
        tok, text, kw, n = ToyTokenizer(512), TEXT * 2, gold["kw"], gold["max_tokens"]
        rec = Recorder(oracle_method("h2o_l2"))
        got = {"baseline": evaluate_with_compression(model, tok, text, max_tokens=n,
                                                     show_progress=False),
               "h2o_l2": evaluate_with_compression(model, tok, text, compress_fn=rec,
                                                   compress_kwargs=kw, max_tokens=n,
                                                   skip_layers=[0], show_progress=False)}
        monkeypatch.setattr(EA, "h2o_attention_compress", oracle_compress)
        got["h2o_attention"] = EA.evaluate_with_attention_compression(
            model, tok, text, h2o_manager=OracleManager(**kw), max_tokens=n, skip_layers=[0],
            show_progress=False, **kw)
    finally:
        torch.set_num_threads(prev)
    for name, ref in gold["runs"].items():
        for f in ("perplexity", "accuracy", "num_tokens", "final_cache_size"):
            assert got[name][f] == ref[f], (name, f, got[name][f], ref[f])
    # every compress call: the same input keys and the same kept positions as the reference's
    assert rec.steps == unpack(gold["steps"]["h2o_l2"])


def _gold():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                       "eval_attention.json")))


@pytest.mark.parametrize("i", range(len(_gold()["methods"])))
def test_compression_loop_reproduces_reference_golden(i):
    """Every method configuration of test_ppl_parity through the reference's own
    evaluate_with_compression (eval_attention.json "methods") and through the package's, over
    the oracle's compress: identical perplexity, accuracy, token count and cache size."""
    from kvcompress.evaluate import evaluate_with_compression
    from test_ppl_parity import oracle_compress as oracle_method
    gold = _gold()
    _same_host(gold)
    ref = gold["methods"][i]
    prev = torch.get_num_threads()
    torch.set_num_threads(gold["threads"])
    try:
        model = toy_model(torch.float32, "cpu", layers=gold["layers"])
        rec = Recorder(oracle_method(ref["name"]))
        got = evaluate_with_compression(model, ToyTokenizer(512), TEXT * 2,
                                        compress_fn=rec, compress_kwargs=ref["kwargs"],
                                        max_tokens=gold["max_tokens"], skip_layers=[0],
                                        show_progress=False)
    finally:
        torch.set_num_threads(prev)
    for f in ("perplexity", "accuracy", "num_tokens", "final_cache_size"):
        assert got[f] == ref[f], (ref["name"], ref["kwargs"], f, got[f], ref[f])
    # every compress call: the same input keys and the same kept positions as the reference's
    assert rec.steps == unpack(ref["steps"])


def _to_gpu(t):
    return None if t is None else t.to("cuda:0")


def _engine_bridge(name):
    """compress_fn for a CPU model: the layers go to the GPU, through the engine, and back."""
    from kvcompress.methods import get_compress_fn
    fn = get_compress_fn(name)

    def run(kv_list, **kw):
        out = fn([(_to_gpu(k), _to_gpu(v)) for k, v in kv_list], **kw)
        return [(k.cpu(), v.cpu()) for k, v in out]
    return run


class _EngineManagerBridge:
    """The engine's H2OAttentionManager (state on the GPU) behind a CPU model's loop."""

    def __init__(self, **kw):
        from kvcompress.methods.h2o_attention import H2OAttentionManager
        self.inner = H2OAttentionManager(num_layers=3, num_heads=4, **kw)
        self.inner.reduction_threads = THREADS

    def reset(self):
        self.inner.reset()

    def update_attention_scores(self, attentions, skip_layers=()):
        self.inner.update_attention_scores(
            None if attentions is None else tuple(_to_gpu(a) for a in attentions), skip_layers)


def _engine_h2o_attention_compress(kv_list, attention_scores=None, h2o_manager=None, **kw):
    from kvcompress.methods.h2o_attention import h2o_attention_compress
    out = h2o_attention_compress(
        [(_to_gpu(k), _to_gpu(v)) for k, v in kv_list],
        attention_scores=None if attention_scores is None else
        tuple(_to_gpu(a) for a in attention_scores),
        h2o_manager=h2o_manager.inner, **kw)
    return [(k.cpu(), v.cpu()) for k, v in out]


@pytest.mark.gpu
def test_engine_loops_with_cpu_model_match_oracle_loops(monkeypatch):
    """The golden runs' loops with the model on this host's CPU and every compression on the HIP
    engine, against the same loops over the oracle on the same host: identical perplexity,
    accuracy and cache size for every method and the attention-score run.  (On the host that
    made eval_attention.json the oracle loops equal the unmodified reference's runs --
    test_loops_reproduce_reference_golden / test_compression_loop_reproduces_reference_golden;
    the CPU forward's rounding differs between host CPUs, so the GPU box compares like with
    like.)"""
    from kvcompress import _engine
    from kvcompress import evaluate_attention as EA
    from kvcompress.evaluate import evaluate_with_compression
    from test_ppl_parity import oracle_compress as oracle_method
    gold = _gold()
    prev = torch.get_num_threads()
    torch.set_num_threads(gold["threads"])
    fields = ("perplexity", "accuracy", "num_tokens", "final_cache_size")
    try:
        model = toy_model(torch.float32, "cpu", layers=gold["layers"])
        tok, text, n = ToyTokenizer(512), TEXT * 2, gold["max_tokens"]
        for ref in gold["methods"]:
            a, b = (evaluate_with_compression(model, tok, text, compress_fn=fn,
                                              compress_kwargs=ref["kwargs"], max_tokens=n,
                                              skip_layers=[0], show_progress=False)
                    for fn in (_engine_bridge(ref["name"]), oracle_method(ref["name"])))
            for f in fields:
                assert a[f] == b[f], (ref["name"], ref["kwargs"], f, a[f], b[f])
        kw = gold["kw"]
        monkeypatch.setattr(EA, "h2o_attention_compress", _engine_h2o_attention_compress)
        a = EA.evaluate_with_attention_compression(model, tok, text,
                                                   h2o_manager=_EngineManagerBridge(**kw),
                                                   max_tokens=n, skip_layers=[0],
                                                   show_progress=False, **kw)
        monkeypatch.setattr(EA, "h2o_attention_compress", oracle_compress)
        b = EA.evaluate_with_attention_compression(model, tok, text,
                                                   h2o_manager=OracleManager(**kw),
                                                   max_tokens=n, skip_layers=[0],
                                                   show_progress=False, **kw)
        for f in fields:
            assert a[f] == b[f], ("h2o_attention", f, a[f], b[f])
    finally:
        torch.set_num_threads(prev)
    assert _engine.device_status(0) == 0


@pytest.mark.gpu
def test_engine_loop_selections_match_reference_steps():
    """The reference's loops step by step, on this host (eval_attention.json "steps", recorded
    by tests/golden/gen_eval_attention.py from the unmodified reference): the same loop with the
    model on this host's CPU and every compress call on the HIP engine, each call recorded the
    same way (tests/golden/step_digest.py).  At every step whose input keys equal the
    reference's -- i.e. until this host's CPU forward first rounds differently -- the engine must
    have kept exactly the reference's positions; a run whose keys never diverge must also give
    the reference's perplexity.  The first diverging step of every method is reported
    (KVC_LOOP_REPORT=path writes the report as JSON): there the engine's every earlier selection
    equalled the reference's, so the caches were identical, and the keys differ because the new
    token's forward did."""
    import json
    import os
    from kvcompress import _engine
    from kvcompress.evaluate import evaluate_with_compression
    from gen_eval_attention import cpu_model
    gold = _gold()
    prev = torch.get_num_threads()
    torch.set_num_threads(gold["threads"])
    fields = ("perplexity", "accuracy", "num_tokens", "final_cache_size")
    runs = [("h2o_l2", gold["kw"], gold["steps"]["h2o_l2"], gold["runs"]["h2o_l2"])]
    runs += [(m["name"], m["kwargs"], m["steps"], m) for m in gold["methods"]]
    report = {"host_cpu": cpu_model(), "golden_cpu": gold["cpu_model"], "runs": []}
    try:
        model = toy_model(torch.float32, "cpu", layers=gold["layers"])
        for name, kw, steps, ref in runs:
            rec = Recorder(_engine_bridge(name))
            got = evaluate_with_compression(model, ToyTokenizer(512), TEXT * 2, compress_fn=rec,
                                            compress_kwargs=kw, max_tokens=gold["max_tokens"],
                                            skip_layers=[0], show_progress=False)
            want = unpack(steps)
            n, div, bad = first_divergence(rec.steps, want)
            report["runs"].append({"method": name, "kwargs": kw, "steps": len(want),
                                   "steps_with_equal_keys": n, "first_key_divergence": div,
                                   "selection_mismatches_before_it": bad,
                                   "ppl": got["perplexity"], "ref_ppl": ref["perplexity"]})
            assert not bad, (name, kw, "engine selections differ from the reference's", bad[:5])
            assert len(rec.steps) == len(want)
            if div is None:  # this host's forward reproduced every step's keys
                for f in fields:
                    assert got[f] == ref[f], (name, kw, f, got[f], ref[f])
    finally:
        torch.set_num_threads(prev)
        path = os.environ.get("KVC_LOOP_REPORT")
        if path:
            with open(path, "w") as f:
                json.dump(report, f, indent=1)
        print(json.dumps(report))
    assert _engine.device_status(0) == 0


def _rows():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "eval_loop_rows.npz"))


def _replay_case(name, fn):
    from gen_eval_attention import ROW_LAYERS
    gold = _gold()
    ref = next(m for m in gold["methods"] if m["name"] == name)
    kw = dict(ref["kwargs"], skip_layers=[0])
    got = replay(fn, _rows()[f"{name}_rows"], gold["layers"], ROW_LAYERS, kw)
    want = [pd for _, pd in unpack(ref["steps"])]
    assert len(got) == len(want) == gold["max_tokens"] - 1
    return got, want


@pytest.mark.parametrize("name", ["snapkv_lite", "l2_compress"])
def test_oracle_replays_reference_loop_selections(name):
    """Host-independent: the reference loop's compress calls re-run from its recorded K rows
    (eval_loop_rows.npz, no model forward) with the oracle keep, at every one of the 699 steps,
    the positions the reference kept."""
    from test_ppl_parity import oracle_compress as oracle_method
    got, want = _replay_case(name, oracle_method(name))
    assert got == want, [i for i, (a, b) in enumerate(zip(got, want)) if a != b][:5]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["snapkv_lite", "l2_compress"])
def test_engine_replays_reference_loop_selections(name):
    """The same replay with every compress call on the HIP engine: the engine keeps the
    reference's positions at all 699 steps of the loop whose perplexity differs on the GPU box's
    CPU (its forward rounds the first token's keys differently:
    test_engine_loop_selections_match_reference_steps reports step 0 as the first divergence)."""
    from kvcompress import _engine
    got, want = _replay_case(name, _engine_bridge(name))
    assert got == want, [i for i, (a, b) in enumerate(zip(got, want)) if a != b][:5]
    assert _engine.device_status(0) == 0
