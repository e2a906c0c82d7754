"""Golden fixture for the attention-score evaluation loop (build container only):

    cd /tmp && PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_eval_attention.py

Runs the UNMODIFIED reference's kvcompress/evaluate_attention.py loop -- per token a forward with
output_attentions=True, the manager's update, h2o_attention_compress past the budget (with its
second accumulation) and the manager reset (:128-195) -- plus compare_h2o_methods' two other runs
(baseline and h2o_l2 through the reference evaluate_with_compression), on CPU with a seeded
random-weight GPT-NeoX (tests/test_ppl_parity.py's toy_model, fp32) and its toy tokenizer, at
torch.set_num_threads(THREADS).  Two compatibility shims, neither touching the algorithm: the
reference's normalize_kv_cache cannot unpack transformers-5 caches, so its modules
get a version that reads cache.layers[i].keys / .values; and transformers 5 returns attention
weights only from eager attention, whose mask it no longer cuts to each layer's key length (the
4.x eager kernels did), so the attention run uses the package's kvc_eager
(kvcompress/utils.py key_length_attention, loaded by file path).  Writes data only
(eval_attention.json): each run's perplexity, accuracy, token count and final cache size, and
the same for every method configuration of tests/test_ppl_parity.py (CASES) through the
reference's evaluate_with_compression, with the generating host's CPU model (the CPU forward's
rounding is host-dependent: the tests that replay these runs skip on another CPU).  Since round
6 every compress call of the h2o_l2 run and of the method runs is also recorded step by step
(tests/golden/step_digest.py: a digest of the call's input keys and of the positions it kept,
recovered from position-encoding values), so that another host can check the engine's
selections against the reference's at every step where its forward reproduces the keys, and
name the first step where it does not; and for the snapkv_lite and l2_compress runs every K
row the model appended is kept (eval_loop_rows.npz), which replays their compress calls on the
reference's exact inputs on any host (step_digest.replay).
"""
import importlib.util
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

THREADS = 8
MAX_TOKENS = 700
KW = dict(start_size=4, heavy_hitter_size=16, recent_size=40)
FIELDS = ("perplexity", "accuracy", "num_tokens", "final_cache_size")
# the method runs whose every appended K row is kept (eval_loop_rows.npz), so that another host
# can replay their compress calls on the reference's exact keys (step_digest.replay): layers 1-2
# (layer 0 is skipped by every run, and passed through untouched)
ROW_METHODS = ("snapkv_lite", "l2_compress")
ROW_LAYERS = (1, 2)


def cpu_model():
    """The host CPU's model name: the CPU model forward's rounding depends on the BLAS / oneDNN
    kernels torch dispatches for it, so the runs are pinned to the host that made them."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _v5_normalize(past_key_values):
    layers = getattr(past_key_values, "layers", None)
    if layers is not None and all(hasattr(l, "keys") and hasattr(l, "values") for l in layers):
        return [(l.keys, l.values) for l in layers]
    return list(past_key_values)


def main():
    sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, HERE]
    from step_digest import Recorder
    torch.set_num_threads(THREADS)
    import kvcompress  # the reference (PYTHONPATH=/root/reference)
    assert os.path.realpath(kvcompress.__file__).startswith("/root/reference"), kvcompress.__file__
    import kvcompress.evaluate as R_eval
    import kvcompress.evaluate_attention as R_attn
    from kvcompress.methods import h2o_l2_compress
    from kvcompress.methods.h2o_attention import H2OAttentionManager
    for name, mod in list(sys.modules.items()):
        if name.startswith("kvcompress") and hasattr(mod, "normalize_kv_cache"):
            mod.normalize_kv_cache = _v5_normalize
    spec = importlib.util.spec_from_file_location(
        "kvc_utils_build", os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd",
                                        "kvcompress", "utils.py"))
    ours = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ours)
    from test_ppl_parity import TEXT, ToyTokenizer, toy_model

    model = toy_model(torch.float32, "cpu", layers=3)
    tok = ToyTokenizer(512)
    text = TEXT * 2
    runs = {}
    r = R_eval.evaluate_with_compression(model, tok, text, compress_fn=None,
                                         max_tokens=MAX_TOKENS, show_progress=False)
    runs["baseline"] = r
    rec = Recorder(h2o_l2_compress)
    r = R_eval.evaluate_with_compression(model, tok, text, compress_fn=rec,
                                         compress_kwargs=KW, max_tokens=MAX_TOKENS,
                                         skip_layers=[0], show_progress=False)
    runs["h2o_l2"] = r
    steps = {"h2o_l2": rec.packed()}
    mgr = H2OAttentionManager(num_layers=3, num_heads=4, **KW)
    with ours.key_length_attention(model, need_weights=True):
        r = R_attn.evaluate_with_attention_compression(model, tok, text, h2o_manager=mgr,
                                                       max_tokens=MAX_TOKENS, skip_layers=[0],
                                                       show_progress=False, **KW)
    runs["h2o_attention"] = r
    # every method of test_ppl_parity.CASES through the reference's own evaluate loop
    from kvcompress.methods import get_compress_fn
    from test_ppl_parity import CASES
    methods = []
    rows = {}
    for name, kw in CASES:
        rec = Recorder(get_compress_fn(name))
        if name in ROW_METHODS:
            rec.new_rows(ROW_LAYERS)
        r = R_eval.evaluate_with_compression(model, tok, text, compress_fn=rec,
                                             compress_kwargs=kw, max_tokens=MAX_TOKENS,
                                             skip_layers=[0], show_progress=False)
        methods.append({"name": name, "kwargs": kw, **{f: r[f] for f in FIELDS},
                        "steps": rec.packed()})
        if name in ROW_METHODS:
            rows[name] = np.stack(rec.rows)
    out = {"threads": THREADS, "max_tokens": MAX_TOKENS, "kw": KW, "layers": 3,
           "cpu_model": cpu_model(), "cpu_capability": torch.backends.cpu.get_cpu_capability(),
           "text": "TEXT * 2", "runs": {k: {f: v[f] for f in FIELDS} for k, v in runs.items()},
           "methods": methods, "steps": steps}
    json.dump(out, open(os.path.join(HERE, "eval_attention.json"), "w"), indent=1)
    np.savez_compressed(os.path.join(HERE, "eval_loop_rows.npz"),
                        **{f"{k}_rows": v for k, v in rows.items()})
    print(json.dumps(out["runs"]), json.dumps([{f: m[f] for f in FIELDS} for m in methods]))


if __name__ == "__main__":
    main()
