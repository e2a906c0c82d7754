"""scripts/benchmark.py (the reference CLI surface over this package): method configurations
match the reference's build_methods_config for the same command lines (golden, generated from
the unmodified reference by tests/golden/gen_cli_configs.py), and the CLI runs end to end on a
random-weight model (offline)."""
import importlib.util
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd", "scripts", "benchmark.py")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "cli_configs.json")))


def _cli():
    spec = importlib.util.spec_from_file_location("kvc_cli", CLI)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("case", GOLD, ids=[" ".join(c["argv"]) for c in GOLD])
def test_methods_config_matches_reference(case):
    mod = _cli()
    args = mod.build_parser().parse_args(case["argv"])
    got = [{"name": m["name"],
            "fn": None if m["compress_fn"] is None else m["compress_fn"].__name__,
            "kwargs": m["kwargs"]} for m in mod.build_methods_config(args)]
    assert got == case["methods"]


def test_requires_a_method():
    mod = _cli()
    with pytest.raises(SystemExit):
        mod.main([])


def _small_run(mod, extra):
    return mod.main(["--random_model", "pythia-tiny", "--synthetic_text", "--num_samples", "1",
                     "--max_tokens", "80", "--max_new_tokens", "4", "--num_warmup", "1"] + extra)


def test_baseline_runs_offline_on_cpu(capsys):
    mod = _cli()
    res = _small_run(mod, ["--compare_new"])  # the reference's --compare_new adds only baseline
    assert [r["method"] for r in res] == ["baseline"]
    assert np.isfinite(res[0]["perplexity"]) and res[0]["final_cache_size"] == 79
    assert "Benchmark completed!" in capsys.readouterr().out


@pytest.mark.gpu
def test_cli_end_to_end_on_gpu(capsys):
    mod = _cli()
    res = _small_run(mod, ["--method", "fix_size_l2", "--fix_kv_sizes", "32",
                           "--keep_ratios", "0.5", "--skip_layers", "0"])
    names = [r["method"] for r in res]
    assert names == ["baseline", "recent_only_32", "fix32_keep_low_kr=0.5"]
    for r in res:
        assert np.isfinite(r["perplexity"])
    assert res[1]["final_cache_size"] == 32 and res[2]["final_cache_size"] == 32
    assert "Benchmark completed!" in capsys.readouterr().out


H2O_CLI = os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd", "scripts",
                       "test_h2o_attention.py")


def _h2o_cli():
    spec = importlib.util.spec_from_file_location("kvc_h2o_cli", H2O_CLI)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_h2o_cli_defaults_match_reference():
    """scripts/test_h2o_attention.py:95-107 of the reference: argument names and defaults."""
    a = _h2o_cli().build_parser().parse_args([])
    assert (a.model_id, a.max_tokens, a.heavy_hitter_sizes, a.compare, a.skip_layers) == \
        ("EleutherAI/pythia-2.8b", 1500, "32,64,128", False, "0,1")


@pytest.mark.gpu
def test_h2o_cli_compare_on_gpu(capsys):
    mod = _h2o_cli()
    mod.main(["--random_model", "pythia-tiny", "--synthetic_text", "--compare", "--max_tokens",
              "560", "--heavy_hitter_sizes", "32", "--skip_layers", "0"])
    out = capsys.readouterr().out
    assert "h2o_attention_hh32" in out and "H2O-Attention:" in out
    assert "Test completed!" in out


@pytest.mark.gpu
def test_cli_stable_tie_policy_on_gpu(capsys):
    """--tie_policy stable (extension): the run uses the stable selections and the previous
    policy is restored afterwards."""
    from kvcompress import _engine
    mod = _cli()
    res = _small_run(mod, ["--method", "fix_size_l2", "--fix_kv_sizes", "32", "--keep_ratios",
                           "0.0", "--skip_layers", "0", "--tie_policy", "stable", "--no_baseline",
                           "--no_recent_only"])
    assert res and all(r["final_cache_size"] == 32 for r in res)
    assert "Tie policy: stable" in capsys.readouterr().out
    assert _engine.tie_policy == "reference"
