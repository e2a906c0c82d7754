"""Golden method configurations of the reference CLI (build container only).

    cd /tmp && PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python /root/repo/tests/golden/gen_cli_configs.py

Imports the UNMODIFIED reference scripts/benchmark.py as a module (its import-time code only
defines functions) and records build_methods_config(args) for a set of command lines:
name, compress function name and kwargs of every entry -> tests/golden/cli_configs.json.
"""
import importlib.util
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/scripts/benchmark.py"
assert os.path.abspath(os.environ.get("PYTHONPATH", "").split(":")[0]) == "/root/reference"

ARGVS = [
    ["--method", "l2_compress"],
    ["--method", "l2_compress", "--keep_ratios", "1.0,0.5", "--prune_after", "50"],
    ["--method", "l2_compress", "--keep_ratios", "1.0,0.5", "--no_baseline"],
    ["--method", "fix_size_l2"],
    ["--method", "fix_size_l2", "--fix_kv_sizes", "128", "--strategies", "keep_low,keep_high,random",
     "--keep_ratios", "0.0,0.5", "--no_recent_only"],
    ["--method", "streaming_llm"],
    ["--method", "streaming_llm", "--start_size", "8", "--recent_sizes", "100"],
    ["--method", "h2o_l2"],
    ["--method", "h2o_l2", "--heavy_hitter_sizes", "16", "--h2o_recent_size", "100"],
    ["--method", "snapkv_lite"],
    ["--method", "snapkv_lite", "--snapkv_keep_sizes", "256,512", "--observation_windows", "8"],
    ["--method", "pyramid_kv"],
    ["--method", "pyramid_kv", "--base_sizes", "128", "--layer_decay", "0.8", "--min_size", "16",
     "--pyramid_profile", "linear"],
    ["--method", "adaptive_l2"],
    ["--method", "adaptive_l2", "--target_sizes", "128", "--soft_limit", "64", "--hard_limit", "256"],
    ["--compare_all"],
    ["--compare_all", "--no_baseline"],
    ["--compare_new"],
]


def main():
    spec = importlib.util.spec_from_file_location("ref_cli", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    import argparse

    # the reference builds its parser inside main(); re-create it by intercepting parse_args
    captured = {}

    class Stop(Exception):
        pass

    orig = argparse.ArgumentParser.parse_args

    def grab(self, args=None, namespace=None):
        captured["parser"] = self
        raise Stop()
    argparse.ArgumentParser.parse_args = grab
    try:
        mod.main()
    except Stop:
        pass
    finally:
        argparse.ArgumentParser.parse_args = orig
    parser = captured["parser"]
    out = []
    for argv in ARGVS:
        args = parser.parse_args(argv)
        cfg = mod.build_methods_config(args)
        out.append({"argv": argv, "methods": [
            {"name": m["name"],
             "fn": None if m["compress_fn"] is None else m["compress_fn"].__name__,
             "kwargs": m["kwargs"]} for m in cfg]})
    json.dump(out, open(os.path.join(HERE, "cli_configs.json"), "w"), indent=1)
    print(len(out), "command lines")


if __name__ == "__main__":
    main()
