#!/bin/bash
# One GPU-box runner for every measurement this repo takes (replaces the round-1/2 one-off
# scripts).  Usage:  bash tools/gpu.sh STEP [STEP ...]   with STEP one of
#   test       pytest -m gpu (the driver's parity tier)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (headline, default K/W, CPU baseline + PPL leg)   -> bench.json
#   quick      python bench.py --steps 20 --warmup 5 --no-cpu-baseline          -> quick.json
#   trace      rocprofv3 --kernel-trace --stats of `bench.py --steps 20 --warmup 5`, plus the
#              idle time between engine kernels (tools/trace_gaps.py)           -> prof/, gaps.json
#   decode     per-token decode steps (tools/decode_bench.py)                   -> decode.json
#   workloads  every bench.py workload at N=1                                   -> workloads.jsonl
#   pmc        FETCH/WRITE traffic + SQ counters (tools/pmc_round.sh)
#   shard      per-rank cost of the N=8 strong split (cfg4 / cfg5 workloads, --as-shard R/8 for
#              the first and last rank) + a rocprofv3 trace of the last rank's cfg5 pyramid step
#                                                                               -> shard.jsonl, shardprof/
#   dtypes     the headline in fp32 and fp16 K/V                                -> dtypes.jsonl
#   ab:NAME    the A/B recipe NAME of tools/ab_recipes.txt: library variants (built beforehand by
#              tools/build_variant.sh from tools/ab_variants.txt) on bench.py workloads, each
#              line tagged with the recipe                                        -> ab.jsonl
#   h2olong    rocprofv3 kernel stats of the long h2o_attention call
#              (tools/h2o_long_profile.py)                                        -> h2oprof/
#   heap       tools/heap_probe (register heap select vs std::partial_sort)      -> heap_probe.jsonl
#   sq:LIB     SQ issue / wait counters of the headline SELECT_GATHER kernel with library LIB
#              (kvcompress/_lib/LIB.so; two rocprofv3 --pmc passes of 8 SQ counters) -> sq_LIB.json
#   tie        both tie policies (reference / stable, KVC_TIE_POLICY) on the bench workloads and
#              the 8-way split's last rank                                     -> tie_ab.jsonl
#   stamps:stable  s_memtime phases of the stable selection (diagnostic build
#              tools/build_stamps.sh first; SEL_ALGO=2)                         -> stable_stamps.jsonl
#   gatherprobe  tools/row_gather_probe (160-B row gathers, load shapes) timed, then FETCH_SIZE
#              and the TCC read-request counters per shape (one rocprofv3 pass each)
#                                                                                -> gprobe/
#   icache:LIB[:WORKLOAD]  SQC instruction-cache + issue counters of SELECT_GATHER with library LIB
#              on a bench.py workload (default the headline), one rocprofv3 --pmc pass -> ic_*.json
# Every GPU step runs under its own time limit and the first failure ends the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
O="$R/gpurun_out"
LIBDIR="$R/cs3602-llm-inference-acceleration_amd/kvcompress/_lib"
mkdir -p "$O"
cd "$R"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
          -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
      tail -2 "$O/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
          || { tail -20 "$O/smoke.log"; exit 1; }
      grep smoke "$O/smoke.log" ;;
    bench)
      timeout -k 10 500 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
      cat "$O/bench.json" ;;
    quick)
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/quick.json" \
          2> "$O/quick.err" || { tail "$O/quick.err"; exit 1; }
      cat "$O/quick.json" ;;
    trace)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
          --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 \
          --no-cpu-baseline > "$O/prof.log" 2>&1 ) || { tail "$O/prof.log"; exit 1; }
      python3 tools/trace_gaps.py "$(find "$O/prof" -name '*kernel_trace.csv' | head -1)" > "$O/gaps.json" \
          && cat "$O/gaps.json" ;;
    decode)
      timeout -k 10 300 python tools/decode_bench.py > "$O/decode.json" 2> "$O/decode.err" \
          || { tail "$O/decode.err"; exit 1; }
      cat "$O/decode.json" ;;
    workloads)
      : > "$O/workloads.jsonl"
      for w in ${WORKLOADS:-fix512-s16384 fix512-s4096 fix512-s4096-d80 streaming-s16384 h2o-s16384 snapkv-s16384 pyramid-s16384 l2-s16384 adaptive-s16384}; do
        timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline \
            >> "$O/workloads.jsonl" 2>> "$O/workloads.err" || { tail "$O/workloads.err"; exit 1; }
      done
      cat "$O/workloads.jsonl" ;;
    tie)
      : > "$O/tie_ab.jsonl"
      for w in fix512-s16384 fix512-s4096 fix512-s4096-d80 h2o-s16384 snapkv-s16384 pyramid-s16384 adaptive-s16384; do
        for pol in reference stable; do
          KVC_TIE_POLICY=$pol timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 \
              --no-cpu-baseline > "$O/tie_one.json" 2> "$O/tie_one.err" || { tail "$O/tie_one.err"; exit 1; }
          python3 -c "import json; d=json.load(open('$O/tie_one.json')); print(json.dumps({'workload': '$w', 'policy': '$pol', 'ms_per_step': d['ms_per_step'], 'kernel_ms_per_step': d['kernel_ms_per_step']}))" >> "$O/tie_ab.jsonl"
        done
      done
      for w in cfg4-h2o-l32 cfg5-snapkv-l32 cfg5-pyramid-l32; do
        for pol in reference stable; do
          KVC_TIE_POLICY=$pol timeout -k 10 200 python bench.py --workload $w --as-shard 7/8 --steps 50 \
              --warmup 5 --no-cpu-baseline > "$O/tie_one.json" 2> "$O/tie_one.err" || { tail "$O/tie_one.err"; exit 1; }
          python3 -c "import json; d=json.load(open('$O/tie_one.json')); print(json.dumps({'workload': '$w', 'shard': '7/8', 'policy': '$pol', 'ms_per_step': d['ms_per_step'], 'kernel_ms_per_step': d['kernel_ms_per_step']}))" >> "$O/tie_ab.jsonl"
        done
      done
      cat "$O/tie_ab.jsonl" ;;
    stamps:stable)
      : > "$O/stable_stamps.jsonl"
      for cfg in "" "SEL_L=4 SEL_S=15936 SEL_K=64" "SEL_S=4096"; do
        env SEL_ALGO=2 $cfg timeout -k 10 120 python tools/select_stamps.py >> "$O/stable_stamps.jsonl" \
            2> "$O/ss.err" || { tail "$O/ss.err"; exit 1; }
      done
      cat "$O/stable_stamps.jsonl" ;;
    shard)
      : > "$O/shard.jsonl"
      for w in cfg4-h2o-l32 cfg5-snapkv-l32 cfg5-pyramid-l32; do
        for r in 0 7; do
          timeout -k 10 200 python bench.py --workload $w --as-shard $r/8 --steps 50 --warmup 5 \
              --no-cpu-baseline >> "$O/shard.jsonl" 2>> "$O/shard.err" || { tail "$O/shard.err"; exit 1; }
        done
      done
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
          --output-format csv -d "$O/shardprof" -o run -- python3 "$R/bench.py" --workload cfg5-pyramid-l32 \
          --as-shard 7/8 --steps 50 --warmup 5 --no-cpu-baseline > "$O/shardprof.log" 2>&1 ) \
          || { tail "$O/shardprof.log"; exit 1; }
      python3 tools/trace_gaps.py "$(find "$O/shardprof" -name '*kernel_trace.csv' | head -1)" timed > "$O/shard_gaps.json" \
          && cat "$O/shard.jsonl" "$O/shard_gaps.json" ;;
    dtypes)
      : > "$O/dtypes.jsonl"
      for d in fp32 fp16; do
        timeout -k 10 200 python bench.py --dtype $d --steps 20 --warmup 5 --no-cpu-baseline \
            >> "$O/dtypes.jsonl" 2>> "$O/dtypes.err" || { tail "$O/dtypes.err"; exit 1; }
      done
      cat "$O/dtypes.jsonl" ;;
    pmc)
      bash tools/pmc_round.sh > "$O/pmc_round.out" 2>&1 || { tail -20 "$O/pmc_round.out"; exit 1; }
      tail -c 3000 "$O/pmc_round.out" ;;
    ab:*)
      name="${step#ab:}"
      line=$(grep -E "^$name[[:space:]]" tools/ab_recipes.txt) || { echo "recipe $name not in tools/ab_recipes.txt"; exit 2; }
      libs=""; wls="fix512-s16384"; reps="1 2"; args=""; test=""
      for f in $line; do
        case "$f" in
          libs=*) libs="${f#libs=}" ;;
          workloads=*) wls="${f#workloads=}" ;;
          reps=*) reps=$(seq 1 "${f#reps=}") ;;
          args=*) args="${f#args=}"; args="${args//+/ }" ;;
          test=*) test="${f#test=}" ;;
        esac
      done
      if [ -n "$test" ]; then
        last="${libs##*,}"
        KVC_LIB="$LIBDIR/$last.so" timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
            tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread \
            -p no:cacheprovider > "$O/ab_pytest.log" 2>&1 || { tail -30 "$O/ab_pytest.log"; exit 1; }
        tail -1 "$O/ab_pytest.log"
      fi
      for rep in $reps; do
        for lib in ${libs//,/ }; do
          for w in ${wls//,/ }; do
            KVC_LIB="$LIBDIR/$lib.so" timeout -k 10 200 python bench.py --workload $w --steps 20 \
                --warmup 5 --no-cpu-baseline $args > "$O/ab_one.json" 2> "$O/ab.err" || { tail "$O/ab.err"; exit 1; }
            echo "{\"recipe\": \"$name\", \"rep\": $rep, \"lib\": \"$lib\", \"workload\": \"$w\", \"args\": \"$args\", \"r\": $(cat "$O/ab_one.json")}" >> "$O/ab.jsonl"
          done
        done
      done
      python3 tools/ab_summary.py "$O/ab.jsonl" "$name" ;;
    h2olong)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
          --output-format csv -d "$O/h2oprof" -o run -- python3 "$R/tools/h2o_long_profile.py" \
          > "$O/h2oprof.log" 2>&1 ) || { tail "$O/h2oprof.log"; exit 1; }
      grep ms_per_call "$O/h2oprof.log"
      python3 tools/ab_summary.py --kernel-stats "$O/h2oprof/run_kernel_stats.csv" ;;
    heap)
      timeout -k 10 120 tools/heap_probe > "$O/heap_probe.jsonl" 2>&1 || { cat "$O/heap_probe.jsonl"; exit 1; }
      cat "$O/heap_probe.jsonl" ;;
    gatherprobe)
      G="$O/gprobe"; mkdir -p "$G"
      timeout -k 10 120 tools/row_gather_probe > "$G/times.json" 2> "$G/times.err" || { cat "$G/times.err"; exit 1; }
      cat "$G/times.json"
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 60 rocprofv3 -L > "$G/counters.txt" 2>&1 ) || true
      grep -o -E "TCC_EA0_RDREQ[A-Z0-9_]*|TCC_REQ|TCC_READ|TCC_MISS|TCC_HIT" "$G/counters.txt" | sort -u > "$G/tcc_names.txt" || true
      cat "$G/tcc_names.txt"
      passes="FETCH_SIZE"
      grep -qx TCC_EA0_RDREQ "$G/tcc_names.txt" && grep -qx TCC_EA0_RDREQ_32B "$G/tcc_names.txt" && passes="$passes TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_32B_sum"
      grep -qx TCC_MISS "$G/tcc_names.txt" && grep -qx TCC_HIT "$G/tcc_names.txt" && passes="$passes TCC_HIT_sum,TCC_MISS_sum"
      grep -qx TCC_EA0_RDREQ_64B "$G/tcc_names.txt" && grep -qx TCC_EA0_RDREQ_128B "$G/tcc_names.txt" && passes="$passes TCC_EA0_RDREQ_64B_sum,TCC_EA0_RDREQ_128B_sum"
      for ps in $passes; do
        ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc ${ps//,/ } --output-format csv \
            -d "$G/pmc_${ps%%,*}" -o run -- "$R/tools/row_gather_probe" 2 > "$G/pmc_${ps%%,*}.log" 2>&1 ) \
            || { tail "$G/pmc_${ps%%,*}.log"; exit 1; }
      done
      python3 tools/pmc_bykernel.py "$G" ;;
    sq:*)
      lib="${step#sq:}"
      for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"; do
        tag="sq_${lib}_${set%% *}"
        ( cd /tmp && export TMPDIR=/tmp && KVC_LIB="$LIBDIR/$lib.so" timeout -s KILL 120 rocprofv3 --pmc $set \
            --kernel-include-regex "select_gather" --output-format csv -d "$O/$tag" -o run \
            -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$O/$tag.log" 2>&1 ) \
            || { tail "$O/$tag.log"; exit 1; }
      done
      python3 tools/pmc_summary.py "$O/sq_${lib}_SQ_WAVE_CYCLES" "$O/sq_${lib}_SQ_LDS_BANK_CONFLICT" > "$O/sq_$lib.json" \
          && cat "$O/sq_$lib.json" ;;
    icache:*)
      # icache:LIB[:WORKLOAD] -- instruction-cache and issue counters of SELECT_GATHER (one pass)
      spec="${step#icache:}"; lib="${spec%%:*}"; wl="fix512-s16384"
      [ "$spec" != "$lib" ] && wl="${spec#*:}"
      tag="ic_${lib}_${wl}"
      ( cd /tmp && export TMPDIR=/tmp && KVC_LIB="$LIBDIR/$lib.so" timeout -s KILL 120 rocprofv3 --pmc \
          SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES \
          SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY \
          --kernel-include-regex "select_gather" --output-format csv -d "$O/$tag" -o run \
          -- python3 "$R/bench.py" --workload "$wl" --steps 2 --warmup 1 --no-cpu-baseline > "$O/$tag.log" 2>&1 ) \
          || { tail "$O/$tag.log"; exit 1; }
      python3 tools/pmc_summary.py "$O/$tag" > "$O/$tag.json" && cat "$O/$tag.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
