#!/bin/bash
# One parameterised GPU-box pass (replaces the per-round tools/r0*_*.sh scripts of rounds 3-5).
# Each GPU step runs under its own time limit and the first failing step ends the script.
#
#   bash tools/gpu_pass.sh check  <tag> [tests|notests] [ab|noab] [pmc|nopmc]
#        -m gpu tests, smoke, the default bench, a headline-only kernel trace
#        (tools/headline_trace.py), optionally a same-box A/B against tools/ab_prev (headline and
#        the notebook-size frame; tools/ab_lib.sh prepare) and the headline PMC passes
#   bash tools/gpu_pass.sh cutoff <tag> [configs...]
#        the observation-GP cutoff line beside the dense step at configs 2 / 3 / 5 (default all)
#   bash tools/gpu_pass.sh spread <tag> [configs...]
#        the cutoff on spread clouds (bench.py --cutoff-spread): dense vs cutoff launches from
#        resynced >= 1000-ancestor clouds at three spreads (default configs 2 3 5)
#   bash tools/gpu_pass.sh cutoff-ab <tag> [configs...]
#        same-box A/B of the cutoff kernel: the working tree against tools/ab_prev (spread clouds
#        at each config, the config-2 cutoff line, and the bits of a 5-frame cutoff trajectory)
#   bash tools/gpu_pass.sh cutoff-pmc <tag>
#        PMC passes of the config-2 bench with its cutoff line (dense and cutoff kernels)
#   bash tools/gpu_pass.sh spread-split <tag> [spread] [policies...]
#        the cutoff on a spread cloud at configs 2 / 3 / 5 under each tile scheduling policy
#   bash tools/gpu_pass.sh spread-pmc <tag> [config] [spread]
#        PMC passes of one dense and one cutoff launch from a spread cloud (default config 5, 0.2 l)
#   bash tools/gpu_pass.sh configs <tag> [configs...]
#        bench.py on the other BASELINE configurations with their cpu_baseline (default 3 4 5)
# Output under gpurun_out/<tag>/; COMMIT (the evidence commit) stamps the summaries.
set -o pipefail
mode=${1:?mode}; tag=${2:?tag}; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
commit=$(cat COMMIT 2>/dev/null || echo unknown)
HEAD_ARGS="--no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup"
COUNTERS_A="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
COUNTERS_B="TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"

show() {  # one summary line of a bench JSON
  python -c "import json,sys;d=json.load(open(sys.argv[1]));st=d.get('stages_ms_per_step',{});print(sys.argv[2], '%.4g'%d['value'], round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), {k: round(v,4) for k,v in st.items()}, json.dumps(d.get('cutoff'))[:600] if d.get('cutoff') else '')" "$1" "$2"
}

case $mode in
check)
  tests=${1:-tests}; ab=${2:-noab}; pmc=${3:-nopmc}
  if [ "$tests" = tests ]; then
    timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 1200 --timeout-method thread > $out/pytest.log 2>&1 \
      || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
    tail -2 $out/pytest.log
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
      || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
    tail -1 $out/smoke.log
  fi
  timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err \
    || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
  show $out/bench.json bench
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -- python bench.py --steps 100 --warmup 5 $HEAD_ARGS > $out/kt.log 2>&1 \
    || { echo "kernel trace failed rc=$?"; tail -20 $out/kt.log; exit 1; }
  python tools/headline_trace.py $out/kt --steps 100 --warmup 5 --commit "$commit" \
    --command "rocprofv3 --kernel-trace --stats -- python bench.py --steps 100 --warmup 5 $HEAD_ARGS" --out $out/headline_obs.json
  if [ "$ab" = ab ]; then
    for r in 1 2 3; do
      for v in new prev; do
        dir=.; [ $v = prev ] && dir=tools/ab_prev
        (cd $dir && timeout -k 10 240 python -u bench.py --steps 300 $HEAD_ARGS) > $out/ab_${v}_$r.json 2> $out/ab_${v}_$r.err \
          || { echo "ab $v failed"; tail -5 $out/ab_${v}_$r.err; exit 1; }
        show $out/ab_${v}_$r.json "headline $v"
        (cd $dir && timeout -k 10 240 python -u bench.py --config 1 --no-cpu-baseline --bank 0) > $out/c1_${v}_$r.json 2> $out/c1_${v}_$r.err \
          || { echo "c1 $v failed"; tail -5 $out/c1_${v}_$r.err; exit 1; }
        show $out/c1_${v}_$r.json "notebook $v"
      done
    done
  fi
  if [ "$pmc" = pmc ]; then
    BENCH_ARGS="--spread-steps 0 --replay-steps 0 --no-nodedup" bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
      "$COUNTERS_A" "$COUNTERS_B" || exit 1
    python tools/pmc_summary.py $out/pmc --commit "$commit" \
      --command "bench.py --steps 2 --warmup 1 --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup" \
      --out $out/pmc_summary.json > $out/pmc_summary.txt 2>&1 || { echo "pmc summary failed"; exit 1; }
  fi
  ;;
cutoff)
  for c in ${*:-2 3 5}; do
    case $c in
      2) args="--steps 100 $HEAD_ARGS"; lim=400 ;;
      3) args="--config 3 --steps 10 --no-cpu-baseline --no-nodedup --cutoff-steps 10"; lim=600 ;;
      5) args="--config 5 --steps 5 --warmup 2 --no-cpu-baseline --no-nodedup --cutoff-steps 5"; lim=900 ;;
    esac
    timeout -k 10 $lim python -u bench.py $args > $out/c$c.json 2> $out/c$c.err \
      || { echo "config $c failed rc=$?"; tail -5 $out/c$c.err; exit 1; }
    show $out/c$c.json "config $c"
  done
  ;;
spread)
  for c in ${*:-2 3 5}; do
    lim=600; [ "$c" = 5 ] && lim=1000
    timeout -k 10 $lim python -u bench.py --config $c --cutoff-spread --no-cpu-baseline > $out/spread_c$c.json 2> $out/spread_c$c.err \
      || { echo "spread config $c failed rc=$?"; tail -8 $out/spread_c$c.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));[print('config', sys.argv[2], json.dumps(r)) for r in d['cutoff_spread']['rows']]" $out/spread_c$c.json $c
  done
  ;;
cutoff-ab)
  mkdir -p tools/ab_prev/tools && cp tools/cutoff_hash.py tools/ab_prev/tools/
  for c in ${*:-2 3 5}; do
    for v in new prev; do
      dir=.; [ $v = prev ] && dir=tools/ab_prev
      (cd $dir && timeout -k 10 300 python -u tools/cutoff_hash.py --config $c --frames 4) > $out/hash_${v}_c$c.txt 2>&1 \
        || { echo "hash $v c$c failed"; tail -5 $out/hash_${v}_c$c.txt; exit 1; }
      echo "hash $v c$c $(tail -1 $out/hash_${v}_c$c.txt)"
    done
  done
  for r in 1 2; do
    for c in ${*:-2 3 5}; do
      for v in new prev; do
        dir=.; [ $v = prev ] && dir=tools/ab_prev
        lim=600; [ "$c" = 5 ] && lim=1000
        (cd $dir && timeout -k 10 $lim python -u bench.py --config $c --cutoff-spread --no-cpu-baseline) > $out/spread_${v}_c${c}_$r.json 2> $out/spread_${v}_c${c}_$r.err \
          || { echo "spread $v c$c failed"; tail -8 $out/spread_${v}_c${c}_$r.err; exit 1; }
        python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], [(r['spread_ell'], round(r['cutoff_obs_launch_ms'],3), round(r['dense_obs_launch_ms'],3), round(r['executed_frac_of_peak'],3)) for r in d['cutoff_spread']['rows']])" $out/spread_${v}_c${c}_$r.json "spread $v c$c r$r"
      done
    done
    for v in new prev; do
      dir=.; [ $v = prev ] && dir=tools/ab_prev
      (cd $dir && timeout -k 10 300 python -u bench.py --steps 40 --cutoff-steps 20 $HEAD_ARGS) > $out/c2_${v}_$r.json 2> $out/c2_${v}_$r.err \
        || { echo "c2 $v failed"; tail -5 $out/c2_${v}_$r.err; exit 1; }
      show $out/c2_${v}_$r.json "c2 $v r$r"
    done
  done
  ;;
cutoff-pmc)
  BENCH_ARGS="--spread-steps 0 --replay-steps 0 --no-nodedup --cutoff-steps 2" bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
    "$COUNTERS_A" "$COUNTERS_B" || exit 1
  python tools/pmc_summary.py $out/pmc --commit "$commit" \
    --command "bench.py --steps 2 --warmup 1 --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup --cutoff-steps 2" \
    --out $out/pmc_summary.json > $out/pmc_summary.txt 2>&1 || { echo "pmc summary failed"; exit 1; }
  ;;
spread-split)
  # the cutoff's tile scheduling policies on spread clouds: spread-split <tag> <spread> <policies...>
  sp=${1:-0.2}; shift
  for c in 2 3 5; do
    for pol in ${*:-auto chunks}; do
      lim=300; [ "$c" = 5 ] && lim=600
      timeout -k 10 $lim python -u bench.py --config $c --cutoff-spread --no-cpu-baseline --cutoff-spread-at $sp \
          --cutoff-spread-reps 2 --cutoff-split $pol > $out/spread_c${c}_$pol.json 2> $out/spread_c${c}_$pol.err \
        || { echo "spread c$c $pol failed"; tail -8 $out/spread_c${c}_$pol.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], [(r['spread_ell'], round(r['cutoff_obs_launch_ms'],3), round(r['dense_obs_launch_ms'],3), round(r['mfma_groups_run_fraction'],3), round(r['executed_frac_of_peak'],3)) for r in d['cutoff_spread']['rows']])" $out/spread_c${c}_$pol.json "c$c $pol"
    done
  done
  ;;
spread-pmc)
  # PMC passes of one spread-cloud dense + cutoff launch pair: spread-pmc <tag> <config> [spread]
  c=${1:-5}; sp=${2:-0.2}
  args="--config $c --cutoff-spread --cutoff-spread-at $sp --cutoff-spread-reps 1"
  BENCH_ARGS="$args" bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
    "$COUNTERS_A" "$COUNTERS_B" || exit 1
  python tools/pmc_summary.py $out/pmc --commit "$commit" \
    --command "bench.py --steps 2 --warmup 1 --no-cpu-baseline $args" \
    --out $out/pmc_summary.json > $out/pmc_summary.txt 2>&1 || { echo "pmc summary failed"; exit 1; }
  ;;
configs)
  for c in ${*:-3 4 5}; do
    timeout -k 10 600 python -u bench.py --config $c > $out/c$c.json 2> $out/c$c.err || { echo "config $c failed"; tail -5 $out/c$c.err; exit 1; }
    python -c "import json;d=json.load(open('$out/c$c.json'));cb=d.get('cpu_baseline') or {};print('config $c', round(d['ms_per_step'],2), 'ms/step', '%.4g' % d['value'], 'frac', round(d['roofline']['frac'],3), 'cpu', cb.get('value'), cb.get('cores'))"
  done
  ;;
*) echo "unknown mode $mode"; exit 2 ;;
esac
echo done
