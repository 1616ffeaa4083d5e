#!/bin/bash
# Round-5 GPU-box pass: gpu tests, smoke, the default bench, a headline-only kernel trace
# (tools/headline_trace.py), optionally a same-box A/B against tools/ab_prev (headline and the
# notebook-size frame) and the headline-only PMC passes.  Each GPU step has its own time limit;
# the first failing step ends the script.
# Usage (on the box): bash tools/r05_check.sh <tag> [tests|notests] [ab|noab] [pmc|nopmc]
set -o pipefail
tag=${1:-r05}; tests=${2:-tests}; ab=${3:-noab}; pmc=${4:-nopmc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
commit=$(cat COMMIT 2>/dev/null || echo unknown)
HEAD_ARGS="--no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup"
if [ "$tests" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
    || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
  tail -1 $out/smoke.log
fi
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err \
  || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('bench', '%.4g'%d['value'], round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), {k: round(v,4) for k,v in d['stages_ms_per_step'].items()})"
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
      python -c "import json,sys;d=json.load(open(sys.argv[1]));st=d['stages_ms_per_step'];print('headline', sys.argv[2], round(d['ms_per_step'],4), 'obs', round(d['roofline']['launch_ms'],4), 'switch', round(st['switch'],4), 'resample', round(st['resample'],4))" $out/ab_${v}_$r.json $v
      (cd $dir && timeout -k 10 240 python -u bench.py --config 1 --no-cpu-baseline --bank 0) > $out/c1_${v}_$r.json 2> $out/c1_${v}_$r.err \
        || { echo "c1 $v failed"; tail -5 $out/c1_${v}_$r.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));print('notebook', sys.argv[2], round(d['ms_per_step'],4), 'untimed', d['ms_per_frame_without_timing_events']['value'])" $out/c1_${v}_$r.json $v
    done
  done
fi
if [ "$pmc" = pmc ]; then
  BENCH_ARGS="--spread-steps 0 --replay-steps 0 --no-nodedup" bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
    "TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" || exit 1
  python tools/pmc_summary.py $out/pmc --commit "$commit" \
    --command "bench.py --steps 2 --warmup 1 --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup" \
    --out $out/pmc_summary.json > $out/pmc_summary.txt 2>&1 || { echo "pmc summary failed"; exit 1; }
fi
echo done
