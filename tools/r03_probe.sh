#!/bin/bash
# Round-3 first GPU pass: GPU tests, the notebook-mode bench (config 1) with its kernel
# trace, and a short sweep of the predictive observation stream (config 2) for the ESS.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
out=gpurun_out/r03_probe
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u bench.py --config 1 > $out/c1.json 2> $out/c1.err \
  || { echo "bench c1 failed rc=$?"; tail -20 $out/c1.err; exit 1; }
cat $out/c1.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c1prof -- python -u bench.py --config 1 --steps 50 --warmup 5 --no-cpu-baseline --bank 0 --no-nodedup > $out/c1prof.json 2> $out/c1prof.err \
  || { echo "rocprof c1 failed rc=$?"; tail -20 $out/c1prof.err; exit 1; }
for lam in 1.0 0.3 0.1; do
  timeout -k 10 300 python -u bench.py --stream predictive --y-lambda $lam --steps 30 --warmup 5 --no-cpu-baseline --no-nodedup > $out/pred_$lam.json 2> $out/pred_$lam.err \
    || { echo "bench predictive $lam failed rc=$?"; tail -20 $out/pred_$lam.err; exit 1; }
  python -c "import json;d=json.load(open('$out/pred_$lam.json'));print('lambda $lam', round(d['ms_per_step'],3), 'ms', 'ess_frac', d['ess_frac_last'], 'rows', d['dyn_rows_last'], d['stream_check'], d['stages_ms_per_step'])"
done
timeout -k 10 120 tools/microbench/store_hazard > $out/store_hazard.txt 2>&1 \
  || { echo "store_hazard failed rc=$?"; cat $out/store_hazard.txt; exit 1; }
cat $out/store_hazard.txt
for g in 0 1; do
  if [ $g = 1 ]; then export GPMDM_DYN_EXACT_GRID=1; fi
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-nodedup > $out/grid_$g.json 2> $out/grid_$g.err \
    || { echo "bench grid $g failed rc=$?"; tail -20 $out/grid_$g.err; exit 1; }
  python -c "import json;d=json.load(open('$out/grid_$g.json'));print('exact_grid $g', round(d['ms_per_step'],3), d['stages_ms_per_step'], d['dyn_rows_last'])"
done
unset GPMDM_DYN_EXACT_GRID
echo done
