#!/bin/bash
# Round-3 kernel A/B pass: the cleaned gp_tile.h against the pre-split source (tile_ab.sh,
# bitwise hashes + timings at d = 3 / 8 / 16) and the dynamics-tile shapes (dyn_ab.sh).
set -o pipefail
out=gpurun_out/r03_ab
mkdir -p $out
export TMPDIR=/tmp
if [ -n "${TILE_AB:-}" ]; then
  timeout -k 10 700 bash tools/microbench/tile_ab.sh run > $out/tile_ab.txt 2>&1 \
    || { echo "tile_ab failed rc=$?"; tail -20 $out/tile_ab.txt; exit 1; }
  cat $out/tile_ab.txt
fi
timeout -k 10 600 bash tools/dyn_ab.sh $out/dynab 2>&1 | tee $out/dyn_ab.txt
for lam in 0.05 0.03; do
  timeout -k 10 300 python -u bench.py --stream predictive --y-lambda $lam --steps 30 --warmup 5 --no-cpu-baseline > $out/pred_$lam.json 2> $out/pred_$lam.err \
    || { echo "bench predictive $lam failed rc=$?"; tail -20 $out/pred_$lam.err; exit 1; }
  python -c "import json;d=json.load(open('$out/pred_$lam.json'));print('lambda $lam', round(d['ms_per_step'],3), 'ms', 'ess_frac', d['ess_frac_last'], 'rows', d['dyn_rows_last']['breakdown_mean'], d['stages_ms_per_step'], 'nodedup', d['nodedup']['ms_per_step'], d['nodedup']['dyn_gemm_tflops'])"
done
echo done
