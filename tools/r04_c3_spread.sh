#!/bin/bash
# Config 3's spread line at smaller observation-GP output scales (its 128 observation
# dimensions make the likelihood sharper than config 2's).  Usage: bash tools/r04_c3_spread.sh <tag> "<lambdas>"
set -o pipefail
out=gpurun_out/${1:-r04_c3}; lams=${2:-"0.02 0.005"}
mkdir -p $out
for lam in $lams; do
  timeout -k 10 600 python -u bench.py --config 3 --steps 10 --warmup 3 --spread-steps 10 --spread-lambda $lam \
    --no-cpu-baseline --replay-steps 0 --no-nodedup > $out/config3_spread_$lam.json 2> $out/err_$lam.txt || exit 1
  python - $out/config3_spread_$lam.json $lam <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); sp = r["spread"]
print(sys.argv[2], f"{sp['ms_per_step']:.2f} ms ess {sp['ess_frac_last']:.3g} rows {sp['dyn_rows_mean']:.0f} "
      f"dyn {sp['dyn_gemm_tflops']:.1f} TF/s replay_matches {sp['replay_matches']}", flush=True)
PY
done
