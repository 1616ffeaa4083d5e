#!/bin/bash
# Round 5: the cutoff line on the spread cloud (config 2's model with exp(y_log_lambdas) =
# 0.05 and the observation stream drawn from the filter's own predictive distribution: ESS
# ~8-15%), beside the same stream's dense step.
set -o pipefail
out=gpurun_out/${1:-r05_cs}; mkdir -p $out
timeout -k 10 600 python -u bench.py --stream predictive --y-lambda 0.05 --steps 30 --cutoff-steps 20 --no-cpu-baseline \
  --no-nodedup --replay-steps 0 --spread-steps 0 > $out/c2_spread.json 2> $out/c2_spread.err \
  || { echo "spread cutoff failed rc=$?"; tail -5 $out/c2_spread.err; exit 1; }
python -c "import json;d=json.load(open('$out/c2_spread.json'));print('dense', round(d['ms_per_step'],3), 'ess', d.get('ess_last'), json.dumps(d.get('cutoff'))[:700])"
