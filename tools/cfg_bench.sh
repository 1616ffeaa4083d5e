#!/bin/bash
# bench.py on the other BASELINE configurations (per-GPU share of P), short runs.
set -o pipefail
mkdir -p gpurun_out/cfgb
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 4 --warmup 3 --no-cpu-baseline > gpurun_out/cfgb/c$c.json 2> gpurun_out/cfgb/c$c.err || { echo "config $c failed"; tail -5 gpurun_out/cfgb/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/cfgb/c$c.json'));print('config $c', round(d['ms_per_step'],2), 'ms/step', '%.4g' % d['value'], 'frac', round(d['roofline']['frac'],3))"
done
