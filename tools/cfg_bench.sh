#!/bin/bash
# bench.py on the other BASELINE configurations (per-GPU share of P for the 8-GPU ones),
# each with its cpu_baseline (a 1000-particle sample of the numpy oracle above N = 2000).
# Usage (on the box): bash tools/cfg_bench.sh <outdir> [configs...]
set -o pipefail
out=${1:-gpurun_out/cfgb}; shift
cfgs=${*:-3 4 5}
mkdir -p $out
for c in $cfgs; do
  timeout -k 10 600 python -u bench.py --config $c > $out/c$c.json 2> $out/c$c.err || { echo "config $c failed"; tail -5 $out/c$c.err; exit 1; }
  python -c "import json;d=json.load(open('$out/c$c.json'));cb=d.get('cpu_baseline') or {};print('config $c', round(d['ms_per_step'],2), 'ms/step', '%.4g' % d['value'], 'frac', round(d['roofline']['frac'],3), 'cpu', cb.get('value'), cb.get('cores'))"
done
