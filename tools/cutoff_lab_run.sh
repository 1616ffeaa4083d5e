#!/bin/bash
set -o pipefail
out=gpurun_out/${LAB:-lab1}; mkdir -p $out
for c in ${CFGS:-2 5}; do
  for v in ${VARS:-cur v1 v2 v3 v4}; do
    dir=.; [ $v != cur ] && dir=tools/ab_$v
    lim=400; [ $c = 5 ] && lim=600
    (cd $dir && timeout -k 10 $lim python -u bench.py --config $c --cutoff-spread --no-cpu-baseline) > $out/${v}_c$c.json 2> $out/${v}_c$c.err || { echo "$v c$c failed"; tail -5 $out/${v}_c$c.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], [(r['spread_ell'], round(r['cutoff_obs_launch_ms'],3), round(r['dense_obs_launch_ms'],3), round(r['mfma_groups_run_fraction'],3)) for r in d['cutoff_spread']['rows']])" $out/${v}_c$c.json "$v c$c"
  done
done
