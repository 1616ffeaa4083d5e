#!/bin/bash
# GPU tests, then a same-box A/B of the replay line at P = 100k (bench.py --rng torch) and the
# notebook-size line between the working tree and tools/ab_prev.
set -o pipefail
out=${OUT:-gpurun_out/r04_rab}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1; tail -2 $out/pytest.log
grep -q " passed" $out/pytest.log && ! grep -q "failed" $out/pytest.log || exit 1
for r in 1 2 3; do
  for v in new prev; do
    dir=.; [ $v = prev ] && dir=tools/ab_prev
    (cd $dir && timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --rng torch --spread-steps 0 --replay-steps 0 --no-nodedup) > $out/rep_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print('replay100k', sys.argv[2], round(r['ms_per_step'],4), 'obs', round(r['roofline']['launch_ms'],4))" $out/rep_${v}_$r.json $v
  done
done
