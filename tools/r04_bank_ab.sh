#!/bin/bash
# Same-box A/B of the notebook-size lines (bench.py --config 1: single filter and the 39-filter
# bank) between the working tree and tools/ab_prev, after the GPU tests.
set -o pipefail
out=${OUT:-gpurun_out/r04_bank}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1; tail -2 $out/pytest.log
grep -q " passed" $out/pytest.log && ! grep -q "failed" $out/pytest.log || exit 1
for r in 1 2 3; do
  for v in new prev; do
    dir=.; [ $v = prev ] && dir=tools/ab_prev
    (cd $dir && timeout -k 10 300 python -u bench.py --config 1 --no-cpu-baseline) > $out/c1_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], 'single', round(r['ms_per_step'],4), 'bank', round((r.get('bank') or {}).get('ms_per_frame', 0),4))" $out/c1_${v}_$r.json $v
  done
done
