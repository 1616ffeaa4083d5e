#!/bin/bash
# Small-filter fusion check: bitwise test against the multi-kernel path, notebook latency
# (config 1) fused and unfused, and the kernel-trace summary of the fused run.
set -o pipefail
out=gpurun_out/r03_small
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python bench.py --config 1 > $out/c1_fused.json 2> $out/c1_fused.err || { echo "bench fused failed"; tail -20 $out/c1_fused.err; exit 1; }
GPMDM_NO_SMALL_PATH=1 GPMDM_OBS_SMALL_TILES=0 timeout -k 10 300 python bench.py --config 1 > $out/c1_multi.json 2> $out/c1_multi.err || { echo "bench multi failed"; tail -20 $out/c1_multi.err; exit 1; }
python -c "
import json
for t in ('fused','multi'):
    j=json.loads(open('$out/c1_'+t+'.json').read().splitlines()[-1]); print(t, j['ms_per_step'], j['value'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c1 -- python bench.py --config 1 > $out/c1_prof.log 2>&1 || { echo "rocprof failed"; tail -20 $out/c1_prof.log; exit 1; }
find $out/prof -name '*kernel_stats.csv'
echo done
