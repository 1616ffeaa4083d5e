#!/bin/bash
# Round-4 GPU pass: selected GPU tests (pytest -k), then the default bench (optional).
# Usage (on the box): bash tools/r04_check.sh <tag> "<pytest files>" [bench-args | -]
set -o pipefail
tag=${1:-r04}; files=${2:-tests}; bargs=${3:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $files -m gpu -x -v -s --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; grep -E "PASSED|FAILED|Error|assert" $out/pytest.log | tail -30; tail -30 $out/pytest.log; exit 1; }
grep -E "passed|failed" $out/pytest.log | tail -2
if [ "$bargs" != "-" ]; then
  timeout -k 10 600 python -u bench.py $bargs > $out/bench.json 2> $out/bench.err \
    || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
  python - $out/bench.json <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
print({k: r.get(k) for k in ("value", "ms_per_step", "n_gpus")}, "frac", round(r["roofline"]["frac"], 4))
for k in ("replay", "spread", "nodedup", "library_exchange"):
    if r.get(k):
        print(k, {kk: r[k].get(kk) for kk in ("ms_per_step", "value", "vs_headline", "host_threads", "prefetch_hits", "prefetch_misses", "serial_draws_ms_per_frame", "bitwise_equal_to_process_group_filter") if kk in r[k]})
PY
fi
