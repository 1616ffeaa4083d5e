#!/bin/bash
# PMC passes for the hot kernels (one counter group per rocprofv3 run, kernel trace only).
# Usage (on the GPU box): bash tools/pmc_passes.sh <outdir> "<pass1 counters>" "<pass2 counters>" ...
# (BENCH_ARGS="--config 3" profiles another configuration)
set -o pipefail
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for counters in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d $out/pass$i -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $out/pass$i.log 2>&1 || { echo "pass $i ($counters) failed rc=$?"; exit 1; }
  echo "pass $i ok: $counters"
done
