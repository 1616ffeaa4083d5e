#!/bin/bash
# Round 5: the whole GPU suite, then the cutoff line at configs 2, 3 and 5 (tools/r05_cutoff_bench.sh).
# Usage (on the box): bash tools/r05_suite_cutoff.sh <tag>
set -o pipefail
tag=${1:-r05_sc}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash tools/r05_cutoff_bench.sh $tag/cb
