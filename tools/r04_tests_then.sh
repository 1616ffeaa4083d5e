#!/bin/bash
# Selected GPU tests, then (optionally) one more script.  Each step under its own time limit.
# Usage (on the box): bash tools/r04_tests_then.sh <tag> "<test files>" [script args...]
set -o pipefail
tag=$1; files=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|error" $out/pytest.log | head -20; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
if [ $# -gt 0 ]; then
  "$@" || { echo "step failed rc=$?"; exit 1; }
fi
