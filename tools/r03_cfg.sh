#!/bin/bash
# GPU tests at the current tree, then the other BASELINE configurations with their CPU baselines.
set -o pipefail
out=gpurun_out/r03_cfg
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash tools/cfg_bench.sh $out/cfgb 3 4 5
echo done
