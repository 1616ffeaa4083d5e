#!/bin/bash
# Round 5: SQ_INSTS_MFMA (executed MFMA instructions) of the cutoff kernel at configs 3 and 5,
# beside the dense observation kernel, from one rocprofv3 --pmc pass of each bench line.
# Usage (on the box): bash tools/r05_cutoff_mfma.sh <tag>
set -o pipefail
tag=${1:-r05_cm}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for c in 3 5; do
  timeout -k 10 900 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $out/c$c -- \
    python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-nodedup --cutoff-steps 3 > $out/c$c.log 2>&1 \
    || { echo "config $c pass failed rc=$?"; tail -5 $out/c$c.log; exit 1; }
  echo "config $c ok"
done
