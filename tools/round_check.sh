#!/bin/bash
# GPU-box pass for a round's evidence: gpu tests, smoke, default bench, rocprofv3 kernel
# stats of the bench, PMC passes of the bench.  Each GPU step has its own time limit; the
# first failing step ends the script.
# Usage (on the box): bash tools/round_check.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r02}; skip=${2:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ -z "$skip" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/pytest.log 2>&1 \
    || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
  tail -2 $out/pytest.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
    || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
  tail -1 $out/smoke.log
fi
timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err \
  || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -- python bench.py --steps 100 --no-cpu-baseline > $out/kt.log 2>&1 \
  || { echo "kernel trace failed rc=$?"; tail -20 $out/kt.log; exit 1; }
bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" || exit 1
echo done
