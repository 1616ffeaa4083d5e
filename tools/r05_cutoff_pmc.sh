#!/bin/bash
# Round 5: the cutoff tests, then PMC passes of the config-2 bench with its cutoff line (the
# dense observation kernel and k_obs_cutoff in the same run), summarised per kernel.
# Usage (on the box): bash tools/r05_cutoff_pmc.sh <tag> <commit>
set -o pipefail
tag=${1:-r05_cpmc}; commit=${2:-unknown}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_obs_cutoff.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
BENCH_ARGS="--spread-steps 0 --replay-steps 0 --no-nodedup --cutoff-steps 2" bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit 1
python tools/pmc_summary.py $out/pmc --commit "$commit" \
  --command "bench.py --steps 2 --warmup 1 --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup --cutoff-steps 2" \
  --out $out/pmc_summary.json > $out/pmc_summary.txt 2>&1 || { echo "pmc summary failed"; exit 1; }
echo done
