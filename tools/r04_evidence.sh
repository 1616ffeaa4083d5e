#!/bin/bash
# Round-4 evidence pass: PMC counters of the headline bench command (one rocprofv3 run per
# counter group) and the spread (non-collapsing) lines of configs 3 and 4.
# Usage (on the box): bash tools/r04_evidence.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_ev}
mkdir -p $out
export TMPDIR=/tmp
BENCH_ARGS="--spread-steps 0 --replay-steps 0" bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" || exit 1
for cfg in 3 4; do
  timeout -k 10 600 python -u bench.py --config $cfg --steps 10 --warmup 3 --spread-steps 10 --no-cpu-baseline \
    --replay-steps 0 --no-nodedup > $out/config${cfg}_spread.json 2> $out/config${cfg}_spread.err \
    || { echo "config $cfg failed rc=$?"; tail -20 $out/config${cfg}_spread.err; exit 1; }
  python - $out/config${cfg}_spread.json $cfg <<'PY'
import json, sys
r = json.load(open(sys.argv[1])); sp = r.get("spread") or {}
print(f"config {sys.argv[2]}: headline {r['value']:.4g} ({r['ms_per_step']:.2f} ms, ess {r.get('ess_frac_last'):.3g}, obs frac {r['roofline']['frac']:.3f}) "
      f"| spread {sp.get('value', 0):.4g} ({sp.get('ms_per_step', 0):.2f} ms, ess {sp.get('ess_frac_last', 0):.3g}, rows {sp.get('dyn_rows_mean', 0):.0f}, "
      f"dyn {sp.get('dyn_gemm_tflops', 0):.1f} TF/s)", flush=True)
PY
done
