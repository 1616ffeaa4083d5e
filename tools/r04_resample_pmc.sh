#!/bin/bash
# PMC counters of the replicated resample kernels at P_total = 800k (tools/scale_sim.py --ranks
# 4 8), one rocprofv3 pass per counter group.  Usage: bash tools/r04_resample_pmc.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_rpmc}
mkdir -p $out
export TMPDIR=/tmp
i=0
for counters in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_WAVES" \
                "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --kernel-include-regex "k_resample|k_rows_ll|k_ubucket|k_guide" \
    --output-format csv -d $out/pass$i -- python -u tools/scale_sim.py --ranks 4 8 > $out/pass$i.log 2>&1 \
    || { echo "pass $i failed"; tail -5 $out/pass$i.log; exit 1; }
  echo "pass $i ok: $counters"
done
python tools/pmc_summary.py $out > $out/summary.txt && cat $out/summary.txt
