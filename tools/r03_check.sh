#!/bin/bash
# Round-3 evidence pass at the current build: smoke, the default bench line (as the driver
# runs it), the rocprofv3 kernel-trace stats of the bench, a 2-rank gloo rehearsal of the
# multi-rank bench path, and the PMC passes of the observation / dynamics tiles.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
tag=${1:-r03_check}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
  || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err \
  || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('bench', '%.4g' % d['value'], round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'launch_ms', round(d['roofline']['launch_ms'],4), 'cpu', d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('cores'), 'spread', d.get('spread',{}).get('ms_per_step'), d.get('spread',{}).get('ess_frac_last'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -- python -u bench.py --steps 100 --no-cpu-baseline --spread-steps 0 > $out/kt_bench.json 2> $out/kt.err \
  || { echo "kernel trace failed rc=$?"; tail -20 $out/kt.err; exit 1; }
find $out/kt -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
head -6 $out/kernel_stats.csv | cut -c1-160
bash tools/rehearse_ranks.sh 2 > $out/rehearsal2.txt 2>&1 || { echo "rehearsal failed"; cat $out/rehearsal2.txt | tail -20; exit 1; }
tail -3 $out/rehearsal2.txt | cut -c1-400
BENCH_ARGS="--spread-steps 0" bash tools/pmc_passes.sh $out/pmc "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" || exit 1
echo done
