#!/bin/bash
# Per-kernel times of the multi-rank step's replicated work: tools/scale_sim.py --ranks at
# N = 1 and N = 8 (8 simulated ranks of 100k particles on one GPU), each under its own
# rocprofv3 kernel trace.  Usage (on the box): bash tools/r04_replicated.sh <tag> [steps] [Ns]
# (environment switches of the library pass through, e.g. GPMDM_NO_COOP_SEARCH=1 for an A/B)
set -o pipefail
out=gpurun_out/${1:-repl}; steps=${2:-10}; ns=${3:-"1 8"}
mkdir -p $out
export TMPDIR=/tmp
for n in $ns; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_n$n -- \
    python -u tools/scale_sim.py --ranks $steps $n > $out/sim_n$n.txt 2> $out/sim_n$n.err \
    || { echo "scale_sim N=$n failed rc=$?"; tail -20 $out/sim_n$n.err; exit 1; }
  find $out/prof_n$n -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats_n$n.csv \;
  grep "GPU ms per step" $out/sim_n$n.txt
  python - $out/kernel_stats_n$n.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"].split("(")[0][:60]
    if "gp_tile" in name:
        continue
    print(f"  {name:60s} calls {int(r['Calls']):6d} avg {float(r['AverageNs']) / 1e3:8.2f} us")
PY
done
