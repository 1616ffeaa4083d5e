#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, rocprofv3 kernel stats.  Each step has its own
# time limit; the first failing step ends the script.
# Usage (on the box): bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
tag=${1:-chk}; kexpr=${2:-}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
kargs=(); [ -n "$kexpr" ] && kargs=(-k "$kexpr")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${kargs[@]}" > $out/pytest.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -40 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
  || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err \
  || { echo "bench failed rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
cd /tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -- python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $out/prof_bench.json 2> $out/prof.err \
  || { echo "rocprof failed rc=$?"; tail -20 $out/prof.err; exit 1; }
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \;
head -12 $out/kernel_stats.csv | cut -c1-200
