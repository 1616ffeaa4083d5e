#!/bin/bash
# Round 5: the observation-GP cutoff line (bench.py "cutoff") at configs 2, 3 and 5 on one GPU.
set -o pipefail
out=gpurun_out/${1:-r05_cb}; mkdir -p $out
timeout -k 10 400 python -u bench.py --steps 100 --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup \
  > $out/c2.json 2> $out/c2.err || { echo "config 2 failed"; tail -5 $out/c2.err; exit 1; }
python -c "import json;d=json.load(open('$out/c2.json'));print('c2', round(d['ms_per_step'],3), json.dumps(d.get('cutoff')))"
timeout -k 10 600 python -u bench.py --config 3 --steps 10 --no-cpu-baseline --no-nodedup --cutoff-steps 10 \
  > $out/c3.json 2> $out/c3.err || { echo "config 3 failed"; tail -5 $out/c3.err; exit 1; }
python -c "import json;d=json.load(open('$out/c3.json'));print('c3', round(d['ms_per_step'],3), json.dumps(d.get('cutoff')))"
timeout -k 10 900 python -u bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --no-nodedup --cutoff-steps 5 \
  > $out/c5.json 2> $out/c5.err || { echo "config 5 failed"; tail -5 $out/c5.err; exit 1; }
python -c "import json;d=json.load(open('$out/c5.json'));print('c5', round(d['ms_per_step'],3), json.dumps(d.get('cutoff')))"
