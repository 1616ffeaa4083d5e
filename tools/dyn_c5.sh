#!/bin/bash
# Config 5 (N = 2e4, d = 16, C = 8, P = 125k per GPU): the de-duplicated dynamics pass on the
# narrow 16 x 256 image (AUTO), its 32 / 64-row family, and the wide (observation-shaped) image.
# Usage (on the box): bash tools/dyn_c5.sh <tag> [variants] [steps]
set -o pipefail
out=gpurun_out/${1:-dync5}; vs=${2:-"auto wide mt2 mt4"}; steps=${3:-20}
mkdir -p $out
export TMPDIR=/tmp
for v in $vs; do
  case $v in
    auto) envs=""; extra="";;
    wide) envs=""; extra="--dyn-tiles wide";;
    *) envs="GPMDM_DYN_MT=${v#mt}"; extra="--dyn-tiles narrow";;
  esac
  env $envs timeout -k 10 500 python -u bench.py --config 5 --steps $steps --warmup 5 --no-cpu-baseline --replay-steps 0 \
    --spread-steps 0 --no-nodedup $extra > $out/c5_$v.json 2> $out/c5_$v.err || { echo "bench c5 $v failed rc=$?"; tail -5 $out/c5_$v.err; exit 1; }
  python - $out/c5_$v.json $v <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
st = r["stages_ms_per_step"]; dr = r.get("dyn_rows_last") or {}
print(f"cfg 5 {sys.argv[2]:5s} step {r['ms_per_step']:.2f} dyn {st['dyn_gemm']:.3f} ms rows {dr.get('breakdown_mean', 0):.0f} "
      f"({dr.get('dyn_gemm_tflops', 0):.1f} TF/s) obs frac {r['roofline']['frac']:.3f} ess {r.get('ess_frac_last'):.3g}", flush=True)
PY
done
