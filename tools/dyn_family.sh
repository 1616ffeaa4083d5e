#!/bin/bash
# Dynamics-tile shapes of one column blocking (256 columns: 16x256, 32x256, 64x256 -- bitwise
# the same results) against the default pair (narrow 16x256 + wide observation-shaped image),
# config 2 (headline + spread + nodedup lines) and config 5.  Usage: bash tools/dyn_family.sh <tag>
set -o pipefail
out=gpurun_out/${1:-dynfam}
mkdir -p $out
export TMPDIR=/tmp
for cfg in 2 5; do
  steps=100; [ $cfg = 5 ] && steps=5
  for geo in default 4,1,4 4,2,4 4,4,4; do
    if [ $geo = default ]; then envs=""; else envs="GPMDM_DYN_GEO=$geo GPMDM_DYNW_GEO=$geo"; fi
    env $envs timeout -k 10 400 python -u bench.py --config $cfg --steps $steps --no-cpu-baseline --replay-steps 0 \
      > $out/c${cfg}_${geo//,/x}.json 2> $out/c${cfg}_${geo//,/x}.err || { echo "bench c$cfg $geo failed rc=$?"; tail -5 $out/c${cfg}_${geo//,/x}.err; exit 1; }
    python - $out/c${cfg}_${geo//,/x}.json $cfg $geo <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
st = r["stages_ms_per_step"]; nd = r.get("nodedup") or {}; sp = r.get("spread") or {}
print(f"cfg {sys.argv[2]} geo {sys.argv[3]:8s} step {r['ms_per_step']:.3f} dyn {st['dyn_gemm']:.4f} rows {r['dyn_rows_last']['breakdown_mean']:.0f} "
      f"({r['dyn_rows_last']['dyn_gemm_tflops']:.1f} TF/s) | nodedup dyn {nd.get('stages_ms_per_step', {}).get('dyn_gemm', 0):.4f} "
      f"({nd.get('dyn_gemm_tflops', 0):.1f} TF/s) | spread dyn {sp.get('stages_ms_per_step', {}).get('dyn_gemm', 0):.4f} "
      f"rows {sp.get('dyn_rows_mean', 0):.0f} ({sp.get('dyn_gemm_tflops', 0):.1f} TF/s)")
PY
  done
done
