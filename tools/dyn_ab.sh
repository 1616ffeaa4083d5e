#!/bin/bash
# Dynamics-GP tile A/B on the GPU box (config 2): the headline filter's de-duplicated
# dynamics stage and the nodedup (every particle) line under tile-shape overrides
# (GPMDM_DYN_GEO / GPMDM_DYNW_GEO "nw,mt,ntw", capi.hip) and the exact-grid diagnostic.
# Usage: bash tools/dyn_ab.sh <outdir> [extra bench args, e.g. --stream predictive --y-lambda 0.3]
set -o pipefail
out=${1:-gpurun_out/dynab}; shift
mkdir -p $out
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline $BARGS > $out/$name.json 2> $out/$name.err \
    || { echo "$name failed rc=$?"; tail -20 $out/$name.err; exit 1; }
  python - "$out/$name.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); st = d["stages_ms_per_step"]; nd = d.get("nodedup") or {}
print(f"{sys.argv[2]:>14}: {d['ms_per_step']:.3f} ms/step  dyn_gemm {st['dyn_gemm']:.4f} ms  rows {d['dyn_rows_last']['breakdown_mean']:.0f}"
      f"  {d['dyn_rows_last']['dyn_gemm_tflops']:.1f} TF/s  | nodedup {nd.get('ms_per_step', 0):.3f} ms  dyn_gemm "
      f"{nd.get('stages_ms_per_step', {}).get('dyn_gemm', 0):.4f} ms  {nd.get('dyn_gemm_tflops', 0):.1f} TF/s  ess {d['ess_frac_last']:.4f}"
      f"  post {d['posterior_last']}")
PY
}
BARGS="--spread-steps 0 $*"
run base X=0
if [ -n "${DYN_AB_RUNS:-}" ]; then
  # "name:VAR=value name2:VAR=value ..." instead of the default list
  for spec in $DYN_AB_RUNS; do run "${spec%%:*}" "${spec#*:}"; done
else
  if [ -z "${DYN_AB_SHORT:-}" ]; then
    run exact GPMDM_DYN_EXACT_GRID=1
    run n16x512 GPMDM_DYN_GEO=4,1,8
    run n32x256 GPMDM_DYN_GEO=4,2,4
    run w32x1024 GPMDM_DYNW_GEO=8,2,8
    run n32x512 GPMDM_DYN_GEO=4,2,8
  fi
  run n16x1024 GPMDM_DYN_GEO=4,1,16
  run w16x1024 GPMDM_DYNW_GEO=4,1,16
fi
run base2 X=0
