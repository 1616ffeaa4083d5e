#!/bin/bash
# Dynamics-tile heights on the 16 x 256 image (16 / 32 / 64 particle rows per workgroup:
# bitwise the same results) against the default pair (narrow 16x256 + wide observation-
# shaped image for every-particle passes), on config 2 (headline, spread and nodedup lines)
# and config 5.  Usage: bash tools/dyn_family.sh <tag> [configs]
set -o pipefail
out=gpurun_out/${1:-dynfam}; cfgs=${2:-"2 5"}
mkdir -p $out
export TMPDIR=/tmp
for cfg in $cfgs; do
  steps=100; [ $cfg = 5 ] && steps=5
  for v in default mt1 mt2 mt4; do
    case $v in
      default) envs=""; extra="";;
      *) envs="GPMDM_DYN_MT=${v#mt}"; extra="--dyn-tiles narrow";;
    esac
    env $envs timeout -k 10 400 python -u bench.py --config $cfg --steps $steps --no-cpu-baseline --replay-steps 0 $extra \
      > $out/c${cfg}_$v.json 2> $out/c${cfg}_$v.err || { echo "bench c$cfg $v failed rc=$?"; tail -5 $out/c${cfg}_$v.err; exit 1; }
    python - $out/c${cfg}_$v.json $cfg $v <<'PY'
import json, sys
r = json.load(open(sys.argv[1]))
st = r["stages_ms_per_step"]; nd = r.get("nodedup") or {}; sp = r.get("spread") or {}
print(f"cfg {sys.argv[2]} {sys.argv[3]:8s} step {r['ms_per_step']:.3f} dyn {st['dyn_gemm']:.4f} rows {r['dyn_rows_last']['breakdown_mean']:.0f} "
      f"({r['dyn_rows_last']['dyn_gemm_tflops']:.1f} TF/s) | nodedup dyn {nd.get('stages_ms_per_step', {}).get('dyn_gemm', 0):.4f} "
      f"({nd.get('dyn_gemm_tflops', 0):.1f} TF/s) | spread dyn {sp.get('stages_ms_per_step', {}).get('dyn_gemm', 0):.4f} "
      f"rows {sp.get('dyn_rows_mean', 0):.0f} ({sp.get('dyn_gemm_tflops', 0):.1f} TF/s)", flush=True)
PY
  done
done
