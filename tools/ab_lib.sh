#!/bin/bash
# Same-box A/B of two builds of the library on the headline bench: the working tree
# (repo root) against a copy of another revision's package under tools/ab_prev/
# (gpmdm_amd/ with its built .so, and bench.py; made by `tools/ab_lib.sh prepare <worktree>`).
# Usage on the GPU box: bash tools/ab_lib.sh run <outdir> [rounds] [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
if [ "$1" = prepare ]; then
  src=$2; rm -rf tools/ab_prev; mkdir -p tools/ab_prev
  cp -rp "$src/gpmdm_amd" "$src/include" "$src/bench.py" tools/ab_prev/
  rm -rf tools/ab_prev/gpmdm_amd/_build tools/ab_prev/gpmdm_amd/__pycache__
  echo "prepared tools/ab_prev from $src ($(git -C "$src" rev-parse --short HEAD))"
  exit 0
fi
out=${2:-gpurun_out/ab_lib}; rounds=${3:-2}; shift 3 2>/dev/null
args=${*:---steps 300 --no-cpu-baseline --spread-steps 0 --no-nodedup}
mkdir -p "$out"
for r in $(seq "$rounds"); do
  for v in new prev; do
    dir=.; [ $v = prev ] && dir=tools/ab_prev
    (cd $dir && timeout -k 10 240 python -u bench.py $args) > "$out/${v}_$r.json" 2> "$out/${v}_$r.err" || { echo "$v failed"; tail -5 "$out/${v}_$r.err"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));st=d['stages_ms_per_step'];print(sys.argv[2], round(d['ms_per_step'],4), '%.4g'%d['value'], 'obs', round(d['roofline']['launch_ms'],4), 'switch', round(st['switch'],4), 'dyn', round(st['dyn_gemm'],4), 'resample', round(st['resample'],4))" "$out/${v}_$r.json" "$v"
  done
done
