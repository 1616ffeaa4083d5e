set -o pipefail
mkdir -p gpurun_out/dynab
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export GPMDM_DYN16=1; else unset GPMDM_DYN16; fi
  timeout -k 10 200 python -u bench.py --steps 50 --no-cpu-baseline > gpurun_out/dynab/b$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/dynab/b$v.json'));print('dyn16=$v', d['stages_ms_per_step']['dyn_gemm'], d['ms_per_step'])"
done
