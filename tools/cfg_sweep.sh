set -o pipefail
mkdir -p gpurun_out/cfg
for spec in "3 0" "3 1" "5 0" "5 3" "5 2"; do
  set -- $spec
  GPMDM_TILE_SHAPE=$2 timeout -k 10 240 python -u bench.py --config $1 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/cfg/c$1_s$2.json 2> gpurun_out/cfg/c$1_s$2.err || { echo "fail $spec"; tail -5 gpurun_out/cfg/c$1_s$2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/cfg/c$1_s$2.json'));print('cfg $1 shape $2', round(d['ms_per_step'],2), 'ms', d['roofline']['frac'], d['stages_ms_per_step'])"
done
