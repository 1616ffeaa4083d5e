set -o pipefail
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 120 python -u bench.py --gpus 2 --steps 3 > gpurun_out/r04a/refuse.out 2> gpurun_out/r04a/refuse.err; echo "refuse rc=$?"
tail -2 gpurun_out/r04a/refuse.err
timeout -k 10 400 python -u bench.py --gpus 2 --rehearse-gloo --steps 5 --warmup 2 --no-cpu-baseline --no-nodedup > gpurun_out/r04a/gloo2.json 2> gpurun_out/r04a/gloo2.err || { echo "rehearsal failed rc=$?"; tail -30 gpurun_out/r04a/gloo2.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/r04a/gloo2.json')); print({k: r[k] for k in ('n_gpus','world_size_backend','backend','launcher','exchange','rehearsal','value','ms_per_step')})"
timeout -k 10 300 python -u bench.py --steps 50 --no-cpu-baseline > gpurun_out/r04a/bench1.json 2> gpurun_out/r04a/bench1.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/r04a/bench1.err; exit 1; }
python -c "import json; r=json.load(open('gpurun_out/r04a/bench1.json')); print({k: r[k] for k in ('n_gpus','launcher','exchange','value','ms_per_step')}, r['roofline']['frac'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_checkpoint.py tests/test_gpu_systematic_stats.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04a/pytest_new.log 2>&1 || { echo "new tests failed rc=$?"; tail -40 gpurun_out/r04a/pytest_new.log; exit 1; }
tail -15 gpurun_out/r04a/pytest_new.log
