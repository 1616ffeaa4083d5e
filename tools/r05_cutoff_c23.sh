set -o pipefail
out=gpurun_out/${1:-r05_v8}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_obs_cutoff.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
timeout -k 10 400 python -u bench.py --steps 30 --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup > $out/c2.json 2> $out/c2.err || { echo "c2 failed"; exit 1; }
python -c "import json;d=json.load(open('$out/c2.json'));c=d['cutoff'];print('c2', round(c['ms_per_step'],3), round(c['obs_launch_ms'],3))"
timeout -k 10 600 python -u bench.py --config 3 --steps 10 --no-cpu-baseline --no-nodedup --cutoff-steps 10 > $out/c3.json 2> $out/c3.err || { echo "c3 failed"; exit 1; }
python -c "import json;d=json.load(open('$out/c3.json'));c=d['cutoff'];print('c3', round(c['ms_per_step'],3), round(c['obs_launch_ms'],3))"
