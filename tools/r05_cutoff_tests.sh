set -o pipefail
out=gpurun_out/r05_c; mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_obs_cutoff.py tests/test_gpu_large_configs.py -x -v --timeout 900 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -25 $out/pytest.log
[ $rc = 0 ] || exit $rc
