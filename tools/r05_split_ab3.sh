set -o pipefail
out=gpurun_out/split_ab3; mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_obs_cutoff.py tests/test_gpu_bank.py::test_bank_with_cutoff_equals_independent_cutoff_filters "tests/test_gpu_large_configs.py::test_large_config_cutoff_vs_oracle" > $out/pytest.txt 2>&1 || { tail -20 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
timeout -k 10 300 python -u tools/cutoff_split_ab.py --config 2 --P 20000,100000 --rounds 1 > $out/config2.txt 2>&1 || { tail -5 $out/config2.txt; exit 1; }
grep -h '^{' $out/config2.txt | python -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['config'], r['P'], r['split'], '%.4f'%(r['obs_launch_ms']+r['obs_finish_ms']))
"
