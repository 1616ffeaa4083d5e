set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/cutkt2; mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_obs_cutoff.py tests/test_gpu_bank.py::test_bank_with_cutoff_equals_independent_cutoff_filters tests/test_gpu_checkpoint.py > $out/pytest.txt 2>&1 || { tail -20 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
for sp in none tail; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$sp -- python tools/cutoff_psweep.py --ps 100000 --steps 40 --split $sp > $out/log_$sp.txt 2>&1 || exit 1
done
