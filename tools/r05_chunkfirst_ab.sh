set -o pipefail
out=gpurun_out/chunkfirst; mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_obs_cutoff.py tests/test_gpu_bank.py::test_bank_with_cutoff_equals_independent_cutoff_filters "tests/test_gpu_large_configs.py::test_large_config_cutoff_vs_oracle" > $out/pytest.txt 2>&1 || { tail -20 $out/pytest.txt; exit 1; }
tail -1 $out/pytest.txt
for r in 1 2; do
  for v in new prev; do
    root=.; [ $v = prev ] && root=tools/ab_prev
    timeout -k 10 150 python -u $root/tools/cutoff_psweep.py --ps 98304,100000 --steps 60 > $out/c2_${v}_$r.txt 2>&1 || { tail -5 $out/c2_${v}_$r.txt; exit 1; }
    grep '^{' $out/c2_${v}_$r.txt | sed "s/^/c2 $v /"
    timeout -k 10 200 python -u $root/tools/cutoff_psweep.py --config 3 --ps 100000 --steps 10 --warmup 4 > $out/c3_${v}_$r.txt 2>&1 || { tail -5 $out/c3_${v}_$r.txt; exit 1; }
    grep '^{' $out/c3_${v}_$r.txt | sed "s/^/c3 $v /"
    timeout -k 10 300 python -u $root/tools/cutoff_psweep.py --config 5 --ps 125000 --steps 6 --warmup 3 > $out/c5_${v}_$r.txt 2>&1 || { tail -5 $out/c5_${v}_$r.txt; exit 1; }
    grep '^{' $out/c5_${v}_$r.txt | sed "s/^/c5 $v /"
  done
done
