set -o pipefail
out=${OUT:-gpurun_out/r04_zc}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1; tail -2 $out/pytest.log
grep -q " passed" $out/pytest.log && ! grep -q "failed" $out/pytest.log || exit 1
for r in 1 2 3; do
  for v in new prev; do
    dir=.; [ $v = prev ] && dir=tools/ab_prev
    (cd $dir && timeout -k 10 300 python -u bench.py --config 1 --no-cpu-baseline --bank 0) > $out/c1_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], r['ms_per_step'], r.get('untimed_ms_per_step'))" $out/c1_${v}_$r.json $v
  done
done
for r in 1 2; do
  for v in new prev; do
    dir=.; [ $v = prev ] && dir=tools/ab_prev
    (cd $dir && timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --no-cpu-baseline --rng torch --spread-steps 0 --replay-steps 0) > $out/rep_${v}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print('replay100k', sys.argv[2], r['ms_per_step'])" $out/rep_${v}_$r.json $v
  done
done
