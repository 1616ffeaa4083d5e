set -o pipefail
out=gpurun_out/chunkfirst3; mkdir -p $out
for r in 1 2; do
  for v in new prev; do
    root=.; [ $v = prev ] && root=tools/ab_prev
    (cd $root && timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-nodedup --cutoff-steps 8) > $out/c5_${v}_$r.json 2> $out/c5_${v}_$r.err || { tail -5 $out/c5_${v}_$r.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['cutoff'];print('c5', sys.argv[2], round(c['ms_per_step'],3), round(c['obs_launch_ms'],3), round(c['executed_frac_of_peak'],3))" $out/c5_${v}_$r.json $v
  done
done
