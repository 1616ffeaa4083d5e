set -o pipefail
out=gpurun_out/split_ab; mkdir -p $out
for c in 2 3 5; do
  timeout -k 10 300 python -u tools/cutoff_split_ab.py --config $c > $out/config$c.txt 2>&1 || { tail -5 $out/config$c.txt; exit 1; }
  grep '^{' $out/config$c.txt
done
