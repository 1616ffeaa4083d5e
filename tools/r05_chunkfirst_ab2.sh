set -o pipefail
out=gpurun_out/chunkfirst2; mkdir -p $out
for v in new prev; do
  root=.; [ $v = prev ] && root=tools/ab_prev
  for c in 2 3 5; do
    P=100000; [ $c = 5 ] && P=30000
    timeout -k 10 200 python -u $root/tools/cutoff_hash.py --config $c --P $P > $out/hash_${v}_$c.txt 2>&1 || { tail -5 $out/hash_${v}_$c.txt; exit 1; }
    tail -1 $out/hash_${v}_$c.txt | sed "s/^/$v /"
  done
done
for r in 1 2 3; do
  for v in new prev; do
    root=.; [ $v = prev ] && root=tools/ab_prev
    timeout -k 10 300 python -u $root/tools/cutoff_psweep.py --config 5 --ps 125000 --steps 20 --warmup 4 > $out/c5_${v}_$r.txt 2>&1 || { tail -5 $out/c5_${v}_$r.txt; exit 1; }
    grep '^{' $out/c5_${v}_$r.txt | sed "s/^/c5 $v /"
  done
done
