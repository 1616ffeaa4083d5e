set -o pipefail
out=gpurun_out/split_ab2; mkdir -p $out
timeout -k 10 300 python -u tools/cutoff_split_ab.py --config 2 --P 20000,98304,100000,106496,131072 --rounds 2 > $out/config2.txt 2>&1 || { tail -5 $out/config2.txt; exit 1; }
timeout -k 10 300 python -u tools/cutoff_split_ab.py --config 3 --P 98304,120000 --rounds 1 > $out/config3.txt 2>&1 || { tail -5 $out/config3.txt; exit 1; }
grep -h '^{' $out/config2.txt $out/config3.txt | python -c "
import sys,json
from collections import defaultdict
d=defaultdict(list)
for l in sys.stdin:
    r=json.loads(l); d[(r['config'],r['P'],r['split'])].append(r['obs_launch_ms']+r['obs_finish_ms'])
for k in sorted(d): print(k, ['%.4f'%v for v in d[k]])
"
