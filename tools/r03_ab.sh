#!/bin/bash
# Round-3 kernel A/B pass: the cleaned gp_tile.h against the pre-split source (tile_ab.sh,
# bitwise hashes + timings at d = 3 / 8 / 16) and the dynamics-tile shapes (dyn_ab.sh).
set -o pipefail
out=gpurun_out/r03_ab
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 bash tools/microbench/tile_ab.sh run > $out/tile_ab.txt 2>&1 \
  || { echo "tile_ab failed rc=$?"; tail -20 $out/tile_ab.txt; exit 1; }
cat $out/tile_ab.txt
timeout -k 10 600 bash tools/dyn_ab.sh $out/dynab 2>&1 | tee $out/dyn_ab.txt
echo done
