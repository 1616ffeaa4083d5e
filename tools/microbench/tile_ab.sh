#!/bin/bash
# Build tile_ab.hip against gp_tile.h as of several commits (WT = the working tree), here:
#   bash tools/microbench/tile_ab.sh build <commit>[:MACRO,...]...
# and run them alternately on the GPU box:  bash tools/microbench/tile_ab.sh run
set -e
cd "$(dirname "$0")/../.."
out=tools/microbench/ab
if [ "$1" = build ]; then
  shift; rm -rf $out; mkdir -p $out
  # a build spec is <commit|WT>[:MACRO[,MACRO...]] -- the macros are defined for that build
  # (A/B candidates kept behind #ifdef in the working tree), e.g. WT:GPMDM_EXP_SHIFT
  for spec in "$@"; do
    c=${spec%%:*}; defs=""; name=$c
    if [ "$spec" != "$c" ]; then
      for m in $(echo ${spec#*:} | tr ',' ' '); do defs="$defs -D$m"; done
      name=${c}_$(echo ${spec#*:} | tr ',' '_')
    fi
    src=/tmp/tile_ab_src/$c; rm -rf $src; mkdir -p $src
    if [ $c = WT ]; then cp -r gpmdm_amd include $src/; else git archive $c gpmdm_amd/csrc include | tar -x -C $src; fi
    for d in 3 8 16; do
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I $src/include -DTB_D=$d $defs \
        "-DGP_TILE_H=\"$src/gpmdm_amd/csrc/gp_tile.h\"" tools/microbench/tile_ab.hip -o $out/tile_ab_d${d}_$name &
    done
  done
  wait; ls $out
else
  # timings alternate between the builds; the first round also prints a hash of each
  # build's production-variant q partials and means (TB_QHASH): equal hashes = bitwise equal
  for r in 1 2; do
    h=$([ $r = 1 ] && echo 1 || true)
    for b in $out/tile_ab_d16_*; do echo "== $b"; TB_QHASH=$h timeout -k 10 170 $b 125000 20000 256 | grep -E "median|qhash"; done
    for b in $out/tile_ab_d8_*; do echo "== $b"; TB_QHASH=$h timeout -k 10 120 $b 100000 10000 128 | grep -E "median|qhash"; done
    for b in $out/tile_ab_d3_*; do echo "== $b"; TB_QHASH=$h timeout -k 10 60 $b | grep -E "median|qhash"; done
  done
fi
