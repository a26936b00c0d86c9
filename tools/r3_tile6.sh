#!/bin/bash
# Tile shapes at the 4-GPU blocks (72 strip-rows per SIMD) against the split
# pipelines (2071): is there a tile shape worth a threshold move?
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile6
mkdir -p $O
export TMPDIR=/tmp HEAT_TB_TRACE=1
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep "gcells\|heat tb" $O/$name.log | cut -c1-150; }
for blk in "2048 8192" "4096 4096"; do set -- $blk
  step 200 v2071_${1}x${2} python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 2071 --waves 0 --iters 480 --rounds 7
  for shp in "13 8" "16 8" "24 8" "32 8" "12 16"; do set -- $blk $shp
    HEAT_TB_TILE_ROWS=$3 HEAT_TB_TILE_WAVES=$4 step 200 t${3}x${4}_${1}x${2} python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 131088 --waves 0 --iters 480 --rounds 7
  done
done
echo done
