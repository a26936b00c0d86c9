#!/bin/bash
# 4-GPU per-rank blocks (72 strip-rows per SIMD) with the mixed-shift tile:
# forced tile shapes vs the split pipelines, interior sweeps (same process)
# and whole-solver plates with plate edges.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile9
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep "gcells" $O/$name.log | cut -c1-110; }
for blk in "2048 8192" "4096 4096"; do set -- $blk
  for shp in "16 8" "13 8"; do set -- $blk $shp
    HEAT_TB_TILE_ROWS=$3 HEAT_TB_TILE_WAVES=$4 step 200 t${3}x${4}_${1}x${2} python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 131088,2071 --waves 0 --iters 480 --rounds 7
  done
  timeout -k 10 200 python bench.py --nx $1 --ny $2 --steps 10 --warmup 3 > $O/b${1}x${2}.log 2>&1 || exit 1
  HEAT_TB_VARIANT=131088 HEAT_TB_TILE_ROWS=16 HEAT_TB_TILE_WAVES=8 timeout -k 10 200 python bench.py --nx $1 --ny $2 --steps 10 --warmup 3 > $O/b${1}x${2}_t16.log 2>&1 || exit 1
  echo "plate $1x$2 default $(tail -1 $O/b${1}x${2}.log | cut -c90-115) tile16x8 $(tail -1 $O/b${1}x${2}_t16.log | cut -c90-115)"
done
echo done
