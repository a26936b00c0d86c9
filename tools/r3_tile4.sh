#!/bin/bash
# Tile shapes at the 8-GPU blocks: two independent workgroups per CU (14 x 8,
# 4 waves per SIMD from two tiles) vs one 16-wave workgroup (12 x 16) vs 24 x 8.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile4
mkdir -p $O
export TMPDIR=/tmp HEAT_TB_TRACE=1
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep "gcells\|heat tb" $O/$name.log | cut -c1-150; }
for shp in "14 8" "12 16" "24 8"; do set -- $shp
  for blk in "1024 8192" "2048 4096" "1192 8192"; do set -- $shp $blk
    HEAT_TB_TILE_ROWS=$1 HEAT_TB_TILE_WAVES=$2 step 200 s${1}x${2}_${3}x${4} python tools/tb_sweep.py --n $4 --nx $3 --interior --depths 12 --variants 131088 --waves 0 --iters 480 --rounds 7
  done
done
echo done
