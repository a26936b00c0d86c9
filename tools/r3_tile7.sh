#!/bin/bash
# Two-workgroup tile shapes at the 1- and 2-GPU blocks against the split
# pipelines (2071).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile7
mkdir -p $O
export TMPDIR=/tmp HEAT_TB_TRACE=1
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep "gcells\|heat tb" $O/$name.log | cut -c1-150; }
for blk in "4096 8192" "8192 8192" "2048 8192"; do set -- $blk
  step 200 v2071_${1}x${2} python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 2071 --waves 0 --iters 480 --rounds 7
  for shp in "14 8" "16 8"; do set -- $blk $shp
    HEAT_TB_TILE_ROWS=$3 HEAT_TB_TILE_WAVES=$4 step 200 t${3}x${4}_${1}x${2} python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 131088,2071 --waves 0 --iters 480 --rounds 7
  done
done
echo done
