#!/bin/bash
# Tile lane shifts: ds_bpermute (1, default) vs mixed DPP-left / bpermute-right
# (2) vs DPP (0), separate processes interleaved, two repeats; the tile tests
# under the mixed build.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile8
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep "gcells\|passed" $O/$name.log | cut -c1-120; }
HEAT_TB_TILE_XL=2 step 300 t_tile_xl2 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tile.py
for rep in 1 2; do
  for xl in 1 2 0; do
    for blk in "1024 8192" "2048 4096"; do set -- $blk
      HEAT_TB_TILE_XL=$xl step 200 xl${xl}_${1}x${2}_$rep python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 131088 --waves 0 --iters 480 --rounds 7
    done
  done
done
for xl in 1 2; do
  HEAT_TB_TILE_XL=$xl timeout -k 10 200 python bench.py --nx 1024 --steps 20 --warmup 5 > $O/b1024_xl$xl.log 2>&1 || exit 1
  echo "b1024 xl$xl $(tail -1 $O/b1024_xl$xl.log | cut -c90-130)"
done
echo done
