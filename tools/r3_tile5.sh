#!/bin/bash
# Tile planner with the 13 x 8 shape and the recalibrated cost model: auto
# choice vs forced shapes at the 8-GPU blocks and the deep-halo pass, then
# the tile tests and the whole-solver per-rank plates.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile5
mkdir -p $O
export TMPDIR=/tmp HEAT_TB_TRACE=1
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep "gcells\|heat tb\|passed\|failed" $O/$name.log | cut -c1-150; }
step 300 t_tile python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tile.py
for blk in "1024 8192" "2048 4096" "1192 8192" "1536 8192"; do set -- $blk
  step 200 auto_${1}x${2} python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 131088 --waves 0 --iters 480 --rounds 7
  HEAT_TB_TILE_ROWS=12 HEAT_TB_TILE_WAVES=16 step 200 f12x16_${1}x${2} python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 12 --variants 131088 --waves 0 --iters 480 --rounds 7
done
unset HEAT_TB_TRACE
for blk in "1024 8192" "2048 4096"; do set -- $blk
  step 200 b${1}x${2} python bench.py --nx $1 --ny $2 --steps 20 --warmup 5
  tail -1 $O/b${1}x${2}.log | cut -c1-150
done
echo done
