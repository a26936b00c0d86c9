#!/bin/bash
# Tile kernel: barrier halfway through each step (early / late neighbour
# rows) vs the round-3 first version (barrier at the step boundary), A/B in
# separate processes on one box (abprev/ = the previous build), then tests.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile3
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep gcells $O/$name.log | cut -c1-120; }
step 300 t_tile python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tile.py
for rep in 1 2; do
for shp in "1024 8192" "2048 4096"; do set -- $shp
  HEAT_PY_ROOT=$PWD/abprev step 200 old_${1}x${2}_$rep python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 8,12 --variants 131088 --waves 0 --iters 480 --rounds 5
  step 200 new_${1}x${2}_$rep python tools/tb_sweep.py --n $2 --nx $1 --interior --depths 8,12 --variants 131088,23 --waves 0 --iters 480 --rounds 5
done; done
step 200 b1024 python bench.py --nx 1024 --steps 20 --warmup 5
tail -1 $O/b1024.log | cut -c1-200
echo done
