#!/bin/bash
# Round-3 workgroup-tile kernel, second pass: tests with the 16-wave shape,
# then shape x depth at the 8-GPU per-rank blocks (time = memory phase +
# depth x step: the depth sweep separates the two).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile2
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep -v amdgpu.ids $O/$name.log | grep gcells | cut -c1-140; }
export HEAT_TB_TRACE=1
step 300 t_tile python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tile.py tests/test_tb_tuning.py
for sh in "24 8" "12 16" "16 8"; do set -- $sh
  HEAT_TB_TILE_ROWS=$1 HEAT_TB_TILE_WAVES=$2 step 200 k_${1}x${2}_1024 python tools/tb_sweep.py --n 8192 --nx 1024 --interior --depths 2,4,8,12 --variants 131088 --waves 0 --iters 480 --rounds 5
  HEAT_TB_TILE_ROWS=$1 HEAT_TB_TILE_WAVES=$2 step 200 k_${1}x${2}_2048x4096 python tools/tb_sweep.py --n 4096 --nx 2048 --interior --depths 12 --variants 131088,23 --waves 0 --iters 480 --rounds 5
done
step 200 auto_1024 python tools/tb_sweep.py --n 8192 --nx 1024 --interior --depths 8,12 --variants 131088,23,2071 --waves 0 --iters 480 --rounds 5
step 200 auto_1536 python tools/tb_sweep.py --n 8192 --nx 1536 --interior --depths 12 --variants 131088,23,2071 --waves 0 --iters 480 --rounds 5
step 200 auto_4096 python tools/tb_sweep.py --n 4096 --nx 4096 --interior --depths 12 --variants 131088,23,2071 --waves 0 --iters 480 --rounds 5
echo done
