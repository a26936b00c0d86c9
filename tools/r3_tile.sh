#!/bin/bash
# Round-3 workgroup-tile kernel: numerics tests, then the tile vs the
# streaming kernels at the per-rank block shapes of 1-8 GPU runs (interleaved
# rounds in one process, tools/tb_sweep.py), and the tile height sweep.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tile
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep -v amdgpu.ids $O/$name.log | tail -12 | cut -c1-260; }
export HEAT_TB_TRACE=1
step 300 t_tile python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tile.py
VS="23,2071,131088,393232"
step 200 s1024 python tools/tb_sweep.py --n 8192 --nx 1024 --interior --depths 12 --variants $VS --waves 0 --iters 480 --rounds 5
step 200 s2048x4096 python tools/tb_sweep.py --n 4096 --nx 2048 --interior --depths 12 --variants $VS --waves 0 --iters 480 --rounds 5
step 200 s2048x8192 python tools/tb_sweep.py --n 8192 --nx 2048 --interior --depths 12 --variants $VS --waves 0 --iters 480 --rounds 5
step 200 s8192 python tools/tb_sweep.py --n 8192 --depths 12 --variants $VS --waves 0 --iters 480 --rounds 5
for r in 12 16 24; do
  HEAT_TB_TILE_ROWS=$r step 200 r${r}_1024 python tools/tb_sweep.py --n 8192 --nx 1024 --interior --depths 8,12 --variants 131088,393232 --waves 0 --iters 480 --rounds 5
done
echo done
