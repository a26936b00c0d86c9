#!/bin/bash
# Round-3 A/B 3: classic plans with a direct segment call (vs round 2), and
# deeper two-wave level-split pipelines (14 = 7+7, 16 = 8+8) at 8192^2.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3ab3
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -14 $O/$name.log; }
HEADPY=build/ab_head
step 300 t_kern python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_converge_gated.py
step 300 sw8192 python tools/tb_sweep.py --n 8192 --depths 12,14,16 --variants 2071 --waves 0 --iters 480 --rounds 7
step 300 sw8192_head env HEAT_PY_ROOT=$HEADPY python tools/tb_sweep.py --n 8192 --depths 12 --variants 2071 --waves 0 --iters 480 --rounds 7
step 300 sw8192_b python tools/tb_sweep.py --n 8192 --depths 12,16 --variants 2071 --waves 0 --iters 480 --rounds 7
step 300 sw2048x8192 python tools/tb_sweep.py --n 8192 --nx 2048 --interior --depths 12,14,16 --variants 2071 --waves 0 --iters 480 --rounds 5
step 300 bench python bench.py --steps 20 --warmup 5
step 300 bench16 python bench.py --steps 20 --warmup 5 --tb-depth 16
step 300 bench14 python bench.py --steps 20 --warmup 5 --tb-depth 14
echo "all done"
