#!/bin/bash
# Round-3 kernel A/B: residual-at-level cost, linear (balanced) plans vs the
# classic (strip, chunk) plans, the round-2 build (build/ab_head) as baseline.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3ab
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -12 $O/$name.log; }
HEADPY=build/ab_head
step 300 t_kern python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_converge_gated.py
step 200 res_new python tools/res_cost.py --n 8192 --depth 12 --variants 2071,23 --levels 0,12,8,6,4,2
step 200 res_head env HEAT_PY_ROOT=$HEADPY python tools/res_cost.py --n 8192 --depth 12 --variants 2071,23 --levels 0,12
step 300 sw8192 python tools/tb_sweep.py --n 8192 --depths 12 --variants 2071,34839,23,32791 --waves 0 --iters 480 --rounds 5
step 300 sw8192_head env HEAT_PY_ROOT=$HEADPY python tools/tb_sweep.py --n 8192 --depths 12 --variants 2071,23 --waves 0 --iters 480 --rounds 5
step 300 sw1024 python tools/tb_sweep.py --n 8192 --nx 1024 --interior --depths 12 --variants 2071,34839,23,32791 --waves 0 --iters 480 --rounds 5
step 300 sw2048x4096 python tools/tb_sweep.py --n 4096 --nx 2048 --interior --depths 12 --variants 2071,34839,23,32791 --waves 0 --iters 480 --rounds 5
step 300 sw16384x131072 python tools/tb_sweep.py --n 131072 --nx 16384 --interior --depths 12 --variants 2071,34839,23,32791 --waves 0 --iters 240 --rounds 3
step 400 sw131072 python tools/tb_sweep.py --n 131072 --depths 12 --variants 2071,34839 --waves 0 --iters 120 --rounds 3
echo "all done"
