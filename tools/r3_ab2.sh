#!/bin/bash
# Round-3 A/B 2: residual at the pass end (cheap NaN-safe max) vs round 2,
# per-depth pass cost, automatic linear plans, convergence-on bench rows.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3ab2
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -14 $O/$name.log; }
HEADPY=build/ab_head
step 300 t_kern python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_converge_gated.py tests/test_gpu_solver.py
step 200 res_new python tools/res_cost.py --n 8192 --depths 12,8,7 --variants 2071,23
step 200 res_head env HEAT_PY_ROOT=$HEADPY python tools/res_cost.py --n 8192 --depths 12,8,7 --variants 2071,23
step 300 sw8192 python tools/tb_sweep.py --n 8192 --depths 12 --variants 2071,23 --waves 0 --iters 480 --rounds 5
step 300 sw8192_head env HEAT_PY_ROOT=$HEADPY python tools/tb_sweep.py --n 8192 --depths 12 --variants 2071,23 --waves 0 --iters 480 --rounds 5
step 300 sw16384x131072 python tools/tb_sweep.py --n 131072 --nx 16384 --interior --depths 12 --variants 2071,67607,23,65559 --waves 0 --iters 240 --rounds 3
step 400 sw131072 python tools/tb_sweep.py --n 131072 --depths 12 --variants 2071,67607 --waves 0 --iters 120 --rounds 3
step 300 bench python bench.py --steps 20 --warmup 5
step 300 ref python bench.py --steps 10 --warmup 2 --init ref-wrap
step 300 ref_c20 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 20
step 300 ref_c50 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 50
step 400 big python bench.py --nx 131072 --ny 131072 --iters-per-step 1000 --steps 1 --warmup 1 --no-verify
step 400 big_c50 python bench.py --nx 131072 --ny 131072 --iters-per-step 1000 --steps 1 --warmup 1 --no-verify --converge --check-interval 50
echo "all done"
