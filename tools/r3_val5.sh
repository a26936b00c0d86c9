#!/bin/bash
# One residual atomic per tile workgroup: tests, convergence-on benches at
# the 8-GPU per-rank plate.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3val5
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -1 $O/$name.log | cut -c1-180; }
step 300 t_tile python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tile.py tests/test_gpu_converge_gated.py tests/test_gpu_solver.py
step 200 ref_1024 python bench.py --nx 1024 --init ref-wrap --steps 10 --warmup 3
step 200 ref_1024_c20 python bench.py --nx 1024 --init ref-wrap --converge --check-interval 20 --steps 10 --warmup 3
step 200 ref_1024_c50 python bench.py --nx 1024 --init ref-wrap --converge --check-interval 50 --steps 10 --warmup 3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_c20 -o run -- python3 $OLDPWD/bench.py --nx 1024 --init ref-wrap --converge --check-interval 20 --steps 3 --warmup 1 > $OLDPWD/$O/prof_c20.log 2>&1 || { tail -30 $OLDPWD/$O/prof_c20.log; exit 1; }
echo done
