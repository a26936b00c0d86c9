#!/bin/bash
# Even remainder passes only for tile-sized runs: solver tests, the
# convergence-on benches at 8192^2 and the 8-GPU per-rank plate.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3val7
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -1 $O/$name.log | cut -c1-180; }
step 600 pytest python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_gpu_converge_gated.py tests/test_gpu_loopback.py tests/test_gpu_tile.py
for nx in 8192 1024; do
  step 200 ref_$nx python bench.py --nx $nx --init ref-wrap --steps 10 --warmup 3
  step 200 ref_${nx}_c20 python bench.py --nx $nx --init ref-wrap --converge --check-interval 20 --steps 10 --warmup 3
  step 200 ref_${nx}_c50 python bench.py --nx $nx --init ref-wrap --converge --check-interval 50 --steps 10 --warmup 3
done
echo done
