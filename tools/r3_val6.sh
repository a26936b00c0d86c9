#!/bin/bash
# One residual atomic per workgroup in every TB kernel: GPU tests, bench,
# convergence-on benches (reference init, checks every 20 / 50) at 8192^2 and
# at the 8-GPU per-rank plate.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3val6
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -1 $O/$name.log | cut -c1-180; }
step 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 300 bench python bench.py --steps 20 --warmup 5
for nx in 8192 1024; do
  step 200 ref_$nx python bench.py --nx $nx --init ref-wrap --steps 10 --warmup 3
  step 200 ref_${nx}_c20 python bench.py --nx $nx --init ref-wrap --converge --check-interval 20 --steps 10 --warmup 3
  step 200 ref_${nx}_c50 python bench.py --nx $nx --init ref-wrap --converge --check-interval 50 --steps 10 --warmup 3
done
echo done
