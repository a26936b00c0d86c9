#!/bin/bash
# GPU check of the device-judged convergence path + its bench A/B, then the
# translation/cache counter passes of tools/pmc_shapes.sh.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3g
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -2 $O/$name.log; }
step 300 t_gated python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_converge_gated.py tests/test_gpu_solver.py
step 600 t_all python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
step 300 bench python bench.py --steps 20 --warmup 5
step 300 ref python bench.py --steps 10 --warmup 2 --init ref-wrap
step 300 ref_c20 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 20
step 300 ref_c20_host env HEAT_HOST_CHECKS=1 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 20
step 300 ref_c50 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 50
step 300 ref_c50_host env HEAT_HOST_CHECKS=1 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 50
bash tools/pmc_shapes.sh
