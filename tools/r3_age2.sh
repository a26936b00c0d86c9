#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3age2
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -12 $O/$name.log; }
step 200 t_kern python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py
step 300 a16384 python tools/age_sweep.py --n 131072 --nx 16384 --interior --iters 240 --sets ";1.8,1.8,1.2,1;2.2,2.1,1.2,1;2.4,2.2,1.3,1;2.0,1.9,1.3,1;1.7,1" --rounds 3
step 400 a131072 python tools/age_sweep.py --n 131072 --iters 120 --sets ";2.2,2.1,1.2,1;1.7,1" --rounds 3
step 400 big python bench.py --nx 131072 --ny 131072 --iters-per-step 1000 --steps 1 --warmup 1 --no-verify
step 400 big_c50 python bench.py --nx 131072 --ny 131072 --iters-per-step 1000 --steps 1 --warmup 1 --no-verify --converge --check-interval 50 --init ref-wrap
step 300 bench python bench.py --steps 20 --warmup 5
echo done
