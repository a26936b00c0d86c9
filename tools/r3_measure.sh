#!/bin/bash
# Round-3 baseline measurements for the config-5 / convergence gaps:
#   counter list, 8192^2 bench with and without checks (interval 20 / 50),
#   per-cell kernel throughput at the 1-GPU and per-rank interior shapes
#   (incl. the 16384 x 131072 slab of a 1-D 8-GPU 131072^2 run),
#   131072^2 on one GPU with and without the interval-50 check.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3m
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -30 $O/$name.log; exit 1; }
  tail -3 $O/$name.log; }
step 60 counters rocprofv3 -L
step 300 bench python bench.py --steps 20 --warmup 5
step 300 bench_c20 python bench.py --steps 10 --warmup 2 --converge --check-interval 20
step 300 bench_c50 python bench.py --steps 10 --warmup 2 --converge --check-interval 50
step 300 sweep_8192 python tools/tb_sweep.py --n 8192 --nx 8192 --interior --depths 12 --variants 23,2071 --waves 0 --iters 480 --rounds 3
step 300 sweep_1024 python tools/tb_sweep.py --n 8192 --nx 1024 --interior --depths 12 --variants 23,2071 --waves 0 --iters 480 --rounds 3
step 300 sweep_2048x4096 python tools/tb_sweep.py --n 4096 --nx 2048 --interior --depths 12 --variants 23,2071 --waves 0 --iters 480 --rounds 3
step 300 sweep_16384x131072 python tools/tb_sweep.py --n 131072 --nx 16384 --interior --depths 12 --variants 23,2071 --waves 0 --iters 480 --rounds 3
step 400 big python bench.py --nx 131072 --ny 131072 --iters-per-step 1000 --steps 1 --warmup 1 --no-verify
step 400 big_c50 python bench.py --nx 131072 --ny 131072 --iters-per-step 1000 --steps 1 --warmup 1 --no-verify --converge --check-interval 50
echo "all done"
