#!/bin/bash
# Round-3 A/B 4: full GPU tests, waves per SIMD at the 8-GPU per-rank blocks,
# convergence-on bench rows with the direct-call kernel, MFMA kernel numbers.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3ab4
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -14 $O/$name.log; }
step 600 t_all python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
step 300 w1024 python tools/tb_sweep.py --n 8192 --nx 1024 --interior --depths 12,8 --variants 23 --waves 1008,1536,2048,3072 --iters 480 --rounds 5
step 300 w2048x4096 python tools/tb_sweep.py --n 4096 --nx 2048 --interior --depths 12,8 --variants 23 --waves 1008,1536,2048,3072 --iters 480 --rounds 5
step 200 kb python tools/kernel_bench.py --n 8192 --steps 40
step 300 bench python bench.py --steps 20 --warmup 5
step 300 ref python bench.py --steps 10 --warmup 2 --init ref-wrap
step 300 ref_c20 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 20
step 300 ref_c50 python bench.py --steps 10 --warmup 2 --init ref-wrap --converge --check-interval 50
KERNELS=mfma bash tools/pmc_mfma.sh
echo "all done"
