#!/bin/bash
# Round-3 run 5: XCD-ordered single-step kernels (LDS, MFMA) with counters,
# the multi-rank RCCL bench path (shared transport, RCCL fields in the JSON).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3ab5
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -14 $O/$name.log; }
step 400 t_sub python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_loopback.py tests/test_gpu_solver.py tests/test_gpu_rccl_multirank.py
step 200 kb python tools/kernel_bench.py --n 8192 --steps 40
KERNELS="mfma lds" bash tools/pmc_mfma.sh || exit 1
bash tools/rccl_rehearsal.sh "2 4" --steps 3 --warmup 1 || exit 1
cp gpurun_out/rccl_rehearsal_n*.json gpurun_out/rccl_rehearsal_n*.err $O/ 2>/dev/null
step 300 bench python bench.py --steps 20 --warmup 5
echo "all done"
