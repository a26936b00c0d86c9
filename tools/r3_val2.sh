#!/bin/bash
# Round-3: tile auto-selection for every even depth on small launches.
# GPU tests, the per-rank-shape benches, the 8-rank RCCL rehearsal of the
# 8-GPU bench path (1024-row blocks: the tile kernel under RCCL graphs).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3val2
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -2 $O/$name.log | cut -c1-300; }
step 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 200 b1024 python bench.py --nx 1024 --steps 20 --warmup 5
step 200 b2048x4096 python bench.py --nx 2048 --ny 4096 --steps 20 --warmup 5
HEAT_TB_TRACE=1 step 200 b1024_trace python bench.py --nx 1024 --steps 2 --warmup 1
bash tools/rccl_rehearsal.sh "8" --steps 3 --warmup 1 || exit 1
cp gpurun_out/rccl_rehearsal_n8.json gpurun_out/rccl_rehearsal_n8.err $O/
echo done
