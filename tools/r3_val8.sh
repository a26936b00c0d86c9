#!/bin/bash
# Final round-3 validation: whole GPU suite, smoke, bench (8192^2), the 8-GPU
# per-rank plates, the 8-rank RCCL rehearsal of the bench path.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3val8
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -1 $O/$name.log | cut -c1-200; }
step 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 200 smoke python -c "import __graft_entry__ as g; g.smoke()"
step 300 bench python bench.py --steps 20 --warmup 5
step 200 b1024 python bench.py --nx 1024 --steps 20 --warmup 5
step 200 b2048x4096 python bench.py --nx 2048 --ny 4096 --steps 20 --warmup 5
bash tools/rccl_rehearsal.sh "8" --steps 3 --warmup 1 > $O/rehearsal8.log 2>&1 || { tail -30 $O/rehearsal8.log; exit 1; }
cp gpurun_out/rccl_rehearsal_n8.json $O/
grep -o '"verified": [a-z]*' $O/rccl_rehearsal_n8.json
echo done
