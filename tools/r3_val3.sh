#!/bin/bash
# After the tile threshold change (< 64 strip-rows per SIMD): GPU tests,
# per-rank-shape benches, tile counters.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3val3
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -1 $O/$name.log | cut -c1-250; }
step 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 200 b1536 python bench.py --nx 1536 --steps 20 --warmup 5
step 200 b1024 python bench.py --nx 1024 --steps 20 --warmup 5
step 300 bench python bench.py --steps 20 --warmup 5
bash tools/pmc_tile.sh > $O/pmc.log 2>&1 || { tail -30 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
echo done
