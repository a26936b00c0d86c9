#!/bin/bash
# Round 6 final tree (after the r6z revert of the plain-row unit)
# then the driver's round-end sequence on one box: GPU tests,
# smoke(), the driver-style bench and a kernel-trace profile of the bench.
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r6fin
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_$i.log 2>&1 || { cat $OUT/bench_$i.log; exit 1; }
  tail -1 $OUT/bench_$i.log
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$OUT/prof -o run -- python3 $OLDPWD/bench.py --steps 5 --warmup 2 > $OLDPWD/$OUT/prof.log 2>&1 || { tail -30 $OLDPWD/$OUT/prof.log; exit 1; }
cd $OLDPWD
tail -1 $OUT/prof.log
