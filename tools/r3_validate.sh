#!/bin/bash
# Round-3 validation of the tree with the workgroup-tile kernel: the whole GPU
# test suite, bench.py at the headline 8192^2 and at the 8-GPU per-rank block
# shapes run as one-GPU plates (tile default vs the round-2 single-wave
# kernel, HEAT_TB_VARIANT=23), and a rocprofv3 kernel-stats profile.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3val
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -3 $O/$name.log | cut -c1-400; }
step 900 pytest python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step 300 bench python bench.py --steps 20 --warmup 5
step 200 b1024 python bench.py --nx 1024 --steps 20 --warmup 5
HEAT_TB_VARIANT=23 step 200 b1024_v23 python bench.py --nx 1024 --steps 20 --warmup 5
step 200 b2048x4096 python bench.py --nx 2048 --ny 4096 --steps 20 --warmup 5
HEAT_TB_VARIANT=23 step 200 b2048x4096_v23 python bench.py --nx 2048 --ny 4096 --steps 20 --warmup 5
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof -o run -- python3 $OLDPWD/bench.py --nx 1024 --steps 3 --warmup 1 > $OLDPWD/$O/prof.log 2>&1 || { tail -30 $OLDPWD/$O/prof.log; exit 1; }
cd $OLDPWD && find $O/prof -name "*kernel_stats*" | head -3
echo done
