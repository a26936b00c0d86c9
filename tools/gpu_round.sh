#!/bin/bash
# One GPU-box session: tests, bench, kernel profile.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
run() { echo "== $*" ; "$@"; }
if [[ $STAGE == all || $STAGE == test ]]; then
  run timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
  tail -5 gpurun_out/pytest_gpu.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  run timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verbose > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
  cat gpurun_out/bench.log
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  cd /tmp && run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/prof -o run -- python3 $OLDPWD/bench.py --steps 2 --warmup 1 > $OLDPWD/gpurun_out/prof.log 2>&1 || { tail -30 $OLDPWD/gpurun_out/prof.log; exit 1; }
  cd $OLDPWD
  find gpurun_out/prof -name "*stats*" | head
fi
