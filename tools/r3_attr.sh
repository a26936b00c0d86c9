#!/bin/bash
# Small-block attribution: one launch's wave timeline vs the wall time per
# pass of back-to-back launches (gap), plus the plan's row/column redundancy.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3attr
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -3 $O/$name.log | cut -c1-600; }
step 120 tl8192 python tools/wave_timeline.py --nx 8192 --ny 8192 --depth 12
step 120 tl1024 python tools/wave_timeline.py --nx 1024 --ny 8192 --depth 12 --interior
step 120 tl1024w2 python tools/wave_timeline.py --nx 1024 --ny 8192 --depth 12 --interior --waves 2048
step 120 tl1024k8 python tools/wave_timeline.py --nx 1024 --ny 8192 --depth 8 --interior
step 120 tl2048x4096 python tools/wave_timeline.py --nx 2048 --ny 4096 --depth 12 --interior
step 120 tl2048x8192 python tools/wave_timeline.py --nx 2048 --ny 8192 --depth 12 --interior
echo done
