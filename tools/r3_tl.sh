#!/bin/bash
# Per-wave timelines of the default kernel (how much of each launch the
# SIMDs sit idle): 8192^2 plate and the 8-GPU per-rank block.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3tl
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -3 $O/$name.log; }
step 120 tl8192 python tools/wave_timeline.py --nx 8192 --ny 8192 --depth 12
step 120 tl1024 python tools/wave_timeline.py --nx 1024 --ny 8192 --depth 12 --interior
step 120 tl2048 python tools/wave_timeline.py --nx 2048 --ny 8192 --depth 12 --interior
echo done
