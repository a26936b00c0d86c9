#!/bin/bash
# Over-subscribed plans, continued: blocks with plate edges, 16384^2, the
# 4-GPU 1-D rank, 131072^2 with short edge sub-boxes.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3over2
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep -v amdgpu.ids $O/$name.log | grep -v '^\[heat' | tail -20 | cut -c1-200; }
export HEAT_TB_TRACE=1
step 400 e16384 python tools/age_sweep.py --n 131072 --nx 16384 --iters 240 --rounds 3 --sets "@-1@0;@67607@8192;@67607@8192@0.05;@34839@8192;@34839@4096;@67607@8192@0.01"
step 300 p16384 python tools/age_sweep.py --n 16384 --iters 480 --rounds 5 --sets "@-1@0;@67607@4096;@67607@8192;@67607@4096@0.1;@34839@4096;@34839@8192"
step 400 i32768 python tools/age_sweep.py --n 131072 --nx 32768 --interior --iters 120 --rounds 3 --sets "@-1@0;@67607@4096;@67607@8192;@67607@16384;@34839@8192"
step 500 b131072 python tools/age_sweep.py --n 131072 --iters 120 --rounds 2 --sets "@-1@0;@34839@8192;@34839@16384;@67607@8192@0.02;@67607@16384@0.02"
echo done
