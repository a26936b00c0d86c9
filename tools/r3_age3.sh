#!/bin/bash
# Planner trace per shape, then age weights of the linear plans:
# 2-part ratios vs 4-part sets at the 1-D 8-GPU rank shape and at 131072^2.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3age3
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep -v amdgpu.ids $O/$name.log | tail -14 | cut -c1-300; }
export HEAT_TB_TRACE=1
step 300 a16384 python tools/age_sweep.py --n 131072 --nx 16384 --interior --iters 240 --rounds 3 \
  --sets ";2.0,1.95,1.15,1;2.2,2.1,1.2,1;2.4,2.2,1.3,1;2.6,2.4,1.3,1;2.0,1;2.3,1;2.6,1;1.7,1"
step 300 a8192 python tools/age_sweep.py --n 8192 --iters 480 --rounds 5 --sets ";2.2,2.1,1.2,1;2.0,1"
step 400 a131072 python tools/age_sweep.py --n 131072 --iters 120 --rounds 3 --sets ";2.0,1;2.3,1;1.5,1;2.0,1.95,1.15,1"
echo done
