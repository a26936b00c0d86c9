#!/bin/bash
# Over-subscribed plans: more work units than resident pipelines, so the
# dispatcher back-fills SIMDs that finish early (classic = 67607, linear =
# 34839, age-paired classic = 67863), against the default planner.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3over
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep -v amdgpu.ids $O/$name.log | grep -v '^\[heat' | tail -20 | cut -c1-200; }
export HEAT_TB_TRACE=1
S="@-1@0;2.6,2.4,1.3,1@-1@0;@67607@2048;@67607@3072;@67607@4096;@67607@6144;@67607@8192;@34839@2048;@34839@4096;@34839@8192;1.7,1@67863@4096;1.7,1@67863@8192"
step 400 o16384 python tools/age_sweep.py --n 131072 --nx 16384 --interior --iters 240 --rounds 3 --sets "$S"
step 300 o8192 python tools/age_sweep.py --n 8192 --iters 480 --rounds 5 --sets "@-1@0;@67607@3072;@67607@4096;1.7,1@67863@4096;@34839@4096"
step 500 o131072 python tools/age_sweep.py --n 131072 --iters 120 --rounds 2 --sets "@-1@0;@67607@4096;@67607@8192;@34839@4096;@34839@8192;1.7,1@67863@8192"
echo done
