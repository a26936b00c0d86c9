#!/bin/bash
# Small per-rank blocks (8-GPU strong-scaling shapes): one wave per SIMD
# (the default) vs two per SIMD with age-weighted chunk pairs, and the
# level-split pipelines at one / two pipelines per SIMD.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3small
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  grep -v amdgpu.ids $O/$name.log | tail -14 | cut -c1-300; }
export HEAT_TB_TRACE=1
S="@23@0;1,1@279@2048;1.4,1@279@2048;1.7,1@279@2048;2.0,1@279@2048;2.4,1@279@2048;@2071@1024;1.7,1@2327@1024;1.7,1@2327@2048;@2071@0"
step 300 s1024k12 python tools/age_sweep.py --n 8192 --nx 1024 --interior --depth 12 --iters 480 --rounds 5 --sets "$S"
step 300 s2048x4096k12 python tools/age_sweep.py --n 4096 --nx 2048 --interior --depth 12 --iters 480 --rounds 5 --sets "$S"
S8="@23@0;1,1@279@2048;1.4,1@279@2048;1.7,1@279@2048;2.0,1@279@2048;@2071@1024;1.7,1@2327@1024;1.7,1@2327@2048"
step 300 s1024k8 python tools/age_sweep.py --n 8192 --nx 1024 --interior --depth 8 --iters 480 --rounds 5 --sets "$S8"
echo done
