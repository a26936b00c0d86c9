#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3age
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name: $*";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -12 $O/$name.log; }
step 300 a8192 python tools/age_sweep.py --n 8192 --sets ";2,1.95,1.15,1;1.8,1.8,1.2,1;1.6,1.6,1.25,1;2.2,2.1,1.2,1;1.7,1;1.9,1;1.5,1" --rounds 7
step 300 a2048 python tools/age_sweep.py --n 8192 --nx 2048 --interior --sets ";2,1.95,1.15,1;1.8,1.8,1.2,1;1.6,1.6,1.25,1;1.7,1" --rounds 5
step 300 a16384 python tools/age_sweep.py --n 131072 --nx 16384 --interior --iters 240 --sets ";2,1.95,1.15,1;1.7,1;1,1" --rounds 3
echo done
