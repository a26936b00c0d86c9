#!/bin/bash
# Plate-edge ranks of 2- and 4-GPU runs as one-GPU plates: default variant
# choice vs the tile kernel forced (HEAT_TB_VARIANT=131088) vs one wave per
# chunk (23), whole bench.py solver.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3edges
mkdir -p $O
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; echo "== $name";
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; tail -40 $O/$name.log; exit 1; }
  tail -1 $O/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['verified'])"; }
for shp in "2048 8192" "4096 4096" "4096 8192" "1536 8192"; do set -- $shp
  step 200 b${1}x${2} python bench.py --nx $1 --ny $2 --steps 10 --warmup 3
  HEAT_TB_VARIANT=131088 step 200 b${1}x${2}_tile python bench.py --nx $1 --ny $2 --steps 10 --warmup 3
  HEAT_TB_VARIANT=23 step 200 b${1}x${2}_v23 python bench.py --nx $1 --ny $2 --steps 10 --warmup 3
done
echo done
