#!/bin/bash
# A/B of TB kernel variants at the per-rank slab shapes (VARIANTS, depth by shape).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/sweep_variants.jsonl
: > $OUT
for spec in ${SHAPES:-"8192:12" "4096:12" "2048:8" "1024:8"}; do
  nx=${spec%%:*}; d=${spec##*:}
  if [[ $nx == 8192 ]]; then plate=""; else plate="--plate-nx 8192 --gx0 $(( (8192 - nx) / 2 ))"; fi
  timeout -k 10 200 python tools/tb_sweep.py --nx $nx --n 8192 $plate --depths $d \
      --variants ${VARIANTS:-23,535,1047,1559} --waves 0 --iters 480 --rounds 5 >> $OUT 2>>gpurun_out/sweep_variants.err || exit 1
done
cat $OUT
