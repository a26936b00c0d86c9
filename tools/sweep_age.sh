#!/bin/bash
# Age-pair ratio sweep (older:younger rows of a chunk pair at 2 waves/SIMD)
# over the per-rank slab shapes that run two waves per SIMD, plus the wave
# timeline of each shape at the default ratio.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/sweep_age.jsonl
: > $OUT
for ratio in ${RATIOS:-1.0 1.5 2.0 2.5 3.0}; do
  for spec in "8192 12" "4096 12" "2048 8"; do
    set -- $spec
    if [[ $1 == 8192 ]]; then plate=""; else plate="--plate-nx 8192 --gx0 $(( (8192 - $1) / 2 ))"; fi
    HEAT_TB_AGE_RATIO=$ratio timeout -k 10 120 python tools/tb_sweep.py --nx $1 --n 8192 $plate --depths $2 \
        --variants 23 --waves 0 --iters 480 --rounds 5 2>>gpurun_out/sweep_age.err | \
        python3 -c "import sys,json; [print(json.dumps({**json.loads(l), 'age_ratio': $ratio})) for l in sys.stdin]" >> $OUT || exit 1
  done
done
cat $OUT
