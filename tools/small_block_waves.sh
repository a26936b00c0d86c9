#!/bin/bash
# Waves sweep of the two depth-12 kernels on the 8-GPU per-rank blocks.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/small_waves.jsonl
for shape in "--nx 1024 --n 8192 --interior" "--nx 2048 --n 4096 --interior"; do
  timeout -k 10 200 python tools/tb_sweep.py $shape --depths 12 --variants 23,2071 \
    --waves 512,768,1024,1280,1536,2048 --rounds 5 --iters 480 >> gpurun_out/small_waves.jsonl 2>> gpurun_out/small_waves.err || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/small_waves.jsonl'):
    if 'gcells' in l:
        d = json.loads(l); print(d['nx'], d['variant'], d['depth'], d['waves'], d['gcells_s'])"
