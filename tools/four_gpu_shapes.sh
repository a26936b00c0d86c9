#!/bin/bash
# The 4-GPU per-rank blocks (2048 x 8192 slab, 4096 x 4096 2-D) at depth 12:
# single-wave vs split pipelines, waves auto / whole rounds.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/four_gpu_shapes.jsonl
for shape in "--nx 2048 --n 8192 --interior" "--nx 4096 --n 4096 --interior"; do
  timeout -k 10 200 python tools/tb_sweep.py $shape --depths 12 --variants 23,2071 \
    --waves 0,1024,2048,4096 --rounds 5 --iters 480 >> gpurun_out/four_gpu_shapes.jsonl 2>> gpurun_out/four_gpu_shapes.err || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/four_gpu_shapes.jsonl'):
    if 'gcells' in l:
        d = json.loads(l); print(d['nx'], d['variant'], d['depth'], d['waves'], d['gcells_s'])"
