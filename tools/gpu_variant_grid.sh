#!/bin/bash
# Variant x depth grid at the 1-GPU and per-rank shapes (one process per shape).
# Usage: tools/gpu_variant_grid.sh "VARIANTS" "DEPTHS" [tag]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=${1:-2071,23}; D=${2:-8,12}; TAG=${3:-vgrid}
: > gpurun_out/${TAG}.jsonl
for shape in "--nx 8192 --n 8192" "--nx 1024 --n 8192 --interior" "--nx 2048 --n 4096 --interior" "--nx 4096 --n 8192 --interior"; do
  timeout -k 10 200 python tools/tb_sweep.py $shape --depths $D --variants $V --waves 0 \
    --rounds 5 --iters 480 >> gpurun_out/${TAG}.jsonl 2>> gpurun_out/${TAG}.err || exit 1
done
python3 - gpurun_out/${TAG}.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if "gcells" in l:
        d = json.loads(l)
        print(d["nx"], d.get("n", ""), d["variant"], d["depth"], d["gcells_s"], d["min"], d["max"])
PY
