#!/bin/bash
# Quick kernel A/B on one GPU: tb_sweep at the 1- and 8-GPU per-rank shapes.
# Usage: tools/gpu_ab.sh "VARIANTS_8192" "VARIANTS_SMALL" [tag]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V1=${1:-2071}; V2=${2:-23}; TAG=${3:-ab}
timeout -k 10 200 python tools/tb_sweep.py --nx 8192 --n 8192 --depths 12 --variants $V1 --waves 0 --rounds 7 --iters 240 > gpurun_out/${TAG}_8192.txt 2>&1 || exit 1
timeout -k 10 200 python tools/tb_sweep.py --nx 1024 --n 8192 --interior --depths 8 --variants $V2 --waves 0 --rounds 5 --iters 240 > gpurun_out/${TAG}_1024.txt 2>&1 || exit 1
grep -h gcells gpurun_out/${TAG}_*.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['nx'], d['variant'], d['depth'], d['waves'], d['gcells_s'], d['min'], d['max'])"
