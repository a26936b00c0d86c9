#!/bin/bash
# bench.py (1 GPU, the headline config) against two engine builds (HEAT_LIB),
# alternated ROUNDS times.  Usage: tools/gpu_bench_ab.sh BASE.so NEW.so [tag] [rounds]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
A=$1; B=$2; TAG=${3:-benchab}; ROUNDS=${4:-3}
: > gpurun_out/${TAG}.jsonl
for r in $(seq "$ROUNDS"); do
  for lib in "$A" "$B"; do
    HEAT_LIB=$lib timeout -k 10 150 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_last.txt 2>&1 || exit 1
    tail -1 gpurun_out/${TAG}_last.txt | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(json.dumps({'lib': '$lib', 'value': d['value'], 'ms': d['ms_per_step']}))" >> gpurun_out/${TAG}.jsonl || exit 1
  done
done
cat gpurun_out/${TAG}.jsonl
