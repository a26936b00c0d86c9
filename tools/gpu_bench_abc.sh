#!/bin/bash
# bench.py (1 GPU) over several "LIB[:VAR=value]" configurations, alternated
# ROUNDS times (HEAT_LIB selects the engine build, the optional VAR=value is
# put in the environment).  Usage: tools/gpu_bench_abc.sh TAG ROUNDS CONF...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=$1; ROUNDS=$2; shift 2
: > gpurun_out/${TAG}.jsonl
for r in $(seq "$ROUNDS"); do
  for conf in "$@"; do
    lib=${conf%%:*}; setting=""
    [[ $conf == *:* ]] && setting=${conf#*:}
    env HEAT_LIB=$lib $setting timeout -k 10 150 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_last.txt 2>&1 || exit 1
    tail -1 gpurun_out/${TAG}_last.txt | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(json.dumps({'conf': '$conf', 'value': d['value'], 'ms': d['ms_per_step'], 'verified': d['verified']}))" >> gpurun_out/${TAG}.jsonl || exit 1
  done
done
cat gpurun_out/${TAG}.jsonl
