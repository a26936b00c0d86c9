#!/bin/bash
# bench.py (1 GPU) with and without one environment setting, alternated.
# Usage: tools/gpu_bench_env_ab.sh "VAR=value [VAR2=value]" [rounds]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
SETTING=$1; ROUNDS=${2:-3}
for r in $(seq "$ROUNDS"); do
  for mode in base env; do
    if [[ $mode == env ]]; then
      env $SETTING timeout -k 10 150 python bench.py --steps 10 --warmup 3 > gpurun_out/envab_last.txt 2>&1 || exit 1
    else
      timeout -k 10 150 python bench.py --steps 10 --warmup 3 > gpurun_out/envab_last.txt 2>&1 || exit 1
    fi
    echo "$mode $(tail -1 gpurun_out/envab_last.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["verified"])')"
  done
done
