#!/bin/bash
# One gpurun session as a list of steps, each under its own time limit.
#
#   tools/gpu_run.sh TAG "NAME|SECONDS|COMMAND" ["NAME|SECONDS|COMMAND" ...]
#
# Every step runs `bash -c COMMAND` from the repo root under
# `timeout -k 10 SECONDS`, with stdout+stderr in gpurun_out/TAG/NAME.log; the
# last line of each log is echoed (a JSON result line for bench.py).  The
# session stops at the first failing step (no retries: a GPU fault, abort,
# segfault or time limit ends the call, SURVEY §5 / gpurun rules).  A NAME
# that repeats gets a numeric suffix, so interleaved A/B rounds keep every log.
#
# Examples (see tools/README.md for the sessions of each round):
#   gpurun --timeout 900 -- bash tools/gpu_run.sh r4ab \
#     "r2|200|cd abprev/r2 && python bench.py --steps 20 --warmup 5" \
#     "r3|200|cd abprev/r3 && python bench.py --steps 20 --warmup 5"
#   gpurun -- bash tools/gpu_run.sh r4t "tests|900|python -u -m pytest tests -m gpu -x -q \
#     --timeout 120 --timeout-method thread"
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:?usage: gpu_run.sh TAG "NAME|SECONDS|COMMAND" ...}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
declare -A seen
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  n=${seen[$name]:-0}
  seen[$name]=$((n + 1))
  log=$O/$name.log
  [[ $n -gt 0 ]] && log=$O/${name}_$n.log
  echo "== $name ($secs s): $cmd"
  start=$(date +%s%N)
  timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  end=$(date +%s%N)
  echo "   rc=$rc  $(( (end - start) / 1000000 )) ms"
  if [[ $rc -ne 0 ]]; then
    echo "FAILED $name (rc $rc)"
    tail -40 "$log"
    exit 1
  fi
  tail -1 "$log" | cut -c1-400
done
echo "all steps done"
