#!/bin/bash
# Build A/B on one GPU: the same kernel sweeps against two engine builds
# (HEAT_LIB), alternated twice to cancel drift.
# Usage: tools/gpu_lib_ab.sh BASE.so NEW.so [tag]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
A=$1; B=$2; TAG=${3:-libab}
: > gpurun_out/${TAG}.txt
for round in 1 2; do
  for lib in "$A" "$B"; do
    for shape in "--nx 8192 --n 8192" "--nx 1024 --n 8192 --interior" "--nx 2048 --n 4096 --interior"; do
      echo "# $lib $shape" >> gpurun_out/${TAG}.txt
      HEAT_LIB=$lib timeout -k 10 120 python tools/tb_sweep.py $shape --depths 12 --variants -1 \
        --waves 0 --rounds 5 --iters 240 >> gpurun_out/${TAG}.txt 2>&1 || exit 1
    done
  done
done
python3 - gpurun_out/${TAG}.txt <<'PY'
import json, sys
lib = None
for l in open(sys.argv[1]):
    if l.startswith("# "):
        lib = l.split()[1]
    elif "gcells" in l:
        d = json.loads(l)
        print(lib.split("/")[-1], d["nx"], d["variant"], d["depth"], d["gcells_s"], d["min"], d["max"])
PY
