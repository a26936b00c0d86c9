#!/bin/bash
# Counter passes for the workgroup-tile kernel vs one wave per chunk at the
# 8-GPU per-rank block (1024 x 8192 inside a larger plate, depth 12), each
# pass its own rocprofv3 run (tools/prof_counters.sh), then a markdown summary.
set -o pipefail
cd "$(dirname "$0")/.."
for cfg in "131088 tile_kernel" "23 tb_kernel"; do set -- $cfg; v=$1
  ARGS="--n 8192 --nx 1024 --interior --depth 12 --variant $v --waves 0 --launches 8" bash tools/prof_counters.sh || exit 1
  rm -rf gpurun_out/pmc_tile_$v && mv gpurun_out/pmc gpurun_out/pmc_tile_$v
  python3 tools/prof_summary.py --pmc gpurun_out/pmc_tile_$v --match $2 --out gpurun_out/pmc_tile_$v.md || exit 1
done
echo done
