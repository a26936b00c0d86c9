#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
rm -rf gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof.log 2>&1) || { tail -20 gpurun_out/prof.log; exit 1; }
bash tools/prof_counters.sh || exit 1
python tools/prof_summary.py --trace gpurun_out/prof --pmc gpurun_out/pmc --match "tb_kernel<8, 3>" --title "bench.py 8192^2 fp32, 1 MI355X, default TB kernel (K=8, ring3+ramp, scalar build, edge modes)" --out gpurun_out/summary.md
