#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 1; }
grep metric gpurun_out/bench.log
rm -rf gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof.log 2>&1) || { tail -20 gpurun_out/prof.log; exit 1; }
ARGS="--depth 8 --variant 7 --waves 0 --launches 6" bash tools/prof_counters.sh || exit 1
python tools/prof_summary.py --trace gpurun_out/prof --pmc gpurun_out/pmc --match "tb_kernel<8, 3>" --title "bench.py 8192^2 fp32, 1 MI355X, default TB kernel (depth 8, ring3+ramp, scalar)" --out gpurun_out/summary.md | head -40
