#!/bin/bash
# Round 5, session o: counters of the 8192^2 solver with streaming rows
# (default, nt 1) and with plain rows (HEAT_TB_NT=0): HBM bytes, L2 hits,
# issue / wait shares, each pass its own rocprofv3 run (kernel trace +
# counters only), then a kernel-stats trace of the default bench.
set -o pipefail
cd "$(dirname "$0")/.."
export PROG=bench.py ARGS="--steps 2 --warmup 1 --no-verify"
OUT=pmc_r5o_nt bash tools/prof_counters.sh || exit 1
HEAT_TB_NT=0 OUT=pmc_r5o_plain bash tools/prof_counters.sh || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_r5o -o t -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/trace_r5o.log 2>&1 || exit 1
echo done
