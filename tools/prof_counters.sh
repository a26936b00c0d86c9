#!/bin/bash
# Hardware-counter passes for the TB kernel (each pass its own rocprofv3 run,
# kernel-trace + counters only).  Output: gpurun_out/pmc/<pass>/...csv
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
ARGS=${ARGS:-"--depth 8 --variant -1 --waves 0 --launches 6"}
# PROG: the Python program profiled (default tools/tb_one.py with ARGS), e.g.
# PROG="bench.py" ARGS="--nx 1024 --steps 2 --warmup 1 --no-verify" (the whole
# solver: resident tile launches).  OUT: output directory under gpurun_out.
PROG=${PROG:-tools/tb_one.py}
OUT=${OUT:-pmc}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
cd /tmp
i=0
while read -r line; do
  [[ -z $line ]] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $R/gpurun_out/$OUT/p$i -o p$i -- python3 $R/$PROG $ARGS > $R/gpurun_out/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $R/gpurun_out/$OUT/p$i.log; exit 1; }
done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INST_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_COUNT
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD
PASSES
echo "pmc passes done: $i"
