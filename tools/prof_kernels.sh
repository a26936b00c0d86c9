#!/bin/bash
# Counter passes (kernel-trace + --pmc only) for each stencil kernel family.
# Output: gpurun_out/kprof/<kernel>_<pass>/
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/kprof
export TMPDIR=/tmp
cd /tmp
for k in ${KERNELS:-tb lds mfma naive}; do
  j=0
  for ctr in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    j=$((j+1))
    timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/kprof/${k}_$j -o p -- python3 $R/tools/kernel_one.py --kernel $k --launches 6 > $R/gpurun_out/kprof/${k}_$j.log 2>&1 || { echo "pass $k/$j failed"; tail -20 $R/gpurun_out/kprof/${k}_$j.log; exit 1; }
  done
done
echo done
