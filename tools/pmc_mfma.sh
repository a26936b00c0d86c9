#!/bin/bash
# Counters of the single-step kernel families at 8192^2 (the MFMA kernel with
# LDS-staged operands vs the LDS-tiled VALU kernel and the naive one): MFMA
# busy, LDS bank conflicts, VALU, HBM bytes.  One rocprofv3 run per pass,
# kernel trace + counters only.  Output: gpurun_out/pmc_mfma/<kernel>_p<i>/
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/pmc_mfma
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
PASSES=(
"SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
"FETCH_SIZE"
"WRITE_SIZE"
)
for k in ${KERNELS:-mfma lds naive}; do
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $p --kernel-trace --output-format csv -d $O/${k}_p$i -o p -- python3 $R/tools/kernel_one.py --kernel $k --n 8192 --launches 6 > $O/${k}_p$i.log 2>&1 || { echo "pass $k $i failed"; tail -20 $O/${k}_p$i.log; exit 1; }
  done
done
echo "pmc mfma done"
