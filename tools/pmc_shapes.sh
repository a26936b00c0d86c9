#!/bin/bash
# Translation / cache counters of the default TB kernel at three shapes: the
# 8192^2 plate, the 16384 x 131072 slab (1-D 8-GPU rank of 131072^2) and the
# whole 131072^2 plate on one GPU.  One rocprofv3 run per (shape, pass),
# kernel trace + counters only.  Output: gpurun_out/pmc_shapes/<shape>_p<i>/
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/pmc_shapes
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
PASSES=(
"TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
"TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES"
)
for shape in ${SHAPES:-"8192:8192" "16384:131072" "131072:131072"}; do
  nx=${shape%%:*}; ny=${shape##*:}
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $p --kernel-trace --output-format csv -d $O/${nx}x${ny}_p$i -o p -- python3 $R/tools/tb_one.py --nx $nx --n $ny --depth 12 --variant -1 --launches 4 --interior > $O/${nx}x${ny}_p$i.log 2>&1 || { echo "pass $shape $i failed"; tail -20 $O/${nx}x${ny}_p$i.log; exit 1; }
  done
done
echo "pmc shapes done"
