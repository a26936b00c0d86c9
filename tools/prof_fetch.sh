#!/bin/bash
# FETCH_SIZE / L2 hit of the TB kernel for a list of variants (one rocprofv3
# counter run per variant and counter group).  Output: gpurun_out/fetch/
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
mkdir -p gpurun_out/fetch
export TMPDIR=/tmp
cd /tmp
for v in ${VARIANTS:-7 23}; do
  j=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    j=$((j+1))
    timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/gpurun_out/fetch/v${v}_$j -o p -- python3 $R/tools/tb_one.py --depth 8 --variant $v --waves 0 --launches 6 > $R/gpurun_out/fetch/v${v}_$j.log 2>&1 || { tail -20 $R/gpurun_out/fetch/v${v}_$j.log; exit 1; }
  done
done
echo done
