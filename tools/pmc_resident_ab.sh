#!/bin/bash
# Counter passes of the resident tiles on the 8-GPU rank plate (1024 x 8192,
# bench.py's whole solver) for the default and an alternative: another
# engine build (LIB2, a path: round 6's per-wave readiness build) or an
# environment setting (VAR=value, e.g. HEAT_TB_TILE_XL=2: round 5's lane
# shifts).  Each pass is its own rocprofv3 run (kernel trace + counters only).
#   bash tools/pmc_resident_ab.sh build/ab/libheat_perwave.so [OUTDIR]
#   bash tools/pmc_resident_ab.sh HEAT_TB_TILE_XL=2 pmc_xl
# Output: gpurun_out/<OUTDIR, default pmc_res>/{default,alt}/p<pass>/...csv
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
ALT=${1:?usage: pmc_resident_ab.sh LIB2|VAR=value [OUTDIR]}
export TMPDIR=/tmp
OUT=$R/gpurun_out/${2:-pmc_res}
mkdir -p "$OUT"
cd /tmp
for lib in default alt; do
  unset HEAT_LIB
  if [[ $lib == alt && $ALT == *=* ]]; then export "${ALT?}"
  elif [[ $lib == alt ]]; then export HEAT_LIB=$R/$ALT; fi
  i=0
  while read -r line; do
    [[ -z $line ]] && continue
    i=$((i+1))
    d=$OUT/$lib/p$i
    mkdir -p "$d"
    timeout -k 10 240 rocprofv3 --pmc $line --kernel-trace --output-format csv -d "$d" -o p$i -- \
      python3 $R/bench.py --nx 1024 --steps 2 --warmup 1 --no-verify > "$d.log" 2>&1 \
      || { echo "$lib pass $i failed"; tail -20 "$d.log"; exit 1; }
  done <<'PASSES'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_INSTS_SALU GRBM_COUNT
PASSES
done
echo "pmc passes done"
