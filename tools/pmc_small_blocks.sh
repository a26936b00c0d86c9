set -o pipefail
for cfg in "23 12 0" "23 12 2048" "87 8 2048"; do
  set -- $cfg
  ARGS="--n 8192 --nx 1024 --interior --depth $2 --variant $1 --waves $3 --launches 6" bash tools/prof_counters.sh > /dev/null || exit 1
  mkdir -p gpurun_out/pmc_$1_$2_$3 && mv gpurun_out/pmc/* gpurun_out/pmc_$1_$2_$3/
done
