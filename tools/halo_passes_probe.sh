#!/bin/bash
# Passes per halo exchange (deep-halo sync schedule) on one GPU: N loopback
# ranks (threads) share the device, so this measures the exchange's
# synchronisation cost against redundant ghost compute, not xGMI.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for g in ${GPUS:-2 4 8}; do for m in ${MS:-2 4 8 16}; do
  timeout -k 5 120 ./build/heat --gpus $g --nx 8192 --ny 8192 --steps 2000 --init random --decomp rows \
      --out none --json --halo-passes $m > gpurun_out/m_${g}_${m}.json 2>&1 || exit 1
  echo "{\"gpus\": $g, \"halo_passes\": $m, \"run\": $(tail -1 gpurun_out/m_${g}_${m}.json)}"
done; done
