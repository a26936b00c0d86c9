#!/bin/bash
# Strong-scaling curve of the headline benchmark (8192^2, 1000-iteration steps)
# at 1/2/4/8 GPUs of one node, one rank per GPU over RCCL/xGMI.
#   bash bench/scaling.sh [STEPS] [WARMUP]    -> bench/results/scaling_<N>.json
set -o pipefail
cd "$(dirname "$0")/.."
STEPS=${1:-10}; WARMUP=${2:-2}
NG=$(python3 -c "import torch; print(torch.cuda.device_count())")
mkdir -p bench/results
for N in 1 2 4 8; do
  [ "$N" -gt "$NG" ] && break
  if [ "$N" = 1 ]; then
    timeout -k 10 900 python3 bench.py --steps $STEPS --warmup $WARMUP > bench/results/scaling_1.json || exit 1
  else
    timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N \
      --steps $STEPS --warmup $WARMUP > bench/results/scaling_$N.json || exit 1
  fi
  tail -1 bench/results/scaling_$N.json
done
