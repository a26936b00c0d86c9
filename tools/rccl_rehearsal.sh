#!/bin/bash
# Multi-rank RCCL rehearsal on ONE GPU: bench.py as N torchrun ranks that all
# use device 0.  Each rank claims its own RCCL host id (HEAT_RCCL_HOST_PER_RANK,
# see bench.py), so RCCL's duplicate-GPU check passes and the ranks exchange
# over the socket transport on loopback.  Everything else is the multi-GPU
# bench path: torch's nccl process group, the autotune, the engine's own RCCL
# communicator, grouped ncclSend/ncclRecv and ncclAllReduce captured in the
# segment hipGraphs, and the checksum verification against a 1-rank run.
# Throughput is NOT an N-GPU number (N ranks share one GPU and talk over TCP).
#   tools/rccl_rehearsal.sh "2 4" [extra bench.py args]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
NS=${1:-"2 4"}
shift || true
export HEAT_RCCL_HOST_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
port=29610
for n in $NS; do
  port=$((port + 7))
  echo "== $n ranks"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus "$n" --verbose "$@" \
      > gpurun_out/rccl_rehearsal_n$n.json 2> gpurun_out/rccl_rehearsal_n$n.err
  rc=$?
  cat gpurun_out/rccl_rehearsal_n$n.json
  tail -5 gpurun_out/rccl_rehearsal_n$n.err
  [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
done
