#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit 1
echo "== rccl same-device probe"
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1
echo "probe rc=$?"; grep -E "OK|ok|FAILED|rror" gpurun_out/rccl_probe.log | head -20
echo "== bench"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 && cat gpurun_out/bench.log | grep metric
