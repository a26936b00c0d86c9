#!/bin/bash
# Round 5, session g: one kernel-argument load per pass for the resident
# check index; A/B of the gated segment length; a kernel-trace + roctx
# timeline of the 8-rank RCCL rehearsal (one rocprofv3 per rank).
B="python bench.py --steps 20 --warmup 5 --nx 1024 --ny 8192 --init ref-wrap"
R=$PWD
steps=(
 "tests|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_converge_gated.py"
 "u|120|$B"
 "c20_1024|120|$B --converge --check-interval 20"
 "c20_512|120|HEAT_SEG_STEPS=512 $B --converge --check-interval 20"
 "c50_1024|120|$B --converge --check-interval 50"
 "c50_512|120|HEAT_SEG_STEPS=512 $B --converge --check-interval 50"
 "u|120|$B"
 "c20_1024|120|$B --converge --check-interval 20"
 "c20_512|120|HEAT_SEG_STEPS=512 $B --converge --check-interval 20"
 "c50_1024|120|$B --converge --check-interval 50"
 "c50_512|120|HEAT_SEG_STEPS=512 $B --converge --check-interval 50"
 "probe|120|build/probes/stencil_chain"
 "diag_nostore|120|HEAT_TB_VARIANT=3095 python bench.py --steps 20 --warmup 5 --no-verify"
 "diag_nostore_cached|120|HEAT_TB_VARIANT=7167 python bench.py --steps 20 --warmup 5 --no-verify"
 "bench|120|python bench.py --steps 20 --warmup 5"
 "timeline8|600|HEAT_ROCTX=1 HEAT_RCCL_HOST_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29677 --no-python rocprofv3 --kernel-trace --marker-trace --output-format csv -d $R/gpurun_out/r5g/tl -o rank_%pid% -- python3 $R/bench.py --gpus 8 --steps 2 --warmup 1 --no-autotune --no-verify --verbose"
)
exec bash tools/gpu_run.sh r5g "${steps[@]}"
