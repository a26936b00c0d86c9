bash tools/gpu_run.sh r5a \
 "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "gated|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_converge_gated.py tests/test_gpu_resident.py" \
 "bench|180|python bench.py --steps 20 --warmup 5" \
 "giveup2|400|HEAT_RCCL_HOST_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 HEAT_TB_RESIDENT=2 HEAT_TEST_RES_GIVEUP_RANK=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --nx 2048 --ny 2048 --steps 5 --warmup 2 --verbose" \
 "rcclmr|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl_multirank.py" \
 "plan184k|60|build/heat --nx 184000 --ny 184000 --plan" \
 "big184k_tb|400|build/heat --nx 184000 --ny 184000 --steps 100 --init random --seed 7 --out-format checksum --out gpurun_out/r5a/big184k_tb.json --json" \
 "big184k_lds|600|build/heat --nx 184000 --ny 184000 --steps 100 --init random --seed 7 --kernel lds --out-format checksum --out gpurun_out/r5a/big184k_lds.json --json" \
 "cfg34ab|900|python tools/cfg34_ab.py . abprev/r3 --rounds 2"
