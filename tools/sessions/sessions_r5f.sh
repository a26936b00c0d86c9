#!/bin/bash
# Round 5, session f: enqueued (async) bench steps, 1024-step gated segments,
# 64 checks per resident span; RCCL rehearsals of the bench path.
B="python bench.py --steps 20 --warmup 5"
export HEAT_RCCL_HOST_PER_RANK_UNUSED=0
steps=(
 "tests|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_solver.py tests/test_gpu_resident.py tests/test_gpu_converge_gated.py tests/test_gpu_rccl_multirank.py"
 "bench|180|$B"
 "bench2|180|$B"
 "b1024|120|$B --nx 1024 --ny 8192"
 "b1024_ref_c20|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "b1024_ref_c50|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 50"
 "b2048|120|$B --nx 2048 --ny 4096"
 "b2048x8192|120|$B --nx 2048 --ny 8192"
 "b4096|120|$B --nx 4096 --ny 4096"
 "b4096x8192|120|$B --nx 4096 --ny 8192"
 "b8192_ref_c20|120|$B --init ref-wrap --converge --check-interval 20"
 "b8192_ref_c50|120|$B --init ref-wrap --converge --check-interval 50"
 "rehearse|600|bash tools/rccl_rehearsal.sh '2 4' --steps 5 --warmup 2"
)
exec bash tools/gpu_run.sh r5f "${steps[@]}"
