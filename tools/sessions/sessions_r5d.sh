#!/bin/bash
# Round 5, session d: deferred residual atomics in resident spans, the judge
# with the gate in registers.
B="python bench.py --steps 20 --warmup 5"
R=$PWD
P="rocprofv3 --kernel-trace --stats --output-format csv"
steps=(
 "tests|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_converge_gated.py"
 "b1024_ref|120|$B --nx 1024 --ny 8192 --init ref-wrap"
 "b1024_ref_c20|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "b1024_ref_c50|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 50"
 "b2048_ref|120|$B --nx 2048 --ny 4096 --init ref-wrap"
 "b2048_ref_c20|120|$B --nx 2048 --ny 4096 --init ref-wrap --converge --check-interval 20"
 "b8192_ref_c20|120|$B --init ref-wrap --converge --check-interval 20"
 "prof_c20|240|cd /tmp && $P -d $R/gpurun_out/r5d/prof_c20 -o p -- python3 $R/bench.py --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20 --steps 5 --warmup 2 --no-verify"
 "b1024_ref_c20b|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "b1024_refb|120|$B --nx 1024 --ny 8192 --init ref-wrap"
)
exec bash tools/gpu_run.sh r5d "${steps[@]}"
