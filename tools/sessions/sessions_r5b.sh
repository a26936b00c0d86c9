#!/bin/bash
# Round 5, session b: resident checks at inner even levels (depth 12 kept),
# the resident depth sweep on the 8-GPU rank plates, regression bench.
B="python bench.py --steps 20 --warmup 5"
steps=(
 "tests|900|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_converge_gated.py tests/test_gpu_tile.py"
 "bench|180|$B"
 "b1024_ref|120|$B --nx 1024 --ny 8192 --init ref-wrap"
 "b1024_ref_c20|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 20"
 "b1024_ref_c50|120|$B --nx 1024 --ny 8192 --init ref-wrap --converge --check-interval 50"
 "b2048_ref_c20|120|$B --nx 2048 --ny 4096 --init ref-wrap --converge --check-interval 20"
 "b8192_ref_c20|120|$B --init ref-wrap --converge --check-interval 20"
)
for d in 8 10 12 16; do
  steps+=("d${d}_1024|120|HEAT_TB_DEPTH=$d $B --nx 1024 --ny 8192")
  steps+=("d${d}_2048|120|HEAT_TB_DEPTH=$d $B --nx 2048 --ny 4096")
done
steps+=("b1024_ref_again|120|$B --nx 1024 --ny 8192 --init ref-wrap")
exec bash tools/gpu_run.sh r5b "${steps[@]}"
