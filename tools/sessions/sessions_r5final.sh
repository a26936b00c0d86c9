#!/bin/bash
# Round 5, final tree: smoke, every GPU test, the driver-style bench (twice),
# the checked-plate rows, the RCCL rehearsals (2 / 4 / 8 ranks on one GPU)
# and a kernel-stats trace of the bench.
B="python bench.py --steps 20 --warmup 5"
steps=(
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'"
 "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
 "bench|120|$B"
 "bench|120|$B"
 "ref|120|$B --init ref-wrap"
 "c20|120|$B --init ref-wrap --converge --check-interval 20"
 "c50|120|$B --init ref-wrap --converge --check-interval 50"
 "rehearsal|900|bash tools/rccl_rehearsal.sh '2 4 8'"
 "trace|240|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r5final/trace -o t -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2"
)
exec bash tools/gpu_run.sh r5final "${steps[@]}"
