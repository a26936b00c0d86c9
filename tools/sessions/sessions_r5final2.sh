#!/bin/bash
# Round 5, final tree (second pass, after the streaming inner-level residual
# units): smoke, every GPU test, the bench twice, the checked rows.
B="python bench.py --steps 20 --warmup 5"
steps=(
 "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'"
 "tests|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
 "bench|120|$B"
 "bench|120|$B"
 "ref|120|$B --init ref-wrap"
 "c20|120|$B --init ref-wrap --converge --check-interval 20"
 "c50|120|$B --init ref-wrap --converge --check-interval 50"
)
exec bash tools/gpu_run.sh r5final2 "${steps[@]}"
