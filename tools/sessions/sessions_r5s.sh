#!/bin/bash
# Round 5, session s: odd chunks streamed bottom-up (variant bit 32,
# kAltDirection: the 2K rows two adjacent chunks both read come at the same
# time, from L2) with the streaming rows, against the default, 8192^2.
B="python bench.py --steps 20 --warmup 5"
steps=()
for r in 1 2 3; do
  steps+=("bench|120|$B" "alt|120|HEAT_TB_VARIANT=2103 $B")
done
exec bash tools/gpu_run.sh r5s "${steps[@]}"
