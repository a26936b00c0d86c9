#!/bin/bash
# Round 5, session ac: the 288 GB sizing with the final round-5 build
# (streaming rows): 184000^2 (271 GB of device memory), 100 steps -- hash
# against the committed LDS-kernel run (cbf95a893f5f2ea6,
# profiles/r5_raw/big184k_lds.json) -- and 1000 steps timed.
steps=(
 "big184k_tb|400|build/heat --nx 184000 --ny 184000 --steps 100 --init random --seed 7 --out-format checksum --out gpurun_out/r5ac/big184k_tb.json --json"
 "big184k_1000|400|build/heat --nx 184000 --ny 184000 --steps 1000 --init random --seed 7 --out-format checksum --out gpurun_out/r5ac/big184k_1000.json --json"
)
exec bash tools/gpu_run.sh r5ac "${steps[@]}"
