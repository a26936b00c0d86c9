#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
DEPTHS=8,10,12,16 VARIANTS=0,2,4,6 WAVES=-1,-2 bash tools/gpu_sweep.sh
