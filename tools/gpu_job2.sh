#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_sweep.sh && bash tools/prof_counters.sh
