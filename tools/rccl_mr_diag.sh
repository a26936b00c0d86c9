#!/bin/bash
# One-GPU multi-rank RCCL variants (tools/rccl_mr_diag.py), stopping at the
# first failure (a crash ends the GPU work of the call).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONFAULTHANDLER=1
r() { echo "== $*"; timeout -k 10 120 python -u tools/rccl_mr_diag.py "$@" > gpurun_out/diag.out 2>&1; rc=$?; grep -E "^(OK|MISMATCH)|Fatal|Error|error" gpurun_out/diag.out | grep -v "NCCL WARN" | head -5; return $rc; }
r 2 '{"decomp":"rows","schedule":"overlap"}' &&
r 2 '{"decomp":"rows","schedule":"pipeline"}' &&
r 2 '{"px":1,"py":2,"schedule":"overlap"}' &&
r 3 '{"decomp":"rows","schedule":"pipeline"}'
