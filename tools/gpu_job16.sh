#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python tools/tb_sweep.py --n 8192 --depths 1,2,4,8 --variants 7 --waves=-1,-2,-4 > gpurun_out/s.log 2>&1 || exit 1
cat gpurun_out/s.log | cut -c1-150
python - <<'PY'
import torch, time
x = torch.empty(8192*8512, device='cuda'); y = torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); t=time.perf_counter()
for _ in range(50): y.copy_(x)
torch.cuda.synchronize(); dt=(time.perf_counter()-t)/50
print("torch copy 279MB: %.2f TB/s" % (2*x.numel()*4/dt/1e12))
PY
