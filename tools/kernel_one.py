#!/usr/bin/env python3
"""A few launches of one stencil kernel on an n x n field (a profiling target).

    python tools/kernel_one.py --kernel mfma --n 8192 --launches 10
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parallel_heat_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", choices=["naive", "lds", "mfma", "tb"], default="tb")
ap.add_argument("--n", type=int, default=8192)
ap.add_argument("--launches", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda", 0)
g = ops.Geom(nx=a.n, ny=a.n)
x = ops.Field(a.n, a.n, 8, dev)
y = ops.Field(a.n, a.n, 8, dev)
ops.init_field(x, g, "random", 1)
ops.init_field(y, g, "random", 1)
step = {"naive": lambda s, d: ops.naive_step(s, d, g), "lds": lambda s, d: ops.lds_step(s, d, g),
        "mfma": lambda s, d: ops.mfma_step(s, d, g), "tb": lambda s, d: ops.tb_step(s, d, g, 8)}[a.kernel]
for _ in range(a.launches):
    step(x, y)
    x, y = y, x
torch.cuda.synchronize()
print("done")
