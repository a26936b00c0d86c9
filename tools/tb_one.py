#!/usr/bin/env python3
"""Run a few TB kernel launches of one configuration (a profiling target)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parallel_heat_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8192)
ap.add_argument("--depth", type=int, default=8)
ap.add_argument("--variant", type=int, default=2)
ap.add_argument("--waves", type=int, default=0)
ap.add_argument("--launches", type=int, default=10)
ap.add_argument("--nx", type=int, default=0, help="rows (default --n)")
ap.add_argument("--interior", action="store_true",
                help="the block sits inside a larger plate (a middle rank's block)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
nx = a.nx or a.n
g = ops.Geom(nx=nx, ny=a.n) if not a.interior else ops.Geom(nx=4 * nx, ny=4 * a.n, gx0=nx, gy0=a.n)
x = ops.Field(nx, a.n, a.depth, dev)
y = ops.Field(nx, a.n, a.depth, dev)
ops.init_field(x, g, "random", 1)
ops.init_field(y, g, "random", 1)
for i in range(a.launches):
    ops.tb_step(x, y, g, a.depth, waves_target=a.waves, variant=a.variant)
    x, y = y, x
torch.cuda.synchronize()
print("done")
