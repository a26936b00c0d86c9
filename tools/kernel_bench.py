#!/usr/bin/env python3
"""Time the single-step kernels (naive, lds[fp32|mpi]) against the TB kernel
on one GPU: Gcells/s of cell-updates, median of rounds.

    python tools/kernel_bench.py --n 8192 --steps 40
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parallel_heat_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = ops.Geom(nx=a.n, ny=a.n)
    x = ops.Field(a.n, a.n, 8, dev)
    y = ops.Field(a.n, a.n, 8, dev)
    ops.init_field(x, g, "random", 1)
    ops.init_field(y, g, "random", 1)
    kinds = {
        "naive": lambda s, d: ops.naive_step(s, d, g),
        "lds_fp32": lambda s, d: ops.lds_step(s, d, g),
        "lds_mpi": lambda s, d: ops.lds_step(s, d, g, numerics="mpi"),
        "mfma": lambda s, d: ops.mfma_step(s, d, g),
        "tb8": None,
    }
    res = {k: [] for k in kinds}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds + 1):
        for k, f in kinds.items():
            s, d = x, y
            e0.record()
            if f is None:
                for _ in range(a.steps // 8):
                    ops.tb_step(s, d, g, 8)
                    s, d = d, s
            else:
                for _ in range(a.steps):
                    f(s, d)
                    s, d = d, s
            e1.record()
            e1.synchronize()
            res[k].append(a.n * a.n * a.steps / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    for k, v in res.items():
        v = v[1:]  # first round = warm-up
        print(json.dumps({"kernel": k, "n": a.n, "gcells_s": round(statistics.median(v), 1),
                          "hbm_tb_s_equiv": round(statistics.median(v) * 8 / 1e3, 3)
                          if k != "tb8" else None}))


if __name__ == "__main__":
    main()
