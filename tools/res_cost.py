#!/usr/bin/env python3
"""Cost of a convergence check in TB passes: ms per pass with and without the
fused residual, per variant and pass depth (interleaved rounds, median).  A
check cuts its segment's passes (12,12,12,7,7 for 50 steps), so the depths of
the cut passes matter as much as the residual itself.

    python tools/res_cost.py --n 8192 --depths 12,8,7 --variants 2071,23
"""
import argparse
import json
import os
import statistics
import sys

# HEAT_PY_ROOT: time another copy of the package (a previous build).
sys.path.insert(0, os.environ.get("HEAT_PY_ROOT") or
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from parallel_heat_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--nx", type=int, default=0)
    ap.add_argument("--depths", default="12,8,7")
    ap.add_argument("--variants", default="-1")
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nx = a.nx or a.n
    depths = [int(x) for x in a.depths.split(",")]
    H = max(depths)
    g = ops.Geom(nx=nx, ny=a.n)
    x = ops.Field(nx, a.n, H, dev)
    y = ops.Field(nx, a.n, H, dev)
    ops.init_field(x, g, "random", 1)
    ops.init_field(y, g, "random", 1)
    resid = torch.zeros(4, dtype=torch.int32, device=dev)
    combos = [(int(v), k, r) for v in a.variants.split(",") for k in depths for r in (False, True)]

    def launch(c, src, dst):
        v, k, r = c
        if k > 8 and k != 12:
            return
        ops.tb_step(src, dst, g, k, resid=resid if r else None,
                    variant=v if (k == 12 or v < 0 or not v & 2048 or k == 8) else -1)

    for c in combos:
        launch(c, x, y)
    torch.cuda.synchronize()
    res = {c: [] for c in combos}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for c in combos:
            src, dst = x, y
            e0.record()
            for _ in range(a.passes):
                launch(c, src, dst)
                src, dst = dst, src
            e1.record()
            e1.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.passes)
    for c, t in res.items():
        v, k, r = c
        med = statistics.median(t)
        base = statistics.median(res[(v, k, False)])
        print(json.dumps({"variant": v, "depth": k, "resid": r, "ms_per_pass": round(med, 4),
                          "ms_per_step": round(med / k, 5),
                          "tcells_s": round(nx * a.n * k / (med * 1e-3) / 1e12, 3),
                          "vs_no_resid": round(med / base, 4)}))


if __name__ == "__main__":
    main()
