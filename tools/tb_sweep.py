#!/usr/bin/env python3
"""A/B sweep of the temporally blocked kernel on one GPU (interleaved rounds in
one process, median of rounds).  Prints Gcells/s per (variant, depth, waves).

    python tools/tb_sweep.py --n 8192 --depths 4,6,8 --variants 0,1,2,3 --waves 1024,2048,4096
"""
import argparse
import itertools
import json
import os
import statistics
import sys

# HEAT_PY_ROOT: import another copy of the package (e.g. a previous build,
# for an A/B in one session).
sys.path.insert(0, os.environ.get("HEAT_PY_ROOT") or
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from parallel_heat_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--nx", type=int, default=0, help="rows (default --n)")
    ap.add_argument("--depths", default="4,6,8")
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--waves", default="2048")
    ap.add_argument("--iters", type=int, default=200, help="steps per timed sample")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--plate-nx", type=int, default=0,
                    help="treat the block as rows [gx0, gx0+nx) of a plate with this many rows")
    ap.add_argument("--gx0", type=int, default=0)
    ap.add_argument("--interior", action="store_true",
                    help="place the block inside a larger plate: no wave touches the boundary")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = args.n
    nx = args.nx or n
    depths = [int(x) for x in args.depths.split(",")]
    variants = [int(x) for x in args.variants.split(",")]
    waves = [int(x) for x in args.waves.split(",")]
    H = max(depths)
    g = ops.Geom(nx=nx, ny=n) if not args.interior else ops.Geom(nx=4 * nx, ny=4 * n, gx0=nx, gy0=n)
    if args.plate_nx:
        g = ops.Geom(nx=args.plate_nx, ny=n, gx0=args.gx0)
    a = ops.Field(nx, n, H, dev)
    b = ops.Field(nx, n, H, dev)
    ops.init_field(a, g, "random", 1)
    ops.init_field(b, g, "random", 1)
    combos = list(itertools.product(variants, depths, waves))
    res = {c: [] for c in combos}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for c in combos:  # warm-up / first-launch costs
        v, k, w = c
        ops.tb_step(a, b, g, k, waves_target=w, variant=v)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for c in combos:
            v, k, w = c
            passes = max(1, args.iters // k)
            src, dst = a, b
            ev0.record()
            for _ in range(passes):
                ops.tb_step(src, dst, g, k, waves_target=w, variant=v)
                src, dst = dst, src
            ev1.record()
            ev1.synchronize()
            ms = ev0.elapsed_time(ev1)
            res[c].append(nx * n * passes * k / (ms * 1e-3) / 1e9)
    rows = []
    for c in combos:
        v, k, w = c
        med = statistics.median(res[c])
        rows.append({"variant": v, "pipe": (["ring3", "ring4", "ring2", "ring3ramp"][v & 3] + ("+pf6" if v & 8 else "")), "build": "scalar" if v & 4 else "packed",
                     "depth": k, "waves": w, "gcells_s": round(med, 1),
                     "min": round(min(res[c]), 1), "max": round(max(res[c]), 1),
                     "nx": nx, "ny": n,
                     "ms_per_1000": round(nx * n * 1000 / (med * 1e9) * 1e3, 3)})
    rows.sort(key=lambda r: -r["gcells_s"])
    for r in rows:
        print(json.dumps(r))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
