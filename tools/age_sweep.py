#!/usr/bin/env python3
"""A/B of the age-group row weights of the TB planner (ops.set_tb_tuning, one
process, interleaved rounds, median Gcells/s).  Weight sets are ';'-separated
lists of comma-separated weights ("" = the built-in default), each optionally
followed by @variant, @waves_target and @edge_frac (defaults: --variant, 0 =
auto, the current tuning).

    python tools/age_sweep.py --n 8192 --sets ";2,1.95,1.15,1;1.7,1"
    python tools/age_sweep.py --nx 1024 --interior --sets "@23;1.6,1@279@2048"
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
    ap.add_argument("--nx", type=int, default=0)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--sets", default=";1.7,1")
    ap.add_argument("--interior", action="store_true")
    ap.add_argument("--iters", type=int, default=480)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nx = a.nx or a.n
    k = a.depth
    g = ops.Geom(nx=nx, ny=a.n) if not a.interior else ops.Geom(nx=4 * nx, ny=4 * a.n, gx0=nx, gy0=a.n)
    x = ops.Field(nx, a.n, k, dev)
    y = ops.Field(nx, a.n, k, dev)
    ops.init_field(x, g, "random", 1)
    ops.init_field(y, g, "random", 1)
    base = ops.tb_tuning()
    ef0 = base.edge_frac
    sets = []
    for spec in a.sets.split(";"):
        parts = spec.split("@")
        w = [float(x) for x in parts[0].split(",")] if parts[0].strip() else []
        v = int(parts[1]) if len(parts) > 1 and parts[1].strip() else a.variant
        wt = int(parts[2]) if len(parts) > 2 and parts[2].strip() else 0
        ef = float(parts[3]) if len(parts) > 3 and parts[3].strip() else None
        sets.append((w, v, wt, ef))
    passes = max(1, a.iters // k)
    res = {i: [] for i in range(len(sets))}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds + 1):
        for i, (w, v, wt, ef) in enumerate(sets):
            base.age_weights = w
            base.edge_frac = ef0 if ef is None else ef
            ops.set_tb_tuning(base)
            src, dst = x, y
            e0.record()
            for _ in range(passes):
                ops.tb_step(src, dst, g, k, waves_target=wt, variant=v)
                src, dst = dst, src
            e1.record()
            e1.synchronize()
            if r:
                res[i].append(nx * a.n * passes * k / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    for i, (w, v, wt, ef) in enumerate(sets):
        print(json.dumps({"weights": w or "default", "variant": v, "waves": wt, "edge_frac": ef, "nx": nx, "ny": a.n, "depth": k,
                          "gcells_s": round(statistics.median(res[i]), 1),
                          "min": round(min(res[i]), 1), "max": round(max(res[i]), 1)}))


if __name__ == "__main__":
    main()
