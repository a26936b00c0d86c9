#!/usr/bin/env python3
"""Cost of the fused convergence residual in a TB pass: ms per pass without a
residual, with the residual at the last level, and at inner levels (a check
that falls inside the pass), per variant, interleaved rounds, median.

    python tools/res_cost.py --n 8192 --depth 12 --variants -1,23 --levels 0,12,8,6,4
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.environ.get("HEAT_PY_ROOT") or
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from parallel_heat_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--nx", type=int, default=0)
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--variants", default="-1")
    ap.add_argument("--levels", default="0,12,8,6,4", help="0 = no residual")
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    nx = a.nx or a.n
    k = a.depth
    g = ops.Geom(nx=nx, ny=a.n)
    x = ops.Field(nx, a.n, k, dev)
    y = ops.Field(nx, a.n, k, dev)
    ops.init_field(x, g, "random", 1)
    ops.init_field(y, g, "random", 1)
    resid = torch.zeros(4, dtype=torch.int32, device=dev)
    combos = [(int(v), int(lv)) for v in a.variants.split(",") for lv in a.levels.split(",")]
    has_level = "res_level" in ops.tb_step.__code__.co_varnames

    def launch(v, lv, src, dst):
        kw = {"variant": v}
        if lv > 0:
            kw["resid"] = resid
            if has_level:
                kw["res_level"] = lv
            elif lv != k:
                return False
        ops.tb_step(src, dst, g, k, **kw)
        return True

    ok = {c: launch(c[0], c[1], x, y) for c in combos}
    torch.cuda.synchronize()
    res = {c: [] for c in combos if ok[c]}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for c in res:
            src, dst = x, y
            e0.record()
            for _ in range(a.passes):
                launch(c[0], c[1], src, dst)
                src, dst = dst, src
            e1.record()
            e1.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.passes)
    base = {v: statistics.median(res[(v, 0)]) for v, lv in res if lv == 0 and (v, 0) in res}
    for c, t in res.items():
        med = statistics.median(t)
        row = {"variant": c[0], "res_level": c[1], "ms_per_pass": round(med, 4),
               "tcells_s": round(nx * a.n * k / (med * 1e-3) / 1e12, 3)}
        if c[0] in base:
            row["vs_no_resid"] = round(med / base[c[0]], 4)
        print(json.dumps(row))


if __name__ == "__main__":
    main()
