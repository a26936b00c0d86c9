#!/usr/bin/env python3
"""Same-box A/B of the BASELINE config 3 / 4 rehearsals across two builds.

    python tools/cfg34_ab.py ROOT [ROOT2 ...] [--repeats 3] [--rounds 2]

Each ROOT is a tree holding a `parallel_heat_amd` package with its built
libheat.so (the current repo, or a saved round's tree such as abprev/r3).
Config 3 (16384^2, 2 ranks, rows) and config 4 (32768^2, 8 ranks, 2-D 4x2,
overlap schedule) run as threads of one process on the ONE GPU (loopback
transport), exactly like `bench/run_configs.py --rehearse-1gpu`, but with an
untimed first run (graph capture, first-touch) and `--repeats` timed 1000-step
runs per rank; the time of a repeat is the max over ranks.  The roots run in a
child process each, interleaved `--rounds` times, so box drift shows up as
spread rather than as a difference between builds.  One JSON line per
(root, config, round) on stdout.
"""
import argparse
import json
import os
import subprocess
import sys

CONFIGS = {
    "c3": dict(world=2, nx=16384, ny=16384, decomp="rows", schedule="auto"),
    "c4": dict(world=8, nx=32768, ny=32768, decomp="2d", schedule="overlap"),
}

CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from parallel_heat_amd import HeatConfig
from parallel_heat_amd.parallel.group import run_group
spec = json.loads(sys.argv[2]); repeats = int(sys.argv[3])
kw = dict(nx=spec["nx"], ny=spec["ny"], steps=1000, init="random", seed=1234, backend="hip",
          decomp=spec["decomp"])
if spec["schedule"] != "auto":
    kw["schedule"] = spec["schedule"]
cfg = HeatConfig(**kw)
def fn(s):
    s.run(1000)
    return [s.run(1000).seconds for _ in range(repeats)]
res = run_group(cfg, spec["world"], fn)
per = [max(r[i] for r in res) for i in range(repeats)]
best = min(per)
print(json.dumps({"seconds": [round(x, 6) for x in per],
                  "mcells_per_s": round(spec["nx"] * spec["ny"] * 1000 / best / 1e6, 1)}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("roots", nargs="+")
    ap.add_argument("--configs", default="c3,c4")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    for rnd in range(a.rounds):
        for c in a.configs.split(","):
            for root in a.roots:
                root = os.path.abspath(root)
                env = dict(os.environ, HEAT_NO_AUTOBUILD="1")
                env.pop("HEAT_LIB", None)
                p = subprocess.run([sys.executable, "-c", CHILD, root, json.dumps(CONFIGS[c]),
                                    str(a.repeats)], capture_output=True, text=True, env=env,
                                   timeout=900)
                out = [l for l in p.stdout.splitlines() if l.startswith("{")]
                rec = {"root": root, "config": c, "round": rnd}
                if p.returncode == 0 and out:
                    rec.update(json.loads(out[-1]))
                else:
                    rec["error"] = (p.stderr or p.stdout)[-600:]
                print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
