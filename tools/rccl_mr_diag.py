"""Diagnose the multi-rank RCCL path on one GPU, one variant per invocation:
    python tools/rccl_mr_diag.py WORLD 'json of HeatConfig overrides' [chunks]
Runs the ranks (tests/dist_worker.py, transport rccl, one host id per rank)
and compares with the single-rank run; prints OK/MISMATCH."""
import json
import os
import sys
import tempfile
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from parallel_heat_amd import HeatConfig, HeatSolver  # noqa: E402
from tests.dist_worker import run_world  # noqa: E402


def main():
    world = int(sys.argv[1])
    kw = json.loads(sys.argv[2])
    chunks = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [45]
    base = {**dict(nx=150, ny=300, steps=0, init="random", seed=5, backend="hip", tb_depth=8),
            **kw}
    with tempfile.TemporaryDirectory() as d:
        res = run_world(world, base, 0, Path(d), transport="rccl", chunks=chunks)
    with HeatSolver(HeatConfig(**{**base, "decomp": "auto", "px": 0, "py": 0})) as s:
        s.run(sum(chunks))
        ref = s.gather()
    ok = np.array_equal(res["grid"], ref)
    print(f"{'OK' if ok else 'MISMATCH'} world={world} {kw} chunks={chunks}", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
