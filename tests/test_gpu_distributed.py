"""Multi-rank GPU paths on ONE MI355X: two ranks share cuda:0 and exchange
halos through host-staged torch.distributed (gloo).  This runs the real GPU
kernels, pack/unpack and the staged exchange path under a real decomposition;
results must equal the single-rank GPU run bit for bit."""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver

from .dist_worker import run_world

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,kw", [
    (2, dict(decomp="rows")),
    (2, dict(px=1, py=2)),
    (4, dict(decomp="auto")),
    (3, dict(decomp="rows", kernel="naive", tb_depth=2)),
])
def test_gpu_two_ranks_one_device(gpu, tmp_path, world, kw):
    base = dict(nx=150, ny=300, steps=0, init="random", seed=2, backend="hip", tb_depth=8)
    base.update(kw)
    res = run_world(world, base, 45, tmp_path, transport="torch")
    with HeatSolver(HeatConfig(**{**base, "decomp": "auto", "px": 0, "py": 0})) as s:
        s.run(45)
        ref = s.gather()
    assert np.array_equal(res["grid"], ref)
