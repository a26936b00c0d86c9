"""Multi-rank GPU paths on ONE MI355X: ranks share cuda:0 and exchange halos
through host-staged torch.distributed (gloo).  This runs the real GPU kernels,
pack/unpack and all three pass schedules (sync deep-halo, exchange-first
overlap, boundary-first pipeline, the overlap ones with the comm stream
running concurrently with the interior kernel) under a real decomposition;
results must equal the single-rank GPU run bit for bit.

By default these runs capture their segments into hipGraphs with the staged
exchange as a host node, i.e. the multi-rank graph path RCCL runs take
(graphs keyed by segment length, parity and ghost state; deep halos carried
across replays) runs here with world > 1; `use_graph=False` keeps the eager
path covered."""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver

from .dist_worker import run_world

pytestmark = pytest.mark.gpu

BASE = dict(nx=150, ny=300, steps=0, init="random", seed=2, backend="hip", tb_depth=8)


def single(base, steps):
    with HeatSolver(HeatConfig(**{**base, "decomp": "auto", "px": 0, "py": 0})) as s:
        r = s.run(steps)
        return s.gather(), r


@pytest.mark.parametrize("schedule", ["sync", "overlap", "pipeline"])
@pytest.mark.parametrize("world,kw", [
    (2, dict(decomp="rows")),
    (2, dict(px=1, py=2)),
    (4, dict(decomp="auto")),
    (3, dict(decomp="rows", kernel="naive", tb_depth=2)),
])
def test_gpu_ranks_one_device(gpu, tmp_path, world, kw, schedule):
    base = {**BASE, **kw, "schedule": schedule}
    res = run_world(world, base, 45, tmp_path, transport="torch")
    ref, _ = single(base, 45)
    assert np.array_equal(res["grid"], ref)


@pytest.mark.parametrize("schedule,m", [("sync", 0), ("sync", 2), ("sync", 1), ("pipeline", 0)])
def test_gpu_chunked_runs(gpu, tmp_path, schedule, m):
    # Runs of 5, 1, 17, 22 steps: passes shallower than the halo, ghost
    # validity carried across run() calls.
    base = {**BASE, "decomp": "auto", "schedule": schedule, "halo_passes": m}
    res = run_world(4, base, 0, tmp_path, transport="torch", chunks=[5, 1, 17, 22])
    ref, _ = single(BASE, 45)
    assert np.array_equal(res["grid"], ref)


@pytest.mark.parametrize("schedule,decomp", [("sync", dict(decomp="rows")),
                                             ("sync", dict(px=1, py=2)),
                                             ("pipeline", dict(decomp="rows"))])
def test_gpu_distributed_convergence(gpu, tmp_path, schedule, decomp):
    # 2 x (20 x 26) or 2 x (40 x 13) blocks; ny % 4 != 0 so the TB kernel's
    # last lane spills past the box (excluded from the residual).
    kw = dict(nx=40, ny=26, steps=40000, converge=True, check_interval=20, eps=1e-3,
              backend="hip", tb_depth=8, schedule=schedule)
    res = run_world(2, {**kw, **decomp}, 40000, tmp_path, transport="torch")
    ref, r = single(kw, 40000)
    assert bool(res["conv"]) == r.converged
    assert int(res["conv_at"]) == r.converged_at and int(res["done"]) == r.steps_done
    assert np.array_equal(res["grid"], ref)


@pytest.mark.parametrize("world,kw", [(2, dict(decomp="rows", schedule="sync")),
                                      (4, dict(decomp="auto", schedule="pipeline"))])
def test_gpu_ranks_one_device_eager(gpu, tmp_path, world, kw):
    base = {**BASE, **kw, "use_graph": False}
    res = run_world(world, base, 45, tmp_path, transport="torch")
    ref, _ = single(base, 45)
    assert np.array_equal(res["grid"], ref)


@pytest.mark.parametrize("converge", [False, True])
def test_gpu_graph_replay_bench_shape(gpu, tmp_path, converge):
    # bench.py's shape in miniature: rows slabs, auto depth and halo, runs of
    # one "step" (100 iterations) replayed several times from cached graphs,
    # with and without the residual all-reduce of the convergence check.
    base = dict(nx=512, ny=384, steps=0, init="random", seed=1234, backend="hip",
                decomp="rows", converge=converge, check_interval=50, eps=1e-12)
    res = run_world(2, base, 0, tmp_path, transport="torch", chunks=[100] * 5)
    with HeatSolver(HeatConfig(**{**base, "decomp": "auto"})) as s:
        for _ in range(5):
            s.run(100)
        ref, h = s.gather(), s.checksum()["hash"]
    assert int(res["done"]) == 500
    assert np.array_equal(res["grid"], ref)
    assert str(res["hash"]) == h


def test_gpu_autotune_staged(gpu, tmp_path):
    # The multi-GPU autotune of bench.py, with two GPU ranks sharing cuda:0
    # (host-staged halos in captured graphs instead of RCCL).
    from .dist_worker import run_tune

    res = run_tune(2, dict(nx=256, ny=512, steps=0, init="random", seed=3, backend="hip"),
                   tmp_path, transport="torch")
    assert res["choices"][0] == res["choices"][1]
    assert {(r["px"], r["py"]) for r in res["table"]} == {(2, 1), (1, 2)} or \
        {(r["px"], r["py"]) for r in res["table"]} == {(2, 1)}
    assert all("ms_per_1000_iters" in r for r in res["table"])
