"""Multi-process decomposition invariance on CPU: world 2..4 ranks over
torch.distributed (gloo) must reproduce the single-rank run bit for bit, for
1-D and 2-D decompositions, odd sizes with remainders, deep halos, and
convergence.  (The reference was validated only by inspecting output files.)"""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver

from .dist_worker import run_world

BASE = dict(nx=37, ny=45, steps=0, init="random", seed=11, backend="cpu")


def single(cfg_kwargs, steps):
    with HeatSolver(HeatConfig(**{**cfg_kwargs, "tb_depth": 1, "decomp": "auto", "px": 0,
                                  "py": 0})) as s:
        r = s.run(steps)
        return s.gather(), r


@pytest.mark.parametrize("world,decomp,depth", [(2, "rows", 1), (2, "2d", 1), (3, "rows", 2),
                                                (4, "auto", 1), (4, "auto", 3), (4, "rows", 4)])
def test_invariance_gloo(tmp_path, world, decomp, depth):
    kw = {**BASE, "decomp": decomp, "tb_depth": depth}
    if decomp == "2d" and world == 2:
        kw.update(px=1, py=2)  # column split: exercises packed E/W halos
    res = run_world(world, kw, 29, tmp_path)
    ref, _ = single(BASE, 29)
    assert int(res["done"]) == 29
    assert np.array_equal(res["grid"], ref)


@pytest.mark.parametrize("world,kw", [
    (2, dict(decomp="rows", tb_depth=2, halo_passes=3)),
    (2, dict(px=1, py=2, tb_depth=1, halo_passes=4)),
    (4, dict(decomp="auto", tb_depth=3, halo_passes=2)),
    (3, dict(decomp="rows", tb_depth=5, halo_passes=9)),   # clamped to the block size
])
def test_deep_halo_invariance_gloo(tmp_path, world, kw):
    # One exchange per halo_passes passes; ghost cells computed redundantly.
    res = run_world(world, {**BASE, **kw}, 0, tmp_path, chunks=[7, 1, 13, 8])
    ref, _ = single(BASE, 29)
    assert np.array_equal(res["grid"], ref)
    if kw["halo_passes"] <= 4:
        # The last chunk (8 steps) needs at most ceil(8 / (k*m)) + 1 exchanges.
        km = kw["tb_depth"] * kw["halo_passes"]
        assert int(res["exchanges"]) <= -(-8 // km) + 1


def test_deep_halo_convergence_gloo(tmp_path):
    kw = dict(nx=24, ny=30, steps=20000, converge=True, check_interval=20, eps=1e-3,
              backend="cpu", tb_depth=2, halo_passes=3)
    res = run_world(4, kw, 20000, tmp_path)
    ref, r = single(kw, 20000)
    assert bool(res["conv"]) and r.converged
    assert int(res["conv_at"]) == r.converged_at
    assert np.array_equal(res["grid"], ref)


def test_invariance_chunked_runs(tmp_path):
    kw = {**BASE, "tb_depth": 3}
    res = run_world(4, kw, 0, tmp_path, chunks=[5, 1, 17])
    ref, _ = single(BASE, 23)
    assert np.array_equal(res["grid"], ref)


def test_explicit_gloo_group(tmp_path):
    # HeatSolver(..., transport="torch", group=<gloo group>): bench.py's
    # fallback when the engine's RCCL communicator cannot be created.
    kw = {**BASE, "tb_depth": 2}
    res = run_world(2, kw, 19, tmp_path, transport="torch_subgroup")
    ref, _ = single(BASE, 19)
    assert np.array_equal(res["grid"], ref)


def test_convergence_distributed(tmp_path):
    kw = dict(nx=24, ny=30, steps=20000, converge=True, check_interval=20, eps=1e-3,
              backend="cpu", tb_depth=2)
    res = run_world(4, kw, 20000, tmp_path)
    ref, r = single(kw, 20000)
    assert bool(res["conv"]) and r.converged
    assert int(res["conv_at"]) == r.converged_at
    assert np.array_equal(res["grid"], ref)


def test_mpi_compat_distributed(tmp_path):
    kw = {**BASE, "compat": "mpi", "steps": 10}
    res = run_world(2, kw, None, tmp_path)
    assert int(res["done"]) == 11


def test_scatter_then_run_distributed(tmp_path):
    kw = dict(nx=31, ny=27, steps=0, init="zero", backend="cpu", decomp="auto")
    res = run_world(3, kw, 12, tmp_path)
    ref, _ = single(dict(nx=31, ny=27, steps=0, init="random", seed=77, backend="cpu"), 12)
    assert np.array_equal(res["grid"], ref)


def test_autotune_collective_gloo(tmp_path):
    # Four ranks time rows slabs vs the 2x2 grid x {sync (m default, m=2),
    # overlap}; every rank must come out with the same choice, and the
    # table must list every candidate with a time.
    from .dist_worker import run_tune

    res = run_tune(4, dict(nx=64, ny=64, steps=0, init="random", seed=3, backend="cpu",
                           tb_depth=2), tmp_path)
    assert all(c == res["choices"][0] for c in res["choices"])
    layouts = {(r["px"], r["py"]) for r in res["table"]}
    assert layouts == {(4, 1), (2, 2)}
    assert len(res["table"]) == 6
    assert all(r["ms_per_1000_iters"] > 0 for r in res["table"])


def test_autotune_shared_transport_gloo(tmp_path):
    # bench.py's multi-GPU path: ONE engine transport per rank for every
    # autotune candidate and the final solver (one communicator per run).
    from .dist_worker import run_tune

    kw = dict(nx=40, ny=36, steps=0, init="random", seed=5, backend="cpu", tb_depth=2)
    res = run_tune(2, kw, tmp_path, transport="shared")
    assert all(c == res["choices"][0] for c in res["choices"])
    assert all(r["ms_per_1000_iters"] > 0 for r in res["table"])
    got = np.load(str(tmp_path / f"tune_2_{__import__('os').getpid()}.json") + ".npy")
    ref, _ = single(kw, 29)
    assert np.array_equal(got, ref)
