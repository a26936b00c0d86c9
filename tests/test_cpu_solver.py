"""CPU oracle backend of the native engine vs the NumPy reference, halo-depth
invariance, convergence schedules (canonical / mpi / cuda compat), checkpoint."""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver
from parallel_heat_amd.models import reference as R


def run(cfg, steps=None):
    with HeatSolver(cfg) as s:
        r = s.run(steps)
        return s.gather(), r


@pytest.mark.parametrize("nx,ny,steps,init", [(20, 20, 100, "ref-wrap"), (256, 256, 100, "ref-wrap"),
                                              (37, 53, 60, "random"), (3, 9, 10, "random")])
def test_cpu_matches_numpy(nx, ny, steps, init):
    cfg = HeatConfig(nx=nx, ny=ny, steps=steps, init=init, seed=4, backend="cpu")
    g, r = run(cfg)
    ref, done, _ = R.run_np(nx, ny, steps, init=init, seed=4)
    assert r.steps_done == steps == done
    # FMA (engine) vs separately rounded float32 (NumPy): a few ulps.
    scale = max(1.0, float(np.abs(ref).max()))
    assert np.abs(g - ref).max() <= 2e-6 * scale


def test_boundary_ring_fixed():
    cfg = HeatConfig(nx=30, ny=40, steps=50, init="random", seed=1, backend="cpu")
    g, _ = run(cfg)
    g0 = R.init_grid(30, 40, "random", 1)
    for sl in (np.s_[0, :], np.s_[-1, :], np.s_[:, 0], np.s_[:, -1]):
        assert np.array_equal(g[sl], g0[sl])


@pytest.mark.parametrize("depth", [2, 3, 5])
def test_halo_depth_invariance_single_rank(depth):
    cfg = HeatConfig(nx=41, ny=29, steps=23, init="random", backend="cpu")
    a, _ = run(cfg)
    b, _ = run(cfg.replace(tb_depth=depth))
    assert np.array_equal(a, b)


def test_threads_invariance():
    cfg = HeatConfig(nx=64, ny=80, steps=20, init="random", backend="cpu")
    a, _ = run(cfg.replace(threads=1))
    b, _ = run(cfg.replace(threads=4))
    assert np.array_equal(a, b)


@pytest.mark.parametrize("compat", ["none", "mpi", "cuda"])
def test_convergence_schedule_matches_reference_semantics(compat):
    cfg = HeatConfig(nx=24, ny=30, steps=20000, converge=True, check_interval=20, eps=1e-3,
                     backend="cpu", compat=compat)
    g, r = run(cfg)
    ref, done, conv_at = R.run_np(24, 30, 20000, converge=True, check_interval=20, eps=1e-3,
                                  compat=compat)
    assert r.converged and conv_at > 0
    assert r.converged_at == conv_at
    if compat == "cuda":
        assert (r.converged_at - 1) % 20 == 0   # checks after steps 1, 21, 41, ...
    else:
        assert r.converged_at % 20 == 0
    assert r.last_resid < 1e-3 or (compat == "mpi" and r.last_resid <= 1e-3)


def test_not_converged_runs_all_steps_and_mpi_adds_one():
    cfg = HeatConfig(nx=40, ny=40, steps=100, converge=True, check_interval=20, backend="cpu")
    _, r = run(cfg)
    assert not r.converged and r.steps_done == 100 and r.checks == 5
    _, r = run(cfg.replace(compat="mpi"))
    assert r.steps_done == 101  # STEPS+1 iterations


def test_run_in_chunks_equals_one_run():
    cfg = HeatConfig(nx=50, ny=60, steps=0, init="random", backend="cpu", tb_depth=3)
    with HeatSolver(cfg) as s:
        for n in (7, 1, 13, 9):
            s.run(n)
        a = s.gather()
    b, _ = run(cfg.replace(tb_depth=1), 30)
    assert np.array_equal(a, b)


def test_checkpoint_resume_cpu(tmp_path):
    cfg = HeatConfig(nx=33, ny=47, steps=40, init="random", backend="cpu")
    full, _ = run(cfg)
    with HeatSolver(cfg) as s:
        s.run(15)
        s.save(str(tmp_path / "c.bin"))
    with HeatSolver(cfg) as s:
        s.load(str(tmp_path / "c.bin"))
        assert s.step == 15
        s.run(25)
        assert np.array_equal(s.gather(), full)


def test_checksum_and_local_views():
    cfg = HeatConfig(nx=17, ny=19, steps=5, init="random", backend="cpu")
    with HeatSolver(cfg) as s:
        s.run()
        g = s.gather()
        assert np.array_equal(s.local(), g)
        c = s.checksum()
        assert c["count"] == 17 * 19
        assert abs(c["sum"] - float(g.astype(np.float64).sum())) < 1e-6 * abs(c["sum"]) + 1e-6
        assert c["max"] == float(g.max()) and c["min"] == float(g.min())
        s.load_local(np.zeros_like(g), step=0)
        assert not s.gather().any()


def test_nan_detected():
    cfg = HeatConfig(nx=16, ny=16, steps=100, converge=True, check_interval=5, backend="cpu")
    with HeatSolver(cfg) as s:
        g = s.local()
        g[5, 5] = np.nan
        s.load_local(g)
        with pytest.raises(Exception, match="non-finite"):
            s.run()


def test_invalid_config():
    with pytest.raises(ValueError):
        HeatConfig(nx=0).validate()
    with pytest.raises(ValueError):
        HeatConfig(init="bogus").validate()


def test_scatter_single_rank():
    cfg = HeatConfig(nx=21, ny=34, steps=0, init="zero", backend="cpu")
    from parallel_heat_amd.models import reference as R
    g0 = R.init_grid(21, 34, "random", 9)
    with HeatSolver(cfg) as s:
        s.scatter(g0, step=3)
        assert s.step == 3
        assert np.array_equal(s.gather(), g0)
        s.run(10)
        a = s.gather()
    with HeatSolver(cfg.replace(init="random", seed=9)) as s:
        s.run(10)
        assert np.array_equal(s.gather(), a)


@pytest.mark.parametrize("nx,ny,steps,init", [(20, 20, 101, "ref-wrap"), (480, 64, 12, "ref-wrap"),
                                              (37, 53, 60, "random")])
def test_mpi_numerics_bitwise_vs_numpy_emulation(nx, ny, steps, init):
    # numerics="mpi" reproduces the reference MPI program's arithmetic
    # (fp32 neighbour sums, double combine, one rounding) bit for bit.
    cfg = HeatConfig(nx=nx, ny=ny, steps=steps, init=init, seed=3, backend="cpu",
                     numerics="mpi", threads=2)
    g, _ = run(cfg)
    ref, _, _ = R.run_np(nx, ny, steps, init=init, seed=3, numerics="mpi")
    assert np.array_equal(g, ref)
    # and it is a genuinely different rounding from the canonical fp32 FMA form
    g32, _ = run(cfg.replace(numerics="fp32"))
    assert np.abs(g32 - ref).max() <= 1e-5 * max(1.0, float(np.abs(ref).max()))


def test_mpi_numerics_convergence_vs_numpy_emulation():
    kw = dict(nx=20, ny=20, steps=10000, converge=True, check_interval=20, eps=1e-3)
    g, r = run(HeatConfig(**kw, backend="cpu", numerics="mpi", compat="mpi"))
    ref, done, conv_at = R.run_np(**kw, compat="mpi", numerics="mpi")
    assert r.converged and r.converged_at == conv_at
    assert np.array_equal(g, ref)


@pytest.mark.parametrize("world", [2, 4])
def test_mpi_numerics_decomposition_invariance(tmp_path, world):
    from .dist_worker import run_world
    kw = dict(nx=40, ny=36, steps=0, init="random", seed=5, backend="cpu", numerics="mpi",
              tb_depth=2, halo_passes=2)
    res = run_world(world, kw, 25, tmp_path)
    ref, _, _ = R.run_np(40, 36, 25, init="random", seed=5, numerics="mpi")
    assert np.array_equal(res["grid"], ref)


def test_phase_timing_cpu(tmp_path):
    cfg = HeatConfig(nx=64, ny=64, steps=40, converge=True, check_interval=10, backend="cpu",
                     phase_timing=True)
    with HeatSolver(cfg) as s:
        r = s.run()
    assert r.t_compute > 0 and r.t_exchange == 0 and r.t_reduce >= 0
    assert r.t_compute <= r.seconds * 1.05 + 1e-3
    from .dist_worker import run_world
    res = run_world(2, dict(nx=40, ny=30, steps=0, backend="cpu", phase_timing=True), 12, tmp_path)
    assert int(res["done"]) == 12
