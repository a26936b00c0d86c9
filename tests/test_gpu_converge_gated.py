"""Device-judged convergence (Solver::run_gated): checks inside temporally
blocked passes, queued segments behind the converging check, the replay of an
overshooting pass -- all bitwise against the CPU oracle, which judges every
check on the host (reference: cuda/cuda_heat.cu:219-236,
mpi/mpi_heat_improved_persistent_stat.c:235-262).  Needs an MI355X."""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver

pytestmark = pytest.mark.gpu


def _run(cfg, steps=None):
    with HeatSolver(cfg) as s:
        r = s.run(steps)
        return s.gather(), r


@pytest.mark.parametrize("depth,interval", [(12, 50), (12, 20), (8, 5), (12, 7), (8, 3),
                                            (5, 13)])
@pytest.mark.parametrize("compat", ["none", "cuda"])
@pytest.mark.parametrize("graph", [True, False])
def test_gated_convergence_bitwise(gpu, depth, interval, compat, graph):
    # ref-wrap init on a small plate converges after a few thousand steps:
    # the converging check falls inside a pass for most (depth, interval).
    cfg = HeatConfig(nx=26, ny=37, steps=40000, converge=True, check_interval=interval,
                     eps=1e-3, init="ref-wrap", backend="hip", tb_depth=depth, compat=compat,
                     use_graph=graph)
    g, r = _run(cfg)
    c, rc = _run(cfg.replace(backend="cpu", tb_depth=1))
    assert r.converged and rc.converged
    assert r.converged_at == rc.converged_at and r.steps_done == rc.steps_done
    assert r.checks == rc.checks
    assert np.float32(r.last_resid) == np.float32(rc.last_resid)
    assert np.array_equal(g, c), np.abs(g - c).max()


def test_gated_mpi_compat(gpu):
    cfg = HeatConfig(nx=30, ny=24, steps=40000, converge=True, check_interval=20, eps=1e-3,
                     init="ref-wrap", backend="hip", tb_depth=12, compat="mpi")
    g, r = _run(cfg)
    c, rc = _run(cfg.replace(backend="cpu", tb_depth=1))
    assert r.converged and r.converged_at == rc.converged_at
    assert np.array_equal(g, c)


def test_gated_not_converged_counts_checks(gpu):
    cfg = HeatConfig(nx=300, ny=200, steps=1000, converge=True, check_interval=50, eps=0.0,
                     init="random", seed=3, backend="hip", tb_depth=12)
    g, r = _run(cfg)
    c, rc = _run(cfg.replace(backend="cpu", tb_depth=1))
    assert not r.converged and r.steps_done == 1000 and r.checks == 20 == rc.checks
    assert np.float32(r.last_resid) == np.float32(rc.last_resid)
    assert np.array_equal(g, c)


def test_gated_continue_after_convergence(gpu):
    # A converged run leaves the state of the converging check; later runs
    # step on from there (and check again) exactly like the oracle.
    cfg = HeatConfig(nx=40, ny=33, steps=0, converge=True, check_interval=30, eps=2e-2,
                     init="ref-wrap", backend="hip", tb_depth=12)
    out = {}
    for backend in ("hip", "cpu"):
        with HeatSolver(cfg.replace(backend=backend, tb_depth=12 if backend == "hip" else 1)) as s:
            r1 = s.run(50000)
            r2 = s.run(77)
            r3 = s.run(5)
            out[backend] = (s.gather(), (r1.converged_at, r2.converged, r2.steps_done,
                                         r3.steps_done, s.step))
    assert out["hip"][1] == out["cpu"][1]
    assert np.array_equal(out["hip"][0], out["cpu"][0])


@pytest.mark.parametrize("kernel", ["lds", "naive"])
def test_gated_single_step_kernels(gpu, kernel):
    cfg = HeatConfig(nx=28, ny=22, steps=40000, converge=True, check_interval=20, eps=1e-3,
                     init="ref-wrap", backend="hip", kernel=kernel, tb_depth=3)
    g, r = _run(cfg)
    c, rc = _run(cfg.replace(backend="cpu", tb_depth=1))
    assert r.converged_at == rc.converged_at
    assert np.array_equal(g, c)


@pytest.mark.parametrize("interval,check", [(10, 1), (11, 1), (9, 1), (50, 5)])
def test_gated_replay_deep_level(gpu, interval, check):
    # A converging check at level 9, 10 or 11 of a depth-12 pass (every 10
    # steps: level 10 of pass [0, 12); every 50: step 250 at level 10 of
    # [240, 252)) on a level-split plate: the replay runs those steps as
    # passes tb_step takes (rl mod 8, then 8), not as one depth-10 pass.
    base = HeatConfig(nx=2048, ny=8192, steps=0, converge=True, check_interval=interval,
                      eps=0.0, init="random", seed=9, backend="cpu", tb_depth=1)
    with HeatSolver(base) as c:
        res = [np.float32(c.run(interval).last_resid) for _ in range(check)]
        want = c.gather()
    eps = float(np.nextafter(res[-1], np.float32(np.inf)))
    cfg = base.replace(backend="hip", tb_depth=12, eps=eps)
    g, r = _run(cfg, 300)
    assert r.converged and r.converged_at == interval * check, (r.converged_at, res)
    assert np.float32(r.last_resid) == res[-1]
    assert np.array_equal(g, want), np.abs(g - want).max()


@pytest.mark.parametrize("check", [2, 4])
def test_gated_split_kernel_check_inside_pass(gpu, check):
    # A plate large enough for the level-split pipelines (>= 64 strip-rows
    # per SIMD at depth 12).  Checks every 20 steps no longer cut the 12-step
    # passes: the check after step 40 is taken at level 4 of pass [36, 48),
    # the one after step 80 at level 8 of pass [72, 84), the one after step 60
    # at the end of pass [48, 60).  eps is set just above the CPU oracle's
    # residual at the chosen check, so the run converges exactly there and
    # its state is the inner-pass replay.
    base = HeatConfig(nx=2048, ny=8192, steps=0, converge=True, check_interval=20, eps=0.0,
                      init="random", seed=9, backend="cpu", tb_depth=1)
    with HeatSolver(base) as c:
        res = [np.float32(c.run(20).last_resid) for _ in range(check)]
        want = c.gather()
    assert all(res[i] > res[i + 1] for i in range(len(res) - 1)), res
    eps = float(np.nextafter(res[-1], np.float32(np.inf)))
    cfg = base.replace(backend="hip", tb_depth=12, eps=eps)
    g, r = _run(cfg, 200)
    assert r.converged and r.converged_at == 20 * check, (r.converged_at, res)
    assert r.checks == check
    assert np.float32(r.last_resid) == res[-1]
    assert np.array_equal(g, want), np.abs(g - want).max()
