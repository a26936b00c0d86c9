"""GPU solver end to end: bitwise equal to the CPU oracle across kernels,
depths, graph/eager, overlap, decompositions and convergence.  Needs an MI355X."""
import numpy as np
import pytest
import torch

from parallel_heat_amd import HeatConfig, HeatSolver

pytestmark = pytest.mark.gpu


def _run(cfg, steps=None):
    with HeatSolver(cfg) as s:
        r = s.run(steps)
        return s.gather(), r


@pytest.mark.parametrize("kernel,depth", [("naive", 1), ("naive", 3), ("tb", 1), ("tb", 5),
                                          ("tb", 8), ("tb", 7), ("lds", 1), ("lds", 4)])
@pytest.mark.parametrize("graph", [True, False])
def test_gpu_equals_cpu(gpu, kernel, depth, graph):
    cfg = HeatConfig(nx=150, ny=333, steps=45, init="random", seed=9, backend="hip",
                     kernel=kernel, tb_depth=depth, use_graph=graph)
    g, r = _run(cfg)
    c, _ = _run(cfg.replace(backend="cpu", tb_depth=1))
    assert r.steps_done == 45
    assert np.array_equal(g, c), np.abs(g - c).max()


@pytest.mark.parametrize("steps", [45, 50, 1000])
def test_gpu_depth12_passes(gpu, steps):
    # Depth 12 with the remainder in near-equal passes of <= 8
    # (45 -> 12,12,12,5,4; 50 -> 12,12,12,7,7; 1000 -> 82 x 12,8,8).
    cfg = HeatConfig(nx=150, ny=333, steps=steps, init="random", seed=4, backend="hip",
                     tb_depth=12)
    g, r = _run(cfg)
    c, _ = _run(cfg.replace(backend="cpu", tb_depth=1))
    assert r.steps_done == steps
    assert np.array_equal(g, c), np.abs(g - c).max()


def test_gpu_auto_depth_tall_block(gpu):
    # Blocks of >= 1024 rows get depth 12 by default, shorter ones depth 8.
    tall = HeatConfig(nx=1100, ny=70, steps=30, init="random", seed=6, backend="hip")
    with HeatSolver(tall) as s:
        assert s.info.tb_depth == 12
        s.run()
        g = s.gather()
    c, _ = _run(tall.replace(backend="cpu"))
    assert np.array_equal(g, c)
    with HeatSolver(tall.replace(nx=1000)) as s:
        assert s.info.tb_depth == 8


def test_reference_init_grid(gpu):
    cfg = HeatConfig(nx=500, ny=500, steps=100, init="ref-wrap", backend="hip")
    g, _ = _run(cfg)
    c, _ = _run(cfg.replace(backend="cpu"))
    assert np.array_equal(g, c)


@pytest.mark.parametrize("compat", ["none", "mpi", "cuda"])
def test_gpu_convergence_matches_cpu(gpu, compat):
    cfg = HeatConfig(nx=24, ny=30, steps=20000, converge=True, check_interval=20, eps=1e-3,
                     init="ref-wrap", backend="hip", compat=compat)
    g, r = _run(cfg)
    c, rc = _run(cfg.replace(backend="cpu"))
    assert r.converged and rc.converged
    assert r.converged_at == rc.converged_at
    assert np.array_equal(g, c)


def test_repeated_runs_graph_cache(gpu):
    cfg = HeatConfig(nx=256, ny=256, steps=0, init="random", backend="hip", tb_depth=8)
    with HeatSolver(cfg) as s:
        for _ in range(3):
            s.run(100)
        g = s.gather()
        assert s.step == 300
    c, _ = _run(cfg.replace(backend="cpu", tb_depth=1), 300)
    assert np.array_equal(g, c)


def test_checkpoint_resume(gpu, tmp_path):
    cfg = HeatConfig(nx=100, ny=120, steps=60, init="random", backend="hip")
    full, _ = _run(cfg)
    with HeatSolver(cfg) as s:
        s.run(25)
        s.save(str(tmp_path / "ck.bin"))
    with HeatSolver(cfg) as s:
        s.load(str(tmp_path / "ck.bin"))
        assert s.step == 25
        s.run(35)
        g = s.gather()
    assert np.array_equal(g, full)


def test_large_grid_smoke(gpu):
    cfg = HeatConfig(nx=4096, ny=4096, steps=64, init="random", backend="hip")
    with HeatSolver(cfg) as s:
        r = s.run()
        cs = s.checksum()
    assert r.steps_done == 64 and np.isfinite(cs["sum"])
    assert torch.cuda.is_available()


def test_device_checksum_matches_host(gpu):
    cfg = HeatConfig(nx=300, ny=517, steps=20, init="random", backend="hip")
    with HeatSolver(cfg) as s:
        s.run()
        cg = s.checksum()
        g = s.gather()
    with HeatSolver(cfg.replace(backend="cpu")) as c:
        c.run()
        cc = c.checksum()
    assert cg["hash"] == cc["hash"] and cg["count"] == cc["count"]
    assert cg["min"] == float(g.min()) and cg["max"] == float(g.max())
    assert abs(cg["sum"] - cc["sum"]) <= 1e-9 * abs(cc["sum"]) + 1e-6


def test_gpu_scatter(gpu):
    from parallel_heat_amd.models import reference as R
    g0 = R.init_grid(64, 300, "random", 5)
    cfg = HeatConfig(nx=64, ny=300, steps=0, init="zero", backend="hip")
    with HeatSolver(cfg) as s:
        s.scatter(g0)
        s.run(17)
        a = s.gather()
    with HeatSolver(cfg.replace(init="random", seed=5)) as s:
        s.run(17)
        assert np.array_equal(s.gather(), a)


def test_gpu_mpi_numerics(gpu):
    # numerics="mpi" runs on the naive kernel (auto-selected) and reproduces
    # the reference MPI program's double arithmetic bit for bit.
    from parallel_heat_amd.models import reference as R
    cfg = HeatConfig(nx=96, ny=130, steps=33, init="random", seed=4, backend="hip",
                     numerics="mpi")
    g, _ = _run(cfg)
    ref, _, _ = R.run_np(96, 130, 33, init="random", seed=4, numerics="mpi")
    assert np.array_equal(g, ref)
    with pytest.raises(Exception, match="naive"):
        HeatSolver(cfg.replace(kernel="tb"))


@pytest.mark.parametrize("edge_frac", ["0.75", "0.5"])
def test_tb_edge_subboxes_bitwise(gpu, tmp_path, edge_frac):
    # HEAT_TB_EDGE_FRAC < 1 plans the plate's top/bottom chunks as separate
    # shorter sub-boxes (off by default since the round-2 edge A/B,
    # profiles/tb_edge_frac_r2.md).  The planner reads it once per process,
    # so run the CLI with it and compare with the CPU oracle's checksum.
    import json
    import os
    import subprocess

    from parallel_heat_amd import _native
    # Tall enough that chunks are longer than the minimum (edge boxes exist).
    args = ["--nx", "8192", "--ny", "1000", "--steps", "30", "--init", "random",
            "--out", "c.json", "--out-format", "checksum"]
    got = {}
    for backend in ("hip", "cpu"):
        d = tmp_path / backend
        d.mkdir()
        env = dict(os.environ, HEAT_TB_EDGE_FRAC=edge_frac)
        subprocess.run([str(_native.CLI_PATH), "--backend", backend] + args, cwd=d, env=env,
                       capture_output=True, text=True, timeout=300, check=True)
        got[backend] = json.loads((d / "c.json").read_text())
    assert got["hip"]["hash"] == got["cpu"]["hash"]


@pytest.mark.parametrize("kw", [dict(nx=300, ny=517), dict(nx=1024, ny=8192)])
def test_enqueued_runs_match_synchronous(gpu, kw):
    # run(wait=False) x 3 then run(0) (bench.py's timed loop) == one run of
    # the same steps: state, step count; state access completes pending runs.
    cfg = HeatConfig(steps=0, init="random", seed=21, backend="hip", **kw)
    with HeatSolver(cfg) as a:
        rs = [a.run(97, wait=False) for _ in range(3)]
        assert all(r.steps_done == 97 for r in rs)
        done = a.run(0)
        assert done.steps_done == 0 and done.resident_giveups == 0
        ga = a.gather()
        a.run(50, wait=False)
        gb = a.gather()  # completes the pending run first
        step_b = a.step
    with HeatSolver(cfg) as b:
        b.run(291)
        want = b.gather()
        b.run(50)
        want_b = b.gather()
    assert np.array_equal(ga, want) and np.array_equal(gb, want_b) and step_b == 341
