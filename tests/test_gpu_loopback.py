"""The device-memory (RCCL-shaped) exchange path on ONE MI355X: ranks are
threads of this process over the loopback transport (stream-ordered D2D
copies, comm stream, events; eager, no staging).  Every pass schedule and
decomposition must reproduce the single-rank GPU run bit for bit, including
convergence, gather, scatter and the device checksum."""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver
from parallel_heat_amd.models import reference as R
from parallel_heat_amd.parallel.group import run_group

pytestmark = pytest.mark.gpu

BASE = dict(nx=150, ny=300, steps=0, init="random", seed=2, backend="hip", tb_depth=8)


def single(cfg, steps):
    with HeatSolver(cfg.replace(decomp="auto", px=0, py=0)) as s:
        r = s.run(steps)
        return s.gather(), r, s.checksum()


def grid_of(results):
    return next(g for g, _ in results if g is not None)


@pytest.mark.parametrize("schedule", ["sync", "overlap", "pipeline"])
@pytest.mark.parametrize("world,kw", [(2, dict(decomp="rows")), (2, dict(px=1, py=2)),
                                      (4, dict(decomp="auto")), (3, dict(decomp="rows")),
                                      (6, dict(decomp="auto")),
                                      (4, dict(decomp="auto", kernel="lds", tb_depth=3))])
def test_loopback_schedules(gpu, world, kw, schedule):
    cfg = HeatConfig(**{**BASE, **kw, "schedule": schedule})
    def fn(s):
        s.run(45)
        return s.gather(), s.info.schedule

    res = run_group(cfg, world, fn)
    ref, _, _ = single(cfg, 45)
    assert np.array_equal(grid_of(res), ref)
    if world == 2 and kw.get("decomp") == "rows":
        assert {sch for _, sch in res} == {schedule}


@pytest.mark.parametrize("m", [0, 1, 2, 3])
def test_loopback_deep_halo_chunked(gpu, m):
    cfg = HeatConfig(**{**BASE, "decomp": "auto", "halo_passes": m})

    def fn(s):
        for n in (5, 1, 17, 22, 8):
            s.run(n)
        return s.gather(), s.checksum()

    res = run_group(cfg, 4, fn)
    ref, _, cs = single(cfg, 53)
    assert np.array_equal(grid_of(res), ref)
    assert all(c == cs for _, c in res)


@pytest.mark.parametrize("schedule", ["sync", "pipeline"])
def test_loopback_convergence(gpu, schedule):
    cfg = HeatConfig(nx=64, ny=40, steps=40000, converge=True, check_interval=20, eps=1e-3,
                     backend="hip", tb_depth=8, decomp="rows", schedule=schedule)
    res = run_group(cfg, 2, lambda s: (s.run(), s.gather()))
    ref, r, _ = single(cfg, 40000)
    for rr, _ in res:
        assert rr.converged == r.converged and rr.converged_at == r.converged_at
        assert rr.steps_done == r.steps_done
    assert np.array_equal(next(g for _, g in res if g is not None), ref)


def test_loopback_scatter_and_naive_kernel(gpu):
    g0 = R.init_grid(90, 70, "random", 13)
    cfg = HeatConfig(nx=90, ny=70, steps=0, init="zero", backend="hip", kernel="naive",
                     tb_depth=3, decomp="auto")

    def fn(s):
        s.scatter(g0 if s.rank == 0 else None)
        s.run(20)
        return s.gather()

    res = run_group(cfg, 4, fn)
    with HeatSolver(HeatConfig(nx=90, ny=70, steps=0, init="random", seed=13,
                               backend="hip")) as s:
        s.run(20)
        want = s.gather()
    assert np.array_equal(next(g for g in res if g is not None), want)


def test_cli_single_process_gpus(gpu, tmp_path):
    # `heat --gpus N`: one process, N ranks as threads (loopback transport).
    import json
    import subprocess

    from parallel_heat_amd import _native
    outs = {}
    for n in (1, 3):
        d = tmp_path / f"g{n}"
        d.mkdir()
        p = subprocess.run([str(_native.CLI_PATH), "--backend", "hip", "--gpus", str(n),
                            "--nx", "130", "--ny", "90", "--steps", "37", "--init", "random",
                            "--out", "c.json", "--out-format", "checksum", "--json"],
                           cwd=d, capture_output=True, text=True, timeout=300, check=True)
        outs[n] = (json.loads((d / "c.json").read_text()), json.loads(p.stdout.splitlines()[-1]))
    assert outs[3][0]["hash"] == outs[1][0]["hash"]
    assert outs[3][1]["ranks"] == 3 and outs[3][1]["transport"] == "loopback"


def test_cli_single_process_rccl(gpu, tmp_path):
    # `heat --gpus N --transport rccl`: one RCCL rank per thread and GPU.  With
    # fewer GPUs than ranks it must refuse cleanly (RCCL rejects two ranks on
    # one device); with enough GPUs it must match the 1-rank hash.
    import json
    import subprocess

    import torch

    from parallel_heat_amd import _native
    ndev = torch.cuda.device_count()
    args = ["--backend", "hip", "--nx", "130", "--ny", "90", "--steps", "37", "--init",
            "random", "--out", "c.json", "--out-format", "checksum", "--json"]
    if ndev < 2:
        p = subprocess.run([str(_native.CLI_PATH), "--gpus", "2", "--transport", "rccl"] + args,
                           cwd=tmp_path, capture_output=True, text=True, timeout=120)
        assert p.returncode == 2 and "one GPU per rank" in p.stderr, p.stderr
        return
    hashes = {}
    for n in (1, 2):
        d = tmp_path / f"g{n}"
        d.mkdir()
        subprocess.run([str(_native.CLI_PATH), "--gpus", str(n), "--transport", "rccl"] + args,
                       cwd=d, capture_output=True, text=True, timeout=300, check=True)
        hashes[n] = json.loads((d / "c.json").read_text())["hash"]
    assert hashes[2] == hashes[1]


def test_loopback_phase_timing(gpu):
    cfg = HeatConfig(**{**BASE, "decomp": "rows", "phase_timing": True, "converge": True,
                        "check_interval": 16})
    res = run_group(cfg, 2, lambda s: s.run(64))
    for r in res:
        assert r.t_compute > 0 and r.t_exchange > 0 and r.t_reduce > 0
        assert r.checks == 4


def test_loopback_mfma_kernel_invariance(gpu):
    cfg = HeatConfig(**{**BASE, "decomp": "auto", "kernel": "mfma", "tb_depth": 4})

    def fn(s):
        s.run(21)
        return s.gather()

    res = run_group(cfg, 4, fn)
    with HeatSolver(cfg.replace(decomp="auto")) as s:
        s.run(21)
        want = s.gather()
    assert np.array_equal(next(g for g in res if g is not None), want)
    ref, _, _ = single(cfg.replace(kernel="tb", tb_depth=8), 21)
    assert np.abs(want - ref).max() <= 1e-3


def test_loopback_failed_rank_unblocks_peers(gpu):
    # Rank 1 dies before its first exchange; rank 0 would wait forever for
    # its halo rows.  The hub is marked failed, rank 0 raises, and run_group
    # reports rank 1's own error.
    cfg = HeatConfig(**{**BASE, "decomp": "rows"})

    def fn(s):
        if s.rank == 1:
            raise ValueError("injected failure on rank 1")
        s.run(45)
        return s.gather()

    with pytest.raises(RuntimeError, match="rank 1 failed: injected failure"):
        run_group(cfg, 2, fn)


@pytest.mark.parametrize("world,kw", [(2, dict(decomp="rows", tb_depth=12)),
                                      (4, dict(decomp="auto", tb_depth=8))])
def test_loopback_vs_torch_fp32(gpu, world, kw):
    # The direct PyTorch anchor for the multi-rank path: a decomposed
    # deep-halo TB run against K applications of the plain fp32 stencil
    # (R.step_torch) on the GPU, tolerance growing with K.
    import torch
    steps = 60
    cfg = HeatConfig(**{**BASE, "nx": 300, "ny": 280, **kw})

    def fn(s):
        s.run(steps)
        return s.gather()

    got = next(g for g in run_group(cfg, world, fn) if g is not None)
    u = torch.from_numpy(R.init_grid(300, 280, "random", BASE["seed"])).cuda()
    for _ in range(steps):
        u = R.step_torch(u)
    torch.testing.assert_close(torch.from_numpy(got), u.cpu(), rtol=2e-6 * steps,
                               atol=1e-5 * steps)
