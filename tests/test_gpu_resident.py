"""Resident workgroup tiles (csrc/kernels/tb_resident.hip): the passes between
two halo exchanges (all passes of a segment on one rank) run as ONE launch
whose tiles stay in VGPRs and trade only their K-deep ghost rings through
flag-guarded exchange fields.  Bitwise against separate per-pass launches
(HEAT_TB_RESIDENT=0) and the CPU oracle, on plates whose tiles touch every
Dirichlet edge, odd shapes, deep-halo multi-rank blocks (loopback ranks,
2-D grids with ghost corners), graph and eager, and checked runs (checks end
a resident span).  Reference: the per-rank compute of
mpi/mpi_heat_improved_persistent_stat.c:162-234.  Needs an MI355X."""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver
from parallel_heat_amd.parallel.group import run_group

pytestmark = pytest.mark.gpu


def _solve(cfg, steps, resident, monkeypatch, chunks=None):
    monkeypatch.setenv("HEAT_TB_RESIDENT", "1" if resident else "0")
    with HeatSolver(cfg) as s:
        res = [s.run(n) for n in (chunks or [steps])]
        return s.gather(), res


@pytest.mark.parametrize("nx,ny,steps,fits", [
    (1024, 8192, 100, True),    # the 8-GPU 1-D per-rank block as a plate
    (2048, 4096, 60, True),     # the 8-GPU 2-D (4 x 2) per-rank block
    (2048, 8192, 60, True),     # the 4-GPU 1-D per-rank block: 20 x 16 tiles (36 x 7)
    (4096, 4096, 60, True),     # the 4-GPU 2-D (2 x 2) per-rank block: 20 x 16 (18 x 14)
    (203, 517, 97, True),       # partial strips and tiles, a short remainder
    (300, 1000, 50, True),
    (40, 70, 36, True),         # fewer rows than one tile
])
def test_resident_plate_bitwise(gpu, monkeypatch, nx, ny, steps, fits):
    cfg = HeatConfig(nx=nx, ny=ny, steps=steps, init="random", seed=11, backend="hip")
    g1, r1 = _solve(cfg, steps, True, monkeypatch)
    g0, r0 = _solve(cfg, steps, False, monkeypatch)
    assert r0[0].resident_passes == 0
    if fits:
        assert r1[0].resident_passes >= 2, r1
    assert np.array_equal(g1, g0), np.abs(g1 - g0).max()
    if nx * ny <= 1 << 20:
        c, _ = _solve(cfg.replace(backend="cpu", tb_depth=1), steps, False, monkeypatch)
        assert np.array_equal(g1, c), np.abs(g1 - c).max()


def test_resident_repeated_runs_graph_and_eager(gpu, monkeypatch):
    # bench.py's pattern: the same segment graph replayed (flags re-zeroed by
    # the last tile of every launch), and the eager path.
    cfg = HeatConfig(nx=1024, ny=8192, steps=0, init="random", seed=3, backend="hip")
    g_graph, rs = _solve(cfg, 0, True, monkeypatch, chunks=[240, 240, 240])
    assert all(r.resident_passes > 0 for r in rs)
    g_eager, _ = _solve(cfg.replace(use_graph=False), 0, True, monkeypatch,
                        chunks=[240, 240, 240])
    g_sep, _ = _solve(cfg, 0, False, monkeypatch, chunks=[240, 240, 240])
    assert np.array_equal(g_graph, g_sep)
    assert np.array_equal(g_eager, g_sep)


@pytest.mark.parametrize("world,kw", [
    (2, dict(nx=2048, ny=2048, decomp="rows")),         # 1024-row blocks, 96-row halos
    (4, dict(nx=1024, ny=1024, px=2, py=2)),             # 2-D: E/W columns and ghost corners
    (3, dict(nx=777, ny=900, decomp="rows")),            # uneven blocks, remainders
])
def test_resident_multirank_deep_halo(gpu, monkeypatch, world, kw):
    # Ranks as threads of one process (loopback transport on the one GPU):
    # each exchange refills an m*K-deep ring and the m passes behind it run
    # as one resident launch over the first pass's (largest) box.  Ranks
    # sharing a GPU never go resident by default (two resident grids could
    # each hold CUs the other's tiles wait for); HEAT_TB_RESIDENT=2 forces it
    # on blocks small enough that every rank's grid fits the GPU at once.
    cfg = HeatConfig(steps=0, init="random", seed=5, backend="hip", **kw)
    monkeypatch.setenv("HEAT_TB_RESIDENT", "1")
    res = run_group(cfg, world, lambda s: s.run(48))
    assert all(r.resident_passes == 0 for r in res)  # shared device: not resident
    monkeypatch.setenv("HEAT_TB_RESIDENT", "2")
    res = run_group(cfg, world, lambda s: (s.run(300), s.gather()))
    assert all(r[0].resident_passes > 0 for r in res), [r[0] for r in res]
    got = next(g for _, g in res if g is not None)
    single = cfg.replace(decomp="auto", px=0, py=0)
    want, _ = _solve(single, 300, False, monkeypatch)
    assert np.array_equal(got, want), np.abs(got - want).max()


@pytest.fixture
def res_shape():
    """Force the resident planner's tile shape (rows per wave, waves)."""
    from parallel_heat_amd import ops
    saved = ops.tb_tuning()

    def set_(rows, waves):
        t = ops.tb_tuning()
        t.tile_rows, t.tile_waves = rows, waves
        ops.set_tb_tuning(t)
    yield set_
    ops.set_tb_tuning(saved)


@pytest.mark.parametrize("world,kw", [
    (1, dict(nx=203, ny=517)),                       # every Dirichlet edge, partial strips
    (1, dict(nx=700, ny=300)),                       # tiles taller than the plate's chunks
    (2, dict(nx=1024, ny=1024, decomp="rows")),      # deep halos through 20 x 16 tiles
    (4, dict(nx=1024, ny=1024, px=2, py=2)),         # 2-D: ghost columns and corners
])
def test_resident_20x16_tiles(gpu, monkeypatch, res_shape, world, kw):
    # The 4-GPU shape (320-row tiles, 16 waves of 20 rows) forced on small
    # blocks, so its edge, remainder and multi-rank paths run on one GPU.
    res_shape(20, 16)
    cfg = HeatConfig(steps=0, init="random", seed=9, backend="hip", **kw)
    monkeypatch.setenv("HEAT_TB_RESIDENT", "2" if world > 1 else "1")
    if world == 1:
        with HeatSolver(cfg) as s:
            r = s.run(200)
            got = s.gather()
        res = [r]
    else:
        out = run_group(cfg, world, lambda s: (s.run(200), s.gather()))
        res = [o[0] for o in out]
        got = next(g for _, g in out if g is not None)
    assert all(r.resident_passes > 0 for r in res), res
    single = cfg.replace(decomp="auto", px=0, py=0, backend="cpu", tb_depth=1)
    want, _ = _solve(single, 200, False, monkeypatch)
    assert np.array_equal(got, want), np.abs(got - want).max()


@pytest.mark.parametrize("interval", [50, 20, 7])
def test_resident_with_checks(gpu, monkeypatch, interval):
    # Checks at even levels ride inside resident spans (every 20 / 50 steps
    # at depth 8 on this plate: levels 4, 8 / 2, 4, 6, 8); a converging check
    # replays the span from its source buffer.  Every 7 steps every other
    # check falls at an odd level (cut passes, no spans).  Converges, bitwise
    # vs the CPU oracle and vs separate passes.
    cfg = HeatConfig(nx=48, ny=96, steps=40000, converge=True, check_interval=interval,
                     eps=1e-3, init="ref-wrap", backend="hip")
    g1, r1 = _solve(cfg, None, True, monkeypatch)
    g0, r0 = _solve(cfg, None, False, monkeypatch)
    c, rc = _solve(cfg.replace(backend="cpu", tb_depth=1), None, False, monkeypatch)
    assert r1[0].converged and r1[0].converged_at == rc[0].converged_at == r0[0].converged_at
    if interval >= 20:
        assert r1[0].resident_passes > 0
    assert np.array_equal(g1, c) and np.array_equal(g0, c)


@pytest.mark.parametrize("world,kw,interval,check", [
    (1, dict(nx=1024, ny=8192), 20, 4),               # depth 12: step 80, level 8 of pass 7
    (1, dict(nx=1024, ny=8192), 20, 1),               # step 20, level 8 of pass 2 (the 2nd of a span)
    (1, dict(nx=1024, ny=8192), 20, 3),               # step 60 ends pass 5
    (1, dict(nx=1024, ny=8192), 50, 2),               # step 100, level 4 of pass 9
    (1, dict(nx=1024, ny=8192), 50, 5),               # step 250, level 10 of pass 21
    (1, dict(nx=2048, ny=8192), 20, 4),               # 20 x 16 tiles (RES 1 build)
    (2, dict(nx=1024, ny=1024, decomp="rows"), 20, 4),  # deep halos: the owned rows only
    (4, dict(nx=1024, ny=1024, px=2, py=2), 50, 1),     # 2-D blocks: owned rows and columns only
])
def test_resident_span_converges_inside(gpu, monkeypatch, world, kw, interval, check):
    # eps just above the CPU oracle's residual at check `check`: the run
    # converges exactly there, at an inner even level or at the end of a pass
    # of a resident span (depth 12 whatever the interval: round 4 forced
    # depth 10), and its state is the span replayed from its source buffer.
    base = HeatConfig(steps=0, converge=True, check_interval=interval, eps=0.0, init="random",
                      seed=4, backend="cpu", tb_depth=1, nx=kw["nx"], ny=kw["ny"])
    with HeatSolver(base) as c:
        res = [np.float32(c.run(interval).last_resid) for _ in range(check)]
        want = c.gather()
    assert all(res[i] > res[i + 1] for i in range(len(res) - 1)), res
    eps = float(np.nextafter(res[-1], np.float32(np.inf)))
    cfg = HeatConfig(steps=0, converge=True, check_interval=interval, eps=eps, init="random",
                     seed=4, backend="hip", **kw)
    monkeypatch.setenv("HEAT_TB_RESIDENT", "2" if world > 1 else "1")
    if world == 1:
        with HeatSolver(cfg) as s:
            r = s.run(400)
            got = s.gather()
    else:
        out = run_group(cfg, world, lambda s: (s.run(400), s.gather()))
        r = out[0][0]
        got = next(g for _, g in out if g is not None)
        assert all(o[0].converged_at == r.converged_at for o in out)
    assert r.resident_passes > 0, r
    if world == 1:
        with HeatSolver(cfg) as s:
            assert s.info.tb_depth == 12
    assert r.converged and r.converged_at == interval * check, (r.converged_at, res)
    assert np.float32(r.last_resid) == res[-1]
    assert np.array_equal(got, want), np.abs(got - want).max()


@pytest.mark.parametrize("interval", [20, 50])
def test_resident_inner_checks_not_converging(gpu, monkeypatch, interval):
    # 1024 x 8192 at depth 12 checking every 20 / 50 steps without converging
    # (eps 0): every check's residual is taken at its level inside a resident
    # span (the last one reported), the state bitwise the separate passes'.
    cfg = HeatConfig(nx=1024, ny=8192, steps=0, converge=True, check_interval=interval,
                     eps=0.0, init="random", seed=6, backend="hip")
    g1, r1 = _solve(cfg, 600, True, monkeypatch)
    g0, r0 = _solve(cfg, 600, False, monkeypatch)
    assert r1[0].resident_passes > 0 and r0[0].resident_passes == 0
    assert not r1[0].converged and r1[0].checks == r0[0].checks == 600 // interval
    assert np.float32(r1[0].last_resid) == np.float32(r0[0].last_resid)
    assert np.array_equal(g1, g0), np.abs(g1 - g0).max()


def test_resident_shape_host_mirror_matches_the_device(gpu):
    # `heat --plan` and parallel/model.py plan resident tiles without a GPU
    # (topology.cpp resident_shape_static: the planner's shapes with gfx950's
    # co-resident workgroups per CU written in); the solver asks the device
    # planner (gpu::tb_resident_shape: the occupancy API).  Same answers.
    import ctypes

    from parallel_heat_amd import _native
    for r in (40, 203, 640, 1024, 1096, 1168, 1192, 1500, 2048, 2120, 2192, 2216, 3000, 4144, 4180):
        for c in (70, 517, 2000, 4096, 4168, 4180, 8192):
            got = []
            for dev in (1, 0):
                v = ctypes.c_int32()
                _native.call("heat_resident_shape", r, c, 12, dev, ctypes.byref(v))
                got.append(v.value)
            assert got[0] == got[1], (r, c, [(g >> 8, g & 255) for g in got])
