"""Workgroup-tile TB kernel (variant bit TILE, csrc/kernels/tb_tile.hip):
bitwise against the CPU oracle for every tile height, lane-shift build and
even depth, on plates with partial strips and tiles, sub-domains with several
boxes, the fused residual (NaN-propagating), the odd-depth fallback, and the
plain PyTorch fp32 anchor over many passes.  Needs an MI355X."""
import numpy as np
import pytest
import torch

from parallel_heat_amd import ops
from parallel_heat_amd.models import reference as R

from .test_gpu_kernels import _cpu_steps, _fields

pytestmark = pytest.mark.gpu

V = ops.TbVariant
TILE = V.TILE | V.XCD_GROUPS
TILE_DPP = TILE | V.TILE_DPP


@pytest.fixture
def tile_rows():
    """Force the tile shape (rows per wave, waves per workgroup) for one
    test, restore after."""
    saved = ops.tb_tuning()

    def set_rows(r, waves=8):
        t = ops.tb_tuning()
        t.tile_rows = r
        t.tile_waves = waves
        ops.set_tb_tuning(t)

    yield set_rows
    ops.set_tb_tuning(saved)


SHAPES = [(12, 8), (13, 8), (14, 8), (16, 8), (20, 8), (24, 8), (28, 8), (32, 8), (12, 16)]


@pytest.mark.parametrize("variant", [TILE, TILE_DPP])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("depth", [2, 4, 8, 12])
def test_tile_bitwise_vs_cpu_oracle(gpu, tile_rows, depth, shape, variant):
    rows, waves = shape
    if waves * rows <= 2 * depth + 4:
        pytest.skip("tile too short for this depth")
    tile_rows(rows, waves)
    lx, ly = 203, 517  # partial strips and tiles, plate edges on every side
    g, a, b = _fields(lx, ly, depth, gpu)
    ops.tb_step(a, b, g, depth, variant=variant)
    torch.cuda.synchronize()
    ref = _cpu_steps(g, lx, ly, depth, depth)
    got = b.owned().cpu()
    assert torch.equal(got, ref), f"max diff {(got - ref).abs().max()}"


@pytest.mark.parametrize("lx,ly", [(7, 9), (40, 70), (2600, 300), (96, 1000)])
def test_tile_shapes(gpu, lx, ly):
    # Blocks shorter than one tile, taller than many, narrower than a strip.
    k = 6
    g, a, b = _fields(lx, ly, k, gpu)
    ops.tb_step(a, b, g, k, variant=TILE)
    torch.cuda.synchronize()
    assert torch.equal(b.owned().cpu(), _cpu_steps(g, lx, ly, k, k))


@pytest.mark.parametrize("shape", [(12, 8), (24, 8), (12, 16)])
def test_tile_subdomain_offsets_and_boxes(gpu, tile_rows, shape):
    # A block in the middle of a larger plate with valid ghost data, five
    # boxes (the deep-halo band shapes of the solver): equals the full plate.
    tile_rows(*shape)
    NX, NY, k = 160, 900, 8
    ox, oy, lx, ly = 40, 256, 70, 500
    g = ops.Geom(nx=NX, ny=NY, gx0=ox, gy0=oy)
    a = ops.Field(lx, ly, k, gpu)
    b = ops.Field(lx, ly, k, gpu)
    ops.init_field(a, g, "random", 5)
    ops.init_field(b, g, "random", 5)
    boxes = [(0, k, 0, ly), (lx - k, lx, 0, ly), (k, lx - k, 0, 8), (k, lx - k, 496, ly),
             (k, lx - k, 8, 496)]
    ops.tb_step(a, b, g, k, boxes=boxes, variant=TILE)
    torch.cuda.synchronize()
    full = _cpu_steps(ops.Geom(nx=NX, ny=NY), NX, NY, 1, k, seed=5)
    assert torch.equal(b.owned().cpu(), full[ox:ox + lx, oy:oy + ly])


def test_tile_interior_block(gpu):
    # Every tile unmasked (MODE 0 path): a block well inside a larger plate.
    NX, NY, k = 700, 1500, 12
    ox, oy, lx, ly = 200, 300, 260, 900
    g = ops.Geom(nx=NX, ny=NY, gx0=ox, gy0=oy)
    a = ops.Field(lx, ly, k, gpu)
    b = ops.Field(lx, ly, k, gpu)
    ops.init_field(a, g, "random", 9)
    ops.init_field(b, g, "random", 9)
    resid = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.tb_step(a, b, g, k, resid=resid, variant=TILE)
    torch.cuda.synchronize()
    prev = _cpu_steps(ops.Geom(nx=NX, ny=NY), NX, NY, 1, k - 1, seed=9)
    full = _cpu_steps(ops.Geom(nx=NX, ny=NY), NX, NY, 1, k, seed=9)
    want = full[ox:ox + lx, oy:oy + ly]
    assert torch.equal(b.owned().cpu(), want)
    assert ops.resid_value(resid) == float((want - prev[ox:ox + lx, oy:oy + ly]).abs().max())


@pytest.mark.parametrize("variant", [TILE, TILE_DPP])
@pytest.mark.parametrize("k", [2, 8, 12])
def test_tile_residual(gpu, k, variant):
    lx, ly = 300, 517
    g, a, b = _fields(lx, ly, k, gpu)
    resid = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.tb_step(a, b, g, k, resid=resid, variant=variant)
    torch.cuda.synchronize()
    prev = _cpu_steps(g, lx, ly, k, k - 1)
    last = _cpu_steps(g, lx, ly, k, k)
    assert torch.equal(b.owned().cpu(), last)
    assert ops.resid_value(resid) == float((last - prev).abs().max())


def test_tile_residual_propagates_nan_and_inf(gpu):
    k, lx, ly = 8, 300, 517
    for bad in (float("nan"), float("inf")):
        g, a, b = _fields(lx, ly, k, gpu)
        a.owned()[150, 200] = bad
        b.owned()[150, 200] = bad
        resid = torch.zeros(1, dtype=torch.int32, device=gpu)
        ops.tb_step(a, b, g, k, resid=resid, variant=TILE)
        torch.cuda.synchronize()
        assert not np.isfinite(ops.resid_value(resid)), bad


@pytest.mark.parametrize("k", [1, 7])
def test_tile_odd_depth_streams(gpu, k):
    # Odd depths (remainder / check-cut passes) fall back to the streaming kernel.
    lx, ly = 203, 517
    g, a, b = _fields(lx, ly, k, gpu)
    ops.tb_step(a, b, g, k, variant=TILE)
    torch.cuda.synchronize()
    assert torch.equal(b.owned().cpu(), _cpu_steps(g, lx, ly, k, k))


@pytest.mark.parametrize("k", [8, 12])
def test_tile_multi_pass_vs_torch_fp32(gpu, k):
    # Direct anchor: passes of the tile kernel against the plain PyTorch fp32
    # stencil (R.step_torch) applied passes * k times on the GPU.
    lx, ly, passes = 600, 777, 5
    g, a, b = _fields(lx, ly, k, gpu)
    u = a.owned().clone().float()
    for _ in range(passes):
        ops.tb_step(a, b, g, k, variant=TILE)
        a, b = b, a
    for _ in range(passes * k):
        u = R.step_torch(u)
    torch.cuda.synchronize()
    n = passes * k
    torch.testing.assert_close(a.owned(), u, rtol=2e-6 * n, atol=1e-5 * n)


def test_tile_solver_bitwise(gpu):
    # The whole solver (graphs, deep halos as 2 loopback ranks) with the tile
    # kernel forced, against the CPU oracle backend.
    from parallel_heat_amd import HeatConfig, HeatSolver

    saved = ops.tb_tuning()
    t = ops.tb_tuning()
    t.variant = int(TILE)
    ops.set_tb_tuning(t)
    try:
        cfg = HeatConfig(nx=300, ny=517, steps=100, init="random", seed=4, backend="hip",
                         device=0, tb_depth=12)
        with HeatSolver(cfg) as s:
            s.run()
            got = s.gather()
    finally:
        ops.set_tb_tuning(saved)
    with HeatSolver(cfg.replace(backend="cpu")) as c:
        c.run()
        want = c.gather()
    assert np.array_equal(got, want)
