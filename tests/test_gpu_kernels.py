"""GPU kernel numerics: every HIP kernel against the CPU oracle (bitwise) and
against plain PyTorch fp32 (tolerance).  Needs an MI355X."""
import numpy as np
import pytest
import torch

from parallel_heat_amd import ops
from parallel_heat_amd.models import reference as R

pytestmark = pytest.mark.gpu


def _fields(lx, ly, halo, dev, nx=None, ny=None, gx0=0, gy0=0, mode="random", seed=3):
    nx = nx or lx
    ny = ny or ly
    g = ops.Geom(nx=nx, ny=ny, gx0=gx0, gy0=gy0)
    a = ops.Field(lx, ly, halo, dev)
    b = ops.Field(lx, ly, halo, dev)
    ops.init_field(a, g, mode, seed)
    ops.init_field(b, g, mode, seed)
    return g, a, b


def _cpu_steps(g, lx, ly, halo, k, mode="random", seed=3):
    a = ops.Field(lx, ly, halo, "cpu")
    b = ops.Field(lx, ly, halo, "cpu")
    ops.init_field(a, g, mode, seed)
    ops.init_field(b, g, mode, seed)
    for _ in range(k):
        ops.naive_step(a, b, g, (0, lx, 0, ly))
        a, b = b, a
    return a.owned().clone()


def test_init_matches_numpy(gpu):
    g, a, _ = _fields(37, 53, 4, gpu, nx=37, ny=53, mode="ref-wrap")
    ref = R.init_grid(37, 53, "ref-wrap")
    assert np.array_equal(a.owned().cpu().numpy(), ref)
    g, a, _ = _fields(40, 64, 8, gpu, nx=40, ny=64, mode="random", seed=11)
    assert np.array_equal(a.owned().cpu().numpy(), R.init_grid(40, 64, "random", 11))


def test_naive_step_vs_torch(gpu):
    g, a, b = _fields(130, 257, 1, gpu)
    u = a.owned().clone()
    ops.naive_step(a, b, g)
    torch.cuda.synchronize()
    ref = R.step_torch(u.float())
    torch.testing.assert_close(b.owned(), ref, rtol=1e-6, atol=1e-4)


# 0/3 packed ring-3 (+ramp), 4/7 scalar; +16 XCD-grouped blocks, +32 odd
# chunks streamed bottom-up (mirrored rows, incl. the plate's top/bottom rows);
# +64 float2 lanes (128-column strips).
@pytest.mark.parametrize("variant", [0, 3, 4, 7, 23, 39, 55, 71, 87, 119])
@pytest.mark.parametrize("depth", [1, 2, 3, 4, 5, 6, 7, 8])
def test_tb_bitwise_vs_cpu_oracle(gpu, depth, variant):
    lx, ly = 203, 517  # odd sizes: partial strips and chunks
    g, a, b = _fields(lx, ly, depth, gpu)
    ops.tb_step(a, b, g, depth, variant=variant)
    torch.cuda.synchronize()
    ref = _cpu_steps(g, lx, ly, depth, depth)
    got = b.owned().cpu()
    assert torch.equal(got, ref), f"max diff {(got - ref).abs().max()}"


@pytest.mark.parametrize("variant,depth", [(7, 12), (23, 12), (55, 12), (279, 12),
                                           (2055, 8), (2071, 8), (2071, 12), (2103, 12),
                                           (2327, 12)])
def test_tb_deep_bitwise_vs_cpu_oracle(gpu, depth, variant):
    # Depth 12 exists in the scalar ring-3+ramp build only (+32 mirrored odd
    # chunks, +256 age pairs); +2048: two-wave level-split pipelines
    # (depths 8 and 12) fed through the LDS ring.
    lx, ly = 203, 517
    g, a, b = _fields(lx, ly, depth, gpu)
    ops.tb_step(a, b, g, depth, variant=variant)
    torch.cuda.synchronize()
    ref = _cpu_steps(g, lx, ly, depth, depth)
    got = b.owned().cpu()
    assert torch.equal(got, ref), f"max diff {(got - ref).abs().max()}"


@pytest.mark.parametrize("variant", [263, 279, 311])  # +256: age-paired chunks forced
@pytest.mark.parametrize("depth", [3, 8, 12])
@pytest.mark.parametrize("waves", [0, 64, 1000, 4096])
def test_tb_age_pairs_bitwise(gpu, depth, variant, waves):
    # Chunk pairs split unevenly between the two waves of a SIMD (older wave
    # longer), odd sizes so pairs are cut by the box end; the tall block makes
    # the planner's own two-waves-per-SIMD choice pair chunks too (waves 0).
    lx, ly = (203, 517) if waves else (2600, 300)
    g, a, b = _fields(lx, ly, depth, gpu)
    ops.tb_step(a, b, g, depth, waves_target=waves, variant=variant)
    torch.cuda.synchronize()
    ref = _cpu_steps(g, lx, ly, depth, depth)
    got = b.owned().cpu()
    assert torch.equal(got, ref), f"max diff {(got - ref).abs().max()}"


@pytest.mark.parametrize("variant", [7, 55, 87, 2071])
@pytest.mark.parametrize("waves", [64, 4096])
def test_tb_chunking_invariance(gpu, waves, variant):
    lx, ly, k = 300, 1000, 8
    g, a, b = _fields(lx, ly, k, gpu)
    ops.tb_step(a, b, g, k, waves_target=waves, variant=variant)
    torch.cuda.synchronize()
    ref = _cpu_steps(g, lx, ly, k, k)
    assert torch.equal(b.owned().cpu(), ref)


def test_tb_subdomain_offsets_and_boxes(gpu):
    # A block in the middle of a larger plate, with valid ghost data all around:
    # the TB result on the owned block equals the same steps on the full plate.
    NX, NY, k = 120, 700, 6
    ox, oy, lx, ly = 30, 256, 50, 300
    g = ops.Geom(nx=NX, ny=NY, gx0=ox, gy0=oy)
    a = ops.Field(lx, ly, k, gpu)
    b = ops.Field(lx, ly, k, gpu)
    ops.init_field(a, g, "random", 5)
    ops.init_field(b, g, "random", 5)
    boxes = [(0, k, 0, ly), (lx - k, lx, 0, ly), (k, lx - k, 0, 8), (k, lx - k, 296, ly),
             (k, lx - k, 8, 296)]
    ops.tb_step(a, b, g, k, boxes=boxes)
    torch.cuda.synchronize()
    full = _cpu_steps(ops.Geom(nx=NX, ny=NY), NX, NY, 1, k, seed=5)
    assert torch.equal(b.owned().cpu(), full[ox:ox + lx, oy:oy + ly])
    c = ops.Field(lx, ly, 8, gpu)
    d = ops.Field(lx, ly, 8, gpu)
    ops.init_field(c, g, "random", 5)
    ops.init_field(d, g, "random", 5)
    ops.tb_step(c, d, g, 8, boxes=[(0, lx, 0, 296), (0, lx, 296, ly)], variant=2071)
    torch.cuda.synchronize()
    full8 = _cpu_steps(ops.Geom(nx=NX, ny=NY), NX, NY, 1, 8, seed=5)
    assert torch.equal(d.owned().cpu(), full8[ox:ox + lx, oy:oy + ly])


@pytest.mark.parametrize("k,variant", [(4, -1), (8, 2071), (12, 2071)])
def test_tb_residual(gpu, k, variant):
    lx, ly = 64, 300
    g, a, b = _fields(lx, ly, k, gpu)
    resid = torch.zeros(1, dtype=torch.int32, device=gpu)
    ops.tb_step(a, b, g, k, resid=resid, variant=variant)
    torch.cuda.synchronize()
    prev = _cpu_steps(g, lx, ly, k, k - 1)
    last = _cpu_steps(g, lx, ly, k, k)
    assert ops.resid_value(resid) == float((last - prev).abs().max())


def test_residual_and_pack_unpack(gpu):
    g, a, b = _fields(33, 70, 2, gpu)
    ops.naive_step(a, b, g)
    r = ops.residual(a, b)
    ref = float((a.owned() - b.owned()).abs().max())
    assert r == ref
    buf = torch.empty(33 * 2, device=gpu)
    ops.pack(a, (0, 33, 10, 12), buf)
    c = ops.Field(33, 70, 2, gpu)
    ops.unpack(buf, c, (0, 33, -2, 0))
    torch.cuda.synchronize()
    assert torch.equal(c.view(0, 33, -2, 0), a.view(0, 33, 10, 12))


@pytest.mark.parametrize("lx,ly", [(203, 517), (33, 256), (5, 7), (64, 1000)])
def test_lds_step_bitwise_vs_cpu_oracle(gpu, lx, ly):
    g, a, b = _fields(lx, ly, 4, gpu)
    r = torch.zeros(4, dtype=torch.int32, device=gpu)
    ops.lds_step(a, b, g, resid=r)
    torch.cuda.synchronize()
    ref = _cpu_steps(g, lx, ly, 4, 1)
    assert torch.equal(b.owned().cpu(), ref)
    want = float((ref - a.owned().cpu()).abs().max())
    assert ops.resid_value(r) == want


def test_lds_step_grown_and_offset_boxes(gpu):
    # A block inside a larger plate, box grown into (valid) ghosts and
    # starting at unaligned columns; compared with the naive kernel.
    NX, NY = 120, 700
    ox, oy, lx, ly, h = 30, 256, 50, 301, 8
    g = ops.Geom(nx=NX, ny=NY, gx0=ox, gy0=oy)
    a = ops.Field(lx, ly, h, gpu)
    b1 = ops.Field(lx, ly, h, gpu)
    b2 = ops.Field(lx, ly, h, gpu)
    for f in (a, b1, b2):
        ops.init_field(f, g, "random", 5)
    for box in [(-5, lx + 7, -6, ly + 3), (3, 40, 1, 297), (0, lx, 0, ly)]:
        ops.lds_step(a, b1, g, box)
        ops.naive_step(a, b2, g, box)
        torch.cuda.synchronize()
        assert torch.equal(b1.data, b2.data)


def test_lds_step_mpi_numerics(gpu):
    lx, ly = 96, 130
    g, a, b = _fields(lx, ly, 1, gpu, mode="random", seed=8)
    u0 = a.owned().cpu().numpy()
    ops.lds_step(a, b, g, numerics="mpi")
    torch.cuda.synchronize()
    assert np.array_equal(b.owned().cpu().numpy(), R.step_np_mpi(u0))


def test_mfma_step_close_to_oracle(gpu):
    lx, ly = 203, 517
    g, a, b = _fields(lx, ly, 4, gpu)
    r = torch.zeros(4, dtype=torch.int32, device=gpu)
    ops.mfma_step(a, b, g, resid=r)
    torch.cuda.synchronize()
    ref = _cpu_steps(g, lx, ly, 4, 1)
    got = b.owned().cpu()
    # exact fp32 products, different association than heat::stencil
    assert (got - ref).abs().max() <= 2e-5
    assert torch.equal(got[0], ref[0]) and torch.equal(got[:, -1], ref[:, -1])  # ring fixed
    assert abs(ops.resid_value(r) - float((got - a.owned().cpu()).abs().max())) == 0.0


def test_mfma_step_tiling_invariance(gpu):
    # Every cell gets the same fmaf chain wherever it falls in a 16x16 tile.
    lx, ly = 150, 300
    g, a, b1 = _fields(lx, ly, 4, gpu)
    b2 = ops.Field(lx, ly, 4, gpu)
    ops.init_field(b2, g, "random", 3)
    ops.mfma_step(a, b1, g)
    for box in [(0, 37, 0, 101), (0, 37, 101, ly), (37, lx, 0, 5), (37, lx, 5, ly)]:
        ops.mfma_step(a, b2, g, box)
    torch.cuda.synchronize()
    assert torch.equal(b1.owned(), b2.owned())
