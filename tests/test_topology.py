"""Topology / decomposition: MPI_Dims_create parity, remainder-aware blocks,
neighbours, layouts (Python mirror == native engine)."""
import ctypes

import pytest

from parallel_heat_amd import _native
from parallel_heat_amd.parallel import topology as T

# MPI_Dims_create(P, 2) results (MPICH/Open MPI agree for these).
MPI_DIMS_2D = {1: [1, 1], 2: [2, 1], 3: [3, 1], 4: [2, 2], 5: [5, 1], 6: [3, 2], 7: [7, 1],
               8: [4, 2], 9: [3, 3], 10: [5, 2], 11: [11, 1], 12: [4, 3], 13: [13, 1],
               14: [7, 2], 15: [5, 3], 16: [4, 4], 18: [6, 3], 24: [6, 4], 30: [6, 5],
               36: [6, 6], 64: [8, 8]}


def native_dims(n, nd):
    arr = (ctypes.c_int * nd)()
    _native.call("heat_dims_create", n, nd, arr)
    return list(arr)


@pytest.mark.parametrize("n,expected", sorted(MPI_DIMS_2D.items()))
def test_dims_create_2d_matches_mpi(n, expected):
    assert T.dims_create(n, 2) == expected
    assert native_dims(n, 2) == expected


@pytest.mark.parametrize("n", [1, 8, 12, 24, 30, 60, 64, 210])
def test_dims_create_3d_balanced(n):
    d = T.dims_create(n, 3)
    assert d == sorted(d, reverse=True)
    assert d[0] * d[1] * d[2] == n
    assert native_dims(n, 3) == d


@pytest.mark.parametrize("n,parts", [(20, 3), (1000, 10), (1001, 10), (7, 7), (8192, 8), (5, 2)])
def test_block_span_remainders(n, parts):
    spans = [T.block_span(n, parts, i) for i in range(parts)]
    assert sum(s for _, s in spans) == n
    assert spans[0][0] == 0
    for (o0, s0), (o1, _) in zip(spans, spans[1:]):
        assert o1 == o0 + s0
    sizes = [s for _, s in spans]
    assert max(sizes) - min(sizes) <= 1
    for i in range(parts):
        o, s = ctypes.c_int64(), ctypes.c_int64()
        _native.call("heat_block_span", n, parts, i, ctypes.byref(o), ctypes.byref(s))
        assert (o.value, s.value) == spans[i]


def test_reference_drops_cells_we_do_not():
    # The reference uses NX/dx with no remainder (mpi/...c:72): 1001 rows on
    # 10 ranks would lose a row.  Ours covers every row.
    assert 1001 // 10 * 10 == 1000
    assert sum(T.block_span(1001, 10, i)[1] for i in range(10)) == 1001


def test_cart_neighbours_row_major():
    c = T.Cart.create(8)  # dims [4, 2]
    assert (c.px, c.py) == (4, 2)
    assert c.coords(5) == (2, 1)
    n, s, w, e = c.neighbors(5)
    assert (n, s, w, e) == (3, 7, 4, T.NO_NEIGHBOR)
    assert c.neighbors(0) == (T.NO_NEIGHBOR, 2, T.NO_NEIGHBOR, 1)


def test_cart_diagonal_neighbours():
    c = T.Cart.create(8)  # dims [4, 2]
    assert c.diagonal_neighbors(5) == (2, T.NO_NEIGHBOR, 6, T.NO_NEIGHBOR)
    assert c.diagonal_neighbors(0) == (T.NO_NEIGHBOR,) * 3 + (3,)
    # Every diagonal pair is mutual and distinct from the edge neighbours
    # (one message per peer per exchange).
    for r in range(8):
        d = c.diagonal_neighbors(r)
        for k, q in enumerate(d):
            if q != T.NO_NEIGHBOR:
                assert c.diagonal_neighbors(q)[3 - k] == r
                assert q not in c.neighbors(r)
    assert T.Cart.create(8, "rows").diagonal_neighbors(3) == (T.NO_NEIGHBOR,) * 4


def test_cart_rows_and_explicit():
    assert (T.Cart.create(8, "rows").px, T.Cart.create(8, "rows").py) == (8, 1)
    c = T.Cart.create(6, px=1, py=6)
    assert (c.px, c.py) == (1, 6)
    with pytest.raises(ValueError):
        T.Cart.create(6, px=4, py=2)


def test_blocks_tile_the_grid():
    nx, ny = 37, 53
    for world, decomp in [(1, "auto"), (4, "auto"), (6, "auto"), (5, "rows"), (8, "2d")]:
        c = T.Cart.create(world, decomp, nx=nx, ny=ny)
        covered = [[0] * ny for _ in range(nx)]
        for r in range(world):
            b = c.block(r, nx, ny)
            for i in range(b.ox, b.ox + b.lx):
                for j in range(b.oy, b.oy + b.ly):
                    covered[i][j] += 1
        assert all(v == 1 for row in covered for v in row)


@pytest.mark.parametrize("lx,ly,h", [(20, 20, 1), (1024, 8192, 8), (7, 5, 3), (100, 333, 16)])
def test_layout_python_matches_native(lx, ly, h):
    p, r, hx, hy = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
    _native.call("heat_layout", lx, ly, h, ctypes.byref(p), ctypes.byref(r), ctypes.byref(hx),
                 ctypes.byref(hy))
    assert T.layout(lx, ly, h) == (p.value, r.value, hx.value, hy.value)
    pitch, rows, hx_, hy_ = T.layout(lx, ly, h)
    assert pitch % 64 == 0 and hy_ % 4 == 0 and hy_ >= h
    assert pitch >= 2 * hy_ + ly + 256


def test_memory_plan_131072_fits_288gb():
    plan = T.memory_plan(131072, 131072, 8, "auto", halo=8)
    assert plan["process_grid"] == (4, 2)
    assert plan["fits_288gb"]
    assert 17e9 < plan["bytes_per_gpu"] < 18e9
