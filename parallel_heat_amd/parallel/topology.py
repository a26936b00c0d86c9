"""Process topology and block decomposition (Python mirror of csrc/src/topology.cpp).

Reference: ``MPI_Dims_create`` / ``MPI_Cart_create`` / ``MPI_Cart_shift`` and the
block sizes at ``mpi/mpi_heat_improved_persistent_stat.c:51-75``.  Unlike the
reference, remainders are distributed and each rank owns only its
block (Q13).  The native engine is the source of truth; this mirror is used
for planning (memory sizing, message sizes) and is tested against it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Tuple

NO_NEIGHBOR = -1
NORTH, SOUTH, WEST, EAST = 0, 1, 2, 3


def dims_create(nnodes: int, ndims: int = 2) -> List[int]:
    """Balanced non-increasing factorisation, as MPI_Dims_create with free dims."""
    if nnodes < 1 or ndims < 1:
        raise ValueError("nnodes and ndims must be >= 1")
    if ndims == 1:
        return [nnodes]
    if ndims == 2:
        d = int(math.isqrt(nnodes))
        while d > 1 and nnodes % d:
            d -= 1
        return [nnodes // d, d]
    primes, n, p = [], nnodes, 2
    while p * p <= n:
        while n % p == 0:
            primes.append(p)
            n //= p
        p += 1
    if n > 1:
        primes.append(n)
    dims = [1] * ndims
    for q in sorted(primes, reverse=True):
        i = dims.index(min(dims))
        dims[i] *= q
    return sorted(dims, reverse=True)


def block_span(n: int, parts: int, index: int) -> Tuple[int, int]:
    """(offset, size) of part `index` of n split into `parts` (remainder first)."""
    base, rem = divmod(n, parts)
    size = base + (1 if index < rem else 0)
    return index * base + min(index, rem), size


@dataclass
class Block:
    rank: int
    cx: int
    cy: int
    ox: int
    oy: int
    lx: int
    ly: int
    nbr: Tuple[int, int, int, int] = field(default=(NO_NEIGHBOR,) * 4)


@dataclass
class Cart:
    world: int
    px: int
    py: int

    @classmethod
    def create(cls, world: int, decomp: str = "auto", px: int = 0, py: int = 0,
               nx: int = 1 << 62, ny: int = 1 << 62) -> "Cart":
        if px > 0 or py > 0:
            px = px if px > 0 else world // py
            py = py if py > 0 else world // px
            if px * py != world:
                raise ValueError(f"process grid {px}x{py} != world {world}")
        elif decomp in ("rows", "1d"):
            px, py = world, 1
        else:
            px, py = dims_create(world, 2)
        if px > nx or py > ny:
            raise ValueError(f"process grid {px}x{py} larger than grid {nx}x{ny}")
        return cls(world, px, py)

    def coords(self, rank: int) -> Tuple[int, int]:
        return rank // self.py, rank % self.py

    def rank_of(self, cx: int, cy: int) -> int:
        if 0 <= cx < self.px and 0 <= cy < self.py:
            return cx * self.py + cy
        return NO_NEIGHBOR

    def neighbors(self, rank: int) -> Tuple[int, int, int, int]:
        cx, cy = self.coords(rank)
        return (self.rank_of(cx - 1, cy), self.rank_of(cx + 1, cy),
                self.rank_of(cx, cy - 1), self.rank_of(cx, cy + 1))

    def diagonal_neighbors(self, rank: int) -> Tuple[int, int, int, int]:
        """(NW, NE, SW, SE): the owners of the ghost corners of deep halos
        (heat::Cart::diagonal_neighbors)."""
        cx, cy = self.coords(rank)
        return (self.rank_of(cx - 1, cy - 1), self.rank_of(cx - 1, cy + 1),
                self.rank_of(cx + 1, cy - 1), self.rank_of(cx + 1, cy + 1))

    def block(self, rank: int, nx: int, ny: int) -> Block:
        cx, cy = self.coords(rank)
        ox, lx = block_span(nx, self.px, cx)
        oy, ly = block_span(ny, self.py, cy)
        return Block(rank, cx, cy, ox, oy, lx, ly, self.neighbors(rank))


def layout(lx: int, ly: int, halo: int) -> Tuple[int, int, int, int]:
    """(pitch, rows, hx, hy) of a local field, as heat::Layout::make."""
    hy = -(-halo // 4) * 4
    pitch = -(-(hy + ly + hy + 256) // 64) * 64
    return pitch, lx + 2 * halo, halo, hy


def memory_plan(nx: int, ny: int, world: int, decomp: str = "auto", halo: int = 8,
                px: int = 0, py: int = 0) -> dict:
    """Bytes per GPU for the two fields of the largest block (288 GB HBM3E sizing)."""
    cart = Cart.create(world, decomp, px, py, nx, ny)
    worst = 0
    for r in range(world):
        b = cart.block(r, nx, ny)
        pitch, rows, _, _ = layout(b.lx, b.ly, halo)
        worst = max(worst, 2 * pitch * rows * 4)
    halo_rows = max(cart.block(r, nx, ny).ly for r in range(world))
    return {
        "process_grid": (cart.px, cart.py),
        "bytes_per_gpu": worst,
        "gb_per_gpu": worst / 1e9,
        "fits_288gb": worst < 288e9 * 0.95,
        "ns_halo_bytes": halo * (layout(1, halo_rows, halo)[0]) * 4,
    }
