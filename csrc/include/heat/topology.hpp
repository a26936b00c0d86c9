// Process topology and block decomposition.
//
// Replaces the reference's MPI Cartesian topology (MPI_Dims_create /
// MPI_Cart_create / MPI_Cart_coords / MPI_Cart_shift,
// mpi/mpi_heat_improved_persistent_stat.c:51-69) and its block sizes
// (mpi/...c:71-75).  Differences by design:
//   * remainders are distributed (the reference silently drops cells when
//     NX or NY is not divisible by the process grid);
//   * every rank allocates only its own block plus a ghost ring
//     (the reference allocates the full global grid on every rank, Q13).
#pragma once

#include <array>
#include <cstdint>
#include <vector>

#include "heat/params.hpp"

namespace heat {

constexpr int kNoNeighbor = -1;  // MPI_PROC_NULL analogue

// Balanced factorisation of nnodes into ndims factors in non-increasing
// order, with the same results as MPI_Dims_create for fully free dims.
std::vector<int> dims_create(int nnodes, int ndims);

// Directions.  North/South are along x (rows, dim 0), West/East along y
// (columns, dim 1).  The reference names them north/south for dim 0 and
// east/west for dim 1 with east = coord-1 (mpi/...c:68-69); we use the
// geographic convention west = lower column index.
enum Dir : int { North = 0, South = 1, West = 2, East = 3 };
// Diagonal neighbours (2-D grids): the owners of the ghost corners that deep
// (k > 1) halos need.
enum Diag : int { NorthWest = 0, NorthEast = 1, SouthWest = 2, SouthEast = 3 };

struct Cart {
  int world = 1;
  int px = 1, py = 1;  // process-grid extents along x (rows) and y (columns)

  Cart() = default;
  Cart(int world_size, DecompKind kind, int px_req, int py_req, int64_t nx, int64_t ny);

  // Row-major rank order like MPI_Cart_create with reorder=0: rank = cx*py + cy.
  std::array<int, 2> coords(int rank) const { return {rank / py, rank % py}; }
  int rank_of(int cx, int cy) const;  // kNoNeighbor if outside (non-periodic)
  std::array<int, 4> neighbors(int rank) const;
  std::array<int, 4> diagonal_neighbors(int rank) const;
};

// 1-D block partition with remainder distribution: the first (n % p) parts
// get one extra element.
struct Span {
  int64_t offset = 0, size = 0;
};
Span block_span(int64_t n, int parts, int index);

// The block a rank owns, in global coordinates.
struct Block {
  int rank = 0;
  int cx = 0, cy = 0;
  int64_t ox = 0, oy = 0;  // global coordinates of the first owned cell
  int64_t lx = 0, ly = 0;  // owned extent
  std::array<int, 4> nbr{kNoNeighbor, kNoNeighbor, kNoNeighbor, kNoNeighbor};
  std::array<int, 4> diag{kNoNeighbor, kNoNeighbor, kNoNeighbor, kNoNeighbor};
};

Block make_block(const Cart& cart, int rank, int64_t nx, int64_t ny);

// Memory layout of one local field: owned block plus a ghost ring of
// `hx` rows and `hy` columns on every side, with the row pitch padded to a
// multiple of 64 floats (256 B) and extra right-hand padding so that the
// 256-column streaming strips of the TB kernel never read past the row.
struct Layout {
  int64_t lx = 0, ly = 0;
  int hx = 0, hy = 0;
  int64_t pitch = 0;  // floats per row
  int64_t rows = 0;   // allocated rows = lx + 2*hx

  static Layout make(int64_t lx, int64_t ly, int halo);
  int64_t elems() const { return rows * pitch; }
  int64_t bytes() const { return elems() * 4; }
  // Offset (in floats) of owned cell (0,0) from the allocation base.
  int64_t origin() const { return int64_t(hx) * pitch + hy; }
  // Offset of local cell (r, c); r and c may be negative (ghost ring).
  int64_t at(int64_t r, int64_t c) const { return origin() + r * pitch + c; }
};

// A rectangle of local cells, [r0, r1) x [c0, c1).
struct Box {
  int64_t r0 = 0, r1 = 0, c0 = 0, c1 = 0;
  int64_t rows() const { return r1 > r0 ? r1 - r0 : 0; }
  int64_t cols() const { return c1 > c0 ? c1 - c0 : 0; }
  bool empty() const { return rows() == 0 || cols() == 0; }
};

}  // namespace heat
