// Process topology / decomposition (see topology.hpp for the reference map).
#include "heat/topology.hpp"

#include <algorithm>
#include <cmath>

#include "heat/common.hpp"

namespace heat {

std::vector<int> dims_create(int nnodes, int ndims) {
  HEAT_CHECK(nnodes >= 1 && ndims >= 1, "nnodes=%d ndims=%d", nnodes, ndims);
  std::vector<int> dims(ndims, 1);
  if (ndims == 1) {
    dims[0] = nnodes;
    return dims;
  }
  if (ndims == 2) {
    // Most balanced split: the largest divisor d <= sqrt(n) gives [n/d, d].
    int d = int(std::sqrt(double(nnodes)));
    while (d > 1 && nnodes % d != 0) --d;
    dims[0] = nnodes / d;
    dims[1] = d;
    return dims;
  }
  // General case: largest prime factors first, each to the smallest dim.
  std::vector<int> primes;
  int n = nnodes;
  for (int p = 2; int64_t(p) * p <= n; ++p)
    while (n % p == 0) { primes.push_back(p); n /= p; }
  if (n > 1) primes.push_back(n);
  std::sort(primes.rbegin(), primes.rend());
  for (int p : primes) *std::min_element(dims.begin(), dims.end()) *= p;
  std::sort(dims.rbegin(), dims.rend());
  return dims;
}

Cart::Cart(int world_size, DecompKind kind, int px_req, int py_req, int64_t nx, int64_t ny)
    : world(world_size) {
  HEAT_CHECK(world_size >= 1, "world size %d", world_size);
  if (px_req > 0 || py_req > 0) {
    if (px_req <= 0) px_req = world_size / py_req;
    if (py_req <= 0) py_req = world_size / px_req;
    HEAT_CHECK(int64_t(px_req) * py_req == world_size,
               "process grid %dx%d does not match world size %d", px_req, py_req, world_size);
    px = px_req;
    py = py_req;
  } else if (kind == DecompKind::Rows) {
    px = world_size;
    py = 1;
  } else {
    auto d = dims_create(world_size, 2);
    px = d[0];
    py = d[1];
  }
  HEAT_CHECK(px <= nx && py <= ny, "process grid %dx%d larger than grid %lldx%lld", px, py,
             (long long)nx, (long long)ny);
}

int Cart::rank_of(int cx, int cy) const {
  if (cx < 0 || cx >= px || cy < 0 || cy >= py) return kNoNeighbor;
  return cx * py + cy;
}

std::array<int, 4> Cart::neighbors(int rank) const {
  auto c = coords(rank);
  std::array<int, 4> n{};
  n[North] = rank_of(c[0] - 1, c[1]);
  n[South] = rank_of(c[0] + 1, c[1]);
  n[West] = rank_of(c[0], c[1] - 1);
  n[East] = rank_of(c[0], c[1] + 1);
  return n;
}

std::array<int, 4> Cart::diagonal_neighbors(int rank) const {
  auto c = coords(rank);
  std::array<int, 4> n{};
  n[NorthWest] = rank_of(c[0] - 1, c[1] - 1);
  n[NorthEast] = rank_of(c[0] - 1, c[1] + 1);
  n[SouthWest] = rank_of(c[0] + 1, c[1] - 1);
  n[SouthEast] = rank_of(c[0] + 1, c[1] + 1);
  return n;
}

Span block_span(int64_t n, int parts, int index) {
  HEAT_CHECK(parts >= 1 && index >= 0 && index < parts, "parts=%d index=%d", parts, index);
  const int64_t base = n / parts, rem = n % parts;
  Span s;
  s.size = base + (index < rem ? 1 : 0);
  s.offset = index * base + std::min<int64_t>(index, rem);
  return s;
}

Block make_block(const Cart& cart, int rank, int64_t nx, int64_t ny) {
  HEAT_CHECK(rank >= 0 && rank < cart.world, "rank %d of %d", rank, cart.world);
  Block b;
  b.rank = rank;
  auto c = cart.coords(rank);
  b.cx = c[0];
  b.cy = c[1];
  auto sx = block_span(nx, cart.px, b.cx);
  auto sy = block_span(ny, cart.py, b.cy);
  b.ox = sx.offset;
  b.lx = sx.size;
  b.oy = sy.offset;
  b.ly = sy.size;
  b.nbr = cart.neighbors(rank);
  b.diag = cart.diagonal_neighbors(rank);
  return b;
}

Layout Layout::make(int64_t lx, int64_t ly, int halo) {
  HEAT_CHECK(lx >= 1 && ly >= 1 && halo >= 1, "lx=%lld ly=%lld halo=%d", (long long)lx,
             (long long)ly, halo);
  Layout L;
  L.lx = lx;
  L.ly = ly;
  L.hx = halo;
  L.hy = int(round_up(halo, 4));  // keeps owned column 0 16-B aligned
  // Left ghost + owned + right ghost, plus one full 256-column strip of slack
  // for the TB kernel's last strip, rounded to 256 B.
  L.pitch = round_up(L.hy + ly + L.hy + 256, 64);
  L.rows = lx + 2 * int64_t(halo);
  return L;
}

}  // namespace heat
