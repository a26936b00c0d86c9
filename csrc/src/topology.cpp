// Process topology / decomposition (see topology.hpp for the reference map).
#include "heat/plan.hpp"
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

Box span_box(const Cart& cart, const Block& b, int depth, int m) {
  const int64_t gr = cart.px > 1 ? int64_t(m - 1) * depth : 0;
  const int64_t gc = cart.py > 1 ? round_down(int64_t(m - 1) * depth, 4) : 0;
  return Box{b.nbr[North] >= 0 ? -gr : 0, b.lx + (b.nbr[South] >= 0 ? gr : 0),
             b.nbr[West] >= 0 ? -gc : 0, b.ly + (b.nbr[East] >= 0 ? gc : 0)};
}

int resident_halo_passes(const Cart& cart, int64_t nx, int64_t ny, int depth, int mmax,
                         const std::function<int(const Box&)>& shape) {
  if (cart.world < 2 || depth < 1) return 0;
  std::vector<Block> blocks;
  std::vector<int> own;
  int64_t min_ext = INT64_MAX;
  for (int r = 0; r < cart.world; ++r) {
    blocks.push_back(make_block(cart, r, nx, ny));
    const Block& b = blocks.back();
    own.push_back(shape(Box{0, b.lx, 0, b.ly}));
    if (own.back() == 0) return 0;
    if (cart.px > 1) min_ext = std::min(min_ext, b.lx);
    if (cart.py > 1) min_ext = std::min(min_ext, b.ly);
  }
  for (int m = int(std::min<int64_t>(mmax, min_ext / depth)); m >= 2; --m) {
    bool ok = true;
    for (size_t i = 0; i < blocks.size() && ok; ++i)
      ok = shape(span_box(cart, blocks[i], depth, m)) == own[i];
    if (ok) return m;
  }
  return 0;
}

int resident_shape_static(const Box& box, int depth, int cus) {
  // (rows per wave, waves per workgroup, workgroups per CU), plan_res's order.
  static constexpr int kShapes[][3] = {{12, 8, 2}, {13, 8, 2}, {14, 8, 2}, {16, 8, 2},
                                       {20, 8, 1}, {24, 8, 1}, {12, 16, 1}, {20, 16, 1}};
  if (box.empty() || depth < 4 || depth % 2 != 0 || box.c0 % 4 != 0) return 0;
  const int64_t W = 256 - 2 * round_up(int64_t(depth), 4);
  // tb_tile.hpp tile_step_estimate: waves per SIMD of the busiest CU x rows.
  auto estimate = [&](int64_t units, int occ, int rows, int waves) {
    const int64_t cap = int64_t(cus) * occ, full = (units - 1) / cap;
    const int64_t busiest = (units - full * cap + cus - 1) / cus;
    auto cost = [&](int64_t tiles) {
      const double wps = double(tiles * waves) / 4.0;
      return wps * rows * (wps >= 4.0 ? 2.7 : 3.1);
    };
    return double(full) * cost(occ) + cost(busiest);
  };
  int best = 0;
  double best_est = 0.0;
  int64_t best_hmax = 0;
  for (const auto& s : kShapes) {
    const int64_t hmax = int64_t(s[0]) * s[1] - 2 * int64_t(depth);
    if (hmax < std::max(depth, 4)) continue;
    const int64_t units = ceil_div(box.cols(), W) * ceil_div(box.rows(), hmax);
    if (units > int64_t(cus) * s[2]) continue;
    const double est = estimate(units, s[2], s[0], s[1]);
    if (best == 0 || est < best_est) {
      best = res_shape(s[0], s[1]);
      best_est = est;
      best_hmax = hmax;
    }
  }
  // tb_resident_fits: every tile but the last of a strip at least K rows.
  if (best != 0 && ceil_div(box.rows(), ceil_div(box.rows(), best_hmax)) < depth) return 0;
  return best;
}

}  // namespace heat
