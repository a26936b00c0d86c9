// Resident workgroup tiles: the tile kernel (tb_tile.hip) with each tile kept
// in VGPRs across the P passes of one launch.
//
// A tile pass of the 8-GPU per-rank blocks costs ~11 us fixed plus ~1.7 us
// per step (profiles/r3_tile.md): every pass relaunches, and every tile
// reloads its whole 8R-row footprint at once (48 MB per pass at 1024 x 8192)
// before any step can start.  Here the grid is one dispatch round (every
// tile co-resident, checked on the host) and stays for P passes:
//
//   pass 0      load the tile from src, as tb_tile.hip does;
//   pass p      K steps in registers; the last step publishes the tile's
//               useful EDGE BANDS (K rows at the top and bottom, KK columns
//               at the left and right of its useful region) into exchange
//               field xb[p & 1] with write-through (sc1) stores, then every
//               wave drains (vmcnt 0), the workgroup barrier, and one lane
//               stores flag[tile] = p + 1 (agent-scope, sc1);
//   pass p + 1  wave 0 polls the flags of the <= 8 neighbour tiles (relaxed
//               sc1 loads, bounded spin) until they reach p + 1, the barrier
//               releases the other waves, and each wave reloads only its
//               GHOST cells -- the K-deep ring around the useful region,
//               which is exactly the neighbours' edge bands -- from
//               xb[p & 1] with sc1 loads (MI355X_MICROARCH.md "Valid forms",
//               first row: sc1 payload both sides, no acquire fence);
//   last pass   stores the useful region to dst, like tb_tile.hip.
//
// Ghost cells outside the launch's box are not reloaded (their registers are
// don't-care, as clamped rows are in tb_tile.hip): on deep-halo blocks the
// invalid region grows from the box edge by K per pass exactly as the
// shrinking boxes of separate passes do (Solver::enqueue_resident).
// Double-buffered exchange fields make the protocol race-free: a tile
// rewrites xb[p & 1] at the end of pass p + 2 only after it has seen every
// neighbour's flag p + 2, i.e. after every neighbour finished the pass p + 1
// that read it.  Flags and the completion counter are zero at every launch:
// zeroed once when the buffers are allocated, then re-zeroed by the tile that
// finishes last (the completion counter tells it; every other tile is past
// its last poll by then), in place of a memset node per launch
// (cdna_hip_programming.md Guideline 16, "Re-initialise every call"); every
// spin is bounded and reports through *err instead of hanging the device.
//
// Results are bitwise those of separate passes (heat::stencil, the same
// Tile code).  Reference: the per-rank compute of
// mpi/mpi_heat_improved_persistent_stat.c:162-234, which this replaces.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>

#include "heat/common.hpp"
#include "heat/plan.hpp"
#include "tb_resident_kern.hpp"

namespace heat::gpu::tbw {

// The lane-shift builds (tb_resident_xl<XL>.hip, compiled in parallel).
bool res_launch_x0(const ResArgs& ra, int rows, int waves, int blocks, hipStream_t st);
bool res_launch_x1(const ResArgs& ra, int rows, int waves, int blocks, hipStream_t st);
bool res_launch_x2(const ResArgs& ra, int rows, int waves, int blocks, hipStream_t st);
int res_occupancy_x0(int rows, int waves);
int res_occupancy_x1(int rows, int waves);
int res_occupancy_x2(int rows, int waves);

namespace {
int occupancy_res(int rows, int waves, int xl) {
  return xl == 1 ? res_occupancy_x1(rows, waves)
         : xl == 2 ? res_occupancy_x2(rows, waves)
                   : res_occupancy_x0(rows, waves);
}

bool launch_res(const ResArgs& ra, int rows, int waves, int xl, int blocks, hipStream_t st) {
  return xl == 1 ? res_launch_x1(ra, rows, waves, blocks, st)
         : xl == 2 ? res_launch_x2(ra, rows, waves, blocks, st)
                   : res_launch_x0(ra, rows, waves, blocks, st);
}

int cached_occupancy_res(int rows, int waves, int xl) {
  static std::map<std::tuple<int, int, int, int>, int> cache;
  static std::mutex mu;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_tuple(dev, rows, waves, xl);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  return cache.emplace(key, occupancy_res(rows, waves, xl)).first->second;
}

struct ResPlan {
  int rows = 0, waves = 0, units = 0;
};

int res_xl(int variant, const TbTuning& tune) {
  // Mixed lane shifts unless a forced variant asks for DPP (variant -1 is the
  // automatic choice, not "every flag": it ran the all-DPP build, 11 % slower
  // than ds_bpermute shifts on 1024 x 8192, profiles/r4_resident.md).
  if (tune.tile_xl >= 0 && tune.tile_xl <= 2) return tune.tile_xl;
  return variant >= 0 && (variant & tbv::kTileDpp) ? 0 : 2;
}

// The shape with the lowest step estimate (tile_step_estimate) among those
// whose tiles are all co-resident (one dispatch round; the occupancy of the
// resident instantiation itself, bounded by its VGPR granule).
ResPlan plan_res(const Box& box, int depth, int xl, const TbTuning& tune) {
  ResPlan best;
  if (box.empty() || depth < 4 || depth % 2 != 0 || box.c0 % 4 != 0) return best;
  const int W = tb_strip_width(depth, 4);
  const int cus = tb_simd_count() / 4;
  double best_est = 0.0;
  struct Shape {
    int rows, waves;
  };
  static constexpr Shape kShapes[] = {{12, 8}, {13, 8}, {14, 8}, {16, 8}, {20, 8}, {24, 8}, {12, 16}, {20, 16}};
  for (const Shape& sh : kShapes) {
    if (tune.tile_rows > 0 && sh.rows != tune.tile_rows) continue;
    if (tune.tile_waves > 0 && sh.waves != tune.tile_waves) continue;
    const int64_t hmax = int64_t(sh.waves) * sh.rows - 2 * int64_t(depth);
    if (hmax < std::max(depth, 4)) continue;
    const int64_t units = ceil_div(box.cols(), W) * ceil_div(box.rows(), hmax);
    const int occ = cached_occupancy_res(sh.rows, sh.waves, xl);
    if (occ <= 0 || units > int64_t(cus) * occ) continue;
    const double est = tile_step_estimate(units, cus, occ, sh.rows, sh.waves);
    if (best.rows == 0 || est < best_est) {
      best_est = est;
      best = ResPlan{sh.rows, sh.waves, int(units)};
    }
  }
  return best;
}
}  // namespace

}  // namespace heat::gpu::tbw

namespace heat::gpu {

bool tb_resident_fits(const Box& box, int depth, int variant) {
  using namespace tbw;
  const TbTuning tune = tb_tuning();
  const ResPlan pl = plan_res(box, depth, res_xl(variant, tune), tune);
  if (pl.rows == 0) return false;
  // Every tile but the last of a strip (and every strip but the last) must
  // be at least K rows (KK columns) deep: a ghost ring comes from the
  // direct neighbours only.
  const int64_t hmax = int64_t(pl.waves) * pl.rows - 2 * int64_t(depth);
  const int64_t n = ceil_div(box.rows(), hmax);
  return ceil_div(box.rows(), n) >= depth;
}

int tb_resident_shape(const Box& box, int depth, int variant) {
  using namespace tbw;
  const TbTuning tune = tb_tuning();
  const ResPlan pl = plan_res(box, depth, res_xl(variant, tune), tune);
  if (pl.rows == 0) return 0;
  const int64_t hmax = int64_t(pl.waves) * pl.rows - 2 * int64_t(depth);
  if (ceil_div(box.rows(), ceil_div(box.rows(), hmax)) < depth) return 0;
  return res_shape(pl.rows, pl.waves);
}

void tb_resident_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
                      int depth, int passes, const TbResidentBuffers& xb, hipStream_t st,
                      int variant, const TbResidentCheck* checks, int nchecks, unsigned* resids,
                      int64_t own_rows, int64_t own_cols) {
  using namespace tbw;
  HEAT_CHECK(passes >= 2, "a resident launch spans >= 2 passes (%d)", passes);
  const TbTuning tune = tb_tuning();
  int xl = res_xl(variant, tune);
  const ResPlan pl = plan_res(box, depth, xl, tune);
  HEAT_CHECK(pl.rows > 0, "resident tiles do not fit box %lldx%lld at depth %d",
             (long long)box.rows(), (long long)box.cols(), depth);
  HEAT_CHECK(pl.units <= xb.max_tiles, "%d resident tiles, flag buffer holds %d", pl.units,
             xb.max_tiles);
  HEAT_CHECK(xb.bytes < (int64_t(1) << 31), "exchange field of %lld bytes (32-bit offsets)",
             (long long)xb.bytes);
  const int64_t hmax = int64_t(pl.waves) * pl.rows - 2 * int64_t(depth);
  ResArgs ra{};
  TbArgs& a = ra.a;
  a.src = src;
  a.dst = dst;
  HEAT_CHECK(nchecks >= 0 && nchecks <= kResMaxChecks && (nchecks == 0 || resids != nullptr),
             "%d checks in a resident launch (at most %d)", nchecks, kResMaxChecks);
  for (int c = 0; c < nchecks; ++c) {
    HEAT_CHECK(checks[c].pass >= 0 && checks[c].pass < passes && checks[c].step >= 2 &&
                   checks[c].step <= depth && checks[c].step % 2 == 0 &&
                   (c == 0 || checks[c].pass > checks[c - 1].pass),
               "resident check %d at pass %d step %d (passes %d, depth %d)", c, checks[c].pass,
               checks[c].step, passes, depth);
    ra.chk_pass[c] = checks[c].pass;
    ra.chk_step[c] = checks[c].step;
  }
  ra.nchk = nchecks;
  ra.resids = resids;
  a.resid = nchecks > 0 ? resids : nullptr;  // selects the RES 1 instantiation
  // Timing diagnostic: the RES 1 build without checks (what the residual
  // instantiation costs by itself, profiles/r5_resident_checks.md).
  static const bool diag_res1 = [] {
    const char* e = std::getenv("HEAT_TB_RES_DIAG_RES1");
    return e && *e && *e != '0';
  }();
  if (diag_res1 && resids) a.resid = resids;
  // Lane shifts: the shape is planned with the mixed shifts (XL 2); a
  // packed-update launch (rows <= kTilePkRows, checked or not) then runs with
  // DPP shifts for both neighbours (XL 0), the packed update's best partner
  // (tools/probes/stencil_chain.hip: packed + DPP 65 vs 73 cycles per row
  // update; 1168 x 8192 plate 4.90 vs 4.62 Tcells/s, 2192 x 4168 4.54 vs
  // 4.43, profiles/r6_raw/r6h/; checks every 20 steps on 1024 x 8192 4.01
  // vs 3.80, r6l; unchecked launches have the left / element-3 right edge
  // modes, tile_dispatch).  The round-4 all-DPP build was 11 % slower with
  // the scalar update, which the taller tiles keep.
  if (variant < 0 && tune.tile_xl < 0 && pl.rows <= kTilePkRows &&
      cached_occupancy_res(pl.rows, pl.waves, 0) >= cached_occupancy_res(pl.rows, pl.waves, xl))
    xl = 0;
  a.res_level = depth;
  a.g = g;
  a.flags = (variant < 0 || (variant & tbv::kXcdGroups)) ? tbdetail::kTbXcdGroups : 0;
  TbBox& t = a.box[0];
  t.r0 = box.r0;
  t.r1 = box.r1;
  t.c0 = box.c0;
  t.c1 = box.c1;
  t.nstrips = int(ceil_div(box.cols(), tb_strip_width(depth, 4)));
  t.nchunks = int(ceil_div(box.rows(), hmax));
  t.chunk_len = int(ceil_div(box.rows(), int64_t(t.nchunks)));
  HEAT_CHECK(t.chunk_len >= depth, "resident tiles of %d rows at depth %d", t.chunk_len, depth);
  t.wave_begin = 0;
  a.nbox = 1;
  a.total_waves = t.nstrips * t.nchunks;
  HEAT_CHECK(a.total_waves == pl.units, "resident plan %d != %d tiles", pl.units, a.total_waves);
  ra.passes = passes;
  ra.depth = depth;
  ra.xbase[0] = xb.base[0];
  ra.xbase[1] = xb.base[1];
  ra.xorigin = xb.origin;
  ra.xbytes = int(xb.bytes);
  HEAT_CHECK(xb.done != nullptr, "resident launch without a completion counter");
  ra.flags = xb.flags;
  ra.done = xb.done;
  ra.err = xb.err;
  ra.own_r1 = nchecks > 0 ? own_rows : box.r1;
  ra.own_c1 = nchecks > 0 ? own_cols : box.c1;
  ra.diag = tune.res_diag;
  // The flags and the completion counter are zero: zeroed once when the
  // buffers are allocated, then by the last tile of every launch.
  if (const char* e = std::getenv("HEAT_TB_TRACE"); e && *e && *e != '0') {
    static std::mutex mu;
    static std::set<std::string> seen;
    char line[200];
    std::snprintf(line, sizeof line, "[heat tb] resident depth %d passes %d rows %d waves %d xl %d tiles %d\n",
                  depth, passes, pl.rows, pl.waves, xl, pl.units);
    std::lock_guard<std::mutex> lk(mu);
    if (seen.insert(line).second) std::fputs(line, stderr);
  }
  HEAT_CHECK(launch_res(ra, pl.rows, pl.waves, xl, pl.units, st), "resident %dx%d not built",
             pl.rows, pl.waves);
  HIP_CHECK(hipGetLastError());
}

}  // namespace heat::gpu
