// Workgroup-tile temporally blocked Jacobi kernel (variant bit kTile).
//
// The register-streaming kernel (tb_stream.inl) gives every wave its own
// (strip, chunk) and pays the trapezoid of classic temporal blocking: each
// chunk recomputes K - l rows beyond both of its ends at level l.  On the
// per-rank blocks of 4-8 GPU runs (1024 x 8192, 2048 x 4096: 36 strip-rows per
// SIMD) that is 1.30x the useful row updates, and there is only room for one
// wave per SIMD, which issues a VALU op every ~4-6 cycles instead of ~2-3
// (profiles/r3_small_blocks.md).
//
// Here a workgroup of NW = 8 (or 16) waves owns one tile: a 256-column strip
// (64 lanes x float4) by NW * R rows, every wave R consecutive rows held in
// VGPRs for the whole launch.  A time step updates all rows in place; the
// only data a wave needs from outside its registers are the last row of the
// wave above and the first row of the wave below, exchanged through LDS (one
// barrier per step, halfway through it, see tile_run).  The tile pays its
// own K-deep ghost ring (2K of NW * R rows, round_up(K, 4) columns per side)
// instead of a trapezoid per wave -- about the same VALU work -- but runs
// 2-4 waves per SIMD (two workgroups per CU up to R = 16) where the
// streaming kernel has room for one (profiles/r3_tile.md).  East/west
// neighbours cross lanes with DPP wave shifts and / or ds_bpermute (XL).
//
// Input rows [r0 - K, r1 + K) and columns [c0 - round_up(K, 4), ...) of each
// box are read (the same footprint as tb_stream.inl); rows of the tile past
// that range load a clamped (valid, don't-care) row: their values only reach
// rows outside the useful range within K steps.  The update is heat::stencil,
// so results are bitwise identical to every other kernel.
//
// Reference kernel this replaces: cuda/cuda_heat.cu:140-163 (one step per
// launch, global memory) and :42-138 (the fused residual).
#include "tb_tile.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <tuple>

#include "heat/common.hpp"

namespace heat::gpu::tbw {

using tbdetail::TbArgs;
using tbdetail::TbBox;

namespace {
bool launch_xl(const TbArgs& args, int depth, int rows, int waves, int xl, hipStream_t st) {
  if (depth < 2 || depth % 2 != 0 || waves * rows <= 2 * depth) return false;
  return xl == 1 ? tile_launch_x1(args, depth, rows, waves, st)
         : xl == 2 ? tile_launch_x2(args, depth, rows, waves, st)
                   : tile_launch_x0(args, depth, rows, waves, st);
}

int occupancy_xl(int rows, int waves, int xl) {
  return xl == 1 ? tile_occupancy_x1(rows, waves)
         : xl == 2 ? tile_occupancy_x2(rows, waves)
                   : tile_occupancy_x0(rows, waves);
}
}  // namespace

bool launch(const TbArgs& args, int depth, int rows, int waves, bool bpermute, hipStream_t st) {
  return launch_xl(args, depth, rows, waves, bpermute ? 1 : 0, st);
}

int occupancy(int rows, int waves, bool bpermute) { return occupancy_xl(rows, waves, bpermute ? 1 : 0); }

namespace {
bool trace_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT_TB_TRACE");
    return e && *e && *e != '0';
  }();
  return on;
}
void trace_once(const std::string& line) {
  static std::mutex mu;
  static std::set<std::string> seen;
  std::lock_guard<std::mutex> lk(mu);
  if (seen.insert(line).second) std::fputs(line.c_str(), stderr);
}
// Resident blocks per CU, cached per (device, rows, waves, shifts).
int cached_occupancy(int rows, int waves, int bp) {
  static std::map<std::tuple<int, int, int, int>, int> cache;
  static std::mutex mu;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_tuple(dev, rows, waves, bp);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  return cache.emplace(key, occupancy_xl(rows, waves, bp)).first->second;
}
}  // namespace

// The launch planner.  A tile is one 256-column strip by NW waves x R rows;
// its useful rows are NW * R - 2 * depth.  The shape comes from the
// instantiated set by the estimated time of the launch: dispatch rounds x
// (rows each SIMD updates per round) x (relative cycles per VALU op: 2.7
// with two or more independent workgroups per CU, 3.1 with one, whose waves
// stall together at its barriers; calibrated on the 8-GPU blocks,
// profiles/r3_tile.md).
void step(const float* src, float* dst, const StencilGeom& g, const Box* boxes, int nbox, int depth,
          unsigned* resid, int res_level, hipStream_t st, int variant, const TbTuning& tune) {
  struct Shape {
    int rows, waves;
  };
  static constexpr Shape kShapes[] = {{12, 8}, {13, 8}, {14, 8}, {16, 8}, {20, 8}, {24, 8}, {28, 8}, {32, 8}, {12, 16}, {20, 16}};
  // Lane shifts: mixed (2: the left shift a DPP wave shift folded into the
  // add, the right one ds_bpermute issued ahead; +3-6 % over ds_bpermute for
  // both, which waited on LDS issue 13 % of the time, profiles/r3_tile.md)
  // unless the variant asks for DPP (0); TbTuning::tile_xl (HEAT_TB_TILE_XL)
  // 0/1/2 overrides.
  const int bp = tune.tile_xl >= 0 && tune.tile_xl <= 2 ? tune.tile_xl : (variant & tbv::kTileDpp) ? 0 : 2;
  const int W = tb_strip_width(depth, 4);
  const int cus = tb_simd_count() / 4;
  Shape best{0, 0};
  double best_est = 0.0;
  for (const Shape& sh : kShapes) {
    if (tune.tile_rows > 0 && sh.rows != tune.tile_rows) continue;
    if (tune.tile_waves > 0 && sh.waves != tune.tile_waves) continue;
    const int64_t hmax = int64_t(sh.waves) * sh.rows - 2 * int64_t(depth);
    if (hmax < std::max(depth, 4)) continue;
    int64_t units = 0;
    for (int b = 0; b < nbox; ++b)
      if (!boxes[b].empty()) units += ceil_div(boxes[b].cols(), W) * ceil_div(boxes[b].rows(), hmax);
    const int occ = cached_occupancy(sh.rows, sh.waves, bp);
    if (occ <= 0) continue;
    const double est = tile_step_estimate(units, cus, occ, sh.rows, sh.waves);
    if (best.rows == 0 || est < best_est) {
      best_est = est;
      best = sh;
    }
  }
  HEAT_CHECK(best.rows > 0, "no tile shape fits depth %d (HEAT_TB_TILE_ROWS=%d, HEAT_TB_TILE_WAVES=%d)",
             depth, tune.tile_rows, tune.tile_waves);
  const int64_t hmax = int64_t(best.waves) * best.rows - 2 * int64_t(depth);
  TbArgs args{};
  args.src = src;
  args.dst = dst;
  args.resid = resid;
  args.res_level = res_level > 0 && res_level < depth ? res_level : depth;
  args.g = g;
  args.flags = (variant & tbv::kXcdGroups) ? tbdetail::kTbXcdGroups : 0;
  int n = 0;
  int64_t units = 0;
  for (int b = 0; b < nbox; ++b) {
    const Box& B = boxes[b];
    if (B.empty()) continue;
    HEAT_CHECK(B.c0 % 4 == 0, "TB box column start %lld not a multiple of 4", (long long)B.c0);
    HEAT_CHECK(n < tbdetail::kMaxBoxes, "too many TB boxes");
    TbBox& t = args.box[n++];
    t.r0 = B.r0;
    t.r1 = B.r1;
    t.c0 = B.c0;
    t.c1 = B.c1;
    t.nstrips = int(ceil_div(B.cols(), W));
    t.nchunks = int(ceil_div(B.rows(), hmax));                 // tiles per strip
    t.chunk_len = int(ceil_div(B.rows(), int64_t(t.nchunks)));  // useful rows per tile
    t.wave_begin = int(units);                                  // first unit (block)
    units += int64_t(t.nstrips) * t.nchunks;
  }
  if (n == 0) return;
  HEAT_CHECK(units < (int64_t(1) << 31), "tile launch too large");
  args.nbox = n;
  args.total_waves = int(units);
  if (trace_enabled()) {
    char line[200];
    std::snprintf(line, sizeof line,
                  "[heat tb] tile depth %d rows %d waves %d bpermute %d boxes %d units %lld tiles0 %d "
                  "len0 %d\n",
                  depth, best.rows, best.waves, int(bp), n, (long long)units, args.box[0].nchunks,
                  args.box[0].chunk_len);
    trace_once(line);
  }
  HEAT_CHECK(launch_xl(args, depth, best.rows, best.waves, bp, st), "tile %dx%d not instantiated",
             best.rows, best.waves);
  HIP_CHECK(hipGetLastError());
}

}  // namespace heat::gpu::tbw
