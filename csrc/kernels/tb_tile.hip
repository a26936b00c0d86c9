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
#include <type_traits>

#include "heat/common.hpp"
#include "tb_tile_core.hpp"

namespace heat::gpu::tbw {

template <int R, int NW, int MODE, int RES, int XL>
__device__ __forceinline__ float tile_run(const TbArgs& a, const TbBox& bx, int strip, int t, int K,
                                          vecf (*xch)[2][NW][64]) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const StencilGeom& g = a.g;
  const int KK = (K + 3) & ~3;
  const int64_t Wd = 256 - 2 * KK;
  const int64_t cbase = bx.c0 + int64_t(strip) * Wd;
  const int64_t cend = min(cbase + Wd, bx.c1);
  const int64_t col = cbase - KK + 4 * lane;
  const bool store_lane = col >= cbase && col < cend;
  const int rc = int(min<int64_t>(cend - col, 4));
  const int64_t ub = bx.r0 + int64_t(t) * bx.chunk_len;  // useful rows [ub, ue)
  const int64_t ue = min(ub + bx.chunk_len, bx.r1);
  const int64_t row0 = ub - K + int64_t(w) * R;         // this wave's first row
  const int64_t rmin = bx.r0 - K, rmax = bx.r1 + K - 1;  // readable rows
  const int64_t pitch = g.pitch;
  const float* __restrict__ src = a.src + (cbase - KK);  // wave-uniform; + 4*lane
  float* __restrict__ dst = a.dst + (cbase - KK);
  const int lo = 4 * lane;

  Tile<R, MODE, RES, XL> T;
  // Row offsets are made opaque (asm) so the compiler neither keeps R 64-bit
  // row offsets alive from the loads to the stores (CSE) nor hoists per-row
  // masks out of the step loop: both spilled SGPRs into VGPR lanes.
  auto ld = [&](int r) {
    int64_t row = min(max(row0 + r, rmin), rmax);
    opaque(row);
    return *reinterpret_cast<const vecf*>(src + row * pitch + lo);
  };
  // The first and last rows go to LDS at step 0: load them first.
  T.u[0] = ld(0);
  T.u[R - 1] = ld(R - 1);
#pragma unroll
  for (int r = 1; r < R - 1; ++r) T.u[r] = ld(r);

  Upd<MODE, XL> up;
  up.cx = to_vgpr(g.cx);
  up.cy = to_vgpr(g.cy);
  // Bit r: row row0 + r is a global interior row (MODE 1) / a useful row.
  auto bits = [](int64_t lo_r, int64_t hi_r) -> unsigned {  // rows [lo_r, hi_r) of 0..R-1
    const int l = int(max<int64_t>(0, min<int64_t>(lo_r, R)));
    const int h = int(max<int64_t>(0, min<int64_t>(hi_r, R)));
    const unsigned top = h >= 32 ? ~0u : (1u << h) - 1u;
    return l >= h ? 0u : top & ~((1u << l) - 1u);
  };
  unsigned rowmask;
  tile_mode_setup(up, g, col, bits(1 - (g.gx0 + row0), g.nx - 1 - (g.gx0 + row0)), rowmask);
  unsigned usemask = bits(ub - row0, ue - row0);
  int64_t off0 = row0 * pitch;  // this wave's first row in dst (the last step stores)
  opaque(off0);
  const int wa = w > 0 ? w - 1 : 0, wb = w < NW - 1 ? w + 1 : NW - 1;
  // Neighbour rows through LDS (TileXc, tb_tile_core.hpp).
  TileXc<NW> xc{xch, w, lane, 1, 0, 0, vecf{}};
  // Step -1 (fictional, bottom-up): early row R - 1, late row 0.
  xch[1][0][w][lane] = T.u[R - 1];
  xch[1][1][w][lane] = T.u[0];
  lds_barrier();
  xc.efirst = xch[1][0][wa][lane];
  // RES 1: the residual of step res_level - 1 (tile_pass_steps).
  const int rs = RES ? a.res_level - 1 : -1;
  tile_pass_steps<RES == 1, 1>(K, rs, [&](auto down_c, auto what_c, auto acc_c, int s) {
    constexpr bool D = decltype(down_c)::value;
    xc.p = s & 1;
    // Down: the last row needs the wave below; so does the next (up) step's first.
    xc.last_w = xc.next_w = D ? wb : wa;
    const vecf first_nb = xc.efirst;
    opaque(rowmask);
    opaque(usemask);
    T.template step<D, decltype(what_c)::value, decltype(acc_c)::value>(
        first_nb, xc, up, rowmask, usemask, store_lane, rc, dst + lo, off0, pitch);
  });
  return T.m;
}


// RES: 0 no residual; 1 the residual of step a.res_level (check passes).
// Separate instantiations: the residual must not cost the plain passes
// registers (one kernel with both bodies spilled 240-680 B per lane).
template <int R, int NW, int XL, int RES>
__global__ __launch_bounds__(64 * NW, (tile_waves_per_simd<R, NW>())) void tile_kernel(TbArgs a, int K) {
  __shared__ vecf xch[2][2][NW][64];  // [step parity][first / last row][wave][lane]
  if (tbdetail::gated(a.g.gate)) return;  // uniform over the launch
  int blk = blockIdx.x;
  if (a.flags & tbdetail::kTbXcdGroups) {
    // Contiguous unit ranges per XCD (blocks b, b+8, ... share one XCD):
    // vertically adjacent tiles of a strip share their K halo rows in L2.
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7, x = blk & 7, j = blk >> 3;
    blk = x * q + min(x, r) + j;
  }
  if (blk >= a.total_waves) return;  // whole workgroup: no barrier is left waiting
  int bi = 0;
#pragma unroll
  for (int j = 1; j < tbdetail::kMaxBoxes; ++j)
    if (j < a.nbox && blk >= a.box[j].wave_begin) bi = j;
  const TbBox& bx = a.box[bi];
  const int u = blk - bx.wave_begin;
  const int strip = u / bx.nchunks, t = u % bx.nchunks;
  const StencilGeom& g = a.g;
  // Dirichlet mode: per wave (tile_mode), the same steps and barriers on every path.
  const int KK = (K + 3) & ~3;
  const int64_t cbase = bx.c0 + int64_t(strip) * (256 - 2 * KK);
  const int64_t gy_lo = g.gy0 + cbase - KK, gy_hi = gy_lo + 255;
  const int64_t ub = bx.r0 + int64_t(t) * bx.chunk_len;
  // This wave's global rows (the mode is per wave, see tile_mode).
  const int64_t wx_lo = g.gx0 + ub - K + int64_t(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * R;
  const int64_t wx_hi = wx_lo + R - 1;
  const float m = tile_dispatch<XL>(tile_mode(g, wx_lo, wx_hi, gy_lo, gy_hi), [&](auto mode_c) {
    return tile_run<R, NW, decltype(mode_c)::value, RES, XL>(a, bx, strip, t, K, xch);
  });
  if constexpr (RES == 1) {
    // One atomic per workgroup: a per-wave atomicMax on the one residual
    // word from ~4000 waves serialised at the memory side (~37 us per check
    // pass at 1024 x 8192, as much as the whole pass).  Non-negative floats
    // (and NaN, sign cleared by fabs) order like their bit patterns.
    __shared__ unsigned wmax[NW];
    unsigned mm = __float_as_uint(m);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mm = max(mm, unsigned(__shfl_xor(int(mm), off)));
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mm;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned r = 0u;
#pragma unroll
      for (int i = 0; i < NW; ++i) r = max(r, wmax[i]);
      atomicMax(a.resid, r);
    }
  }
}

template <int R, int NW, int XL>
void launch_r(const TbArgs& args, int depth, hipStream_t st) {
  if (args.resid != nullptr)
    hipLaunchKernelGGL((tile_kernel<R, NW, XL, 1>), dim3(args.total_waves), dim3(64 * NW), 0, st,
                       args, depth);
  else
    hipLaunchKernelGGL((tile_kernel<R, NW, XL, 0>), dim3(args.total_waves), dim3(64 * NW), 0, st,
                       args, depth);
}

template <int R, int NW, int XL>
int occ_r() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, tile_kernel<R, NW, XL, 0>, 64 * NW, 0) != hipSuccess)
    n = 1;
  // Bound by the VGPR granule as well (the API can over-report by one block).
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(tile_kernel<R, NW, XL, 0>)) == hipSuccess &&
      fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    n = std::min(n, (512 / alloc) / (NW / 4));
  }
  return std::max(1, n);
}

// Instantiated (rows per wave, waves per workgroup).
#define HEAT_TILE_SHAPES(X) X(12, 8) X(13, 8) X(14, 8) X(16, 8) X(20, 8) X(24, 8) X(28, 8) X(32, 8) X(12, 16)

namespace {
bool launch_xl(const TbArgs& args, int depth, int rows, int waves, int xl, hipStream_t st) {
  if (depth < 2 || depth % 2 != 0 || waves * rows <= 2 * depth) return false;
#define HEAT_TILE_CASE(r, nw)                                      \
  if (rows == r && waves == nw) {                                  \
    if (xl == 1) launch_r<r, nw, 1>(args, depth, st);              \
    else if (xl == 2) launch_r<r, nw, 2>(args, depth, st);         \
    else launch_r<r, nw, 0>(args, depth, st);                      \
    return true;                                                   \
  }
  HEAT_TILE_SHAPES(HEAT_TILE_CASE)
#undef HEAT_TILE_CASE
  return false;
}

int occupancy_xl(int rows, int waves, int xl) {
#define HEAT_TILE_CASE(r, nw)                                                           \
  if (rows == r && waves == nw)                                                         \
    return xl == 1 ? occ_r<r, nw, 1>() : xl == 2 ? occ_r<r, nw, 2>() : occ_r<r, nw, 0>();
  HEAT_TILE_SHAPES(HEAT_TILE_CASE)
#undef HEAT_TILE_CASE
  return 0;
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
  static constexpr Shape kShapes[] = {{12, 8}, {13, 8}, {14, 8}, {16, 8}, {20, 8}, {24, 8}, {28, 8}, {32, 8}, {12, 16}};
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
