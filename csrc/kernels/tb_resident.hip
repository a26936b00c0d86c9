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
// that read it.  Flags are zeroed by a memset node before every launch
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
#include "tb_tile.hpp"
#include "tb_tile_core.hpp"

namespace heat::gpu::tbw {

constexpr int kResMaxChecks = kTbResidentMaxChecks;

struct ResArgs {
  TbArgs a;             // box[0]: the launch's box; src: pass 0 input; dst: last pass output
  int passes;           // P >= 2
  int depth;            // K (even)
  float* xbase[2];      // exchange fields (allocation bases, same layout as the field)
  int64_t xorigin;      // owned cell (0, 0) in floats from an allocation base
  int xbytes;           // allocation size (buffer descriptor range, < 2^31)
  unsigned* flags;      // one word per tile, zero at launch (the previous launch's last
                        // tile re-zeroes them, see tile_resident_kernel)
  unsigned* done;       // tiles finished (zero at launch, re-zeroed with the flags)
  unsigned* err;        // non-zero: a neighbour wait gave up (bounded spin)
  int64_t own_r1, own_c1;  // owned block [0, own_r1) x [0, own_c1): the residual's cells
  // Convergence checks inside the launch: check c takes the residual of
  // step chk_step[c] (1..K) of pass chk_pass[c] into resids[c] (RES 1).
  int nchk;
  unsigned* resids;
  int chk_pass[kResMaxChecks], chk_step[kResMaxChecks];
  int diag;             // timing diagnostics (HEAT_TB_RES_DIAG; bits 0-2 give wrong
                        // results): bit 0 no neighbour wait, 1 no ghost reload, 2 no
                        // publish, 3 every tile on the masked path
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Neighbour waits give up after this many polls (~0.3 s with s_sleep 2).
constexpr unsigned kSpinLimit = 1u << 22;

// One max per workgroup into *word (a non-negative float's bits order like
// the float; NaN has its sign cleared by fabs).  Every thread calls it.
template <int NW>
__device__ __forceinline__ void wg_max_atomic(float m, unsigned* word, unsigned* wmax) {
  unsigned mm = __float_as_uint(m);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mm = max(mm, unsigned(__shfl_xor(int(mm), off)));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mm;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned r = 0u;
#pragma unroll
    for (int i = 0; i < NW; ++i) r = max(r, wmax[i]);
    atomicMax(word, r);
  }
  __syncthreads();  // wmax is reused by the next check
}

// RES 1: the residuals of the checks inside the launch (ResArgs::chk_*): a
// check pass accumulates the max under a uniform row mask that is zero in
// every other step (tb_tile_core.hpp), and the workgroup's max goes to its
// word at the end of that pass.  A separate instantiation: the RES 0 kernel
// keeps its register allocation.
template <int R, int NW, int MODE, int XL, int RES>
__device__ __forceinline__ void resident_run(const ResArgs& ra, const TbBox& bx, int strip, int t,
                                             int u, vecf (*xch)[2][NW][64], unsigned* wmax) {
  const TbArgs& a = ra.a;
  const int K = ra.depth;
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
  const int64_t row0 = ub - K + int64_t(w) * R;
  const int64_t rmin = bx.r0 - K, rmax = bx.r1 + K - 1;
  const int64_t pitch = g.pitch;
  const float* __restrict__ src = a.src + (cbase - KK);
  float* __restrict__ dst = a.dst + (cbase - KK);
  const int lo = 4 * lane;

  Tile<R, MODE, RES, XL> T;
  auto ld = [&](int r) {
    int64_t row = min(max(row0 + r, rmin), rmax);
    opaque(row);
    return *reinterpret_cast<const vecf*>(src + row * pitch + lo);
  };
  T.u[0] = ld(0);
  T.u[R - 1] = ld(R - 1);
#pragma unroll
  for (int r = 1; r < R - 1; ++r) T.u[r] = ld(r);

  Upd<MODE, XL> up;
  up.cx = to_vgpr(g.cx);
  up.cy = to_vgpr(g.cy);
  auto bits = [](int64_t lo_r, int64_t hi_r) -> unsigned {  // rows [lo_r, hi_r) of 0..R-1
    const int l = int(max<int64_t>(0, min<int64_t>(lo_r, R)));
    const int h = int(max<int64_t>(0, min<int64_t>(hi_r, R)));
    const unsigned top = h >= 32 ? ~0u : (1u << h) - 1u;
    return l >= h ? 0u : top & ~((1u << l) - 1u);
  };
  unsigned rowmask;
  tile_mode_setup(up, g, col, bits(1 - (g.gx0 + row0), g.nx - 1 - (g.gx0 + row0)), rowmask);
  unsigned usemask = bits(ub - row0, ue - row0);
  // Edge-band rows (published in full width) and ghost rows (reloaded in
  // full width): the K useful rows next to each useful-row boundary, and the
  // K rows beyond it that lie inside the box.
  const unsigned bandmask = usemask & (bits(ub - row0, ub + K - row0) | bits(ue - K - row0, ue - row0));
  const unsigned ghostmask =
      bits(max(ub - K, bx.r0) - row0, ub - row0) | bits(ue - row0, min(ue + K, bx.r1) - row0);
  // Lanes of the column bands: useful lanes within KK of the useful edge
  // (published in every useful row) and overlap lanes inside the box
  // (reloaded in every useful row).
  const bool band_lane = store_lane && (col < cbase + KK || col + 4 > cend - KK);
  const bool ghost_lane = !store_lane && col >= bx.c0 && col < bx.c1;
  const bool box_lane = col >= bx.c0 && col < bx.c1;
  // The last pass's residual: owned cells only (a deep-halo box's edge rows
  // and columns are stale by then).
  const unsigned resmask = bits(max<int64_t>(ub, 0) - row0, min<int64_t>(ue, ra.own_r1) - row0);
  const int res_rc = store_lane && col >= 0 && col < ra.own_c1 ? int(min<int64_t>(ra.own_c1 - col, 4)) : 0;
  // Exchange fields through buffer descriptors (sc1 = write-through stores,
  // L2-coherent loads): the lane's column in the voffset VGPR, the row in the
  // scalar soffset.  Row offsets derive from a base made opaque once per
  // pass (opaque32), so the compiler cannot precompute R per-row offsets
  // across the pass loop (it did, and spilled them to scratch).
  __amdgpu_buffer_rsrc_t xr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) xr[i] = __builtin_amdgcn_make_buffer_rsrc(ra.xbase[i], 0, ra.xbytes, 0x00020000);
  const int vlane = 16 * lane;
  const int xrow0 = int((ra.xorigin + row0 * pitch + (cbase - KK)) * 4);  // this wave's first row
  const int xpitch = int(pitch * 4);

  const int wa = w > 0 ? w - 1 : 0, wb = w < NW - 1 ? w + 1 : NW - 1;
  TileXc<NW> xc{xch, w, lane, 1, 0, 0, vecf{}};
  using Down = std::true_type;
  using Up = std::false_type;

  // The publish sink of a pass's last step: edge bands into xb[p & 1].
  struct Pub {
    __amdgpu_buffer_rsrc_t rs;
    unsigned usemask, bandmask;
    bool store_lane, band_lane;
    int vlane, xrow0, xpitch;
    __device__ __forceinline__ void row(int r, const vecf& v, const vecf&) {
      if ((usemask >> r) & 1u) {
        const bool st = ((bandmask >> r) & 1u) ? store_lane : band_lane;
        if (st)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, vlane,
                                                 xrow0 + r * xpitch, 16);
      }
    }
  };

  // One pass: LDS slots of the fictional step -1, then K steps; the last one
  // publishes the edge bands (LAST false) or stores the box to dst (LAST).
  auto pass = [&](auto last_c, int p) {
    constexpr bool LAST = decltype(last_c)::value;
    xch[1][0][w][lane] = T.u[R - 1];
    xch[1][1][w][lane] = T.u[0];
    lds_barrier();
    xc.efirst = xch[1][0][wa][lane];
    int xr0 = xrow0, xp = xpitch;
    opaque32(xr0);
    opaque32(xp);
    const bool nopub = ra.diag & 4;
    Pub pub{xr[p & 1], usemask, nopub ? 0u : bandmask, nopub ? false : store_lane,
            nopub ? false : band_lane, vlane, xr0, xp};
    int64_t off0 = row0 * pitch;  // this wave's first row in dst (the last pass stores)
    opaque(off0);
    // The check of this pass (at most one), if any.
    int ci = -1;
    if constexpr (RES == 1) {
      for (int c = 0; c < ra.nchk; ++c)
        if (ra.chk_pass[c] == p) ci = c;
    }
    const int rs = ci >= 0 ? ra.chk_step[ci] - 1 : -1;
    tile_pass_steps<RES == 1, LAST ? 1 : 3>(K, rs, [&](auto down_c, auto what_c, auto acc_c, int s) {
      constexpr bool D = decltype(down_c)::value;
      xc.p = s & 1;
      xc.last_w = xc.next_w = D ? wb : wa;
      const vecf first_nb = xc.efirst;
      opaque(rowmask);
      opaque(usemask);
      T.template step<D, decltype(what_c)::value, decltype(acc_c)::value>(
          first_nb, xc, up, rowmask, usemask, store_lane, rc, dst + lo, off0, pitch, &pub, resmask,
          res_rc);
    });
    if constexpr (RES == 1) {
      if (ci >= 0) {
        wg_max_atomic<NW>(T.m, ra.resids + ci, wmax);
        T.m = 0.f;
      }
    }
  };

  // Wait for the neighbours' pass p - 1 bands, then reload the ghost ring.
  auto refill = [&](int p) {
    if (w == 0 && !(ra.diag & 1)) {
      // Wave 0, one lane per neighbour tile: relaxed agent-scope polls
      // (sc1), bounded; a give-up is reported, never waited out.
      const int ns = bx.nstrips, nc = bx.nchunks;
      const int ds = lane < 3 ? -1 : lane < 5 ? 0 : 1;
      const int dt = (lane == 0 || lane == 3 || lane == 5) ? -1 : (lane == 1 || lane == 6) ? 0 : 1;
      const int s2 = strip + ds, t2 = t + dt;
      const bool real = lane < 8 && s2 >= 0 && s2 < ns && t2 >= 0 && t2 < nc;
      const unsigned* f = ra.flags + (real ? s2 * nc + t2 : u);
      for (unsigned spins = 0;; ++spins) {
        const unsigned v =
            real ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : unsigned(p);
        if (__all(v >= unsigned(p))) break;
        if (spins >= kSpinLimit) {
          if (lane == 0) __hip_atomic_fetch_or(ra.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    if (ra.diag & 2) return;
    const __amdgpu_buffer_rsrc_t rs = xr[(p - 1) & 1];
    unsigned gm = ghostmask, um = usemask;
    opaque(gm);
    opaque(um);
    int xr0 = xrow0, xp = xpitch;
    opaque32(xr0);
    opaque32(xp);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool full = (gm >> r) & 1u;
      const bool part = (um >> r) & 1u;
      if ((full && box_lane) || (part && ghost_lane))
        T.u[r] = __builtin_bit_cast(vecf, __builtin_amdgcn_raw_buffer_load_b128(rs, vlane, xr0 + r * xp, 16));
    }
  };

  const int P = ra.passes;
  for (int p = 0; p + 1 < P; ++p) {
    if (p > 0) refill(p);
    pass(std::false_type{}, p);
    // Publish (Guideline 16 R1): every storing wave drains its sc1 stores,
    // the barrier, then ONE lane raises the tile's flag (sc1 store).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(ra.flags + u, unsigned(p + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  refill(P - 1);
  pass(std::true_type{}, P - 1);
}

template <int R, int NW, int XL, int RES>
__global__ __launch_bounds__(64 * NW, (tile_waves_per_simd<R, NW>())) void tile_resident_kernel(
    ResArgs ra) {
  __shared__ vecf xch[2][2][NW][64];  // [step parity][first / last row][wave][lane]
  const TbArgs& a = ra.a;
  if (tbdetail::gated(a.g.gate)) return;  // uniform over the launch: nobody waits
  int blk = blockIdx.x;
  if (a.flags & tbdetail::kTbXcdGroups) {
    const int nb = gridDim.x, q = nb >> 3, r = nb & 7, x = blk & 7, j = blk >> 3;
    blk = x * q + min(x, r) + j;
  }
  // The grid is exactly the tiles of box[0] (strip-major), all co-resident.
  const TbBox& bx = a.box[0];
  const int strip = blk / bx.nchunks, t = blk % bx.nchunks;
  const StencilGeom& g = a.g;
  const int K = ra.depth, KK = (K + 3) & ~3;
  const int64_t cbase = bx.c0 + int64_t(strip) * (256 - 2 * KK);
  const int64_t gy_lo = g.gy0 + cbase - KK, gy_hi = gy_lo + 255;
  const int64_t ub = bx.r0 + int64_t(t) * bx.chunk_len;
  // This wave's global rows (the mode is per wave, see tile_mode).
  const int64_t wx_lo = g.gx0 + ub - K + int64_t(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * R;
  const int64_t wx_hi = wx_lo + R - 1;
  const int mode = (ra.diag & 8) ? kTileGeneric : tile_mode(g, wx_lo, wx_hi, gy_lo, gy_hi);
  __shared__ unsigned wmax[NW];
  tile_dispatch<XL>(mode, [&](auto mode_c) {
    resident_run<R, NW, decltype(mode_c)::value, XL, RES>(ra, bx, strip, t, blk, xch, wmax);
    return 0.f;
  });
  // Completion: the tile that finishes last (every other tile is past its
  // last flag poll) re-zeroes the flags and the counter for the next launch
  // on this stream, in place of a memset node per launch (~5 us each, as much
  // as a check's whole judge launch).  A gated launch returns above without
  // touching either.
  __shared__ unsigned last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned n = __hip_atomic_fetch_add(ra.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = n + 1 == unsigned(gridDim.x);
  }
  __syncthreads();
  if (last) {
    for (int i = threadIdx.x; i < int(gridDim.x); i += blockDim.x)
      __hip_atomic_store(ra.flags + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(ra.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int R, int NW, int XL>
int occ_res() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, tile_resident_kernel<R, NW, XL, 0>, 64 * NW, 0) !=
      hipSuccess)
    n = 1;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(tile_resident_kernel<R, NW, XL, 0>)) ==
          hipSuccess &&
      fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    n = std::min(n, (512 / alloc) / (NW / 4));
  }
  return std::max(0, n);
}

// Instantiated shapes (rows per wave, waves per workgroup): the tile
// planner's set up to 24 rows per wave (the resident grid must be one
// dispatch round, so only blocks with few tiles qualify).
#define HEAT_RES_SHAPES(X) X(12, 8) X(13, 8) X(14, 8) X(16, 8) X(20, 8) X(24, 8) X(12, 16)

namespace {
int occupancy_res(int rows, int waves, int xl) {
#define HEAT_RES_CASE(r, nw)                                                                \
  if (rows == r && waves == nw)                                                             \
    return xl == 1 ? occ_res<r, nw, 1>() : xl == 2 ? occ_res<r, nw, 2>() : occ_res<r, nw, 0>();
  HEAT_RES_SHAPES(HEAT_RES_CASE)
#undef HEAT_RES_CASE
  return 0;
}

template <int R, int NW, int XL>
void launch_res_x(const ResArgs& ra, int blocks, hipStream_t st) {
  if (ra.a.resid != nullptr)
    hipLaunchKernelGGL((tile_resident_kernel<R, NW, XL, 1>), dim3(blocks), dim3(64 * NW), 0, st, ra);
  else
    hipLaunchKernelGGL((tile_resident_kernel<R, NW, XL, 0>), dim3(blocks), dim3(64 * NW), 0, st, ra);
}

bool launch_res(const ResArgs& ra, int rows, int waves, int xl, int blocks, hipStream_t st) {
#define HEAT_RES_CASE(r, nw)                                          \
  if (rows == r && waves == nw) {                                     \
    if (xl == 1) launch_res_x<r, nw, 1>(ra, blocks, st);              \
    else if (xl == 2) launch_res_x<r, nw, 2>(ra, blocks, st);         \
    else launch_res_x<r, nw, 0>(ra, blocks, st);                      \
    return true;                                                      \
  }
  HEAT_RES_SHAPES(HEAT_RES_CASE)
#undef HEAT_RES_CASE
  return false;
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
  static constexpr Shape kShapes[] = {{12, 8}, {13, 8}, {14, 8}, {16, 8}, {20, 8}, {24, 8}, {12, 16}};
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

void tb_resident_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
                      int depth, int passes, const TbResidentBuffers& xb, hipStream_t st,
                      int variant, const TbResidentCheck* checks, int nchecks, unsigned* resids,
                      int64_t own_rows, int64_t own_cols) {
  using namespace tbw;
  HEAT_CHECK(passes >= 2, "a resident launch spans >= 2 passes (%d)", passes);
  const TbTuning tune = tb_tuning();
  const int xl = res_xl(variant, tune);
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
    HEAT_CHECK(checks[c].pass >= 0 && checks[c].pass < passes && checks[c].step >= 1 &&
                   checks[c].step <= depth && (c == 0 || checks[c].pass > checks[c - 1].pass),
               "resident check %d at pass %d step %d (passes %d, depth %d)", c, checks[c].pass,
               checks[c].step, passes, depth);
    ra.chk_pass[c] = checks[c].pass;
    ra.chk_step[c] = checks[c].step;
  }
  ra.nchk = nchecks;
  ra.resids = resids;
  a.resid = nchecks > 0 ? resids : nullptr;  // selects the RES 1 instantiation
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
