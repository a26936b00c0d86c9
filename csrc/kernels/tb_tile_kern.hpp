// Device code of the workgroup-tile kernel, included by tb_tile_xl{0,1,2}.hip
// (one lane-shift build each, compiled in parallel); the planner and the
// design notes are in tb_tile.hip.
#pragma once

#include <algorithm>
#include <type_traits>

#include "heat/common.hpp"
#include "tb_tile.hpp"
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
  // RES 1: the residual of step res_level - 1: a uniform row mask, zero in
  // every other step (tile_pass_steps ACC_MODE 1).
  const int rs = RES ? a.res_level - 1 : -1;
  unsigned sm = usemask;
  opaque(sm);
  RowStoreSink fin{dst + off0, pitch, sm, store_lane ? 16 * lane : kNoStore};
  tile_pass_steps<RES == 1 ? 1 : 0, 3>(K, [&](auto down_c, auto what_c, auto acc_c, int s) {
    constexpr bool D = decltype(down_c)::value;
    xc.p = s & 1;
    // Down: the last row needs the wave below; so does the next (up) step's first.
    xc.last_w = xc.next_w = D ? wb : wa;
    const vecf first_nb = xc.efirst;
    opaque(rowmask);
    opaque(usemask);
    unsigned rm = s == rs ? ~0u : 0u;
    opaque(rm);
    T.template step<D, decltype(what_c)::value, decltype(acc_c)::value>(
        first_nb, xc, up, rowmask, usemask, store_lane, rc, &fin, rm);
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
#define HEAT_TILE_SHAPES(X) X(12, 8) X(13, 8) X(14, 8) X(16, 8) X(20, 8) X(24, 8) X(28, 8) X(32, 8) X(12, 16) X(20, 16)

// The entry points of one lane-shift build (tb_tile_xl<XL>.hip).
template <int XL>
bool tile_launch_unit(const TbArgs& args, int depth, int rows, int waves, hipStream_t st) {
#define HEAT_TILE_CASE(r, nw)               \
  if (rows == r && waves == nw) {           \
    launch_r<r, nw, XL>(args, depth, st);   \
    return true;                            \
  }
  HEAT_TILE_SHAPES(HEAT_TILE_CASE)
#undef HEAT_TILE_CASE
  return false;
}

template <int XL>
int tile_occupancy_unit(int rows, int waves) {
#define HEAT_TILE_CASE(r, nw) \
  if (rows == r && waves == nw) return occ_r<r, nw, XL>();
  HEAT_TILE_SHAPES(HEAT_TILE_CASE)
#undef HEAT_TILE_CASE
  return 0;
}

}  // namespace heat::gpu::tbw
