// Device code of the resident workgroup tiles, included by
// tb_resident_xl{0,1,2}.hip (one lane-shift build each, compiled in
// parallel); the protocol notes and the planner are in tb_resident.hip.
#pragma once

#include <algorithm>
#include <type_traits>

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
  // level chk_step[c] (even, 2..K; checked on the host) of pass chk_pass[c]
  // into resids[c] (RES 1).
  int nchk;
  unsigned* resids;
  int chk_pass[kResMaxChecks], chk_step[kResMaxChecks];
  int diag;             // timing diagnostics (HEAT_TB_RES_DIAG; bits 0-2 give wrong
                        // results): bit 0 no neighbour wait, 1 no ghost reload, 2 no
                        // publish, 3 every tile on the masked path, 4 plate edge rows
                        // computed as interior rows (what the masked edge waves cost)
};

// Neighbour waits give up after this many polls (~0.3 s with s_sleep 2).
constexpr unsigned kSpinLimit = 1u << 22;

// One max per WAVE into *word (a non-negative float's bits order like the
// float; NaN has its sign cleared by fabs): no workgroup barrier in the
// pass (two per check cost ~1.5 us per check pass); the callers spread the
// waves over kTbResidentSlots words, so an address takes ~130 atomics.
__device__ __forceinline__ void wave_max_atomic_u(float m, unsigned* word) {
  unsigned mm = __float_as_uint(m);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mm = max(mm, unsigned(__shfl_xor(int(mm), off)));
  if ((threadIdx.x & 63) == 0) atomicMax(word, mm);
}

// RES 1: the residuals of the checks inside the launch (ResArgs::chk_*),
// each at an even level of its pass (tile_pass_steps ACC_MODE 3); each
// wave's max goes to the check's word of its slot after the next pass's
// ghost loads (the last pass: at its end).  A separate instantiation: the
// RES 0 kernel keeps its register allocation.
template <int R, int NW, int MODE, int XL, int RES>
__device__ __forceinline__ void resident_run(const ResArgs& ra, const TbBox& bx, int strip, int t,
                                             int u, vecf (*xch)[2][NW][64]) {
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

  // The sinks of a pass's last step: edge bands into xb[p & 1] (Pub), the
  // last pass's useful rows into dst (RowStoreSink).  Both branch-free (see
  // RowStoreSink): with a per-row `if`, tiles of 36-40 rows per wave spilled
  // 660-1000 B/lane, and 20 x 16 tiles 96 B.
  struct Pub {
    __amdgpu_buffer_rsrc_t rs;
    unsigned usemask, bandmask;
    int vs, vb;  // voffset of a core row's / a band row's store (kNoStore: none)
    int xrow0, xpitch;
    __device__ __forceinline__ void row(int r, const vecf& v, const vecf&) {
      const int vo = ((usemask >> r) & 1u) ? (((bandmask >> r) & 1u) ? vs : vb) : kNoStore;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, vo, xrow0 + r * xpitch,
                                             16);
    }
  };

  // A check's wave max waiting for its atomic (RES 1); the next check.
  float pend_m = 0.f;
  int pend_c = -1;
  int next_chk = 0;
  auto flush_resid = [&]() {
    if constexpr (RES == 1) {
      if (pend_c >= 0) {
        const int slot = (u * NW + w) & (kTbResidentSlots - 1);
        wave_max_atomic_u(pend_m, ra.resids + slot * kResMaxChecks + pend_c);
        pend_c = -1;
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
    // Masks opaque per pass: hoisted out of the pass loop, the per-row
    // voffset selects became R loop-invariant VGPRs (and spilled).
    unsigned pum = nopub ? 0u : usemask, pbm = bandmask;
    opaque(pum);
    opaque(pbm);
    Pub pub{xr[p & 1], pum, pbm, store_lane ? vlane : kNoStore, band_lane ? vlane : kNoStore, xr0, xp};
    int64_t off0 = row0 * pitch;  // this wave's first row in dst (the last pass stores)
    opaque(off0);
    RowStoreSink fin{dst + off0, pitch, pum, store_lane ? vlane : kNoStore};
    // The check of this pass (at most one, at an even level), if any: the
    // checks come in pass order, so one kernel-argument load per pass (a scan
    // of all of them was up to 64 dependent scalar loads per pass).
    int ci = -1;
    if constexpr (RES == 1) {
      if (next_chk < ra.nchk && ra.chk_pass[next_chk] == p) ci = next_chk++;
    }
    int acc_step = ci >= 0 ? ra.chk_step[ci] - 1 : -1;  // its step index (odd: an up step)
    opaque32(acc_step);
    unsigned rm = ci >= 0 ? resmask : 0u;  // the check step's residual rows
    opaque(rm);
    tile_pass_steps<RES == 1 ? 3 : 0, 3>(
        K,
        [&](auto down_c, auto what_c, auto acc_c, int s) {
          constexpr bool D = decltype(down_c)::value;
          xc.p = s & 1;
          xc.last_w = xc.next_w = D ? wb : wa;
          const vecf first_nb = xc.efirst;
          opaque(rowmask);
          opaque(usemask);
          // The last step always runs the accumulating body: rows only if
          // the check is there.
          const unsigned rms = s == acc_step ? rm : 0u;
          if constexpr (LAST)
            T.template step<D, decltype(what_c)::value, decltype(acc_c)::value>(
                first_nb, xc, up, rowmask, usemask, store_lane, rc, &fin,
                rms, res_rc);
          else
            T.template step<D, decltype(what_c)::value, decltype(acc_c)::value>(
                first_nb, xc, up, rowmask, usemask, store_lane, rc, &pub,
                rms, res_rc);
        },
        acc_step);
    if constexpr (RES == 1) {
      // Tall tiles: pin the residual here.  Consumed only under `ci >= 0`,
      // its max chain is sunk into that branch (the last step's residual
      // work skipped on passes without a check), which keeps every row's
      // old value of the pass's last step alive until then: 20 x 16 spilled
      // 352 B/lane (108 pinned; checked 2048 x 8192 3.89 -> 4.95 Tcells/s).
      // Short tiles keep the sunk chain: 48 B/lane, 3 % faster on checked
      // 1024 x 8192 than pinned (every pass's last step accumulating).
      if constexpr (R > 16) asm volatile("" : "+v"(T.m));
      if (ci >= 0) {
        // Deferred: the atomic goes out after the next pass's ghost loads
        // (refill), not in front of the publish's vmcnt(0) drain, where ~63
        // atomics per residual word (4032 waves, 64 slots) held every check
        // pass's boundary; the last pass issues it at once.
        pend_m = T.m;
        pend_c = ci;
        T.m = 0.f;
        if constexpr (LAST) flush_resid();
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
    if (ra.diag & 2) {
      flush_resid();
      return;
    }
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
    flush_resid();  // behind the ghost loads: their waits do not include it
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
  const int mode = (ra.diag & 8) ? kTileGeneric : tile_mode(g, wx_lo, wx_hi, gy_lo, gy_hi, ra.diag & 16);
  tile_dispatch<XL, (RES == 0 && R <= kTilePkRows)>(mode, [&](auto mode_c) {
    resident_run<R, NW, decltype(mode_c)::value, XL, RES>(ra, bx, strip, t, blk, xch);
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

template <class Kern>
int occ_kernel(Kern k, int NW) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 64 * NW, 0) != hipSuccess) n = 1;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k)) == hipSuccess && fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    n = std::min(n, (512 / alloc) / (NW / 4));
  }
  return std::max(0, n);
}

// Co-resident tiles per CU: the smaller of the two instantiations (the RES 1
// build takes more VGPRs, e.g. 128 vs 106 at 12 x 8), so a plan accepted for
// an unchecked span stays co-resident when its span carries checks.
template <int R, int NW, int XL>
int occ_res() {
  return std::min(occ_kernel(tile_resident_kernel<R, NW, XL, 0>, NW),
                  occ_kernel(tile_resident_kernel<R, NW, XL, 1>, NW));
}

// Instantiated shapes (rows per wave, waves per workgroup): the tile
// planner's set up to 24 rows per wave (the resident grid must be one
// dispatch round, so only blocks with few tiles qualify), and 20 x 16: 320
// rows per tile, one tile per CU at 4 waves per SIMD, the 4-GPU per-rank
// blocks (2048 x 8192: 36 strips x 7 chunks; 4096 x 4096: 18 x 14).
#define HEAT_RES_SHAPES(X) X(12, 8) X(13, 8) X(14, 8) X(16, 8) X(20, 8) X(24, 8) X(12, 16) X(20, 16)

template <int R, int NW, int XL>
void launch_res_x(const ResArgs& ra, int blocks, hipStream_t st) {
  if (ra.a.resid != nullptr)
    hipLaunchKernelGGL((tile_resident_kernel<R, NW, XL, 1>), dim3(blocks), dim3(64 * NW), 0, st, ra);
  else
    hipLaunchKernelGGL((tile_resident_kernel<R, NW, XL, 0>), dim3(blocks), dim3(64 * NW), 0, st, ra);
}

// The entry points of one lane-shift build (tb_resident_xl<XL>.hip).
template <int XL>
bool res_launch_unit(const ResArgs& ra, int rows, int waves, int blocks, hipStream_t st) {
#define HEAT_RES_CASE(r, nw)                     \
  if (rows == r && waves == nw) {                \
    launch_res_x<r, nw, XL>(ra, blocks, st);     \
    return true;                                 \
  }
  HEAT_RES_SHAPES(HEAT_RES_CASE)
#undef HEAT_RES_CASE
  return false;
}

template <int XL>
int res_occupancy_unit(int rows, int waves) {
#define HEAT_RES_CASE(r, nw) \
  if (rows == r && waves == nw) return occ_res<r, nw, XL>();
  HEAT_RES_SHAPES(HEAT_RES_CASE)
#undef HEAT_RES_CASE
  return 0;
}

}  // namespace heat::gpu::tbw
