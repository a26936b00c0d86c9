// Device building blocks of the workgroup-tile TB kernels (tb_tile.hip: one
// pass per launch; tb_resident.hip: the tile kept in VGPRs across passes).
// See tb_tile.hip for the design.
#pragma once

#include <type_traits>

#include "tb_common.hpp"

namespace heat::gpu::tbw {

using tbdetail::TbArgs;
using tbdetail::TbBox;
typedef float vecf __attribute__((ext_vector_type(4)));

#ifndef HEAT_TILE_PD
#define HEAT_TILE_PD 3  // rows the ds_bpermute lane shifts run ahead
#endif

// Lane l <- lane l-1 / l+1.  Lanes 0 and 63 lie in the strip overlap
// (don't-care values).  XL: 0 both shifts DPP wave shifts (folded into the
// e + w add), 1 both ds_bpermute (issued PD rows ahead), 2 mixed: the left
// shift DPP, the right one ds_bpermute (half the LDS-crossbar issue).
template <int XL>
__device__ __forceinline__ float from_left(float v) {
  if constexpr (XL == 1) {
    const int l = threadIdx.x & 63;
    return __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 63) & 63) << 2, __float_as_int(v)));
  } else {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
  }
}
template <int XL>
__device__ __forceinline__ float from_right(float v) {
  if constexpr (XL >= 1) {
    const int l = threadIdx.x & 63;
    return __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 1) & 63) << 2, __float_as_int(v)));
  } else {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
  }
}

// cx / cy in VGPRs: a VALU op with an SGPR operand issues at half rate.
__device__ __forceinline__ float to_vgpr(float x) {
  float r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
  return r;
}

// A wave-uniform value the compiler must treat as unknown from here on.
// (readfirstlane: values read from the kernel arguments through a dynamic box
// index are not provably uniform to the compiler.)
__device__ __forceinline__ void opaque(unsigned& x) {
  x = __builtin_amdgcn_readfirstlane(x);
  asm volatile("" : "+s"(x));
}
__device__ __forceinline__ void opaque32(int& x) {
  x = __builtin_amdgcn_readfirstlane(x);
  asm volatile("" : "+s"(x));
}
__device__ __forceinline__ void opaque(int64_t& x) {
  unsigned lo = __builtin_amdgcn_readfirstlane(unsigned(uint64_t(x)));
  unsigned hi = __builtin_amdgcn_readfirstlane(unsigned(uint64_t(x) >> 32));
  asm volatile("" : "+s"(lo), "+s"(hi));
  x = int64_t((uint64_t(hi) << 32) | lo);
}

// LDS writes of this wave done, then the workgroup barrier.  Not
// __syncthreads(): its fence would also wait for the wave's outstanding
// global loads (the tile's rows still streaming in at step 0) and stores.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// MODE 0: no cell of the tile is on the plate's fixed ring (or outside it);
// MODE 1: per-lane column masks and a per-row (uniform) mask keep those cells.
template <int MODE, int XL>
struct Upd {
  float cx, cy;
  bool cm[4];
  // wl / er: the west neighbour of element 0 (lane l-1's element 3) and the
  // east neighbour of element 3 (lane l+1's element 0).
  __device__ __forceinline__ vecf apply(const vecf& a, const vecf& b, const vecf& c, float wl,
                                        float er, bool row_ok) const {
    vecf r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float w = j == 0 ? wl : b[j - 1];
      const float e = j == 3 ? er : b[j + 1];
      // The shifted value as the second operand of e + w (fp add commutes):
      // the DPP build folds it into v_add_f32_dpp.
      r[j] = j == 3 ? stencil(b[j], a[j], c[j], e, w, cx, cy) : stencil(b[j], a[j], c[j], w, e, cx, cy);
    }
    if constexpr (MODE == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = (cm[j] && row_ok) ? r[j] : b[j];
    }
    return r;
  }
};

struct TileNoSink;

// RES: 0 no residual; 1 max |new - old| over the rows of `resmask` (a
// runtime mask: zero except in the step that takes the check's residual,
// TbArgs::res_level, the last step or an inner one of a full-depth pass).
template <int R, int MODE, int RES, int XL>
struct Tile {
  vecf u[R];
  float m = 0.f;

  // One time step of this wave's rows, in place, top-down (DOWN) or
  // bottom-up.  first_nb: the outside neighbour of the first row processed
  // (old value, already in a register); the outside neighbour of the last
  // row comes from xc.mid(), called halfway through the step (the step's
  // workgroup barrier), and xc.publish(0 / 1, row) hands the first / last
  // row computed to the neighbour waves.  Alternating the direction every step
  // lets the register allocator put new row r where old row r -/+ 1 was (dead
  // by then) and be back at the loop's assignment after two steps: one
  // direction only needed a copy of every row per step at the back-edge.
  // WHAT 1 (LAST): the launch's last step stores every useful row as soon as
  // it is computed (dst + off0 + r * pitch, this lane's columns if
  // store_lane); WHAT 3: every row goes to sink->row(r, new, old) (the
  // resident kernel's edge-band publish, tb_resident.hip).  With RES 1 any
  // step accumulates max |new - old| over the useful rows in resmask.
  template <bool DOWN, int WHAT, class Xc, class Sink = TileNoSink>
  __device__ __forceinline__ void step(const vecf& first_nb, Xc& xc, const Upd<MODE, XL>& up,
                                       unsigned rowmask, unsigned usemask, bool store_lane, int rc,
                                       float* __restrict__ dst, int64_t off0, int64_t pitch,
                                       Sink* sink = nullptr, unsigned resmask = ~0u,
                                       int res_rc = -1) {
    // Residual window (the resident kernel's deep-halo boxes: the owned block
    // only): rows resmask, res_rc useful columns of this lane (-1: the stored
    // cells, store_lane / rc).
    const bool res_lane = res_rc < 0 ? store_lane : res_rc > 0;
    const int res_cols = res_rc < 0 ? rc : res_rc;
    // Lane shifts of the OLD rows.  ds_bpermute results take ~50+ cycles: the
    // shifts of the row PD places ahead in processing order are issued before
    // a row is computed (scheduling barriers keep that order; unconstrained,
    // the scheduler hoisted every row's shifts and spilled).  DPP shifts fold
    // into the add.
    constexpr int PD = XL >= 1 ? (R - 1 < HEAT_TILE_PD ? R - 1 : HEAT_TILE_PD) : 0;
    float wl[R], er[R];
    auto row_at = [](int i) { return DOWN ? i : R - 1 - i; };
    auto shift = [&](int r) {  // the ds_bpermute shifts, issued ahead
      if constexpr (XL == 1) wl[r] = from_left<XL>(u[r][3]);
      if constexpr (XL >= 1) er[r] = from_right<XL>(u[r][0]);
    };
    if constexpr (XL >= 1) {
#pragma unroll
      for (int i = 0; i < PD; ++i) shift(row_at(i));
    }
    vecf prev = u[row_at(0)];  // old value of the row processed before
    vecf last_nb = first_nb;     // set by xc.mid() before the last row
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = row_at(i);
      if (XL >= 1 && i + PD < R) shift(row_at(i + PD));
      if constexpr (XL != 1) wl[r] = from_left<XL>(u[r][3]);
      if constexpr (XL == 0) er[r] = from_right<XL>(u[r][0]);
      const vecf cur = u[r];
      const vecf outside = i == 0 ? first_nb : last_nb;
      const vecf n = r == 0 ? outside : (DOWN ? prev : u[r - 1]);
      const vecf so = r == R - 1 ? outside : (DOWN ? u[r + 1] : prev);
      u[r] = up.apply(n, cur, so, wl[r], er[r], (rowmask >> r) & 1u);
      if (i == 0) xc.publish(0, u[r]);
      if (i == R - 1) xc.publish(1, u[r]);
      if constexpr (WHAT == 1) {
        if ((usemask >> r) & 1u) {
          if (store_lane) *reinterpret_cast<vecf*>(dst + off0 + r * pitch) = u[r];
        }
      } else if constexpr (WHAT == 3) {
        sink->row(r, u[r], cur);
      }
      if constexpr (RES == 1) {
        if (((usemask & resmask) >> r) & 1u) acc(u[r], cur, res_lane, res_cols);
      }
      prev = cur;
      if (i == R / 2 - 1) last_nb = xc.mid();
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  __device__ __forceinline__ void acc(const vecf& nw, const vecf& old, bool res_lane, int rc) {
    // NaN-propagating max (v_maximum3_f32): a NaN or inf reaches the judge.
    if (res_lane) {
      float d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) d[j] = (j == 0 || rc > j) ? __builtin_fabsf(nw[j] - old[j]) : 0.f;
      m = __builtin_elementwise_maximum(
          m, __builtin_elementwise_maximum(__builtin_elementwise_maximum(d[0], d[1]),
                                           __builtin_elementwise_maximum(d[2], d[3])));
    }
  }
};

// Register budget: waves per SIMD each instantiation must fit.
template <int R, int NW>
constexpr int tile_waves_per_simd() {
  return NW >= 16 ? 4 : R <= 16 ? 4 : 2;
}

struct TileNoSink {
  __device__ __forceinline__ void row(int, const vecf&, const vecf&) {}
};

// Neighbour rows through LDS, one workgroup barrier per step placed HALFWAY
// through the step.  A step publishes the row it computes first (early slot
// E) and the row it computes last (late slot L); with the direction
// alternating, the row a wave needs first in step s + 1 is its neighbour's
// EARLY row of step s (read right after step s's barrier, so it waits in a
// register when step s + 1 starts) and the row it needs last is the
// neighbour's LATE row of step s (read after step s + 1's barrier).  A
// barrier at the step boundary left every wave of the workgroup waiting on
// the LDS read of its first row at once.  Slots are double-buffered by step
// parity; each is rewritten only after the barrier that follows its readers'
// use.
template <int NW>
struct TileXc {
  vecf (*xch)[2][NW][64];
  int w, lane, p, last_w, next_w;
  vecf efirst;
  __device__ __forceinline__ void publish(int late, const vecf& v) { xch[p][late][w][lane] = v; }
  __device__ __forceinline__ vecf mid() {
    lds_barrier();
    const vecf l = xch[p ^ 1][1][last_w][lane];  // neighbour's late row of step s - 1
    efirst = xch[p][0][next_w][lane];             // neighbour's early row of step s
    return l;
  }
};

}  // namespace heat::gpu::tbw
