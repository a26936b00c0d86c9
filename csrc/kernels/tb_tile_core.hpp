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
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#ifndef HEAT_TILE_PD
#define HEAT_TILE_PD 3  // rows the ds_bpermute lane shifts run ahead
#endif
// Waves of at most this many rows take the packed row update (Upd::apply
// PK): on 12-row waves it measured +3-6 % (1024 x 8192 4.06-4.18 vs
// 3.91-3.95, 2048 x 4096 4.17 vs 4.04, session r5j); its pair temporaries
// spilled taller waves (20 x 16: 676 B/lane, 1.04 Tcells/s) and, next to
// the residual code, the 12-row RES 1 builds with ds_bpermute shifts
// (resident XL 2: 48 -> 200 B/lane), which keep the scalar update.  The
// RES 1 builds with DPP shifts (XL 0) take it: resident 12-row checks every
// 20 / 50 steps ran 4.01-4.02 / 4.07 vs 3.80 / 3.83 Tcells/s (1024 x 8192,
// session r6l; 68 B/lane, none of it in a step loop).
constexpr int kTilePkRows = 12;

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

// Dirichlet handling of one WAVE of a tile (wave-uniform: the waves of a
// tile run the same steps and barriers, each on its own path).  Cells outside
// the plate are don't-care (their values only flow further out); only the
// fixed ring must be kept.
//   kTileInterior   none of the wave's rows is a plate edge row and no column
//                   of the tile is a plate edge column (rows outside the plate
//                   are computed like any other: don't-care);
//   kTileGeneric    per-lane column masks AND a per-row (uniform) mask: the
//                   wave holds plate row 0 or nx-1 (or the tile both edge
//                   columns);
//   kTileLeft       plate column 0 is element 0 of one lane: one v_cndmask
//                   per row;
//   kTileRight + e  plate column ny-1 is element e of one lane.
// Edge waves set the pace (a tile waits at every step's barrier for its
// slowest wave, a resident grid for its slowest tile): the generic path
// issues ~36 % more instructions per step than the interior, the column
// modes ~3 % (profiles/r4_resident.md).
constexpr int kTileInterior = 0, kTileGeneric = 1, kTileLeft = 3, kTileRight = 4;

template <int MODE, int XL>
struct Upd {
  float cx, cy;
  bool cm[4];
  // wl / er: the west neighbour of element 0 (lane l-1's element 3) and the
  // east neighbour of element 3 (lane l+1's element 0).
  template <bool PK = false>
  __device__ __forceinline__ vecf apply(const vecf& a, const vecf& b, const vecf& c, float wl,
                                        float er, bool row_ok) const {
    vecf r;
    if constexpr (PK) {
      // Packed f32 (v_pk_add_f32 / v_pk_fma_f32) on the element pairs 0-1
      // and 2-3: the same per-element operations in the same order as
      // stencil() (bitwise equal), ~14.5 VALU per row instead of 24-25; the
      // horizontal e + w sums stay scalar (their operands straddle the
      // pairs; the DPP shift still folds into the first).
      typedef float f2 __attribute__((ext_vector_type(2)));
      const f2 b01 = {b[0], b[1]}, b23 = {b[2], b[3]};
      const f2 ns01 = f2{c[0], c[1]} + f2{a[0], a[1]}, ns23 = f2{c[2], c[3]} + f2{a[2], a[3]};
      const f2 tx01 = __builtin_elementwise_fma(f2(-2.0f), b01, ns01);
      const f2 tx23 = __builtin_elementwise_fma(f2(-2.0f), b23, ns23);
      const f2 ew01 = {b[1] + wl, b[2] + b[0]}, ew23 = {b[3] + b[1], er + b[2]};
      const f2 ty01 = __builtin_elementwise_fma(f2(-2.0f), b01, ew01);
      const f2 ty23 = __builtin_elementwise_fma(f2(-2.0f), b23, ew23);
      const f2 cx2 = f2(cx), cy2 = f2(cy);
      const f2 r01 = __builtin_elementwise_fma(cy2, ty01, __builtin_elementwise_fma(cx2, tx01, b01));
      const f2 r23 = __builtin_elementwise_fma(cy2, ty23, __builtin_elementwise_fma(cx2, tx23, b23));
      r = vecf{r01[0], r01[1], r23[0], r23[1]};
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float w = j == 0 ? wl : b[j - 1];
        const float e = j == 3 ? er : b[j + 1];
        // The shifted value as the second operand of e + w (fp add
        // commutes): the DPP build folds it into v_add_f32_dpp.
        r[j] = j == 3 ? stencil(b[j], a[j], c[j], e, w, cx, cy) : stencil(b[j], a[j], c[j], w, e, cx, cy);
      }
    }
    if constexpr (MODE == kTileGeneric) {
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = (cm[j] && row_ok) ? r[j] : b[j];
    } else if constexpr (MODE == kTileLeft) {
      r[0] = cm[0] ? b[0] : r[0];  // cm[0]: this lane holds plate column 0
    } else if constexpr (MODE >= kTileRight) {
      r[MODE - kTileRight] = cm[0] ? b[MODE - kTileRight] : r[MODE - kTileRight];
    }
    return r;
  }
};

struct TileNoSink;

// A wave's mode from its global rows [wx_lo, wx_hi] and the tile's global
// columns [gy_lo, gy_hi].  Lanes hold 4 columns starting at a global column
// = gy0 (mod 4).
__device__ __forceinline__ int tile_mode(const StencilGeom& g, int64_t wx_lo, int64_t wx_hi,
                                         int64_t gy_lo, int64_t gy_hi, bool no_edge_rows = false) {
  const bool edge_row = !no_edge_rows &&
                        ((wx_lo <= 0 && 0 <= wx_hi) || (wx_lo <= g.nx - 1 && g.nx - 1 <= wx_hi));
  const bool left = gy_lo < 1, right = gy_hi > g.ny - 2;
  if (edge_row || (left && right)) return kTileGeneric;
  if (!left && !right) return kTileInterior;
  if (left) return (g.gy0 & 3) == 0 ? kTileLeft : kTileGeneric;
  return kTileRight + int((g.ny - 1 - g.gy0) & 3);
}

// The K steps of a pass (K even) as (down, up) pairs, the last step's body
// LAST_WHAT: st(down_c, what_c, acc_c, s) for s = 0..K-1.
//   ACC_MODE 0: no residual anywhere;
//   ACC_MODE 1: every step is the accumulating body (acc_c true) and the
//     caller's per-step row mask picks the check's step (a per-row branch in
//     every step: ~16 % slower per pass; the tile kernel's check passes);
//   ACC_MODE 2: only the last step is the accumulating body, its row mask
//     zero unless the pass ends at a check (the resident kernel: its spans
//     take checks at pass ends; the other steps stay free of residual code).
//     Choosing between two last-step bodies per pass, or a body per check
//     step, spilled 80-330 B/lane.
//   ACC_MODE 3: as 2, plus an accumulating UP body inside the loop, taken at
//     step acc_step (odd: an even level, 2..K-2) by a uniform branch; the
//     last step is the accumulating body as in mode 2 (the caller zeroes its
//     row mask unless acc_step == K - 1).  The resident kernel's checks at
//     inner even levels (depth 12, a check every 20 or 50 steps: levels 8,
//     4, 12 / 2, 4, ..., 12), so depth 10 is no longer forced on them.
template <int ACC_MODE, int LAST_WHAT, class StepFn>
__device__ __forceinline__ void tile_pass_steps(int K, StepFn&& st, int acc_step = -1) {
  using Down = std::true_type;
  using Up = std::false_type;
  using Plain = std::integral_constant<int, 0>;
  using Last = std::integral_constant<int, LAST_WHAT>;
  using A = std::integral_constant<bool, ACC_MODE == 1>;
  using AL = std::integral_constant<bool, ACC_MODE != 0>;
  int s = 0;
  if constexpr (ACC_MODE == 3) {
    // The pairs before the check's pair, the check's pair, the rest: two
    // loops of the one plain body around it (a branch between two up
    // bodies inside one loop spilled 556 B/lane, all of it in the loop).
    const int q = (acc_step >= 1 && acc_step + 2 < K) ? acc_step - 1 : K;
    for (; s + 2 < K && s < q; s += 2) {
      st(Down{}, Plain{}, A{}, s);
      st(Up{}, Plain{}, A{}, s + 1);
    }
    if (s == q) {
      st(Down{}, Plain{}, A{}, s);
      st(Up{}, Plain{}, std::true_type{}, s + 1);
      s += 2;
    }
  }
  for (; s + 2 < K; s += 2) {
    st(Down{}, Plain{}, A{}, s);
    st(Up{}, Plain{}, A{}, s + 1);
  }
  st(Down{}, Plain{}, A{}, s);
  st(Up{}, Last{}, AL{}, s + 1);
}

// Calls f(std::integral_constant<int, MODE>) for the tile's mode.  The edge
// modes are built for the mixed lane shifts (XL 2) and, for the unchecked
// resident DPP launches (XL 0, RES 0), the left and the element-3 right
// mode: a plate of a multiple of 4 columns whose local column 0 is global
// column 0 mod 4 (every power-of-two grid and its rank boxes) has its last
// column in element 3.  They cost 12 B/lane on the 12-row RES 0 kernels and
// gained 0-3 % on the 8-GPU rank boxes (2192 x 4168 at 7-pass spans 4.40-4.51
// vs 4.26-4.38, 2048 x 4096 4.42-4.47 vs 4.33-4.36; sessions r6o, r6p); with
// the residual code (RES 1) they spilled 68 -> 172 B/lane.  XL0_EDGES: the
// caller is such a launch (<= kTilePkRows rows: taller DPP builds only run
// when forced; 20 x 16 spilled 20 B/lane with them).  Everything else takes the generic path on its
// edge tiles.
template <int XL, bool XL0_EDGES = false, class F>
__device__ __forceinline__ float tile_dispatch(int mode, F&& f) {
  using std::integral_constant;
  if (mode == kTileInterior) return f(integral_constant<int, kTileInterior>{});
  if constexpr (XL == 0 && XL0_EDGES) {
    if (mode == kTileLeft) return f(integral_constant<int, kTileLeft>{});
    if (mode == kTileRight + 3) return f(integral_constant<int, kTileRight + 3>{});
  }
  if constexpr (XL == 2) {
    switch (mode) {
      case kTileLeft: return f(integral_constant<int, kTileLeft>{});
      case kTileRight + 0: return f(integral_constant<int, kTileRight + 0>{});
      case kTileRight + 1: return f(integral_constant<int, kTileRight + 1>{});
      case kTileRight + 2: return f(integral_constant<int, kTileRight + 2>{});
      case kTileRight + 3: return f(integral_constant<int, kTileRight + 3>{});
      default: break;
    }
  }
  return f(integral_constant<int, kTileGeneric>{});
}

// Mode-dependent setup of an Upd and the tile's row mask (rows row0 + r,
// r < R, that are global interior rows).
template <int MODE, int XL>
__device__ __forceinline__ void tile_mode_setup(Upd<MODE, XL>& up, const StencilGeom& g,
                                                int64_t col, unsigned interior_rows,
                                                unsigned& rowmask) {
  rowmask = MODE == kTileGeneric ? interior_rows : ~0u;
  if constexpr (MODE == kTileGeneric) {
#pragma unroll
    for (int j = 0; j < 4; ++j) up.cm[j] = tbdetail::in_interior(g.gy0 + col + j, g.ny);
  } else if constexpr (MODE == kTileLeft) {
    up.cm[0] = g.gy0 + col == 0;
  } else if constexpr (MODE >= kTileRight) {
    up.cm[0] = g.gy0 + col + (MODE - kTileRight) == g.ny - 1;
  }
}

// RES 1: the instantiation that takes residuals; the step that takes one is
// its own body (step<.., ACC = true>: max |new - old| over the useful rows
// in `resmask`), so the other steps carry no residual code (a per-row
// branch in every step split the rows into basic blocks: 13 % slower).
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
  // WHAT 3: every row goes to sink->row(r, new, old) as soon as it is
  // computed (the last step's stores: RowStoreSink, or the resident
  // kernel's edge-band publish); 0: nothing.  ACC: this step accumulates
  // max |new - old| over the useful rows in resmask.
  template <bool DOWN, int WHAT, bool ACC = false, class Xc, class Sink = TileNoSink>
  __device__ __forceinline__ void step(const vecf& first_nb, Xc& xc, const Upd<MODE, XL>& up,
                                       unsigned rowmask, unsigned usemask, bool store_lane, int rc,
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
      u[r] = up.template apply<(R <= kTilePkRows && (RES == 0 || XL == 0))>(n, cur, so, wl[r], er[r],
                                                                (rowmask >> r) & 1u);
      if (i == 0) xc.publish(0, u[r]);
      if (i == R - 1) xc.publish(1, u[r]);
      if constexpr (WHAT == 3) sink->row(r, u[r], cur);
      if constexpr (ACC) {
        // Branch-free: a uniform branch per row split the step into basic
        // blocks the scheduler cannot interleave.
        acc_sel(u[r], cur, res_lane, res_cols, ((usemask & resmask) >> r) & 1u);
      }
      prev = cur;
      if (i == R / 2 - 1) last_nb = xc.mid();
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // acc without branches: `take` (uniform), res_lane and the lane's element
  // count fold into one select per element (the uniform row bit ANDs into the
  // per-lane masks on the scalar unit), then two NaN-propagating
  // v_maximum3_f32 with abs modifiers: 10 VALU per row (was 14: a select per
  // element, then one for the lane and one for the row).
  __device__ __forceinline__ void acc_sel(const vecf& nw, const vecf& old, bool res_lane, int rc,
                                          bool take) {
    float c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = (take && res_lane && (j == 0 || rc > j)) ? nw[j] - old[j] : 0.f;
    m = __builtin_elementwise_maximum(
        __builtin_elementwise_maximum(m, __builtin_fabsf(c[0])), __builtin_fabsf(c[1]));
    m = __builtin_elementwise_maximum(
        __builtin_elementwise_maximum(m, __builtin_fabsf(c[2])), __builtin_fabsf(c[3]));
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

// The last step's stores of a wave's useful rows to dst, branch-free: one
// buffer resource per row (the strip's 256 columns, built on the scalar
// unit: no 32-bit limit on the field's size) and an out-of-range voffset
// for a lane or row that does not store (the range check drops it).  A
// per-row `if` around a store made every row of the step its own basic
// block; the step's lane shifts were then hoisted ahead of its barrier and
// tall tiles spilled (profiles/r5_spills.md).
constexpr int kNoStore = int(0x80000000u);
struct RowStoreSink {
  float* base;  // the wave's first row, the strip's first column
  int64_t pitch;
  unsigned usemask;
  int vs;  // this lane's voffset (kNoStore: not a stored lane)
  __device__ __forceinline__ void row(int r, const vecf& v, const vecf&) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + r * pitch, 0, 1024, 0x00020000);
    const int vo = ((usemask >> r) & 1u) ? vs : kNoStore;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, vo, 0, 0);
  }
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
