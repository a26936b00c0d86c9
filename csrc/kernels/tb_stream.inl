// Register-streaming temporally blocked Jacobi kernel (the hot kernel).
//
// Included by stencil.hip (namespace heat::gpu::tbp, explicit packed-fp32
// row update) and tb_scalar.hip (namespace heat::gpu::tbs, compiled with
// -fno-slp-vectorize: scalar row update).  The two builds exist so the row
// update's instruction selection can be A/B-timed in one process.
//
// Structure (one wave = one 64*V-column strip x one chunk of rows):
//   lane l holds columns [Vl, Vl+V) of the strip as a float4 (V=4) or a
//   float2 (V=2, the narrow-strip build tb_narrow.hip);
//   level 0 = the input rows, level s = the field after s steps;
//   every loop iteration loads one input row and advances every level by one
//   row, keeping each level's last rows in a register ring;
//   east/west neighbours cross lanes with DPP wave_shr:1 / wave_shl:1.
// LAG selects the pipeline skew: level s works on row i - LAG*s (LAG 0 is the
// 2-slot ring below, skew 1).
//   LAG 1: 3-row rings; the K levels of one iteration form one dependency
//          chain (level s consumes the row level s-1 produced this iteration).
//   LAG 2: 4-row rings; level s consumes only rows produced in earlier
//          iterations, so the K updates of an iteration are independent
//          (K-way instruction-level parallelism) at the cost of 4/3 the
//          ring registers and K more pipeline-fill iterations.
#ifndef HEAT_TB_NS
#error "define HEAT_TB_NS"
#endif
// Columns per lane: 4 (float4, 256-column strips) or 2 (float2, 128-column
// strips: twice the strips, so twice the chunk length at the same wave count
// on small blocks, at 2x the relative strip overlap).
#ifndef HEAT_TB_V
#define HEAT_TB_V 4
#endif
#if HEAT_TB_PACKED && HEAT_TB_V != 4
#error "the packed row update is written for float4 lanes"
#endif
// Row cache policy.  HEAT_TB_NTSTORE / HEAT_TB_NTLOAD 1: non-temporal output
// stores / input-row loads (the streaming build tb_split_nt.hip, taken when
// one pass sweeps more than the MALL holds: the rows a pass writes are read
// back one whole-field sweep later, past L2 and the MALL).  8192^2 bench
// 5.03-5.09 -> 5.24-5.25 Tcells/s, 131072^2 5.53 -> 5.63; but the 4096 x
// 8192 plate (134 MB, inside the MALL) 4.76-4.83 -> 4.66-4.70, so the
// smaller fields keep the plain build (profiles/r5_stores.md).
// (Round 5's buffer-store and fixed-row-store experiment builds,
// profiles/r5_stores.md, were removed in round 6.)
#ifndef HEAT_TB_NTSTORE
#define HEAT_TB_NTSTORE 0
#endif
#ifndef HEAT_TB_NTLOAD
#define HEAT_TB_NTLOAD 0
#endif
// Chained level-split passes (tb_chain.hip, tb_chain_kernel): the cache
// policy of their write-through stores (16 = sc1).
#ifndef HEAT_TB_CHAIN
#define HEAT_TB_CHAIN 0
#endif
#ifndef HEAT_TB_CHAIN_AUX
#define HEAT_TB_CHAIN_AUX 16
#endif
// s_sleep argument between a chained unit's flag polls.
#ifndef HEAT_TB_CHAIN_SLEEP
#define HEAT_TB_CHAIN_SLEEP 1
#endif
#if HEAT_TB_CHAIN && HEAT_TB_V != 4
#error "the chained build stores float4 rows through buffer stores of its own"
#endif

namespace heat::gpu::HEAT_TB_NS {

constexpr int V = HEAT_TB_V;
typedef float vecf __attribute__((ext_vector_type(HEAT_TB_V)));

using heat::gpu::tbdetail::TbArgs;
using heat::gpu::tbdetail::TbBox;
using heat::gpu::tbdetail::in_interior;
using heat::gpu::tbdetail::wave_max_atomic;
using heat::gpu::tbdetail::kSplitRing;

// Lane 0 (from_left) / lane 63 (from_right) has no source lane and reads 0
// (bound_ctrl); those lanes lie in the strip overlap, so the value is
// don't-care.  bound_ctrl lets the compiler fold both shifts into the
// consuming v_add_f32_dpp; with old = 0 and bound_ctrl off it only folded
// wave_shr and materialised wave_shl as v_mov 0 + v_mov_b32_dpp + v_add.
// A DPP wave shift left (lane l <- lane l-1), folded by the compiler into
// the consuming v_add_f32_dpp: the left shift of the mixed build
// (HEAT_TB_BPERMUTE 2), which sends only the right shift through the LDS
// crossbar (the workgroup-tile kernel measured +3-6 % for that split of the
// two shifts between the VALU and LDS pipes, profiles/r3_tile.md).
__device__ __forceinline__ float dpp_wave_shr(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
#if HEAT_TB_BPERMUTE
// Lane shifts through the LDS crossbar (ds_bpermute_b32, no LDS memory):
// DPP wave shifts mixed into the FMA stream stop a second wave per SIMD from
// adding throughput (tools/probes/stencil_chain.hip: ~105 cycles per float4
// row update at 1-4 waves; with ds_bpermute 82 at 2 waves, 71 at 4).  Lane
// 0 / 63 wrap around; they lie in the strip overlap (don't-care).
__device__ __forceinline__ float dpp_from_left(float v) {  // lane l <- lane l-1
  const int l = threadIdx.x & 63;
  return __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 63) & 63) << 2, __float_as_int(v)));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane l <- lane l+1
  const int l = threadIdx.x & 63;
  return __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 1) & 63) << 2, __float_as_int(v)));
}
#else
__device__ __forceinline__ float dpp_from_left(float v) {  // lane l <- lane l-1 (wave_shr:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane l <- lane l+1 (wave_shl:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}
#endif

// A wave-uniform value moved into a VGPR.  A VALU instruction with an SGPR
// operand issues at half rate on gfx950 (tools/probes/valu_rate.hip:
// v_fmac_f32 v,s,v ~4.4 cycles vs ~2.6 for v,v,v at 4 waves/SIMD), and the
// update's two coefficient FMAs would otherwise read cx/cy from SGPRs.  The
// asm result is opaque, so the compiler cannot fold it back into an SGPR.
__device__ __forceinline__ float to_vgpr(float x) {
  float r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
  return r;
}

// One input row element of this lane: row `rowp` (the strip's first
// column), lane offset `lo` floats.
__device__ __forceinline__ vecf ld_in(const float* rowp, int lo) {
#if HEAT_TB_CHAIN
  // Chained passes read rows a neighbour unit (possibly on another XCD)
  // wrote in this launch: sc1 loads (HEAT_TB_CHAIN_AUX), as the resident
  // tiles load their ghosts, so a line this XCD's L2 kept from an earlier
  // pass of the launch is never returned (the writer's sc1 stores and flag
  // pair with them).
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(rowp), 0, 4 * V * 64,
                                                                      0x00020000);
  return __builtin_bit_cast(vecf, __builtin_amdgcn_raw_buffer_load_b128(rs, int(4 * lo), 0, HEAT_TB_CHAIN_AUX));
#elif HEAT_TB_NTLOAD
  return __builtin_nontemporal_load(reinterpret_cast<const vecf*>(rowp + lo));
#else
  return *reinterpret_cast<const vecf*>(rowp + lo);
#endif
}

// Dirichlet handling modes (wave-uniform, chosen per wave in tb_kernel).
// Cells outside the plate are don't-care (their values only ever flow
// further out), so only the boundary ring itself must be kept:
//   MODE 0  interior: no wave cell is on the ring;
//   MODE 1  left edge strip: global column 0 is element 0 of one lane;
//   MODE 2+j right edge strip: global column ny-1 is element j of one lane;
//   MODE 6  generic: per-lane column masks AND the (uniform) row test.
constexpr int kModeGeneric = 6;

template <int MODE>
struct RowUpdate {
  float cx, cy;
  bool cm[V];  // MODE 6: per-column "updatable" masks; MODE 1-5: cm[0] = this
               // lane holds the boundary column
  __device__ __forceinline__ vecf operator()(const vecf& a, const vecf& b, const vecf& c,
                                             bool row_ok) const {
    return apply(a, b, c, dpp_from_left(b[V - 1]), dpp_from_right(b[0]), row_ok);
  }
  // wl / er: the west neighbour of element 0 (lane l-1's last element) and
  // the east neighbour of element V-1 (lane l+1's first), shifted by the caller.
  __device__ __forceinline__ vecf apply(const vecf& a, const vecf& b, const vecf& c, float wl,
                                        float er, bool row_ok) const {
    vecf r;
#if HEAT_TB_PACKED
    const float w = wl;
    const float e = er;
    // Explicit pairs (x,y) and (z,w): v_pk_add_f32 / v_pk_fma_f32 on aligned
    // register pairs; the east+west sums are scalar adds (two of them fuse
    // the DPP lane shift) written straight into aligned pairs.
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 m2 = {-2.0f, -2.0f}, cx2 = {cx, cx}, cy2 = {cy, cy};
    const f2 b01 = {b.x, b.y}, b23 = {b.z, b.w};
    const f2 ns01 = f2{c.x, c.y} + f2{a.x, a.y};
    const f2 ns23 = f2{c.z, c.w} + f2{a.z, a.w};
    const f2 ew01 = {b.y + w, b.z + b.x};
    const f2 ew23 = {b.w + b.y, e + b.z};
    const f2 tx01 = __builtin_elementwise_fma(m2, b01, ns01);
    const f2 tx23 = __builtin_elementwise_fma(m2, b23, ns23);
    const f2 ty01 = __builtin_elementwise_fma(m2, b01, ew01);
    const f2 ty23 = __builtin_elementwise_fma(m2, b23, ew23);
    const f2 r01 = __builtin_elementwise_fma(cy2, ty01, __builtin_elementwise_fma(cx2, tx01, b01));
    const f2 r23 = __builtin_elementwise_fma(cy2, ty23, __builtin_elementwise_fma(cx2, tx23, b23));
    r = vecf{r01.x, r01.y, r23.x, r23.y};
#else
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float w = j == 0 ? wl : b[j - 1];
      const float e = j == V - 1 ? er : b[j + 1];
      // stencil() sums e + w; for the last element pass them swapped (fp add
      // commutes, bitwise identical) so the DPP value is the operand the
      // compiler folds into v_add_f32_dpp, as it does for the first element.
      r[j] = j == V - 1 ? stencil(b[j], a[j], c[j], e, w, cx, cy)
                        : stencil(b[j], a[j], c[j], w, e, cx, cy);
    }
#endif
    if constexpr (MODE == kModeGeneric) {
      // Branch-free: keep b where the row (wave-uniform) or the column
      // (per lane) is not a global interior cell.
#pragma unroll
      for (int j = 0; j < V; ++j) r[j] = (cm[j] && row_ok) ? r[j] : b[j];
    } else if constexpr (MODE == 1) {
      r[0] = cm[0] ? b[0] : r[0];  // one v_cndmask per row and level
    } else if constexpr (MODE >= 2 && MODE - 2 < V) {
      r[MODE - 2] = cm[0] ? b[MODE - 2] : r[MODE - 2];
    }
    return r;
  }
};

// Local row r is a global interior row iff rlo <= r <= rhi (32-bit, uniform).
__device__ __forceinline__ bool row_in(int64_t r, int rlo, int rhi) {
  const int ri = int(r);
  return ri >= rlo && ri <= rhi;
}

template <int N>
__device__ constexpr int modn(int v) {
  return ((v % N) + N) % N;
}

// RS: the level (1..K) whose residual max |new - old| this launch takes (a
// check pass), 0 = none; the other passes get an instantiation without it.
// RS = K (not stage 0) is taken at emit time, next to the store; an inner
// level (or stage 0's last, which goes to the LDS ring) right after the
// level's update, over the unit's output rows [qrb, qrb + qlen): a check
// that falls inside a full-depth pass rides on it instead of cutting the
// pass (LAG 3 pipelines).
// ROLE (the level-split pipeline, tb_split.hip): 0 = the whole pipeline;
// 1 = stage 0, levels 1..K of a two-wave pipeline, emitting its last level
// into the LDS ring of the pair (all lanes, rows [rb, re) of the stage);
// 2 = stage 1, reading its input rows from that ring instead of memory.
template <int K, int LAG, int MODE, int RS, int ROLE = 0>
struct TbStream {
  static constexpr bool ROWCHK = MODE == kModeGeneric;
  static constexpr bool LASTRES = RS == K && ROLE != 1;
  static constexpr bool MIDRES = RS > 0 && !LASTRES;
  static_assert(!MIDRES || LAG == 3, "inner-level residuals need the LAG 3 pipeline");
  // LAG 3 = LAG 1 pipeline with the compile-time ramp (see run()).
  static constexpr int RING = LAG == 0 ? 2 : (LAG == 2 ? 4 : 3);
  // Prefetch distance in rows (LAG 3: part of the 6-row level-0 ring L0).
  static constexpr int PF = RING;
  static constexpr int SKEW = LAG == 2 ? 2 : 1;
  static constexpr int STEP = LAG == 2 ? 2 : 1;  // row skew per level in the ring bodies
  vecf R[K][RING];  // R[s][slot]: rows of level s (level 0 = input rows; LAG 3: s >= 1)
  vecf P[PF];       // prefetch ring (input row i + PF; LAG 0-2)
  vecf L0[LAG == 3 ? 6 : 1];  // LAG 3: level-0 rows t-2 .. t+3 (see lv())
  float m = 0.f;  // residual max |delta| (RES)
  int rc = V;  // elements of this lane inside the box (the residual skips the rest)
  int qrb = 0, qlen = 0;  // MIDRES: the unit's output rows (local, 32-bit)
  // src / dst (run() arguments) point at the strip's first column, the same
  // for every lane (scalar registers); lane l adds lo = V * l elements, so
  // loads and stores use the scalar-base + 32-bit lane-offset addressing
  // and the row arithmetic stays on the scalar unit.
  int lo = 0;
  bool nostore = false;  // diagnostics only (kTbDiagNoStore): timing without the stores
  bool cached_rows = false;  // diagnostics only (kTbDiagCachedRows): loads hit 4 rows

  // Level-split pipeline state (ROLE 1/2): a ring of kSplitRing rows of the
  // boundary level in LDS, this lane's element of each, plus two counters:
  // rows produced by stage 0 and rows released by stage 1.
  vecf* ring = nullptr;           // ring[slot * 64 + lane]
  unsigned* produced = nullptr;   // LDS, written by stage 0
  unsigned* released = nullptr;   // LDS, written by stage 1
  int64_t seq0 = 0;               // row of sequence number qoff (the stage's first_in / rb)
  int64_t qoff = 0;               // sequence number of row seq0 (segments of one unit)
  unsigned seen = 0;              // last counter value observed (polls only when needed)

  __device__ __forceinline__ vecf load_row(const float* __restrict__ src, int64_t row,
                                           int64_t pitch) {
    if constexpr (ROLE == 2) {
      // Ordering: LDS requests of one wave execute in issue order, so only
      // the compiler must keep the data access on the right side of the
      // counter access (asm memory clobbers).  Acquire/release atomics would
      // also wait for this wave's in-flight global loads and stores (vmcnt)
      // and serialise the prefetch.
      const unsigned q = unsigned(row - seq0 + qoff);
      if (q >= seen) {
        unsigned v;
        while ((v = __hip_atomic_load(produced, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <= q)
          __builtin_amdgcn_s_sleep(1);
        // Uniform (every lane read the same word): keeps the per-row test
        // `q >= seen` on the scalar unit instead of a VALU compare + branch.
        seen = __builtin_amdgcn_readfirstlane(v);
      }
      asm volatile("" ::: "memory");
      const vecf x = ring[(q % kSplitRing) * 64 + (threadIdx.x & 63)];
      asm volatile("" ::: "memory");
      // Rows before q are no longer needed (q itself may still be in flight).
      __hip_atomic_store(released, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return x;
    } else {
      if (cached_rows) row = seq0 + (row & 3);  // diagnostics: cache-resident input
      return ld_in(src + row * pitch, lo);
    }
  }

  // FAST: the caller guarantees rb <= ro < re (main-loop groups, see run())
  // and passes ro * pitch as *woff (advanced here by one pitch).
  template <bool FAST = false>
  __device__ __forceinline__ void emit(const vecf& out, const vecf& b, int64_t ro,
                                       float* __restrict__ dst, int64_t pitch, int64_t rb,
                                       int64_t re, bool store_lane, int64_t* woff = nullptr) {
    if constexpr (ROLE == 1) {
      if (FAST || (ro >= rb && ro < re)) {  // every lane: stage 1 needs the overlap columns too
        const unsigned q = unsigned(ro - seq0 + qoff);
        if (q >= seen + kSplitRing) {  // the slot's previous row may still be unread
          unsigned v;
          while ((v = __hip_atomic_load(released, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) +
                     kSplitRing <= q)
            __builtin_amdgcn_s_sleep(1);
          seen = __builtin_amdgcn_readfirstlane(v);
        }
        asm volatile("" ::: "memory");
        ring[(q % kSplitRing) * 64 + (threadIdx.x & 63)] = out;
        asm volatile("" ::: "memory");  // data before the counter (in-order LDS)
        __hip_atomic_store(produced, q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return;
    }
    int64_t off = ro * pitch;
    if constexpr (FAST) {
      off = *woff;
      *woff += pitch;
    }
    if ((FAST || (ro >= rb && ro < re)) && store_lane) {
#if HEAT_TB_CHAIN
      // Chained passes: write-through (sc1) 16-B stores, so a neighbour
      // unit on another XCD reads them after this unit's flag (drained
      // stores, then an sc1 flag store; tb_chain_kernel).
      if (!nostore) {
        typedef unsigned uvec __attribute__((ext_vector_type(V)));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + off, 0, 4 * V * 64, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uvec, out), rs, 4 * lo, 0, HEAT_TB_CHAIN_AUX);
      }
#elif HEAT_TB_NTSTORE
      if (!nostore) __builtin_nontemporal_store(out, reinterpret_cast<vecf*>(dst + off + lo));
#else
      if (!nostore) *reinterpret_cast<vecf*>(dst + off + lo) = out;
#endif
      if constexpr (LASTRES) {
        // max |delta| with the NaN-propagating IEEE-2019 maximum
        // (v_maximum3_f32, abs folded into its inputs): a NaN or inf
        // anywhere reaches the judge.  Columns past the box end (the last
        // lane's spill into padding or stale ghost columns) are written but
        // not counted.
        float d[V];
#pragma unroll
        for (int j = 0; j < V; ++j) d[j] = (j == 0 || rc > j) ? __builtin_fabsf(out[j] - b[j]) : 0.f;
#pragma unroll
        for (int j = 0; j < V; j += 2)
          m = __builtin_elementwise_maximum(m, __builtin_elementwise_maximum(d[j], d[j + 1]));
      }
    }
  }

  // MIDRES: fold max |nw - old| of level-RS row `row` (uniform) into m if
  // the row is one of the unit's output rows (this lane's stored columns).
  __device__ __forceinline__ void acc_mid(const vecf& nw, const vecf& old, int64_t row,
                                          bool store_lane) {
    if (unsigned(int(row) - qrb) < unsigned(qlen) && store_lane) {
      float d[V];
#pragma unroll
      for (int j = 0; j < V; ++j) d[j] = (j == 0 || rc > j) ? __builtin_fabsf(nw[j] - old[j]) : 0.f;
#pragma unroll
      for (int j = 0; j < V; j += 2)
        m = __builtin_elementwise_maximum(m, __builtin_elementwise_maximum(d[j], d[j + 1]));
    }
  }

  // LAG 0 / 1 / 2 iteration (the LAG 3 pipelines use body3).
  template <int U, int Q = U>
  __device__ __forceinline__ void body(int64_t i, int64_t t, const float* __restrict__ src,
                                       float* __restrict__ dst, int64_t pitch, int64_t last_in,
                                       int64_t rb, int64_t re, int rlo, int rhi,
                                       bool store_lane, const RowUpdate<MODE>& upd) {
    if constexpr (LAG == 0) {
      // Slot of row r of level s: (r - first_in) mod 2.  At iteration i level
      // s holds rows i-s-2 (slot (U-s)&1) and i-s-1 (slot (U-s-1)&1).
      vecf c = P[U];
      {
        const int64_t nxt = min(i + RING, last_in);
        P[U] = ld_in(src + nxt * pitch, lo);
      }
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int sa = modn<2>(U - s), sb = modn<2>(U - s - 1);
        const int64_t row = i - s - 1;  // row of level s+1 computed now
        const bool ok = !ROWCHK || row_in(row, rlo, rhi);
        const vecf cn = upd(R[s][sa], R[s][sb], c, ok);
        if (s == K - 1) emit(cn, R[s][sb], row, dst, pitch, rb, re, store_lane);
        R[s][sa] = c;  // level s row i-s replaces the consumed row i-s-2
        c = cn;
      }
    } else {
      R[0][U] = P[Q];
      P[Q] = load_row(src, min(i + PF, last_in), pitch);
      // Levels 1..K-1.  With LAG 2 each reads only slots written in earlier
      // iterations, so the order below carries no dependency.
#pragma unroll
      for (int s = 1; s < K; ++s) {
        const int rs = STEP * s;  // this level's row is i - rs
        const bool ok = !ROWCHK || row_in(i - rs, rlo, rhi);
        R[s][modn<RING>(U - rs)] = upd(R[s - 1][modn<RING>(U - rs - 1)],
                                       R[s - 1][modn<RING>(U - rs)],
                                       R[s - 1][modn<RING>(U - rs + 1)], ok);
      }
      const int rK = STEP * K;
      const int64_t ro = i - rK;  // output row of this iteration
      const bool ok = !ROWCHK || row_in(ro, rlo, rhi);
      const vecf& b = R[K - 1][modn<RING>(U - rK)];
      const vecf out =
          upd(R[K - 1][modn<RING>(U - rK - 1)], b, R[K - 1][modn<RING>(U - rK + 1)], ok);
      emit(out, b, ro, dst, pitch, rb, re, store_lane);
    }
  }

  // LAG 3 rows, by iteration t (input row first_in + t): level 0 row t + d
  // is L0[(t + d) mod 6] -- the three rows level 1 reads plus the three
  // prefetched ones, one ring, so no row is ever copied from a prefetch
  // buffer into the level-0 ring (with separate rings the register
  // allocator rotated them with moves at the loop back-edge, which waited
  // for the row loaded in that same iteration: vmcnt(0) every 3 rows);
  // level s > 0 row t + d is R[s][(t + d) mod 3].  s and d fold to
  // constants once the level loops are unrolled.
  __device__ __forceinline__ vecf& lv(int s, int td) {
    return s == 0 ? L0[modn<6>(td)] : R[s][modn<3>(td)];
  }

  // One LAG 3 iteration, t = T6 (mod 6).  FAST (main-loop groups, see run()):
  // the prefetched row needs no clamp and is read at src + *roff, the output
  // row needs no range test and is written at dst + *woff (both advanced by
  // one pitch per row).
  template <int T6, bool FAST>
  __device__ __forceinline__ void body3(int64_t i, const float* __restrict__ src,
                                        float* __restrict__ dst, int64_t pitch, int64_t last_in,
                                        int64_t rb, int64_t re, int rlo, int rhi,
                                        bool store_lane, const RowUpdate<MODE>& upd,
                                        int64_t* roff, int64_t* woff) {
    // Row t + 3 into the slot of row t - 3 (level 1 now reads t-2 .. t).
    if constexpr (FAST && ROLE != 2) {
      L0[modn<6>(T6 + 3)] = ld_in(src + *roff, lo);
      *roff += pitch;
    } else {
      L0[modn<6>(T6 + 3)] = load_row(src, FAST ? i + 3 : min(i + 3, last_in), pitch);
    }
#if HEAT_TB_BPERMUTE == 2
    // Mixed: the K right shifts through the LDS crossbar, issued up front;
    // each left shift a DPP wave shift at its use (folded into the add).
    float er[K + 1];
#pragma unroll
    for (int s = 1; s <= K; ++s) er[s] = dpp_from_right(lv(s - 1, T6 - s)[0]);
    __builtin_amdgcn_sched_barrier(0);
#define HEAT_TB_UPD(s, a_, b_, c_, ok_) upd.apply(a_, b_, c_, dpp_wave_shr((b_)[V - 1]), er[s], ok_)
#elif HEAT_TB_BPERMUTE
    // Every level's centre row (level s-1, row t - s) was produced in an
    // earlier iteration: issue all 2K lane shifts (LDS crossbar round trips)
    // up front so their latencies overlap, instead of each level waiting on
    // its own pair (where the scheduler otherwise puts them in stage 1).
    float wl[K + 1], er[K + 1];
#pragma unroll
    for (int s = 1; s <= K; ++s) {
      const vecf& mid = lv(s - 1, T6 - s);
      wl[s] = dpp_from_left(mid[V - 1]);
      er[s] = dpp_from_right(mid[0]);
    }
    __builtin_amdgcn_sched_barrier(0);
#define HEAT_TB_UPD(s, a_, b_, c_, ok_) upd.apply(a_, b_, c_, wl[s], er[s], ok_)
#else
#define HEAT_TB_UPD(s, a_, b_, c_, ok_) upd(a_, b_, c_, ok_)
#endif
#pragma unroll
    for (int s = 1; s < K; ++s) {  // level s computes row t - s
      const bool ok = !ROWCHK || row_in(i - s, rlo, rhi);
      lv(s, T6 - s) = HEAT_TB_UPD(s, lv(s - 1, T6 - s - 1), lv(s - 1, T6 - s),
                                  lv(s - 1, T6 - s + 1), ok);
      if constexpr (MIDRES && RS < K) {
        if (s == RS) acc_mid(lv(s, T6 - s), lv(s - 1, T6 - s), i - s, store_lane);
      }
    }
    const int64_t ro = i - K;  // output row of this iteration
    const bool ok = !ROWCHK || row_in(ro, rlo, rhi);
    const vecf& b = lv(K - 1, T6 - K);
    const vecf out = HEAT_TB_UPD(K, lv(K - 1, T6 - K - 1), b, lv(K - 1, T6 - K + 1), ok);
    if constexpr (MIDRES && RS == K) acc_mid(out, b, ro, store_lane);
#undef HEAT_TB_UPD
    emit<FAST>(out, b, ro, dst, pitch, rb, re, store_lane, woff);
  }

  template <int T, int S>
  __device__ __forceinline__ void ramp_levels(int64_t i, int rlo, int rhi, bool store_lane,
                                              const RowUpdate<MODE>& upd) {
    if constexpr (S < K) {
      if constexpr (2 * S <= T) {
        const bool ok = !ROWCHK || row_in(i - S, rlo, rhi);
        lv(S, T - S) = upd(lv(S - 1, T - S - 1), lv(S - 1, T - S), lv(S - 1, T - S + 1), ok);
        // Ramp rows of an inner level can be output rows (t >= K + S).
        if constexpr (MIDRES && S == RS) acc_mid(lv(S, T - S), lv(S - 1, T - S), i - S, store_lane);
      }
      ramp_levels<T, S + 1>(i, rlo, rhi, store_lane, upd);
    }
  }
  template <int T>
  __device__ __forceinline__ void ramp(int64_t first_in, const float* __restrict__ src,
                                       int64_t pitch, int64_t last_in, int rlo, int rhi,
                                       bool store_lane, const RowUpdate<MODE>& upd) {
    if constexpr (T < 2 * K) {
      const int64_t i = first_in + T;
      L0[modn<6>(T + 3)] = load_row(src, min(i + 3, last_in), pitch);
      ramp_levels<T, 1>(i, rlo, rhi, store_lane, upd);
      __builtin_amdgcn_sched_barrier(0);
      ramp<T + 1>(first_in, src, pitch, last_in, rlo, rhi, store_lane, upd);
    }
  }

  __device__ __forceinline__ void run(const float* __restrict__ src, float* __restrict__ dst,
                                      int64_t pitch, int64_t rb, int64_t re, int rlo, int rhi,
                                      bool store_lane, const RowUpdate<MODE>& upd) {
    // src/dst point at the strip's first column (+ lo for this lane); rows
    // are local rows.
    const int64_t first_in = rb - K, last_in = re + K - 1;
    // The last output row (re-1) leaves the pipeline at iteration re-1+SKEW*K.
    const int64_t T = (re - 1 + SKEW * K) - first_in + 1;
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
      for (int j = 0; j < RING; ++j) R[s][j] = vecf(0.f);
    if constexpr (ROLE != 1) seq0 = first_in;
    if constexpr (LAG == 3) {
#pragma unroll
      for (int j = 0; j < 6; ++j)
        L0[j] = j < 3 ? load_row(src, min(first_in + j, last_in), pitch) : vecf(0.f);
      // Pipeline ramp: during iteration t < 2K only levels s <= t/2 compute
      // rows the chunk's output trapezoid needs; a plain loop would compute
      // 2s useless rows per level per chunk (a third of all work for short
      // chunks).  The ramp is unrolled at compile time, one scheduling
      // region per iteration (keeps register pressure at the loop's level).
      ramp<0>(first_in, src, pitch, last_in, rlo, rhi, store_lane, upd);
      constexpr int T0 = 2 * K;
      int64_t t = T0;
      // Main-loop groups t .. t+5 with t + 5 + 3 <= last_in - first_in
      // (= T - 1): every prefetch is an in-range row and every output row
      // first_in + t - K (>= rb from t = 2K on) lies below re, so the group
      // needs neither the clamp nor the range tests (64-bit compares are
      // VALU work plus VALU->branch stalls on gfx950).  The last < 9
      // iterations run checked bodies.
      if (!cached_rows) {
        int64_t roff = (first_in + t + 3) * pitch, woff = (first_in + t - K) * pitch;
        for (; t + 9 <= T; t += 6) {
          const int64_t i = first_in + t;
          body3<(T0 + 0) % 6, true>(i, src, dst, pitch, last_in, rb, re, rlo, rhi, store_lane,
                                    upd, &roff, &woff);
          body3<(T0 + 1) % 6, true>(i + 1, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                    store_lane, upd, &roff, &woff);
          body3<(T0 + 2) % 6, true>(i + 2, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                    store_lane, upd, &roff, &woff);
          body3<(T0 + 3) % 6, true>(i + 3, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                    store_lane, upd, &roff, &woff);
          body3<(T0 + 4) % 6, true>(i + 4, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                    store_lane, upd, &roff, &woff);
          body3<(T0 + 5) % 6, true>(i + 5, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                    store_lane, upd, &roff, &woff);
        }
      }
      for (; t < T; t += 6) {
        const int64_t i = first_in + t;
        body3<(T0 + 0) % 6, false>(i, src, dst, pitch, last_in, rb, re, rlo, rhi, store_lane,
                                   upd, nullptr, nullptr);
        if (t + 1 >= T) break;
        body3<(T0 + 1) % 6, false>(i + 1, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                   store_lane, upd, nullptr, nullptr);
        if (t + 2 >= T) break;
        body3<(T0 + 2) % 6, false>(i + 2, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                   store_lane, upd, nullptr, nullptr);
        if (t + 3 >= T) break;
        body3<(T0 + 3) % 6, false>(i + 3, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                   store_lane, upd, nullptr, nullptr);
        if (t + 4 >= T) break;
        body3<(T0 + 4) % 6, false>(i + 4, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                   store_lane, upd, nullptr, nullptr);
        if (t + 5 >= T) break;
        body3<(T0 + 5) % 6, false>(i + 5, src, dst, pitch, last_in, rb, re, rlo, rhi,
                                   store_lane, upd, nullptr, nullptr);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < PF; ++j) P[j] = load_row(src, min(first_in + j, last_in), pitch);
    for (int64_t t = 0; t < T; t += RING) {
      const int64_t i = first_in + t;
      body<0>(i, t, src, dst, pitch, last_in, rb, re, rlo, rhi, store_lane, upd);
      body<1>(i + 1, t + 1, src, dst, pitch, last_in, rb, re, rlo, rhi, store_lane, upd);
      if constexpr (RING >= 3)
        body<2>(i + 2, t + 2, src, dst, pitch, last_in, rb, re, rlo, rhi, store_lane, upd);
      if constexpr (RING == 4)
        body<3>(i + 3, t + 3, src, dst, pitch, last_in, rb, re, rlo, rhi, store_lane, upd);
    }
  }
};

// Register budget: waves per SIMD each instantiation must keep (the edge
// path and the ramp otherwise inflate the allocation for every wave).
template <int K, int LAG>
constexpr int tb_waves_per_simd() {
  // float2 lanes: half the ring registers.
  if (V == 2) return K <= 4 ? 8 : K <= 6 ? 6 : 5;
  if (LAG == 2) return K <= 4 ? 4 : 2;
  return K <= 2 ? 6 : K <= 4 ? 5 : K <= 6 ? 4 : K <= 8 ? 3 : 2;
}

// Grid position -> (work unit, age half); see kTbAgePairs / kTbXcdGroups.
// `per_block` work units per block (4 waves, or 2 two-wave pipelines).
__device__ __forceinline__ int tb_unit(const TbArgs& a, int per_block, int sub, int& age) {
  // Age pairs (kTbAgePairs): the grid is two halves of one block per CU
  // each; a CU runs block i of the first half (dispatched first: the OLDER
  // wave on each SIMD, which the SIMD's issue arbitration favours) next to
  // block i of the second half.  Wave i of both halves takes the same pair
  // of vertically adjacent chunks, the older one the longer share.
  const bool pairs = a.flags & tbdetail::kTbAgePairs;
  int nb = gridDim.x, blk = blockIdx.x;
  age = 0;
  if (pairs) {
    nb /= a.age_groups;  // the launch makes the grid a multiple of age_groups
    age = min(blk / nb, a.age_groups - 1);
    blk -= age * nb;
  }
  if (a.flags & tbdetail::kTbXcdGroups) {
    const int q = nb >> 3, r = nb & 7, x = blk & 7, j = blk >> 3;
    blk = x * q + min(x, r) + j;
  }
  return blk * per_block + sub;
}

// One segment of a work unit: rows [rb, re) of one strip of box bx.  K1 =
// 0: one wave runs all K levels; K1 > 0: a two-wave pipeline, stage 0
// levels 1..K1 (into the LDS ring), stage 1 levels K1+1..K (`ring`, `cnt`:
// the pair's LDS ring and its two counters; `qoff`: ring sequence number of
// the segment's first row, so consecutive segments of one unit keep the
// ring protocol's numbers monotonic).  RLM > 0: a check pass whose residual
// is taken at pipeline level RLM < K (stage 0 if RLM <= K1); only the
// interior and generic Dirichlet modes are built for it (edge strips take
// the generic path).  Returns this lane's residual max.
template <int K, int LAG, int K1, int RLM = 0>
__device__ __forceinline__ float tb_segment(const TbArgs& a, const TbBox& bx, int strip,
                                               int chunk, int64_t rb, int64_t re, int stage,
                                               vecf* ring, unsigned* cnt, int64_t qoff,
                                               const float* sbase = nullptr,
                                               float* dbase = nullptr) {
  constexpr int KK = (K + V - 1) / V * V;  // strip overlap per side, whole lanes
  constexpr int W = 64 * V - 2 * KK;
  constexpr int K2 = K - K1;               // levels of stage 1
  const int lane = threadIdx.x & 63;
  const int64_t cbase = bx.c0 + int64_t(strip) * W;
  const int64_t cend = min(cbase + W, bx.c1);
  const int64_t col = cbase - KK + V * lane;
  const bool store_lane = col >= cbase && col < cend;

  const StencilGeom& g = a.g;
  // wave-uniform; + lo per lane.  sbase / dbase: the chained launch's
  // ping-pong fields of the current pass (tb_chain_kernel).
  const float* src = (sbase ? sbase : a.src) + (cbase - KK);
  float* dst = (dbase ? dbase : a.dst) + (cbase - KK);
  int64_t pitch = g.pitch;
  const bool want_resid = a.resid != nullptr;

  // Wave-uniform fast path: every row and column the wave touches is a
  // global interior cell, so no Dirichlet masking is needed.
  const int64_t gy_lo = g.gy0 + cbase - KK, gy_hi = gy_lo + 64 * V - 1;
  const int64_t gx_lo = g.gx0 + rb - K, gx_hi = g.gx0 + re + K - 1;
  // Updatable local rows (global 1..nx-2), clamped into int32.
  int rlo = int(max<int64_t>(1 - g.gx0, -(int64_t(1) << 30)));
  int rhi = int(min<int64_t>(g.nx - 2 - g.gx0, int64_t(1) << 30));
  if ((a.flags & tbdetail::kTbAltDirection) && (chunk & 1)) {
    // Stream this chunk bottom-up: mirror rows r -> M - r about the chunk
    // (the same row set [rb-K, re+K) is read, [rb, re) written).
    const int64_t M = rb + re - 1;
    src += M * pitch;
    dst += M * pitch;
    pitch = -pitch;
    const int lo = rlo, hi = rhi;
    rlo = int(max<int64_t>(M - hi, -(int64_t(1) << 30)));
    rhi = int(min<int64_t>(M - lo, int64_t(1) << 30));
  }
  float m = 0.f;
  // Which Dirichlet mode this wave needs (all wave-uniform).
  const bool rows_in = gx_lo >= 1 && gx_hi <= g.nx - 2;
  const bool left = gy_lo < 1, right = gy_hi > g.ny - 2;
  int mode = kModeGeneric;
  if (rows_in && !left && !right) mode = 0;
  else if (rows_in && left && !right && g.gy0 == 0) mode = 1;
  else if (rows_in && right && !left) mode = 2 + int((g.ny - 1 - g.gy0) & (V - 1));
  const int64_t gy = g.gy0 + col;
  auto go2 = [&](auto mode_c, auto res_c) {
    constexpr int MD = decltype(mode_c)::value;
    RowUpdate<MD> upd;
    upd.cx = to_vgpr(g.cx);
    upd.cy = to_vgpr(g.cy);
    if constexpr (MD == kModeGeneric) {
#pragma unroll
      for (int j = 0; j < V; ++j) upd.cm[j] = in_interior(gy + j, g.ny);
    } else if constexpr (MD == 1) {
      upd.cm[0] = gy == 0;  // element 0 of this lane is global column 0
    } else if constexpr (MD >= 2) {
      upd.cm[0] = gy <= g.ny - 1 && g.ny - 1 < gy + V;  // this lane holds column ny-1
    }
    constexpr bool RES = decltype(res_c)::value;
    // Residual level of each stream (0 = none), see TbStream RS.
    constexpr int RS_ALL = RLM > 0 ? RLM : (RES ? K : 0);
    constexpr int RS_ST0 = (RLM > 0 && RLM <= K1) ? RLM : 0;
    constexpr int RS_ST1 = RLM > K1 ? RLM - K1 : ((RLM == 0 && RES) ? K2 : 0);
    if constexpr (K1 == 0) {
      TbStream<K, LAG, MD, RS_ALL> st;
      st.lo = V * lane;
      st.rc = int(min<int64_t>(cend - col, V));
      st.qrb = int(rb);
      st.qlen = int(re - rb);
      st.nostore = a.flags & tbdetail::kTbDiagNoStore;
      st.cached_rows = a.flags & tbdetail::kTbDiagCachedRows;
      st.run(src, dst, pitch, rb, re, rlo, rhi, store_lane, upd);
      m = st.m;
    } else if (stage == 0) {
      // Level-K1 rows [rb - K2, re + K2): exactly what stage 1's trapezoid reads.
      TbStream<K1, LAG, MD, RS_ST0, 1> st;
      st.lo = V * lane;
      st.rc = int(min<int64_t>(cend - col, V));
      st.qrb = int(rb);
      st.qlen = int(re - rb);
      st.ring = ring;
      st.produced = cnt;
      st.released = cnt + 1;
      st.seq0 = rb - K2;
      st.qoff = qoff;
      st.cached_rows = a.flags & tbdetail::kTbDiagCachedRows;
      st.run(src, dst, pitch, rb - K2, re + K2, rlo, rhi, store_lane, upd);
      m = st.m;  // an inner-level residual of stage 0's levels (RS_ST0)
    } else {
      TbStream<K2, LAG, MD, RS_ST1, 2> st;
      st.lo = V * lane;
      st.ring = ring;
      st.produced = cnt;
      st.released = cnt + 1;
      st.qoff = qoff;
      st.rc = int(min<int64_t>(cend - col, V));
      st.qrb = int(rb);
      st.qlen = int(re - rb);
      st.nostore = a.flags & tbdetail::kTbDiagNoStore;
      st.run(src, dst, pitch, rb, re, rlo, rhi, store_lane, upd);
      m = st.m;
    }
  };
  auto go = [&](auto mode_c) {
    if (RLM > 0 || !want_resid) go2(mode_c, std::false_type{});
    else go2(mode_c, std::true_type{});
  };
  if constexpr (RLM > 0) {
    if (mode == 0) go(std::integral_constant<int, 0>{});
    else go(std::integral_constant<int, kModeGeneric>{});
    return m;
  }
  switch (mode) {
    case 0: go(std::integral_constant<int, 0>{}); break;
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 3: go(std::integral_constant<int, 3>{}); break;
    case 4:
      if constexpr (V > 2) go(std::integral_constant<int, 4>{});
      break;
    case 5:
      if constexpr (V > 2) go(std::integral_constant<int, 5>{});
      break;
    default: go(std::integral_constant<int, kModeGeneric>{}); break;
  }
  return m;
}

// Linear (balanced) plans: the launch's boxes are one sequence of strip-rows
// (box-major, strip-major); unit boundaries are multiples of total/units,
// moved to a strip end when they fall within `slack` rows of one (no tiny
// segments, each of which would pay a whole pipeline ramp).
__device__ __forceinline__ int64_t tb_lin_boundary(const TbArgs& a, int64_t x) {
  if (x <= 0 || x >= a.lin_total) return min(max(x, int64_t(0)), a.lin_total);
  int bi = 0;
#pragma unroll
  for (int j = 1; j < tbdetail::kMaxBoxes; ++j)
    if (j < a.nbox && x >= a.box[j].lin0) bi = j;
  const int64_t rows = a.box[bi].r1 - a.box[bi].r0;
  const int64_t r = (x - a.box[bi].lin0) % rows;
  if (r < a.lin_slack) return x - r;
  if (rows - r < a.lin_slack) return x + (rows - r);
  return x;
}

// One work unit.  Classic plans: a (strip, chunk) of a box (with age pairs a
// group of G chunks split between G units).  Linear plans: a range of the
// strip-row sequence, run as consecutive segments (a strip end, a box end
// or a row where the Dirichlet mode changes starts a new segment).
// LIN: 0 classic plans only, 1 linear plans only, 2 either (the launch's
// kTbLinear flag at run time).  The level-split launches instantiate 0 and 1
// separately, so the classic kernel carries no inlined copy of the linear
// segment loop (its register allocation and ramp spills stay those of the
// classic body alone).
template <int K, int LAG, int K1, int RLM = 0, int LIN = 2>
__device__ __forceinline__ void tb_run(const TbArgs& a, int wave, int age, int stage, vecf* ring,
                                       unsigned* cnt, unsigned* wg, int nact) {
  constexpr int K2 = K - K1;
  const int lane = threadIdx.x & 63;
  const bool pairs = a.flags & tbdetail::kTbAgePairs;
  const unsigned long long t_start = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
  float m = 0.f;
  int strip = 0, chunk = wave;
  const bool linear = LIN == 2 ? bool(a.flags & tbdetail::kTbLinear) : LIN == 1;
  int64_t x0 = 0, x1 = 1;  // linear: this unit's strip-row range
  if (linear) {
    const int64_t U = a.total_waves;
    x0 = tb_lin_boundary(a, (a.lin_total * wave) / U);
    x1 = tb_lin_boundary(a, (a.lin_total * (wave + 1)) / U);
    if (pairs) {
      const int64_t span = x1 - x0;
      const int64_t y0 = x0 + (span * a.age_cum[age]) / 1024;
      x1 = x0 + (span * a.age_cum[age + 1]) / 1024;
      x0 = y0;
    }
  }
  if (!linear) {
    // Classic plan: one (strip, chunk) segment, called directly (a loop
    // around the inlined segment body measured ~3 % slower at 8192^2).
    int bi = 0;
#pragma unroll
    for (int j = 1; j < tbdetail::kMaxBoxes; ++j)
      if (j < a.nbox && wave >= a.box[j].wave_begin) bi = j;
    const TbBox& bx = a.box[bi];
    const int w = wave - bx.wave_begin;
    strip = w % bx.nstrips;
    chunk = w / bx.nstrips;
    int64_t rb = bx.r0 + int64_t(chunk) * bx.chunk_len;
    int64_t re = min(rb + bx.chunk_len, bx.r1);
    if (pairs) {
      // Box chunks are groups of G * chunk_len rows; age a takes rows
      // [age_cum[a], age_cum[a+1]) / 1024 of its group.
      const int G = a.age_groups;
      const int64_t p0 = bx.r0 + int64_t(chunk) * G * bx.chunk_len;
      const int64_t p1 = min(p0 + G * int64_t(bx.chunk_len), bx.r1);
      rb = p0 + ((p1 - p0) * a.age_cum[age]) / 1024;
      re = p0 + ((p1 - p0) * a.age_cum[age + 1]) / 1024;
    }
    if (rb < re) m = tb_segment<K, LAG, K1, RLM>(a, bx, strip, chunk, rb, re, stage, ring, cnt, 0);
  } else {
    // Linear plan: as many segments as the unit's range crosses.
    int64_t qoff = 0;
    while (x0 < x1) {
      int bi = 0;
#pragma unroll
      for (int j = 1; j < tbdetail::kMaxBoxes; ++j)
        if (j < a.nbox && x0 >= a.box[j].lin0) bi = j;
      const TbBox& bx = a.box[bi];
      const int64_t rows = bx.r1 - bx.r0;
      const int64_t off = x0 - bx.lin0;
      strip = int(off / rows);
      const int64_t rb = bx.r0 + off % rows;
      int64_t re = min(bx.r1, rb + (x1 - x0));
      // Rows whose K-window reaches the plate's top / bottom row run the
      // masked (generic) path: keep them in segments of their own.
      const int64_t top = 1 - a.g.gx0 + K, bot = a.g.nx - 1 - a.g.gx0 - K;
      if (rb < top && re > top) re = top;
      else if (rb < bot && re > bot) re = bot;
      x0 += re - rb;
      m = __builtin_elementwise_maximum(
          m, tb_segment<K, LAG, K1, RLM>(a, bx, strip, chunk, rb, re, stage, ring, cnt, qoff));
      qoff += (re - rb) + 2 * K2;
    }
  }
  // One contributor per pipeline: the wave whose levels hold the residual.
  constexpr int res_stage = (RLM > 0 && RLM <= K1) ? 0 : 1;
  if (a.resid != nullptr && (K1 == 0 || stage == res_stage))
    tbdetail::group_max_atomic(__float_as_uint(m), a.resid, wg, nact);
  if (a.stamps && lane == 0) {
    const int64_t idx = int64_t(wave) + int64_t(age) * a.total_waves;
    unsigned long long* st = a.stamps + 4 * (K1 == 0 ? idx : 2 * idx + stage);
    st[0] = t_start;
    st[1] = __builtin_amdgcn_s_memrealtime();
    // HW_ID (wave, SIMD, CU, SE ids) and XCC_ID via s_getreg.
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
    st[2] = ((unsigned long long)blockIdx.x << 40) | ((unsigned long long)xcc << 32) | hw;
    st[3] = ((unsigned long long)strip << 32) | unsigned(chunk);
  }
}

template <int K, int LAG>
__global__ __launch_bounds__(256, (tb_waves_per_simd<K, LAG>())) void tb_kernel(TbArgs a) {
  __shared__ unsigned wg[2];  // residual: block max, contributors done
  if (tbdetail::gated(a.g.gate)) return;
  if (threadIdx.x < 2) wg[threadIdx.x] = 0u;
  __syncthreads();
  int age = 0;
  const int wave = tb_unit(a, 4, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), age);
  int nact = 0;  // waves of this block with a unit (all contribute a residual)
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    int ag = 0;
    nact += tb_unit(a, 4, s, ag) < a.total_waves ? 1 : 0;
  }
  if (wave >= a.total_waves) return;
  tb_run<K, LAG, 0>(a, wave, age, 0, nullptr, nullptr, wg, nact);
}

#if HEAT_TB_SPLIT
// Level-split pipeline: a block is two pipelines of two waves; wave 2p runs
// levels 1..K1 of pipeline p's (strip, chunk), wave 2p+1 levels K1+1..K,
// fed through an LDS ring.  Same chunks and ramp as one wave doing all K
// levels, at twice the waves per SIMD (half the ring registers per wave):
// a lone wave issues a VALU op every ~5 cycles, two ~2.5
// (profiles/tb_wave_timeline_r1.md).
template <int K, int K1>
constexpr int tb_split_waves_per_simd() {
  return tb_waves_per_simd<(K1 > K - K1 ? K1 : K - K1), 3>();
}
template <int K, int K1, int RLM = 0, int LIN = 2>
__global__ __launch_bounds__(256, (tb_split_waves_per_simd<K, K1>())) void tb_split_kernel(TbArgs a) {
  __shared__ vecf ring[2][kSplitRing * 64];
  __shared__ unsigned cnt[2][2];
  __shared__ unsigned wg[2];  // residual: block max, contributors done
  if (tbdetail::gated(a.g.gate)) return;  // the same value for every wave of the block
  if (threadIdx.x < 4) cnt[threadIdx.x >> 1][threadIdx.x & 1] = 0;
  if (threadIdx.x < 2) wg[threadIdx.x] = 0u;
  __syncthreads();
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int p = wid >> 1;
  int age = 0;
  const int unit = tb_unit(a, 2, p, age);
  int nact = 0;  // pipelines of this block with a unit (their stage-1 wave contributes)
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    int ag = 0;
    nact += tb_unit(a, 2, q, ag) < a.total_waves ? 1 : 0;
  }
  if (unit >= a.total_waves) return;
  tb_run<K, 3, K1, RLM, LIN>(a, unit, age, wid & 1, ring[p], cnt[p], wg, nact);
}
#endif

#if HEAT_TB_SPLIT && HEAT_TB_CHAIN
// Chained level-split passes (tb_chain.hip): ONE launch runs `passes`
// depth-K passes of a one-box classic plan, ping-ponging between a.src and
// a.dst, with no grid-wide boundary between passes.  A per-pass launch ends
// when its slowest pipeline does (busy fraction 0.81 at 8192^2: the waves of
// a pass end between 135 and 184 us, tools/wave_timeline.py); here a unit
// starts pass p as soon as the units whose rows it reads (and will
// overwrite) finished pass p - 1, and a waiting wave leaves its SIMD's issue
// slots to the waves beside it.
//   unit u = (strip s, chunk group c, age a); flags[u] = passes it finished.
//   Stage 1 (the only wave that stores the unit's rows) drains its sc1
//   stores (s_waitcnt vmcnt(0)), then one lane stores flags[u] = p + 1
//   (sc1, relaxed, agent scope).
//   Stage 0, before pass p >= 1, polls (sc1 loads) the flags of every unit
//   of strips s-1..s+1, groups c-1..c+1, all ages (itself included) until
//   they reach p: their pass p - 1 rows are stored (RAW) and their pass p - 1
//   reads of the field this pass overwrites are done (WAR: a unit's stage 0
//   finishes reading before its stage 1 finishes).  Row loads are
//   non-temporal (they bypass the CU's L1, the only cache that could hold a
//   stale copy; MI355X_MICROARCH inter-workgroup visibility).
//   Bounded polls: a give-up sets *err (grid not co-resident) and the run is
//   reported invalid by the solver, as for resident tiles.
//   The last unit to finish re-zeroes the flags and the counter.
struct ChainArgs {
  int passes;
  unsigned* flags;  // one word per unit (total_waves x age groups), zero at launch
  unsigned* done;   // units finished (zero at launch)
  unsigned* err;    // non-zero: a poll gave up
};
constexpr unsigned kChainSpinLimit = 1u << 22;

template <int K, int K1>
__global__ __launch_bounds__(256, (tb_split_waves_per_simd<K, K1>())) void tb_chain_kernel(TbArgs a,
                                                                                        ChainArgs c) {
  constexpr int K2 = K - K1;
  __shared__ vecf ring[2][kSplitRing * 64];
  __shared__ unsigned cnt[2][2];
  if (tbdetail::gated(a.g.gate)) return;  // uniform over the launch: nobody waits
  if (threadIdx.x < 4) cnt[threadIdx.x >> 1][threadIdx.x & 1] = 0;
  __syncthreads();
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pp = wid >> 1, stage = wid & 1;
  const int lane = threadIdx.x & 63;
  int age = 0;
  const int unit = tb_unit(a, 2, pp, age);
  const bool pairs = a.flags & tbdetail::kTbAgePairs;
  const int G = pairs ? a.age_groups : 1;
  const unsigned nunits = unsigned(a.total_waves) * unsigned(G);
  if (unit < a.total_waves) {
    const TbBox& bx = a.box[0];
    const int strip = unit % bx.nstrips, chunk = unit / bx.nstrips;
    const int ngroups = a.total_waves / bx.nstrips;
    int64_t rb = bx.r0 + int64_t(chunk) * bx.chunk_len;
    int64_t re = min(rb + bx.chunk_len, bx.r1);
    if (pairs) {
      const int64_t p0 = bx.r0 + int64_t(chunk) * G * bx.chunk_len;
      const int64_t p1 = min(p0 + G * int64_t(bx.chunk_len), bx.r1);
      rb = p0 + ((p1 - p0) * a.age_cum[age]) / 1024;
      re = p0 + ((p1 - p0) * a.age_cum[age + 1]) / 1024;
    }
    const int fid = unit + age * a.total_waves;
    // Stage 0: lane l < 9 G watches unit (s + l%3 - 1, c + (l/3)%3 - 1, age l/9).
    int nf = -1;
    if (stage == 0 && lane < 9 * G) {
      const int q = lane % 9, ag = lane / 9;
      const int s2 = strip + q % 3 - 1, c2 = chunk + q / 3 - 1;
      if (s2 >= 0 && s2 < bx.nstrips && c2 >= 0 && c2 < ngroups)
        nf = c2 * bx.nstrips + s2 + ag * a.total_waves;
    }
    const float* src = a.src;
    float* dst = a.dst;
    int64_t qoff = 0;
    for (int p = 0; p < c.passes; ++p) {
      if (stage == 0 && p > 0) {
        for (unsigned spins = 0;; ++spins) {
          const unsigned v =
              nf >= 0 ? __hip_atomic_load(c.flags + nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : unsigned(p);
          if (__all(v >= unsigned(p))) break;
          if (spins >= kChainSpinLimit) {
            if (lane == 0) __hip_atomic_fetch_or(c.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          __builtin_amdgcn_s_sleep(HEAT_TB_CHAIN_SLEEP);
        }
      }
      if (rb < re)
        (void)tb_segment<K, 3, K1>(a, bx, strip, chunk, rb, re, stage, ring[pp], cnt[pp], qoff, src,
                                   dst);
      qoff += (re - rb) + 2 * K2;
      if (stage == 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
          __hip_atomic_store(c.flags + fid, unsigned(p + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const float* t = src;
      src = dst;
      dst = const_cast<float*>(t);
    }
    if (stage == 1) {
      // Every other unit is past its last poll once the counter reaches
      // nunits: the last one re-zeroes the flags (all 64 lanes) and the
      // counter for the next launch.
      unsigned n = 0;
      if (lane == 0) n = __hip_atomic_fetch_add(c.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      n = __builtin_amdgcn_readfirstlane(n);
      if (n + 1 == nunits) {
        for (unsigned i = unsigned(lane); i < nunits; i += 64)
          __hip_atomic_store(c.flags + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 0) __hip_atomic_store(c.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

template <int K, int K1>
int occ_chain_k() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, tb_chain_kernel<K, K1>, 256, 0) != hipSuccess) n = 0;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(tb_chain_kernel<K, K1>)) == hipSuccess &&
      fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    n = std::min(n, std::min(8, 512 / alloc));
  }
  return std::max(0, n);
}
// Blocks per CU the chained kernel keeps resident (0: not built for depth).
int occupancy_chain(int depth) { return depth == 12 ? occ_chain_k<12, 6>() : 0; }
// One launch of `passes` chained depth-12 passes (classic plan, one box).
bool launch_chain(const TbArgs& args, int depth, int passes, unsigned* flags, unsigned* done,
                  unsigned* err, hipStream_t st) {
  if (depth != 12) return false;
  int blocks = int((args.total_waves + 1) / 2);
  if (args.flags & tbdetail::kTbAgePairs) blocks = (blocks + 7) / 8 * 8 * args.age_groups;
  ChainArgs c{passes, flags, done, err};
  hipLaunchKernelGGL((tb_chain_kernel<12, 6>), dim3(blocks), dim3(256), 0, st, args, c);
  return true;
}
#endif

#ifndef HEAT_TB_EXPERIMENT  // experiments instantiate tb_kernel<K, LAG> themselves
template <int K, int LAG>
void launch_k(const TbArgs& args, hipStream_t st) {
  int blocks = int((args.total_waves + 3) / 4);
  // Age groups: each grid part a whole number of 8-block XCD rounds, so a
  // part's local block index has the physical block's XCD (tb_unit).
  if (args.flags & tbdetail::kTbAgePairs) blocks = (blocks + 7) / 8 * 8 * args.age_groups;
  hipLaunchKernelGGL((tb_kernel<K, LAG>), dim3(blocks), dim3(256), 0, st, args);
}

template <int K, int LAG>
int occ_k() {
  // 256-thread blocks put one wave on each SIMD, so blocks/CU = waves/SIMD.
  // The occupancy API can over-report by one block per CU (MI355X_MICROARCH
  // "Residency"), so also bound it by the VGPR allocation granule of 8.
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, tb_kernel<K, LAG>, 256, 0) != hipSuccess)
    n = 1;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(tb_kernel<K, LAG>)) == hipSuccess &&
      fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    n = std::min(n, std::min(8, 512 / alloc));
  }
  return std::max(1, n);
}

#if !HEAT_TB_SPLIT_RL_LO && !HEAT_TB_SPLIT_ONLY  // those units define only split launchers
// Resident 256-thread blocks per CU of the (depth, lag) instantiation.
int occupancy(int depth, int lag) {
#if HEAT_TB_DEEP
  if (lag == 3 && depth == 12) return occ_k<12, 3>();
#endif
  if (lag == 3) {
  switch (depth) {
    case 1: return occ_k<1, 3>();
    case 2: return occ_k<2, 3>();
    case 3: return occ_k<3, 3>();
    case 4: return occ_k<4, 3>();
    case 5: return occ_k<5, 3>();
    case 6: return occ_k<6, 3>();
    case 7: return occ_k<7, 3>();
    case 8: return occ_k<8, 3>();
    default: return 1;
    }
  }
  switch (depth) {
    case 1: return occ_k<1, 1>();
    case 2: return occ_k<2, 1>();
    case 3: return occ_k<3, 1>();
    case 4: return occ_k<4, 1>();
    case 5: return occ_k<5, 1>();
    case 6: return occ_k<6, 1>();
    case 7: return occ_k<7, 1>();
    case 8: return occ_k<8, 1>();
    default: return 1;
  }
}

// Returns false if (depth, lag) is not instantiated.  A 6-row prefetch (the
// round-1 "LAG 4") measured equal to LAG 3's 3 rows
// (profiles/tb_depth_bandwidth_calibration_r1.jsonl: K=8 already moves
// ~4.4 TB/s of the ~4.9 TB/s this access pattern reaches) and was removed.  Only the skew-1
// pipelines (LAG 1, and LAG 3 = LAG 1 + ramp) are instantiated: the skew-2
// (LAG 2) and 2-slot (LAG 0) forms lost every sweep (profiles/tb_sweep_*.json)
// and only cost build time.
bool launch(const TbArgs& args, int depth, int lag, hipStream_t st) {
#if HEAT_TB_DEEP
  // K = 12: 2 waves/SIMD (256 VGPRs; the main loop is spill-free, the
  // unrolled ramp spills a little); 2/3 the HBM bytes per update of K = 8.
  // K = 10 measured between 8 and 12, K = 16 spills in the main loop
  // (profiles/tb_depth_sweep_r1.md).
  if (lag == 3 && depth == 12) {
    launch_k<12, 3>(args, st);
    return true;
  }
#endif
  if (lag == 3) {
  switch (depth) {
    case 1: launch_k<1, 3>(args, st); return true;
    case 2: launch_k<2, 3>(args, st); return true;
    case 3: launch_k<3, 3>(args, st); return true;
    case 4: launch_k<4, 3>(args, st); return true;
    case 5: launch_k<5, 3>(args, st); return true;
    case 6: launch_k<6, 3>(args, st); return true;
    case 7: launch_k<7, 3>(args, st); return true;
    case 8: launch_k<8, 3>(args, st); return true;
    default: return false;
    }
  }
  switch (depth) {
    case 1: launch_k<1, 1>(args, st); return true;
    case 2: launch_k<2, 1>(args, st); return true;
    case 3: launch_k<3, 1>(args, st); return true;
    case 4: launch_k<4, 1>(args, st); return true;
    case 5: launch_k<5, 1>(args, st); return true;
    case 6: launch_k<6, 1>(args, st); return true;
    case 7: launch_k<7, 1>(args, st); return true;
    case 8: launch_k<8, 1>(args, st); return true;
    default: return false;
  }
}

#endif  // !HEAT_TB_SPLIT_RL_LO

#if HEAT_TB_SPLIT && !HEAT_TB_CHAIN
template <int K, int K1, int RLM = 0, int LIN = 2>
void launch_split_k(const TbArgs& args, hipStream_t st) {
  int blocks = int((args.total_waves + 1) / 2);  // two pipelines per block
  if (args.flags & tbdetail::kTbAgePairs) blocks = (blocks + 7) / 8 * 8 * args.age_groups;
  hipLaunchKernelGGL((tb_split_kernel<K, K1, RLM, LIN>), dim3(blocks), dim3(256), 0, st, args);
}
#endif
#if HEAT_TB_SPLIT_RL_LO
// A build unit of inner-level residual kernels (depth 12, levels LO..HI):
// the eleven instantiations are spread over three units that compile in
// parallel (tb_split_rl{a,b,c}.hip).
template <int RL>
bool launch_split_rl_range(const TbArgs& args, int rl, hipStream_t st) {
  if constexpr (RL > HEAT_TB_SPLIT_RL_HI) {
    return false;
  } else {
    if (rl == RL) {
      launch_split_k<12, 6, RL>(args, st);
      return true;
    }
    return launch_split_rl_range<RL + 1>(args, rl, st);
  }
}
bool HEAT_TB_SPLIT_RL_FN(const TbArgs& args, int depth, int rl, hipStream_t st) {
  return depth == 12 && launch_split_rl_range<HEAT_TB_SPLIT_RL_LO>(args, rl, st);
}
#endif
#if HEAT_TB_SPLIT && !HEAT_TB_SPLIT_RL_LO && !HEAT_TB_CHAIN
template <int K, int K1>
int occ_split_k() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, tb_split_kernel<K, K1, 0, 0>, 256, 0) != hipSuccess)
    n = 1;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(tb_split_kernel<K, K1, 0, 0>)) == hipSuccess &&
      fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    n = std::min(n, std::min(8, 512 / alloc));
  }
  return std::max(1, n);
}
// Level-split launches: depth 8 (4 + 4) and 12 (6 + 6).  14 (7 + 7) and
// 16 (8 + 8) were built for an A/B and removed: 3.73 / 3.85 vs 5.02
// Tcells/s at 8192^2, bench 3.83 / 3.80 vs 5.17 (3 waves per SIMD,
// profiles/r3_raw/r3ab3_*.log).
bool launch_split(const TbArgs& args, int depth, hipStream_t st) {
  const int rl = args.res_level;
  if (args.resid != nullptr && rl > 0 && rl < depth)  // a check inside the pass
    return tbx::launch_split_rl_a(args, depth, rl, st) || tbx::launch_split_rl_b(args, depth, rl, st) ||
           tbx::launch_split_rl_c(args, depth, rl, st);
  switch (depth) {
    case 8:
      if (args.flags & tbdetail::kTbLinear) launch_split_k<8, 4, 0, 1>(args, st);
      else launch_split_k<8, 4, 0, 0>(args, st);
      return true;
    case 12:
      if (args.flags & tbdetail::kTbLinear) launch_split_k<12, 6, 0, 1>(args, st);
      else launch_split_k<12, 6, 0, 0>(args, st);
      return true;
    default: return false;
  }
}
// Resident blocks per CU (each block = 2 pipelines = 4 waves).
int occupancy_split(int depth) {
  switch (depth) {
    case 8: return occ_split_k<8, 4>();
    case 12: return occ_split_k<12, 6>();
    default: return 1;
  }
}
#endif
#endif  // HEAT_TB_EXPERIMENT
}  // namespace heat::gpu::HEAT_TB_NS
