// Shared definitions of the temporally blocked kernel builds (tb_stream.inl).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "heat/init_fn.hpp"
#include "heat/kernels.hpp"

namespace heat::gpu::tbdetail {

struct TbBox {
  int64_t r0, r1, c0, c1;
  int nstrips, nchunks, chunk_len, wave_begin;
  int64_t lin0;  // linear plans: strip-rows of the boxes before this one
};

constexpr int kMaxBoxes = 16;
// Rows of the LDS ring between the two stages of a level-split pipeline.
constexpr int kSplitRing = 8;

struct TbArgs {
  const float* src;
  float* dst;
  unsigned* resid;
  StencilGeom g;
  int nbox, total_waves;
  int flags;  // kTbXcdGroups | kTbAltDirection | kTbAgePairs ...
  // Residual level of a check pass (with resid != null): the step, 1..depth,
  // whose max |new - old| is taken.  depth (or 0) = the pass's last step; a
  // smaller level lets a check ride inside a full-depth pass instead of
  // cutting it (tb_step's res_level; tile and level-split kernels).
  int res_level;
  // kTbAgePairs: the grid is age_groups equal parts (dispatch rounds); a
  // group of age_groups vertically adjacent chunks is split between one unit
  // of each part at the cumulative row fractions age_cum[a] / 1024.
  int age_groups;
  int age_cum[5];
  // Diagnostics (null in production): per wave {start, end} of the global
  // 100 MHz s_memrealtime clock, block<<40 | XCC_ID<<32 | HW_ID and
  // strip<<32 | chunk, 4 u64
  // per wave index; see tb_set_stamps().
  unsigned long long* stamps;
  // Linear plans (kTbLinear): total strip-rows of the boxes and the slack
  // (rows) within which a unit boundary moves to a strip end.
  int64_t lin_total;
  int64_t lin_slack;
  TbBox box[kMaxBoxes];
};

// Convergence gate (StencilGeom::gate): once the judge kernel has set it,
// every later stencil launch of the run returns at once (the queued passes
// after the converging check become no-ops).
__device__ __forceinline__ bool gated(const unsigned* gate) {
  return gate != nullptr && *gate != 0u;  // uniform: one scalar load per wave
}

// Launch-time layout options (variant bits 16 and 32, see tb_step):
//   kTbXcdGroups     remap blocks so each XCD (blocks b, b+8, ... under the
//                    observed round-robin placement) gets a contiguous range
//                    of waves: vertically adjacent chunks share one L2.
//   kTbAltDirection  odd chunks stream bottom-up, so the 2K halo rows two
//                    adjacent chunks both read are read at about the same
//                    time (both at the start or both at the end).
constexpr int kTbXcdGroups = 1;
constexpr int kTbAltDirection = 2;
//   kTbAgePairs      age groups: the G blocks a CU holds (dispatch rounds:
//                    grid part a = round a) split each group of G adjacent
//                    chunks unevenly, older (earlier-dispatched) blocks taking
//                    more rows: the SIMD's issue arbitration favours older
//                    waves, so with equal chunks the youngest set the launch
//                    tail (tools/wave_timeline.py by_age_rank,
//                    profiles/tb_split_age_pairs_r2.md).
constexpr int kTbAgePairs = 4;
//   kTbDiagNoStore   diagnostics: skip the output stores (wrong results; a
//                    timing probe of the store traffic; variant bit 1024).
constexpr int kTbDiagNoStore = 8;
//   kTbDiagCachedRows diagnostics: every input row load reads one of the
//                    chunk's first 4 rows (cache-resident; wrong results, a
//                    probe of load latency; variant bit 4096).
constexpr int kTbDiagCachedRows = 16;
//   kTbLinear        balanced plan: unit u takes strip-rows [u, u+1) * total /
//                    units of the box sequence (variant bit 32768), so every
//                    SIMD gets the same work whatever the shape; a unit may
//                    run several segments (strip / box / Dirichlet-mode ends).
constexpr int kTbLinear = 32;
//   kTbStreamRows    level-split launches take the streaming build
//                    (tb_split_nt.hip: non-temporal row loads and stores)
//                    when one pass sweeps more than the MALL holds
//                    (kTbStreamBytes, HEAT_TB_NT overrides).
constexpr int kTbStreamRows = 64;

__device__ __forceinline__ bool in_interior(int64_t g, int64_t n) { return g >= 1 && g <= n - 2; }

__device__ __forceinline__ void wave_max_atomic(unsigned m, unsigned* resid) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, unsigned(__shfl_xor(int(m), off)));
  if ((threadIdx.x & 63) == 0) atomicMax(resid, m);
}

// The same with ONE global atomic per workgroup: every contributing wave
// folds its max into an LDS word wg[0] and counts itself in wg[1]; the last
// of the nact contributors (the count's acquire-release orders all earlier
// folds before it) publishes.  Per-wave atomics on the one residual word
// from thousands of waves serialise at the memory side (~7 ns each: ~37 us
// per check pass at 4000 waves).  No barrier: waves of the block may have
// exited already.  wg must be zeroed (and a barrier passed) at kernel start.
__device__ __forceinline__ void group_max_atomic(unsigned m, unsigned* resid, unsigned* wg, int nact) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, unsigned(__shfl_xor(int(m), off)));
  if ((threadIdx.x & 63) == 0) {
    // Release / acquire at workgroup scope: the memory model (not just the
    // in-order LDS queue of one wave) orders every contributor's max before
    // its count, and the last contributor's count before its read of the max.
    __hip_atomic_fetch_max(wg, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const unsigned n = __hip_atomic_fetch_add(wg + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (int(n) == nact - 1)
      atomicMax(resid, __hip_atomic_load(wg, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
  }
}

}  // namespace heat::gpu::tbdetail

namespace heat::gpu::tbp {
bool launch(const tbdetail::TbArgs& args, int depth, int lag, hipStream_t st);
int occupancy(int depth, int lag);
}
namespace heat::gpu::tbs {
bool launch(const tbdetail::TbArgs& args, int depth, int lag, hipStream_t st);
int occupancy(int depth, int lag);
}
namespace heat::gpu::tbx {  // level-split two-wave pipelines (tb_split.hip)
bool launch_split(const tbdetail::TbArgs& args, int depth, hipStream_t st);
int occupancy_split(int depth);
// Depth-12 launches with the residual at inner level rl (tb_split_rl{a,b,c}.hip:
// levels 1-4, 5-8, 9-11); false if rl is not in the unit's range.
bool launch_split_rl_a(const tbdetail::TbArgs& args, int depth, int rl, hipStream_t st);
bool launch_split_rl_b(const tbdetail::TbArgs& args, int depth, int rl, hipStream_t st);
bool launch_split_rl_c(const tbdetail::TbArgs& args, int depth, int rl, hipStream_t st);
}
namespace heat::gpu::tbc {  // chained level-split passes (tb_chain.hip)
int occupancy_chain(int depth);
bool launch_chain(const tbdetail::TbArgs& args, int depth, int passes, unsigned* flags, unsigned* done,
                  unsigned* err, hipStream_t st);
}
namespace heat::gpu::tbxn {  // level-split pipelines, non-temporal rows (tb_split_nt.hip)
bool launch_split(const tbdetail::TbArgs& args, int depth, hipStream_t st);
}
namespace heat::gpu::tbxm {  // level-split pipelines, mixed DPP / ds_bpermute shifts (tb_split_mixed.hip)
bool launch_split(const tbdetail::TbArgs& args, int depth, hipStream_t st);
int occupancy_split(int depth);
}
namespace heat::gpu::tbn {  // float2 lanes (tb_narrow.hip)
bool launch(const tbdetail::TbArgs& args, int depth, int lag, hipStream_t st);
int occupancy(int depth, int lag);
}
