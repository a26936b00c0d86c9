// Device kernel launchers (gfx950).  Implementations: csrc/kernels/*.hip.
//
// Reference kernels these replace:
//   heat(old,new)              cuda/cuda_heat.cu:140-163  -> naive_step / tb_step
//   heat<threads>(old,new,f)   cuda/cuda_heat.cu:42-138   -> the same kernels with the
//                                                           fused max|delta| residual
//   semi_reduce(f)             cuda/cuda_heat.cu:32-40    -> removed: the residual is a
//                                                           single device word (atomic max)
//   MPI col_type datatype      mpi/...c:82-84             -> pack_box / unpack_box
//   host inidat + H2D copies   cuda/cuda_heat.cu:194-198  -> init_field (device side)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "heat/topology.hpp"

namespace heat::gpu {

// Geometry shared by all stencil kernels.  `src`/`dst` point at local owned
// cell (0,0) of a field allocated with some Layout; (gx0, gy0) are the
// global coordinates of that cell.  Only cells with 1 <= gx <= nx-2 and
// 1 <= gy <= ny-2 are updated (fixed Dirichlet ring); every other
// cell keeps its value.
struct StencilGeom {
  int64_t pitch = 0;
  int64_t gx0 = 0, gy0 = 0;
  int64_t nx = 0, ny = 0;
  float cx = 0.1f, cy = 0.1f;
  int numerics = 0;  // heat::Numerics (naive kernel only; TB is always Fp32)
  // Convergence gate (device word, null = none): a launch whose gate reads
  // non-zero writes nothing (see judge_check).
  const unsigned* gate = nullptr;
};

// Variant flags of the temporally blocked kernel (tb_step's `variant`; the
// same names in parallel_heat_amd.ops.TbVariant).  Bits 0-1 choose the
// register pipeline, the rest the build and the launch layout.
namespace tbv {
enum : int {
  kRing3 = 0,           // 3-row rings, skew 1 (LAG 1)
  kRing4 = 1,           // 4-row rings, skew 2 (LAG 2)
  kRing2 = 2,           // 2-row rings + copy (LAG 0)
  kRamp = 3,            // 3-row rings + compile-time ramp skip (LAG 3)
  kPipeMask = 3,
  kScalar = 4,          // scalar row update build (tbs; depth 12 lives here)
  kPrefetch6 = 8,       // with kRamp: 6-row prefetch (retired, LAG 4)
  kXcdGroups = 16,      // contiguous wave ranges per XCD
  kAltDirection = 32,   // odd chunks stream bottom-up
  kFloat2 = 64,         // float2 lanes, 128-column strips (tbn)
  kForceAgePairs = 256, // age groups even at equal weights (tests)
  kDiagNoStore = 1024,  // diagnostics: no output stores (wrong results)
  kSplit = 2048,        // two-wave level-split pipelines (tbx; depths 8, 12)
  kDiagCachedRows = 4096,  // diagnostics: cache-resident input rows (wrong results)
  kNoAgePairs = 16384,  // never age-group (A/B of the weights)
  kLinear = 32768,      // force the balanced linear plan (equal strip-rows per unit)
  kNoLinear = 65536,    // never switch to it (by default it replaces a classic
                        // plan that fills < 90 % of the launch's units)
  kTile = 131072,       // workgroup tiles: 8 waves x R rows of a strip in VGPRs,
                        // neighbour rows through LDS each step (tbw, tb_tile.hip)
  kTileDpp = 262144,    // with kTile: DPP lane shifts instead of ds_bpermute
  kShiftMixed = 524288, // with kSplit: west shift DPP, east ds_bpermute (tbxm, tb_split_mixed.hip)
  // Defaults: depth <= 8 and small launches at 12; large launches at 12.
  kDefault = kRamp | kScalar | kXcdGroups,  // 23
  kDefaultDeep = kDefault | kSplit,         // 2071
};
}  // namespace tbv

// Depths the temporally blocked kernel is instantiated for.
constexpr int kTbMaxDepth = 8;    // 1..8: every build
// Rows of the older : younger wave of a chunk pair at two waves per SIMD
// (kTbAgePairs; HEAT_TB_AGE_RATIO sets it, <= 1 = off).  Off by default: it
// evens the two waves' finish times (busy fraction 0.77 -> 0.81) but not the
// launch span, which the SIMD's combined issue rate sets
// (profiles/tb_wave_timeline_r1.md).
constexpr double kTbAgeRatio = 1.0;
// Level-split pipelines at two per SIMD: the first-dispatched half of the
// grid takes 1.7x the rows of the second half in each pair of adjacent
// chunks: +4-7 % at 2048..8192-row blocks (profiles/tb_split_age_pairs_r2.md).
constexpr double kTbSplitAgeWeights[2] = {1.7, 1.0};
// Linear plans of split pipelines at four blocks per CU: one share per
// dispatch round (oldest first).
constexpr double kTbLinearAgeWeights[4] = {2.0, 1.95, 1.15, 1.0};
constexpr int kTbDeepDepth = 12;  // + 12: scalar ring-3+ramp build (variant bits 4|3)
bool tb_depth_supported(int k);
// Output columns per 256-column strip at depth k.
// Output columns per TB strip (64 lanes x lane_cols, minus the overlap) and
// the lane width of a variant (4: float4 lanes; variant bit 64: float2).
int tb_strip_width(int k, int lane_cols = 4);
int tb_lane_cols(int variant);

// Fill every allocated cell (owned, ghost ring and padding) of a field with
// the initial condition at its global coordinates (0 outside the plate).
void init_field(float* origin, const Layout& L, int64_t gx0, int64_t gy0, int64_t nx,
                int64_t ny, int mode, uint64_t seed, hipStream_t st);

// One Jacobi step over `box` (local coordinates), one cell per thread.
// If resid != nullptr, atomically max-reduces |new - old| (as float bits)
// over the box into *resid.
void naive_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
                unsigned* resid, hipStream_t st);

// `depth` fused Jacobi steps over up to 5 output boxes in one launch using
// the register-streaming temporally blocked kernel.  Reads rows
// [r0-depth, r1+depth) and columns [c0-round_up(depth,4), ...) of src, so the
// ghost ring must be at least that deep and valid (halo exchanged).
// Box column starts must be multiples of 4.  `waves_target` steers the row
// chunking (parallelism vs. redundant halo work): > 0 absolute wave count,
// 0 default rounds, < 0 that many whole rounds of resident waves.
// `variant`: bits 0-1 pipeline (0: 3-row rings, skew 1; 1: 4-row rings,
// skew 2; 2: 2-row rings + copy; 3: 3-row rings + ramp skip), bit 2
// scalar-update build; -1 = default
// (HEAT_TB_VARIANT or the tuned choice).
// One Jacobi step over `box` from an LDS-staged 32x256 halo tile per
// workgroup (float4 lanes, DPP east/west); honours g.numerics.
void lds_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
              unsigned* resid, hipStream_t st);

// One Jacobi step over `box` as banded matrix products on the fp32 MFMA
// units (v_mfma_f32_16x16x4_f32); rounding differs from heat::stencil.
void mfma_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
               unsigned* resid, hipStream_t st);

// res_level (with resid): the step 1..depth whose max |new - old| is taken;
// 0 = depth (the pass's last step).  Inner levels need tb_mid_residual(depth).
// chain (optional): run chain->passes passes of `depth` steps in ONE launch
// of the chained level-split kernel (tb_chain.hip) when this launch's plan
// qualifies (the streaming split build, one box, no residual, a classic
// plan of one dispatch round, at most chain->max_units units); the passes
// ping-pong between src and dst (an odd count ends in dst).  chain->chained
// reports whether it ran; if not, nothing was launched.
struct TbChain {
  int passes = 1;
  unsigned* flags = nullptr;  // >= max_units words, zero (the launch re-zeroes them)
  unsigned* done = nullptr;   // zero (re-zeroed by the launch)
  unsigned* err = nullptr;    // set non-zero if a unit's poll gave up
  int max_units = 0;
  bool chained = false;
};
void tb_step(const float* src, float* dst, const StencilGeom& g, const Box* boxes, int nbox,
             int depth, unsigned* resid, hipStream_t st, int waves_target = 0, int variant = -1,
             int res_level = 0, TbChain* chain = nullptr);
// Resident workgroup tiles (tb_resident.hip): `passes` passes of `depth`
// steps over ONE box in a single launch whose tiles stay in VGPRs, trading
// only their K-deep ghost rings between passes through two exchange fields
// (same layout as the field) and per-tile flags.  The tiles of the box must
// all be co-resident (tb_resident_fits).  src is read by the first pass only;
// dst receives the last pass's box.  checks: convergence checks inside the
// launch (increasing passes, at most one per pass, each at an even level
// 2 <= checks[c].step <= depth): check c writes the max |delta| of that
// step over the owned block [0, own_rows) x [0, own_cols) into
// resids[slot * kTbResidentMaxChecks + c] (atomic max per wave, 64 slots;
// words zeroed by the caller, kTbResidentSlots * kTbResidentMaxChecks of
// them: judge_check(resids, ..., n, kTbResidentSlots, kTbResidentMaxChecks)).
struct TbResidentBuffers {
  float* base[2] = {nullptr, nullptr};  // exchange field allocations
  int64_t origin = 0;                   // owned cell (0, 0) in floats from base
  int64_t bytes = 0;                    // allocation size
  unsigned* flags = nullptr;            // >= max_tiles words, 16-byte aligned, zeroed once
  int max_tiles = 0;
  unsigned* done = nullptr;             // completion counter, zeroed once
  unsigned* err = nullptr;              // set non-zero if a neighbour wait gave up
};
struct TbResidentCheck {
  int pass = 0, step = 0;
};
constexpr int kTbResidentMaxChecks = 64;  // a 1024-step gated segment checking every 20 steps: 51
bool tb_resident_fits(const Box& box, int depth, int variant = -1);
void tb_resident_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
                      int depth, int passes, const TbResidentBuffers& xb, hipStream_t st,
                      int variant = -1, const TbResidentCheck* checks = nullptr,
                      int nchecks = 0, unsigned* resids = nullptr, int64_t own_rows = 0,
                      int64_t own_cols = 0);

// The automatic variant choice at this depth takes a residual at any inner
// level (depth 12: level-split pipelines or workgroup tiles), so a
// convergence check can ride inside a full-depth pass instead of cutting it.
bool tb_mid_residual(int depth);
// Variant a launch of `depth` uses by default (HEAT_TB_VARIANT overrides).
int tb_default_variant(int depth);
// Variant tb_step picks for a launch of `depth` with this much work
// (strip-rows of 232/256-column float4 strips per SIMD).
int tb_auto_variant(int depth, int64_t strip_rows_per_simd);
// Diagnostics: while set, every tb_step launch writes 4 u64 per wave into buf
// ({start, end} s_memrealtime ticks (100 MHz), block, strip<<32 | chunk);
// waves = buffer capacity in waves.  nullptr switches it off.
void tb_set_stamps(unsigned long long* buf, int64_t waves);
int tb_variant_lag(int variant);
// The variant's build has the kTbDeepDepth instantiation (scalar ring-3+ramp).
bool tb_variant_deep(int variant);
// Bit 2048: each (strip, chunk) runs on a two-wave level-split pipeline
// (depths 8 and 12; scalar ring-3+ramp variants only).
bool tb_variant_split(int variant);
// Launch-planner knobs of the TB kernel.  Defaults are the tuned values;
// each HEAT_TB_* environment variable overrides its field when the process
// first plans a launch (diagnostics and A/B sweeps), and tb_set_tuning()
// replaces the whole set at run time (tests, tools).
struct TbTuning {
  int variant = -1;        // HEAT_TB_VARIANT: force a variant (-1: per launch)
  int rounds = 0;          // HEAT_TB_ROUNDS: whole resident rounds per launch (0: from the work)
  int min_len = 0;         // HEAT_TB_MINLEN: minimum chunk rows (0: max(depth, 8))
  int waves = 0;           // HEAT_TB_WAVES: waves per launch of the solver (0: planner)
  double edge_frac = 1.0;  // HEAT_TB_EDGE_FRAC: top/bottom edge chunk length factor
  // HEAT_TB_AGE_WEIGHTS "w0,w1,.." (or HEAT_TB_AGE_RATIO r = {r, 1}): row
  // shares of the age groups; empty = the built-in weights.
  std::vector<double> age_weights;
  int tile_rows = 0;       // HEAT_TB_TILE_ROWS: rows per wave of kTile launches (0: planner)
  int tile_waves = 0;      // HEAT_TB_TILE_WAVES: waves per kTile workgroup, 8 or 16 (0: planner)
  int tile_xl = -1;        // HEAT_TB_TILE_XL: kTile lane shifts, 0 DPP, 1 ds_bpermute,
                           // 2 mixed (-1: mixed unless the variant has kTileDpp)
  int tile_max_srps = 64;  // HEAT_TB_TILE_MAX: workgroup tiles below this many strip-rows
                           // per SIMD (the automatic variant and Solver::tile_sized)
  int nt = -1;             // HEAT_TB_NT: level-split rows non-temporal (1) or plain (0);
                           // -1: non-temporal when a pass sweeps > kTbStreamBytes
  int res_diag = 0;        // HEAT_TB_RES_DIAG: resident-tile timing diagnostics (bits 0-2
                           // give WRONG results): bit 0 no neighbour wait, 1 no ghost reload,
                           // 2 no publish; bit 3 every tile on the masked (edge) path
};
TbTuning tb_tuning();  // a copy of the current set
void tb_set_tuning(const TbTuning& t);
// Whole rounds of resident waves per launch (TbTuning::rounds; 0 = unset: the
// planner picks waves per SIMD from the work, tb_auto_waves_per_simd).
int tb_default_rounds();
// Resident waves of the TB kernel instantiation on the current device.
int tb_resident_waves(int depth, int variant);
// SIMDs of the current device (CUs x 4).
int tb_simd_count();
// Waves per SIMD the planner uses for a launch with this much work per SIMD
// (strip-rows / SIMDs), at most max_per_simd.
int tb_auto_waves_per_simd(int depth, int64_t strip_rows_per_simd, int max_per_simd);

// Copy a box of a strided field to/from a contiguous buffer (E/W halos).
void pack_box(const float* origin, int64_t pitch, const Box& box, float* buf, hipStream_t st);
// Up to kMaxBoxCopies boxes <-> their contiguous buffers (row-major
// rows x cols) in ONE launch: the packing / unpacking of a whole halo
// exchange (E/W columns and ghost corners).
constexpr int kMaxBoxCopies = 8;
struct BoxCopy {
  Box box;
  float* buf = nullptr;
};
void copy_boxes(float* origin, int64_t pitch, const BoxCopy* copies, int n, bool to_buf,
                hipStream_t st);
void unpack_box(const float* buf, float* origin, int64_t pitch, const Box& box, hipStream_t st);

// Order-independent checksum of the owned block, accumulated on the device
// into out (zeroed by the caller): hash (u64, wrapping sum of
// mix64(global index, bits)), sum (f64), min/max (order-preserving int keys).
struct DeviceChecksum {
  unsigned long long hash;
  double sum;
  int min_key, max_key;
  unsigned long long count;
};
void checksum_block(const float* origin, int64_t pitch, int64_t lx, int64_t ly, int64_t ox,
                    int64_t oy, int64_t ny, DeviceChecksum* out, hipStream_t st);
float checksum_key_to_float(int key);

// Device-side convergence decision (one per check, stream-ordered after the
// residual of the check's pass and its all-reduce): the host never waits on a
// check.  Unless the gate is already closed, judge_check compares the
// residual with eps (compat mpi: double(r) <= eps, mpi/...c:245; otherwise
// r < float(eps), cuda/cuda_heat.cu:67), closes the gate on convergence or on
// a non-finite residual, and zeroes the residual word for the next check.
// Every stencil launch given the gate (StencilGeom::gate = &stop) returns at
// once after that, so passes queued behind the converging check write
// nothing.  The host reads the record after the run.
struct DeviceGate {
  unsigned stop;        // gate word: non-zero once closed
  unsigned reason;      // 1 converged, 2 non-finite residual
  unsigned stop_check;  // ordinal (0-based, since the last reset) of the closing check
  unsigned checks;      // checks judged while open
  unsigned last_bits;   // residual (float bits) of the last judged check
  unsigned pad[3];
};
// n > 1: n consecutive checks judged in order in one launch (the checks of a
// resident span); check i's residual is the max of resid[s * stride + i]
// over s < slots (the span's tiles spread their atomics over `slots` cache
// lines: 500 workgroups on one word serialised ~3.5 us per check).
void judge_check(unsigned* resid, DeviceGate* gate, double eps, bool mpi_compat, hipStream_t st,
                 int n = 1, int slots = 1, int stride = 0);
// The resident span's residual block: kTbResidentSlots lines of
// kTbResidentMaxChecks words (TbResidentBuffers / tb_resident_step resids);
// wave w of tile t adds to slot (t * waves + w) % kTbResidentSlots.
constexpr int kTbResidentSlots = 64;

// Max |a-b| over a box (standalone residual), atomically into *resid.
void residual_box(const float* a, const float* b, int64_t pitch, const Box& box, unsigned* resid,
                  hipStream_t st);

}  // namespace heat::gpu
