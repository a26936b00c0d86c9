// gfx950 (CDNA4) stencil kernels: device init, naive oracle step, the
// register-streaming temporally blocked step (the hot kernel), residual and
// halo pack/unpack.
//
// Design notes (MI355X-first):
//  * Layout is row-major with y contiguous, so a wave64 covers 64 consecutive
//    float4 = 256 columns of one row: every global access is a fully
//    coalesced 1 KiB dwordx4 wave-instruction (the reference maps threadIdx.x
//    to the strided x index, cuda/cuda_heat.cu:46-59, and is uncoalesced).
//  * The hot kernel (tb_kernel) streams a wave down a 256-column strip and
//    keeps K time levels of a 3-row sliding window in VGPRs.  Each input row
//    is loaded from HBM once and leaves after K fused updates, so HBM traffic
//    per cell-update is 8/K bytes instead of 8.  East/west neighbours cross
//    lanes with DPP wave_shr:1 / wave_shl:1 (fused into v_add_f32_dpp): no
//    LDS, no barriers, waves are fully independent.  Strips overlap by
//    2*round_up(K,4) columns and row chunks by 2K rows (redundant halo
//    compute, the trapezoid of classic temporal blocking).
//  * All variants evaluate the identical FMA expression (heat::stencil), so
//    results are bitwise equal across kernels, depths and decompositions.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <iterator>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "heat/common.hpp"
#include "heat/init_fn.hpp"
#include "heat/kernels.hpp"
#include "tb_common.hpp"
#include "tb_exp.hpp"
#include "tb_tile.hpp"

namespace heat::gpu {
namespace {

using tbdetail::in_interior;
using tbdetail::TbArgs;
using tbdetail::TbBox;
using tbdetail::wave_max_atomic;

// --------------------------------------------------------------------------
// init
// --------------------------------------------------------------------------
__global__ void init_kernel(float* base, int64_t pitch, int64_t rows, int64_t hx, int64_t hy,
                            int64_t gx0, int64_t gy0, int64_t nx, int64_t ny, int mode,
                            uint64_t seed) {
  const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= pitch) return;
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    const int64_t gx = gx0 + r - hx, gy = gy0 + c - hy;
    base[r * pitch + c] = init_value(mode, gx, gy, nx, ny, seed);
  }
}

// --------------------------------------------------------------------------
// naive: one cell per thread (independent oracle for the TB kernel)
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void naive_kernel(const float* __restrict__ src,
                                                    float* __restrict__ dst, StencilGeom g,
                                                    Box box, unsigned* resid) {
  const int64_t c = box.c0 + int64_t(blockIdx.x) * 64 + threadIdx.x;
  const int64_t r = box.r0 + int64_t(blockIdx.y) * 4 + threadIdx.y;
  if (tbdetail::gated(g.gate)) return;
  unsigned m = 0;
  if (r < box.r1 && c < box.c1) {
    const int64_t i = r * g.pitch + c;
    const float v = src[i];
    float out = v;
    if (in_interior(g.gx0 + r, g.nx) && in_interior(g.gy0 + c, g.ny))
      out = g.numerics == 1
                ? stencil_mpi(v, src[i - g.pitch], src[i + g.pitch], src[i - 1], src[i + 1], g.cx, g.cy)
                : stencil(v, src[i - g.pitch], src[i + g.pitch], src[i - 1], src[i + 1], g.cx, g.cy);
    dst[i] = out;
    m = __float_as_uint(fabsf(out - v));
  }
  if (resid) wave_max_atomic(m, resid);
}

// --------------------------------------------------------------------------
// pack / unpack / residual
// --------------------------------------------------------------------------
__global__ void pack_kernel(const float* __restrict__ origin, int64_t pitch, Box box,
                            float* __restrict__ buf) {
  const int64_t cols = box.c1 - box.c0, n = (box.r1 - box.r0) * cols;
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n;
       k += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = k / cols, c = k % cols;
    buf[k] = origin[(box.r0 + r) * pitch + box.c0 + c];
  }
}

struct BoxCopies {
  BoxCopy c[kMaxBoxCopies];
};

// blockIdx.y selects the box; rows are grid-strided over blockIdx.x, columns
// over the threads (row segments are contiguous in both the field and the
// buffer).
__global__ __launch_bounds__(128) void box_copy_kernel(float* __restrict__ origin, int64_t pitch,
                                                       BoxCopies a, int to_buf) {
  const BoxCopy& c = a.c[blockIdx.y];
  const int64_t rows = c.box.r1 - c.box.r0, cols = c.box.c1 - c.box.c0;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    float* f = origin + (c.box.r0 + r) * pitch + c.box.c0;
    float* b = c.buf + r * cols;
    for (int64_t j = threadIdx.x; j < cols; j += blockDim.x) {
      if (to_buf) b[j] = f[j];
      else f[j] = b[j];
    }
  }
}

__global__ void unpack_kernel(const float* __restrict__ buf, float* __restrict__ origin,
                              int64_t pitch, Box box) {
  const int64_t cols = box.c1 - box.c0, n = (box.r1 - box.r0) * cols;
  for (int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < n;
       k += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = k / cols, c = k % cols;
    origin[(box.r0 + r) * pitch + box.c0 + c] = buf[k];
  }
}

__global__ __launch_bounds__(256) void residual_kernel(const float* __restrict__ a,
                                                       const float* __restrict__ b,
                                                       int64_t pitch, Box box, unsigned* resid) {
  const int64_t c = box.c0 + int64_t(blockIdx.x) * 64 + threadIdx.x;
  unsigned m = 0;
  if (c < box.c1)
    for (int64_t r = box.r0 + blockIdx.y * 4 + threadIdx.y; r < box.r1; r += gridDim.y * 4)
      m = max(m, __float_as_uint(fabsf(a[r * pitch + c] - b[r * pitch + c])));
  wave_max_atomic(m, resid);
}

__global__ void judge_kernel(unsigned* resids, int n, int slots, int stride, DeviceGate* gate,
                             double eps, int mpi_compat) {
  // One wave: lane s reads (and zeroes) slot s of every check -- all loads
  // issued before the first use --, the max over the slots is a wave
  // reduction, lane 0 judges.  Checks in order: the first converging one
  // closes the gate.
  constexpr int kMax = 32;  // kTbResidentMaxChecks; longer lists loop
  const int lane = threadIdx.x;
  for (int i0 = 0; i0 < n; i0 += kMax) {
    const int m = min(n - i0, kMax);
    unsigned v[kMax];
#pragma unroll
    for (int j = 0; j < kMax; ++j) v[j] = (j < m && lane < slots) ? resids[lane * stride + i0 + j] : 0u;
#pragma unroll
    for (int j = 0; j < kMax; ++j)
      if (j < m && lane < slots) resids[lane * stride + i0 + j] = 0u;
    // The gate in registers for the whole list (a read-modify-write of the
    // gate in memory per check serialised ~0.4 us per check: 10 us for the
    // 27 checks of a resident span).
    DeviceGate gl{};
    if (lane == 0) gl = *gate;
    for (int j = 0; j < m; ++j) {
      unsigned bits = v[j];  // non-negative floats order like their bits
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) bits = max(bits, unsigned(__shfl_xor(int(bits), off)));
      if (lane == 0 && gl.stop == 0u) {
        float r;
        __builtin_memcpy(&r, &bits, 4);
        const unsigned ordinal = gl.checks;
        gl.checks = ordinal + 1u;
        gl.last_bits = bits;
        unsigned why = 0u;
        if ((bits & 0x7F800000u) == 0x7F800000u) why = 2u;  // inf or NaN
        else if (mpi_compat ? double(r) <= eps : r < float(eps)) why = 1u;
        if (why) {
          gl.reason = why;
          gl.stop_check = ordinal;
          gl.stop = 1u;
        }
      }
    }
    if (lane == 0) *gate = gl;
  }
}

__device__ __forceinline__ int float_key(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : (i ^ 0x7FFFFFFF);
}

__global__ __launch_bounds__(256) void checksum_kernel(const float* __restrict__ origin,
                                                       int64_t pitch, int64_t lx, int64_t ly,
                                                       int64_t ox, int64_t oy, int64_t ny,
                                                       DeviceChecksum* out) {
  // Grid-stride over the block; every term is order-independent (wrapping
  // u64 sums, min/max), except the fp64 sum's last bits.  One set of
  // atomics per workgroup: a per-wave atomic on five hot addresses from
  // ~10^5 waves serialised at the memory side (30 ms for 8192^2).
  unsigned long long h = 0, cnt = 0;
  double sum = 0.0;
  int mn = 0x7FFFFFFF, mx = int(0x80000000);
  for (int64_t r = blockIdx.y; r < lx; r += gridDim.y) {
    const float* row = origin + r * pitch;
    const uint64_t gbase = uint64_t(ox + r) * uint64_t(ny) + uint64_t(oy);
    for (int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; c < ly;
         c += int64_t(gridDim.x) * blockDim.x) {
      const float v = row[c];
      const uint32_t bits = __float_as_uint(v);
      h += mix64((gbase + uint64_t(c)) * 0x100000001B3ull ^ bits);
      sum += double(v);
      const int k = float_key(v);
      mn = min(mn, k);
      mx = max(mx, k);
      ++cnt;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    h += __shfl_xor(h, off);
    cnt += __shfl_xor(cnt, off);
    sum += __shfl_xor(sum, off);
    mn = min(mn, __shfl_xor(mn, off));
    mx = max(mx, __shfl_xor(mx, off));
  }
  __shared__ unsigned long long sh_h[4], sh_c[4];
  __shared__ double sh_s[4];
  __shared__ int sh_mn[4], sh_mx[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh_h[w] = h;
    sh_c[w] = cnt;
    sh_s[w] = sum;
    sh_mn[w] = mn;
    sh_mx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < int(blockDim.x >> 6); ++i) {
      h += sh_h[i];
      cnt += sh_c[i];
      sum += sh_s[i];
      mn = min(mn, sh_mn[i]);
      mx = max(mx, sh_mx[i]);
    }
    if (cnt) {
      atomicAdd(&out->hash, h);
      atomicAdd(&out->count, cnt);
      atomicAdd(&out->sum, sum);
      atomicMin(&out->min_key, mn);
      atomicMax(&out->max_key, mx);
    }
  }
}

int grid_1d(int64_t n) { return int(std::min<int64_t>(ceil_div(n, 256), 256 * 16)); }

}  // namespace

bool tb_depth_supported(int k) {
  // 1..8 in every build; 12 in the scalar ring-3+ramp build only
  // (tb_scalar.hip, HEAT_TB_DEEP).
  return (k >= 1 && k <= kTbMaxDepth) || k == kTbDeepDepth;
}

int tb_strip_width(int k, int lane_cols) {
  return 64 * lane_cols - 2 * int(round_up(k, lane_cols));
}
int tb_lane_cols(int variant) { return (variant & tbv::kFloat2) ? 2 : 4; }

int tb_variant_lag(int variant) {
  const int pipe = variant & tbv::kPipeMask;
  if (pipe == tbv::kRamp && (variant & tbv::kPrefetch6)) return 4;  // retired
  switch (pipe) {
    case tbv::kRing4: return 2;
    case tbv::kRing2: return 0;
    case tbv::kRamp: return 3;
    default: return 1;
  }
}

bool tb_variant_split(int variant) {
  // Level-split two-wave pipelines (tb_split.hip; scalar ring-3+ramp).
  return (variant & tbv::kSplit) && tb_variant_deep(variant);
}

bool tb_variant_deep(int variant) {
  return (variant & tbv::kScalar) && !(variant & tbv::kFloat2) && tb_variant_lag(variant) == 3;
}

namespace {
TbTuning tuning_from_env() {
  TbTuning t;
  auto geti = [](const char* n, int def) {
    const char* e = std::getenv(n);
    return e && *e ? std::atoi(e) : def;
  };
  t.variant = geti("HEAT_TB_VARIANT", -1);
  t.rounds = std::max(0, geti("HEAT_TB_ROUNDS", 0));
  t.min_len = std::max(0, geti("HEAT_TB_MINLEN", 0));
  t.waves = std::max(0, geti("HEAT_TB_WAVES", 0));
  t.tile_rows = std::max(0, geti("HEAT_TB_TILE_ROWS", 0));
  t.tile_waves = std::max(0, geti("HEAT_TB_TILE_WAVES", 0));
  t.tile_xl = geti("HEAT_TB_TILE_XL", -1);
  t.res_diag = geti("HEAT_TB_RES_DIAG", 0) & 31;
  t.nt = geti("HEAT_TB_NT", -1);
  t.tile_max_srps = std::max(0, geti("HEAT_TB_TILE_MAX", 64));
  if (const char* e = std::getenv("HEAT_TB_EDGE_FRAC"); e && *e) t.edge_frac = std::atof(e);
  if (const char* e = std::getenv("HEAT_TB_AGE_WEIGHTS"); e && *e) {
    for (const char* q = e; *q;) {
      char* end = nullptr;
      const double v = std::strtod(q, &end);
      if (end == q) break;
      t.age_weights.push_back(v);
      q = *end == ',' ? end + 1 : end;
    }
  } else if (const char* r = std::getenv("HEAT_TB_AGE_RATIO"); r && *r) {
    t.age_weights = {std::atof(r), 1.0};
  }
  return t;
}
std::mutex g_tuning_mu;
TbTuning& tuning_ref() {
  static TbTuning t = tuning_from_env();
  return t;
}
}  // namespace

TbTuning tb_tuning() {
  std::lock_guard<std::mutex> lk(g_tuning_mu);
  return tuning_ref();
}

void tb_set_tuning(const TbTuning& t) {
  std::lock_guard<std::mutex> lk(g_tuning_mu);
  tuning_ref() = t;
}

int tb_default_rounds() { return tb_tuning().rounds; }

namespace {
bool tb_trace_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT_TB_TRACE");
    return e && *e && *e != '0';
  }();
  return on;
}
void tb_trace_once(const char* line) {
  static std::mutex mu;
  static std::vector<std::string> seen;
  std::lock_guard<std::mutex> lk(mu);
  for (const auto& s : seen)
    if (s == line) return;
  seen.emplace_back(line);
  std::fputs(line, stderr);
}
}  // namespace

int tb_simd_count() {
  static std::map<int, int> cache;
  static std::mutex mu;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  return cache.emplace(dev, std::max(1, cus) * 4).first->second;
}

int tb_auto_waves_per_simd(int depth, int64_t strip_rows_per_simd, int max_per_simd) {
  // Fewer, longer chunks for small problems: each chunk pays a ~2K-row
  // pipeline ramp, and more waves per SIMD only buy latency hiding.  The
  // thresholds come from the waves sweep over slab heights 512..8192
  // (tools/sweep_waves.sh, profiles/tb_waves_per_simd_r1.md): at K=8 one
  // wave per SIMD wins below ~48 strip-rows per SIMD, two below ~100.
  int w = max_per_simd;
  if (strip_rows_per_simd < 6 * int64_t(depth)) w = 1;
  else if (strip_rows_per_simd * 2 < 25 * int64_t(depth)) w = 2;
  return std::max(1, std::min(w, max_per_simd));
}

int tb_resident_waves(int depth, int variant) {
  // Cached per (device, depth, variant): CUs x resident blocks per CU x 4 waves.
  static std::map<std::tuple<int, int, int>, int> cache;
  static std::mutex mu;
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto key = std::make_tuple(dev, depth, variant);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int cus = 0;
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int lag = tb_variant_lag(variant);
  if (tb_variant_split(variant)) {
    // Work units are two-wave pipelines, two per block.
    const int occ = (variant & tbv::kShiftMixed)
                        ? tb_exp("the mixed-shift split build (kShiftMixed)").tbxm_occupancy_split(depth)
                        : tbx::occupancy_split(depth);
    const int w = std::max(1, cus * std::max(1, occ) * 2);
    cache.emplace(key, w);
    return w;
  }
  const int per_cu = (variant & tbv::kFloat2)  ? tb_exp("the float2-lane build (kFloat2)").tbn_occupancy(depth, lag)
                     : (variant & tbv::kScalar) ? tbs::occupancy(depth, lag)
                                                : tb_exp("the packed build (no kScalar)").tbp_occupancy(depth, lag);
  const int w = std::max(1, cus * std::max(1, per_cu) * 4);
  cache.emplace(key, w);
  return w;
}

int tb_default_variant(int depth) {
  if (const int v = tb_tuning().variant; v >= 0) return v;
  // Ring-3 + ramp skip, scalar build, XCD-grouped blocks (23); at depth 12
  // on large launches as two-wave level-split pipelines with ds_bpermute
  // lane shifts (2071): +5 % in bench.py, +9-10 % in the interleaved kernel
  // A/B (profiles/tb_wave_timeline_r1.md).  tb_step picks per launch from
  // the work size (tb_auto_variant).
  return depth == kTbDeepDepth ? tbv::kDefaultDeep : tbv::kDefault;
}

int tb_auto_variant(int depth, int64_t strip_rows_per_simd) {
  if (const int v = tb_tuning().variant; v >= 0) return v;
  // The split pipelines need about 64 strip-rows per SIMD to pay for their
  // second wave: below that (the per-rank blocks of 4-8 GPU runs: 1024 x
  // 8192, 2048 x 4096, 1536 x 8192, ...) one wave per (strip, chunk) at
  // depth 12 is 8-12 % faster, above it the split is 2-4 % faster
  // (profiles/tb_block_shapes_r2.md).
  // Below 64 (the 8-GPU blocks 1024 x 8192 and 2048 x 4096 and their
  // deep-halo passes, 1536-row blocks) the workgroup tiles win: +6-10 % over
  // one wave per chunk inside the plate at 36, and +36-38 % on blocks with a
  // plate edge (the first and last rank, whose time the max over ranks
  // reports) at 36 and 54, where one wave per chunk loses 8 % inside the
  // plate (profiles/r3_tile.md).  Even depths only (the tile runs steps in
  // pairs).  From 64 the split pipelines keep the edge ranks within 2 %.
  if (depth >= 4 && depth % 2 == 0 && strip_rows_per_simd < tb_tuning().tile_max_srps)
    return tbv::kTile | tbv::kXcdGroups;
  if (depth == kTbDeepDepth && strip_rows_per_simd < 64) return tbv::kDefault;
  // Depth 8 on whole-GPU plates (the remainder passes of 1000 = 82 x 12 +
  // 8 + 8 at 8192^2: 288 strip-rows per SIMD) as split pipelines too:
  // bench 5.21-5.22 vs 5.19-5.21 interleaved (profiles/r5_stores.md).
  if (depth == 8 && strip_rows_per_simd >= 256) return tbv::kDefaultDeep;
  return tb_default_variant(depth);
}

void init_field(float* origin, const Layout& L, int64_t gx0, int64_t gy0, int64_t nx, int64_t ny,
                int mode, uint64_t seed, hipStream_t st) {
  float* base = origin - L.origin();
  dim3 grid(unsigned(ceil_div(L.pitch, 256)), unsigned(std::min<int64_t>(L.rows, 1024)));
  hipLaunchKernelGGL(init_kernel, grid, dim3(256), 0, st, base, L.pitch, L.rows, int64_t(L.hx),
                     int64_t(L.hy), gx0, gy0, nx, ny, mode, seed);
  HIP_CHECK(hipGetLastError());
}

void naive_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
                unsigned* resid, hipStream_t st) {
  if (box.empty()) return;
  dim3 grid(unsigned(ceil_div(box.cols(), 64)), unsigned(ceil_div(box.rows(), 4)));
  hipLaunchKernelGGL(naive_kernel, grid, dim3(64, 4), 0, st, src, dst, g, box, resid);
  HIP_CHECK(hipGetLastError());
}

namespace {
// Stamp buffers per device: with one host thread per GPU (`heat --gpus N`)
// each rank's launches stamp into its own device's buffer only.
struct Stamps {
  unsigned long long* buf = nullptr;
  int64_t waves = 0;
};
std::mutex g_stamps_mu;
std::map<int, Stamps> g_stamps;

Stamps stamps_of_current_device() {
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_stamps_mu);
  auto it = g_stamps.find(dev);
  return it == g_stamps.end() ? Stamps{} : it->second;
}
}  // namespace

void tb_set_stamps(unsigned long long* buf, int64_t waves) {
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_stamps_mu);
  if (buf) g_stamps[dev] = Stamps{buf, waves};
  else g_stamps.erase(dev);
}

bool tb_mid_residual(int depth) {
  // Depth 12 under the automatic variant choice is always the level-split
  // pipelines (tb_split_rl*.hip) or the workgroup tiles (tb_tile.hip), which
  // take a residual at any inner step; forced variants keep the last step.
  return depth == kTbDeepDepth && tb_tuning().variant < 0;
}

namespace {
std::mutex g_exp_mu;
const TbExpKernels* g_exp = nullptr;
}  // namespace

bool tb_exp_loaded() {
  std::lock_guard<std::mutex> lk(g_exp_mu);
  return g_exp != nullptr;
}

const TbExpKernels& tb_exp(const char* what) {
  std::lock_guard<std::mutex> lk(g_exp_mu);
  HEAT_CHECK(g_exp != nullptr,
             "%s is an experiment kernel build: `make exp`, then load "
             "parallel_heat_amd/_lib/libheat_exp.so (HEAT_EXP=1)", what);
  return *g_exp;
}

// HEAT_TB_SPLIT_PK=1: the streaming level-split launches take the packed-f32
// build (round-6 A/B, an experiment build).
bool split_pk_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT_TB_SPLIT_PK");
    return e && *e && *e != '0';
  }();
  return on;
}

// Field bytes one pass must sweep before the level-split launches stream
// their rows (kTbStreamRows): 3/4 of the 256 MB MALL (4096 x 8192 = 134 MB
// measured faster plain, 8192^2 = 268 MB non-temporal).
constexpr int64_t kTbStreamBytes = int64_t(192) << 20;

void tb_step(const float* src, float* dst, const StencilGeom& g, const Box* boxes, int nbox,
             int depth, unsigned* resid, hipStream_t st, int waves_target, int variant,
             int res_level, TbChain* chain) {
  if (chain) chain->chained = false;
  HEAT_CHECK(nbox >= 0 && nbox <= 5, "nbox=%d", nbox);  // API limit (5 boxes)
  HEAT_CHECK(res_level >= 0 && res_level <= depth, "residual level %d of a depth-%d pass",
             res_level, depth);
  if (res_level == depth || resid == nullptr) res_level = 0;  // 0: the last step
  const bool forced = variant >= 0 || tb_tuning().variant >= 0;
  const TbTuning tune = tb_tuning();
  if (variant < 0) {
    // Both defaults use float4 lanes (same strip width).
    const int W4 = tb_strip_width(depth, 4);
    int64_t rows4 = 0;
    for (int b = 0; b < nbox; ++b)
      if (!boxes[b].empty()) rows4 += ceil_div(boxes[b].cols(), W4) * boxes[b].rows();
    variant = tb_auto_variant(depth, rows4 / tb_simd_count());
    // Even depths only the tile kernel builds (10, 14, 16: checks every 10k
    // steps on tile-sized blocks) stay on it whatever the launch size: a
    // deep-halo box grown past the tile threshold (Solver::tile_sized_at
    // judges the owned block) is still a valid tile launch, only slower.
    if (!tb_depth_supported(depth) && depth % 2 == 0 && depth <= 16)
      variant = tbv::kTile | tbv::kXcdGroups;
  }
  // The tile kernel takes any even depth up to 16 (Solver picks 10 for
  // checks every 10k steps on tile-sized blocks); the streaming kernels the
  // built ones.
  const bool tile_depth = (variant & tbv::kTile) && depth % 2 == 0 && depth <= 16;
  HEAT_CHECK(tb_depth_supported(depth) || tile_depth, "unsupported TB depth %d (variant %d)", depth,
             variant);
  if (variant & tbv::kTile) {
    // The tile kernel runs steps in (down, up) pairs: even depths only; an
    // odd pass (a remainder or a check-cut pass) streams, with the default
    // single-wave build (scalar update + ramp; dropping only the tile bits
    // left the packed build, an experiment kernel since round 6).
    if (depth % 2 == 0) {
      tbw::step(src, dst, g, boxes, nbox, depth, resid, res_level, st, variant, tune);
      return;
    }
    variant = (variant & ~(tbv::kTile | tbv::kTileDpp | 3)) | tbv::kDefault;
  }
  // Inner-level residuals: the level-split build at depth 12 (and the tiles).
  HEAT_CHECK(res_level == 0 || (tb_variant_split(variant) && depth == kTbDeepDepth),
             "a residual at step %d of a depth-%d pass needs the depth-12 level-split or tile "
             "kernel (variant %d%s)", res_level, depth, variant, forced ? ", forced" : "");
  const int lag = tb_variant_lag(variant);
  const int W = tb_strip_width(depth, tb_lane_cols(variant));
  int64_t total_strip_rows = 0;
  for (int b = 0; b < nbox; ++b)
    if (!boxes[b].empty()) total_strip_rows += ceil_div(boxes[b].cols(), W) * boxes[b].rows();
  // Age groups (kTbAgePairs) for launches of whole resident rounds: blocks
  // dispatched earlier issue faster (the SIMD's arbitration favours older
  // waves), so the grid is split into G parts (part a = the a-th share of
  // the dispatch rounds) and older parts get more rows.  Default: two parts
  // at kTbSplitAgeWeights for the level-split pipelines; none (kTbAgeRatio
  // = 1) for single-wave pipelines.  HEAT_TB_AGE_WEIGHTS="w0,w1,..." (2-4
  // parts) or HEAT_TB_AGE_RATIO=r (two parts r : 1) override; "1" = off.
  // Four parts (one per round at 4 blocks per CU) measured slower than two
  // whatever the weights (profiles/tb_split_age_pairs_r2.md).
  const std::vector<double>& env_weights = tune.age_weights;
  const bool split_v = tb_variant_split(variant);
  int G = 0;  // age groups of this launch (0: none)
  std::vector<double> weights;
  auto set_weights = [&](int max_groups) {
    if (!env_weights.empty())
      weights = env_weights;
    else if (split_v)
      weights.assign(std::begin(kTbSplitAgeWeights), std::end(kTbSplitAgeWeights));
    else
      weights = {kTbAgeRatio, 1.0};
    bool uneven = false;
    for (double w : weights) uneven = uneven || w != weights[0] || w <= 0.0;
    G = uneven && int(weights.size()) >= 2 && int(weights.size()) <= max_groups ? int(weights.size()) : 0;
  };
  if (variant & tbv::kForceAgePairs) {  // tests: even weights still group
    set_weights(4);
    if (G == 0) {
      G = 2;
      weights.assign(2, 1.0);
    }
  }
  int bpc = 0;  // blocks per CU of the planned launch (0: set by the caller's waves_target)
  if (waves_target <= 0) {
    // Whole rounds of the resident wave capacity (a partial last round leaves
    // SIMDs idle for the tail of the launch); by default with the number of
    // waves per SIMD chosen from the work per SIMD.
    const int resident = tb_resident_waves(depth, variant);
    const int rounds = waves_target < 0 ? -waves_target : tune.rounds;
    if (rounds > 0) {
      waves_target = rounds * resident;
    } else {
      const int simds = tb_simd_count();
      const int per_simd = tb_auto_waves_per_simd(depth, total_strip_rows / simds,
                                                  std::max(1, resident / simds));
      waves_target = simds * per_simd;
      // Blocks per CU = dispatch rounds: single-wave pipelines put one wave
      // per SIMD in a block, level-split blocks hold two pipelines (4 waves).
      const int blocks_per_cu = split_v ? 2 * per_simd : per_simd;
      bpc = blocks_per_cu;
      if (G == 0 && blocks_per_cu >= 2 && !(variant & tbv::kFloat2) &&
          !(variant & tbv::kNoAgePairs))
        set_weights(blocks_per_cu);
    }
  }
  const bool pairs = G > 0;
  TbArgs args{};
  args.src = src;
  args.dst = dst;
  args.resid = resid;
  args.res_level = res_level > 0 ? res_level : depth;
  args.g = g;
  args.flags = ((variant & tbv::kXcdGroups) ? tbdetail::kTbXcdGroups : 0) |
               ((variant & tbv::kAltDirection) ? tbdetail::kTbAltDirection : 0) |
               ((variant & tbv::kDiagNoStore) ? tbdetail::kTbDiagNoStore : 0) |
               ((variant & tbv::kDiagCachedRows) ? tbdetail::kTbDiagCachedRows : 0);
  // Split rows into chunks so the whole launch has about waves_target waves,
  // but never shorter than 4*depth rows (keeps the redundant 2*depth-row
  // halo reads below ~50 %).
  // Minimum chunk length in rows (multiples of depth; HEAT_TB_MINLEN overrides).
  const int64_t min_len = tune.min_len > 0 ? tune.min_len : std::max<int64_t>(depth, 8);
  int64_t len = std::max<int64_t>(min_len, ceil_div(total_strip_rows, waves_target));
  // Rows whose chunk window reaches the global top/bottom row run the
  // generic (masked) path: HEAT_TB_EDGE_FRAC < 1 gives them shorter chunks,
  // as separate sub-boxes.  Default 1 (no edge sub-boxes) since the round-2
  // main loop: the edge chunks at 0.75 finished ~30 us before the rest of an
  // 8192^2 launch; bench.py 1.0 vs 0.95 / 0.9 / 0.75: +0.4 / +1.2 / +1.2 %
  // (profiles/tb_edge_frac_r2.md).
  const double edge_frac = tune.edge_frac;
  int n = 0, waves = 0;
  auto plan = [&](int64_t L) {
    const int64_t edge_len = std::max<int64_t>(std::min<int64_t>(min_len, L),
                                               int64_t(double(L) * edge_frac));
    n = 0;
    waves = 0;
    auto add = [&](const Box& B, int64_t clen) {
      if (B.empty()) return;
      HEAT_CHECK(n < tbdetail::kMaxBoxes, "too many TB sub-boxes");
      TbBox& t = args.box[n++];
      t.r0 = B.r0;
      t.r1 = B.r1;
      t.c0 = B.c0;
      t.c1 = B.c1;
      t.nstrips = int(ceil_div(B.cols(), W));
      t.chunk_len = int(std::min<int64_t>(clen, B.rows()));
      t.nchunks = int(ceil_div(B.rows(), t.chunk_len));
      if (pairs) {
        // Units are groups of G chunks (G * chunk_len rows), one wave (or
        // pipeline) of each age.
        t.chunk_len = int(std::max<int64_t>(1, ceil_div(std::min<int64_t>(G * clen, B.rows()), G)));
        t.nchunks = int(ceil_div(B.rows(), G * int64_t(t.chunk_len)));
      }
      t.wave_begin = waves;
      waves += t.nstrips * t.nchunks * (pairs ? G : 1);
    };
    for (int b = 0; b < nbox; ++b) {
      const Box& B = boxes[b];
      if (B.empty()) continue;
      HEAT_CHECK(B.c0 % 4 == 0, "TB box column start %lld not a multiple of 4", (long long)B.c0);
      Box mid = B, top{}, bot{};
      if (edge_len < L && B.rows() > 2 * L) {
        // Local rows whose window [r - depth, r + depth] touches global row 0 / nx-1.
        const int64_t top_end = 1 - g.gx0 + depth;          // first row clear of the top
        const int64_t bot_begin = g.nx - 2 - g.gx0 - depth;  // last row clear of the bottom
        if (B.r0 < top_end) {
          const int64_t e = std::min(B.r1, std::max(top_end, B.r0 + edge_len));
          top = Box{B.r0, e, B.c0, B.c1};
          mid.r0 = e;
        }
        if (B.r1 - 1 > bot_begin && mid.r1 > mid.r0) {
          const int64_t s0 = std::max(mid.r0, std::min(bot_begin + 1, B.r1 - edge_len));
          bot = Box{s0, B.r1, B.c0, B.c1};
          mid.r1 = s0;
        }
      }
      // Units in plate order (top edge, middle, bottom edge): XCD groups
      // take contiguous unit ranges, so the short edge units land on the
      // first and the last XCD instead of all on the first (which then
      // idled for the last ~15 % of the launch, tools/wave_timeline.py
      // xcd_last_end_us).
      add(top, edge_len);
      add(mid, L);
      add(bot, edge_len);
    }
  };
  bool linear = variant & tbv::kLinear;
  if (!linear) {
    // Keep the total within waves_target (whole resident rounds): a few extra
    // waves would form a nearly empty extra round.
    plan(len);
    for (int it = 0; it < 8 && waves > waves_target; ++it) {
      len = std::max(len + 1, ceil_div(len * int64_t(waves), int64_t(waves_target)));
      plan(len);
    }
    // Few long chunks per strip quantise badly: 565 strips x 131072 rows
    // (131072^2 on one GPU, or a 16384-row slab of it) became 1130 two-wave
    // pipelines for 2048 slots, 2.25 blocks per CU, every chunk touching the
    // plate's top or bottom row (masked path).  Balanced linear plans ran
    // those at 5.16 / 4.65 Tcells/s instead of 3.50 / 4.33; at 8192^2 (the
    // classic plan fills 98 %) they lose 24 %: units that cross a strip end
    // or split off the masked edge rows pay a second pipeline ramp, and in a
    // one-round launch the slowest unit sets the time
    // (profiles/r3_linear_plans.md).
    linear = !(variant & tbv::kNoLinear) && waves < (9 * int64_t(waves_target)) / 10 &&
             total_strip_rows >= 32 * int64_t(depth) * waves_target;
  }
  if (linear) {
    // Balanced plan: the boxes as one strip-row sequence cut into equal
    // ranges, one per unit (per group of G units with age pairs), so every
    // unit -- and every SIMD -- gets the same rows whatever the shape.
    n = 0;
    int64_t total = 0;
    for (int b = 0; b < nbox; ++b) {
      const Box& B = boxes[b];
      if (B.empty()) continue;
      HEAT_CHECK(B.c0 % 4 == 0, "TB box column start %lld not a multiple of 4", (long long)B.c0);
      TbBox& t = args.box[n++];
      t.r0 = B.r0;
      t.r1 = B.r1;
      t.c0 = B.c0;
      t.c1 = B.c1;
      t.nstrips = int(ceil_div(B.cols(), W));
      t.nchunks = 1;
      t.chunk_len = int(std::min<int64_t>(B.rows(), INT32_MAX));
      t.wave_begin = 0;
      t.lin0 = total;
      total += int64_t(t.nstrips) * B.rows();
    }
    if (n == 0) return;
    // Long linear units accumulate the SIMD's age bias: with four blocks
    // per CU every dispatch round gets its own row share
    // (kTbLinearAgeWeights; 16384 x 131072 slab 4.70 -> 5.15 Tcells/s,
    // profiles/r3_raw/r3age_a16384.log).
    if (pairs && env_weights.empty() && split_v && bpc >= 4) {
      weights.assign(std::begin(kTbLinearAgeWeights), std::end(kTbLinearAgeWeights));
      G = int(weights.size());
    }
    const int Gl = pairs ? G : 1;
    const int64_t units = std::max<int64_t>(
        Gl, std::min<int64_t>(waves_target, total / std::max<int64_t>(1, min_len)));
    waves = int(units / Gl * Gl);
    args.lin_total = total;
    args.lin_slack = 2 * int64_t(depth);
    args.flags |= tbdetail::kTbLinear;
  }
  if (n == 0) return;
  args.nbox = n;
  args.total_waves = waves;
  if (pairs) {
    // wave_begin / total_waves count groups (units of one age).
    for (int b = 0; b < n; ++b) args.box[b].wave_begin /= G;
    args.total_waves = waves / G;
    args.flags |= tbdetail::kTbAgePairs;
    args.age_groups = G;
    double tot = 0.0;
    for (double w : weights) tot += w;
    double acc = 0.0;
    args.age_cum[0] = 0;
    for (int a = 0; a < G; ++a) {
      acc += weights[size_t(a)];
      args.age_cum[a + 1] = a + 1 == G ? 1024 : int(std::lround(1024.0 * acc / tot));
    }
  }
  const bool split = tb_variant_split(variant);
  if (split && !(variant & tbv::kShiftMixed)) {
    // Streaming rows when one pass sweeps more field than the MALL (256 MB)
    // holds: its rows come back one sweep later, never from L2 or the MALL.
    int64_t bytes = 0;
    for (int b = 0; b < nbox; ++b)
      if (!boxes[b].empty()) bytes += boxes[b].rows() * g.pitch * int64_t(sizeof(float));
    const bool nt = tune.nt >= 0 ? tune.nt != 0 : bytes > kTbStreamBytes;
    if (nt) args.flags |= tbdetail::kTbStreamRows;
  }
  if (tb_trace_enabled()) {
    // HEAT_TB_TRACE=1: each distinct plan once on stderr (planner checks).
    char line[320];
    std::snprintf(line, sizeof line,
                  "[heat tb] depth %d variant %d boxes %d strip_rows %lld waves_target %d bpc %d "
                  "linear %d units %d age_groups %d cum %d,%d,%d,%d chunk0 %d nchunks0 %d nt %d\n",
                  depth, variant, n, (long long)total_strip_rows, waves_target, bpc,
                  int((args.flags & tbdetail::kTbLinear) != 0), waves, pairs ? G : 0,
                  args.age_cum[1], args.age_cum[2], args.age_cum[3], args.age_cum[4],
                  args.box[0].chunk_len, args.box[0].nchunks,
                  int((args.flags & tbdetail::kTbStreamRows) != 0));
    tb_trace_once(line);
  }
  if (const Stamps sb = stamps_of_current_device(); sb.buf) {
    const int64_t need = int64_t(waves) * (split ? 2 : 1);
    HEAT_CHECK(need <= sb.waves, "stamp buffer holds %lld waves, launch has %lld",
               (long long)sb.waves, (long long)need);
    args.stamps = sb.buf;
  }
  if (chain && chain->passes > 1) {
    // Chained passes: the streaming build's classic one-box plan of one
    // dispatch round (every unit resident: the units poll each other).
    // args.total_waves counts the units of one age group (launch_chain).
    const int G = (args.flags & tbdetail::kTbAgePairs) ? args.age_groups : 1;
    int blocks = (args.total_waves + 1) / 2;
    if (G > 1) blocks = (blocks + 7) / 8 * 8 * G;
    static const int occ = tb_exp("the chained build (HEAT_TB_CHAIN=1)").tbc_occupancy_chain(kTbDeepDepth);
    int dev = 0, cus = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const bool fits = split && !(variant & tbv::kShiftMixed) && (args.flags & tbdetail::kTbStreamRows) &&
                      !(args.flags & tbdetail::kTbLinear) && !(args.flags & tbdetail::kTbAltDirection) &&
                      n == 1 && resid == nullptr && depth == kTbDeepDepth && args.stamps == nullptr &&
                      int64_t(args.total_waves) * G <= chain->max_units && blocks <= cus * occ;
    if (tb_trace_enabled()) {
      char line[320];
      std::snprintf(line, sizeof line,
                    "[heat chain] passes %d split %d mixed %d stream %d linear %d alt %d boxes %d resid %d "
                    "depth %d units %d x %d max %d blocks %d cus %d occ %d -> %d\n",
                    chain->passes, int(split), int((variant & tbv::kShiftMixed) != 0),
                    int((args.flags & tbdetail::kTbStreamRows) != 0),
                    int((args.flags & tbdetail::kTbLinear) != 0),
                    int((args.flags & tbdetail::kTbAltDirection) != 0), n, int(resid != nullptr), depth,
                    args.total_waves, G, chain->max_units, blocks, cus, occ, int(fits));
      tb_trace_once(line);
    }
    if (fits) {
      chain->chained = tb_exp("the chained build (HEAT_TB_CHAIN=1)")
                           .tbc_launch_chain(args, depth, chain->passes, chain->flags, chain->done,
                                             chain->err, st);
      HIP_CHECK(hipGetLastError());
      return;
    }
  }
  bool ok;
  if (split) {
    if (variant & tbv::kShiftMixed)
      ok = tb_exp("the mixed-shift split build (kShiftMixed)").tbxm_launch_split(args, depth, st);
    else if (!(args.flags & tbdetail::kTbStreamRows))
      ok = tbx::launch_split(args, depth, st);
    else if (split_pk_enabled())
      ok = tb_exp("the packed split build (HEAT_TB_SPLIT_PK=1)").tbxnp_launch_split(args, depth, st);
    else
      ok = tbxn::launch_split(args, depth, st);
  } else if (variant & tbv::kFloat2) {
    ok = tb_exp("the float2-lane build (kFloat2)").tbn_launch(args, depth, lag, st);
  } else if (variant & tbv::kScalar) {
    ok = tbs::launch(args, depth, lag, st);
  } else {
    ok = tb_exp("the packed build (no kScalar)").tbp_launch(args, depth, lag, st);
  }
  HEAT_CHECK(ok, "TB depth %d is not instantiated for variant %d (depth %d: scalar ring-3+ramp only)",
             depth, variant, kTbDeepDepth);
  HIP_CHECK(hipGetLastError());
}

void pack_box(const float* origin, int64_t pitch, const Box& box, float* buf, hipStream_t st) {
  if (box.empty()) return;
  hipLaunchKernelGGL(pack_kernel, dim3(grid_1d(box.rows() * box.cols())), dim3(256), 0, st,
                     origin, pitch, box, buf);
  HIP_CHECK(hipGetLastError());
}

void copy_boxes(float* origin, int64_t pitch, const BoxCopy* copies, int n, bool to_buf,
                hipStream_t st) {
  HEAT_CHECK(n >= 0 && n <= kMaxBoxCopies, "copy_boxes: %d boxes", n);
  BoxCopies a{};
  int m = 0;
  int64_t rows = 0;
  for (int i = 0; i < n; ++i) {
    if (copies[i].box.empty()) continue;
    a.c[m++] = copies[i];
    rows = std::max(rows, copies[i].box.rows());
  }
  if (m == 0) return;
  dim3 grid(unsigned(std::min<int64_t>(rows, 2048)), unsigned(m));
  hipLaunchKernelGGL(box_copy_kernel, grid, dim3(128), 0, st, origin, pitch, a, int(to_buf));
  HIP_CHECK(hipGetLastError());
}

void unpack_box(const float* buf, float* origin, int64_t pitch, const Box& box, hipStream_t st) {
  if (box.empty()) return;
  hipLaunchKernelGGL(unpack_kernel, dim3(grid_1d(box.rows() * box.cols())), dim3(256), 0, st,
                     buf, origin, pitch, box);
  HIP_CHECK(hipGetLastError());
}

float checksum_key_to_float(int key) {
  const int i = key >= 0 ? key : (key ^ 0x7FFFFFFF);
  float f;
  std::memcpy(&f, &i, 4);
  return f;
}

void checksum_block(const float* origin, int64_t pitch, int64_t lx, int64_t ly, int64_t ox,
                    int64_t oy, int64_t ny, DeviceChecksum* out, hipStream_t st) {
  if (lx <= 0 || ly <= 0) return;
  // ~8 workgroups per CU in total, grid-stride inside.
  const int64_t gx = std::min<int64_t>(ceil_div(ly, 256), 16);
  dim3 grid(unsigned(gx), unsigned(std::min<int64_t>(lx, std::max<int64_t>(1, 2048 / gx))));
  hipLaunchKernelGGL(checksum_kernel, grid, dim3(256), 0, st, origin, pitch, lx, ly, ox, oy, ny,
                     out);
  HIP_CHECK(hipGetLastError());
}

void judge_check(unsigned* resid, DeviceGate* gate, double eps, bool mpi_compat, hipStream_t st,
                 int n, int slots, int stride) {
  HEAT_CHECK(n >= 1 && slots >= 1 && slots <= 64 && (slots == 1 || stride >= n),
             "judge of %d checks x %d slots", n, slots);
  hipLaunchKernelGGL(judge_kernel, dim3(1), dim3(64), 0, st, resid, n, slots, stride, gate, eps,
                     int(mpi_compat));
  HIP_CHECK(hipGetLastError());
}

void residual_box(const float* a, const float* b, int64_t pitch, const Box& box, unsigned* resid,
                  hipStream_t st) {
  if (box.empty()) return;
  dim3 grid(unsigned(ceil_div(box.cols(), 64)),
            unsigned(std::min<int64_t>(ceil_div(box.rows(), 4), 1024)));
  hipLaunchKernelGGL(residual_kernel, grid, dim3(64, 4), 0, st, a, b, pitch, box, resid);
  HIP_CHECK(hipGetLastError());
}

}  // namespace heat::gpu

extern "C" void heat_register_exp_kernels(const heat::gpu::TbExpKernels* k) {
  std::lock_guard<std::mutex> lk(heat::gpu::g_exp_mu);
  heat::gpu::g_exp = k;
}
