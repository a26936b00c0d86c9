// LDS-staged single-step Jacobi kernel (--kernel lds).
//
// The classic tiled form of the reference's `heat` kernel
// (cuda/cuda_heat.cu:140-163, one cell per thread, global loads only),
// rebuilt for CDNA4: a 256-thread workgroup stages a (32+2) x (256+8) halo
// tile in LDS with coalesced 16-byte loads, then each wave updates 8 rows of
// 256 columns with one float4 per lane: north/centre/south rows come from
// LDS as ds_read_b128, east/west neighbours cross lanes with DPP (the tile's
// edge lanes read the halo columns from LDS).  The residual max|delta| is
// fused (wave max, one atomic per wave).
//
// It is templated on the update arithmetic, so it is also the fast GPU path
// of --numerics mpi (the reference MPI program's double arithmetic), which
// the register-streaming TB kernel does not implement.  For the canonical
// fp32 arithmetic the TB kernel (8 steps per HBM pass) is ~5x faster; this
// kernel reads and writes the field once per step.
#include <hip/hip_runtime.h>

#include "heat/common.hpp"
#include "heat/init_fn.hpp"
#include "heat/kernels.hpp"
#include "tb_common.hpp"

namespace heat::gpu {
namespace {

constexpr int kLdsRows = 32;                 // output rows per tile
constexpr int kLdsCols = 256;                // output columns per tile (64 lanes x float4)
constexpr int kLdsPitch4 = kLdsCols / 4 + 2;  // float4 per LDS row: 1 halo float4 each side

// Round down to a multiple of 4, toward -inf (boxes may start in the ghost ring).
__host__ __device__ inline int64_t floor4(int64_t x) { return x & ~int64_t(3); }

// Lane l <- lane l-1 (wave_shr:1); lane 0, which has no source lane, keeps
// `edge` (bound_ctrl off).  Folding the tile-edge value into the DPP `old`
// operand avoids a lane select, which the compiler may turn into an EXEC
// mask that disables the very lane the shift reads from.
__device__ __forceinline__ float lds_from_left(float v, float edge) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x138, 0xf, 0xf, false));
}
// Lane l <- lane l+1 (wave_shl:1); lane 63 keeps `edge`.
__device__ __forceinline__ float lds_from_right(float v, float edge) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x130, 0xf, 0xf, false));
}

template <int NUMERICS>
__device__ __forceinline__ float lds_update(float c, float n, float s, float w, float e, float cx,
                                            float cy) {
  if constexpr (NUMERICS == 1) return stencil_mpi(c, n, s, w, e, cx, cy);
  return stencil(c, n, s, w, e, cx, cy);
}

template <int NUMERICS>
__global__ __launch_bounds__(256) void lds_kernel(const float* __restrict__ src,
                                                  float* __restrict__ dst, StencilGeom g, Box box,
                                                  int64_t c_base, int ntx, int nty,
                                                  unsigned* resid) {
  __shared__ float4 tile[(kLdsRows + 2) * kLdsPitch4];
  if (tbdetail::gated(g.gate)) return;  // uniform: before the barrier
  // XCD-aware tile order (blocks b, b+8, ... share an XCD): each XCD takes a
  // contiguous row-major range of tiles, so the halo lines of neighbouring
  // tiles are fetched once per XCD L2 instead of once per tile.
  const int nt = ntx * nty, b = blockIdx.x, x8 = b & 7, j = b >> 3;
  const int q = nt >> 3, rem = nt & 7;
  const int t = x8 * q + min(x8, rem) + j;
  const int64_t r0 = box.r0 + int64_t(t / ntx) * kLdsRows;
  const int64_t cb = c_base + int64_t(t % ntx) * kLdsCols;  // multiple of 4
  // Cooperative staging of rows r0-1 .. r0+kLdsRows and float4 columns
  // cb-4 .. cb+kLdsCols+3.  Loads are clamped to the cells the box's
  // stencil can touch (rows [r0box-1, r1box], columns [c0-1, c1]), which
  // keeps every access inside the allocation; clamped values are unused.
  const int64_t lo4 = floor4(box.c0 - 1), hi4 = floor4(box.c1);
  for (int i = threadIdx.x; i < (kLdsRows + 2) * kLdsPitch4; i += 256) {
    const int rr = i / kLdsPitch4, cc = i - rr * kLdsPitch4;
    const int64_t r = min(max(r0 - 1 + rr, box.r0 - 1), box.r1);
    const int64_t c = min(max(cb - 4 + 4 * int64_t(cc), lo4), hi4);
    tile[i] = *reinterpret_cast<const float4*>(src + r * g.pitch + c);
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t col = cb + 4 * lane;
  // Which of this lane's 4 columns are in the box and global-interior.
  bool in[4], upd[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    in[j] = col + j >= box.c0 && col + j < box.c1;
    upd[j] = in[j] && tbdetail::in_interior(g.gy0 + col + j, g.ny);
  }
  const bool full = in[0] && in[3];
  unsigned m = 0;
  for (int k = 0; k < kLdsRows / 4; ++k) {
    const int rr = wave * (kLdsRows / 4) + k;  // output row within the tile
    const int64_t r = r0 + rr;
    if (r >= box.r1) break;
    const float4* trow = tile + (rr + 1) * kLdsPitch4;
    const float4 c = trow[lane + 1];
    const float4 a = tile[rr * kLdsPitch4 + lane + 1];        // north
    const float4 b = tile[(rr + 2) * kLdsPitch4 + lane + 1];  // south
    const float wl = trow[0].w, er = trow[kLdsPitch4 - 1].x;  // tile-edge halo columns
    const float w = lds_from_left(c.w, wl);
    const float e = lds_from_right(c.x, er);
    const bool row_ok = tbdetail::in_interior(g.gx0 + r, g.nx);
    float4 o;
    o.x = (upd[0] && row_ok) ? lds_update<NUMERICS>(c.x, a.x, b.x, w, c.y, g.cx, g.cy) : c.x;
    o.y = (upd[1] && row_ok) ? lds_update<NUMERICS>(c.y, a.y, b.y, c.x, c.z, g.cx, g.cy) : c.y;
    o.z = (upd[2] && row_ok) ? lds_update<NUMERICS>(c.z, a.z, b.z, c.y, c.w, g.cx, g.cy) : c.z;
    o.w = (upd[3] && row_ok) ? lds_update<NUMERICS>(c.w, a.w, b.w, c.z, e, g.cx, g.cy) : c.w;
    float* d = dst + r * g.pitch + col;
    if (full) {
      *reinterpret_cast<float4*>(d) = o;
    } else {
      if (in[0]) d[0] = o.x;
      if (in[1]) d[1] = o.y;
      if (in[2]) d[2] = o.z;
      if (in[3]) d[3] = o.w;
    }
    if (resid) {
      m = max(m, in[0] ? __float_as_uint(fabsf(o.x - c.x)) : 0u);
      m = max(m, in[1] ? __float_as_uint(fabsf(o.y - c.y)) : 0u);
      m = max(m, in[2] ? __float_as_uint(fabsf(o.z - c.z)) : 0u);
      m = max(m, in[3] ? __float_as_uint(fabsf(o.w - c.w)) : 0u);
    }
  }
  if (resid) tbdetail::wave_max_atomic(m, resid);
}

}  // namespace

void lds_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
              unsigned* resid, hipStream_t st) {
  if (box.empty()) return;
  // Tiles start on a float4 column (origin and pitch are 16-byte aligned).
  const int64_t c_base = floor4(box.c0);
  const int ntx = int(ceil_div(box.c1 - c_base, kLdsCols)), nty = int(ceil_div(box.rows(), kLdsRows));
  const dim3 grid(unsigned(ntx) * unsigned(nty));
  if (g.numerics == 1)
    hipLaunchKernelGGL(lds_kernel<1>, grid, dim3(256), 0, st, src, dst, g, box, c_base, ntx, nty,
                       resid);
  else
    hipLaunchKernelGGL(lds_kernel<0>, grid, dim3(256), 0, st, src, dst, g, box, c_base, ntx, nty,
                       resid);
  HIP_CHECK(hipGetLastError());
}

}  // namespace heat::gpu
