// MFMA single-step Jacobi kernel (--kernel mfma): the stencil as two banded
// matrix products on the fp32 matrix cores ("MFMA-packed fp32"),
// with its operands staged through LDS.
//
// For a 16x16 output tile at rows R, columns C:
//   D  = Av · U[R-1 .. R+18, C .. C+15]      (vertical: 5 x v_mfma_f32_16x16x4_f32)
//   D += U[R .. R+15, C-1 .. C+18] · Ah      (horizontal: 5 more)
// with Av[i][i] = cx, Av[i][i+1] = k0 = 1-2cx-2cy, Av[i][i+2] = cx and
// Ah[j][j] = Ah[j+2][j] = cy, zero elsewhere.  fp32 MFMA is exact fp32 and
// evaluates its products as an fmaf chain, so every cell gets the same chain
//   fma(cy,e, fma(cy,w, fma(cx,s, fma(k0,c, cx*n))))   (zero terms are exact no-ops)
// wherever it sits in a tile: the kernel is decomposition invariant bit for
// bit, but its rounding differs from the canonical expression (heat::stencil)
// by an ulp or two, so it is tested against the oracle with a tolerance.
//
// Data path (the reference's heat kernel, cuda/cuda_heat.cu:140-163, reads
// every operand from global memory; round 2's MFMA kernel did too, 11.2 B
// per update): a 256-thread workgroup stages a 66 x 136 halo tile of the
// source in LDS with coalesced 16-byte loads (~4.4 B read per update), then
// each wave computes a 16 x 128 strip as 8 MFMA tiles whose A/B fragments
// come from LDS (ds_read_b32).  The LDS row pitch is 146 floats (18 mod 32
// banks): the vertical B fragment (16 consecutive columns of 4 rows) and the
// horizontal A fragment (one column of 16 rows, two columns per 32-lane
// group) both read with at most 2-way bank conflicts.  The centre value (the
// Dirichlet ring and the residual) also comes from the tile.
//
// Cost: 10 MFMAs (320 SIMD cycles) per 256 cells = 3.3x the issue of the
// canonical VALU form; at one step per pass it is bounded by the ~8.4 B per
// update it moves, i.e. by HBM, like the LDS kernel.  The temporally blocked
// VALU kernel stays the default (README "MFMA").
#include <hip/hip_runtime.h>

#include "heat/common.hpp"
#include "heat/kernels.hpp"
#include "tb_common.hpp"

namespace heat::gpu {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 64;             // output rows per workgroup (4 waves x 16)
constexpr int kCols = 128;            // output columns per workgroup (8 tiles of 16)
constexpr int kTileRows = kRows + 2;  // rows R0-1 .. R0+64 from memory
constexpr int kPadRows = 2;           // + 2 zero rows: the K=20 padding of the last wave's B fragment
constexpr int kLoadCols = kCols + 8;  // float4 columns [cb-4, cb+132)
constexpr int kPitch = 146;           // LDS row pitch in floats: 18 mod 32 banks, 8-byte rows

__host__ __device__ inline int64_t floor4(int64_t x) { return x & ~int64_t(3); }

__global__ __launch_bounds__(256) void mfma_kernel(const float* __restrict__ src,
                                                   float* __restrict__ dst, StencilGeom g, Box box,
                                                   int64_t c_base, int ntx, int nty,
                                                   unsigned* resid) {
  __shared__ float tile[(kTileRows + kPadRows) * kPitch];
  if (tbdetail::gated(g.gate)) return;  // uniform: before the barrier
  // XCD-aware tile order: blocks b, b+8, ... share an XCD (round-robin
  // dispatch, observed), so each XCD takes a contiguous row-major range of
  // tiles and the halo lines of side-by-side tiles hit its L2.
  const int nt = ntx * nty, b = blockIdx.x, x8 = b & 7, j = b >> 3;
  const int q = nt >> 3, r = nt & 7;
  const int t = x8 * q + min(x8, r) + j;
  const int64_t R0 = box.r0 + int64_t(t / ntx) * kRows;
  const int64_t cb = c_base + int64_t(t % ntx) * kCols;  // multiple of 4
  // Stage rows R0-1 .. R0+64 and columns cb-4 .. cb+131: coalesced float4
  // loads, clamped to the cells the box's stencil can touch (rows
  // [r0-1, r1], columns [c0-1, c1]); clamped values are never used.
  const int64_t lo4 = floor4(box.c0 - 1), hi4 = floor4(box.c1);
  constexpr int kQ = kLoadCols / 4;
  for (int i = threadIdx.x; i < kTileRows * kQ; i += 256) {
    const int rr = i / kQ, q = i - rr * kQ;
    const int64_t r = min(max(R0 - 1 + rr, box.r0 - 1), box.r1);
    const int64_t c = min(max(cb - 4 + 4 * int64_t(q), lo4), hi4);
    const float4 v = *reinterpret_cast<const float4*>(src + r * g.pitch + c);
    float2* t = reinterpret_cast<float2*>(tile + rr * kPitch + 4 * q);
    t[0] = make_float2(v.x, v.y);
    t[1] = make_float2(v.z, v.w);
  }
  // The padding rows meet zero coefficients (Av[i][k] = 0 for k > i+2):
  // zeros, not memory, keep the products exact.
  for (int i = threadIdx.x; i < kPadRows * kPitch; i += 256) tile[kTileRows * kPitch + i] = 0.f;
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int64_t R = R0 + wave * 16;  // this wave's first output row
  const float cx = g.cx, cy = g.cy;
  const float k0 = __builtin_fmaf(-2.0f, cy, __builtin_fmaf(-2.0f, cx, 1.0f));
  // Constant operands: Av (A of the vertical products), Ah (B of the horizontal).
  float av[5], ah[5];
#pragma unroll
  for (int kb = 0; kb < 5; ++kb) {
    const int r = 4 * kb + lk;  // K index
    av[kb] = r == li ? cx : r == li + 1 ? k0 : r == li + 2 ? cx : 0.0f;
    ah[kb] = (r == li || r == li + 2) ? cy : 0.0f;
  }
  // LDS row of output row R + i: 1 + 16*wave + i; LDS column of column C + j
  // in tile t: 4 + 16*t + j.
  const float* trow = tile + (1 + wave * 16) * kPitch;
  unsigned m = 0;
  if (R < box.r1) {  // wave-uniform
#pragma unroll 2
    for (int t = 0; t < kCols / 16; ++t) {
      const int tc = 4 + 16 * t;
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 5; ++kb)  // B = U rows R-1+4kb+lk, column C+li
        d = __builtin_amdgcn_mfma_f32_16x16x4f32(
            av[kb], trow[(4 * kb + lk - 1) * kPitch + tc + li], d, 0, 0, 0);
#pragma unroll
      for (int kb = 0; kb < 5; ++kb)  // A = U row R+li, columns C-1+4kb+lk
        d = __builtin_amdgcn_mfma_f32_16x16x4f32(
            trow[li * kPitch + tc - 1 + 4 * kb + lk], ah[kb], d, 0, 0, 0);
      // D: lane holds rows 4*lk+v, column li.
      const int64_t c = cb + 16 * t + li;
      const bool col_in = c >= box.c0 && c < box.c1;
      const bool col_upd = tbdetail::in_interior(g.gy0 + c, g.ny);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int i = 4 * lk + v;
        const int64_t r = R + i;
        if (!col_in || r >= box.r1) continue;
        const float old = trow[i * kPitch + tc + li];
        const float out = (col_upd && tbdetail::in_interior(g.gx0 + r, g.nx)) ? d[v] : old;
        dst[r * g.pitch + c] = out;
        m = max(m, __float_as_uint(fabsf(out - old)));
      }
    }
  }
  if (resid) tbdetail::wave_max_atomic(m, resid);
}

}  // namespace

void mfma_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
               unsigned* resid, hipStream_t st) {
  if (box.empty()) return;
  const int64_t c_base = floor4(box.c0);
  const int ntx = int(ceil_div(box.c1 - c_base, kCols)), nty = int(ceil_div(box.rows(), kRows));
  hipLaunchKernelGGL(mfma_kernel, dim3(unsigned(ntx) * unsigned(nty)), dim3(256), 0, st, src, dst,
                     g, box, c_base, ntx, nty, resid);
  HIP_CHECK(hipGetLastError());
}

}  // namespace heat::gpu
