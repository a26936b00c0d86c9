// MFMA single-step Jacobi kernel (--kernel mfma): the stencil as two banded
// matrix products on the fp32 matrix cores ("MFMA-packed fp32").
//
// For a 16x16 output tile at rows R, columns C:
//   D  = Av · U[R-1 .. R+18, C]        (vertical: 5 x v_mfma_f32_16x16x4_f32)
//   D += U[R, C-1 .. C+18] · Ah        (horizontal: 5 more)
// with Av[i][i] = cx, Av[i][i+1] = k0 = 1-2cx-2cy, Av[i][i+2] = cx and
// Ah[j][j] = Ah[j+2][j] = cy, zero elsewhere.  fp32 MFMA is exact fp32 and
// evaluates its products as an fmaf chain, so every cell gets the same chain
//   fma(cy,e, fma(cy,w, fma(cx,s, fma(k0,c, cx*n))))   (zero terms are exact no-ops)
// wherever it sits in a tile: the kernel is decomposition invariant bit for
// bit, but its rounding differs from the canonical expression (heat::stencil)
// by an ulp or two, so it is tested against the oracle with a tolerance.
//
// Cost: 10 MFMAs (320 SIMD cycles) per 256 cells, 3.3x the VALU issue of the
// canonical form; as a one-step-per-pass kernel it is still HBM-bound, which
// is where it lands next to the LDS kernel (tools/kernel_bench.py).  The TB
// kernel stays the default.
#include <hip/hip_runtime.h>

#include "heat/common.hpp"
#include "heat/kernels.hpp"
#include "tb_common.hpp"

namespace heat::gpu {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTileCols = 4;  // 16x16 tiles per wave along the columns (64 columns)

__global__ __launch_bounds__(256) void mfma_kernel(const float* __restrict__ src,
                                                   float* __restrict__ dst, StencilGeom g, Box box,
                                                   unsigned* resid) {
  if (tbdetail::gated(g.gate)) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t R = box.r0 + (int64_t(blockIdx.y) * 4 + wave) * 16;
  if (R >= box.r1) return;  // wave-uniform
  const int li = lane & 15, lk = lane >> 4;
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
  // Reads are clamped to the cells the box's stencil touches (rows
  // [r0-1, r1], columns [c0-1, c1]): finite values under zero coefficients.
  auto at = [&](int64_t r, int64_t c) {
    r = min(max(r, box.r0 - 1), box.r1);
    c = min(max(c, box.c0 - 1), box.c1);
    return src[r * g.pitch + c];
  };
  unsigned m = 0;
  for (int t = 0; t < kTileCols; ++t) {
    const int64_t C = box.c0 + (int64_t(blockIdx.x) * kTileCols + t) * 16;
    if (C >= box.c1) break;  // wave-uniform
    f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < 5; ++kb)  // B = U rows R-1+4kb+lk, column C+li
      d = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kb], at(R - 1 + 4 * kb + lk, C + li), d, 0, 0, 0);
#pragma unroll
    for (int kb = 0; kb < 5; ++kb)  // A = U row R+li, columns C-1+4kb+lk
      d = __builtin_amdgcn_mfma_f32_16x16x4f32(at(R + li, C - 1 + 4 * kb + lk), ah[kb], d, 0, 0, 0);
    // D: lane holds rows 4*lk+v, column li.
    const int64_t c = C + li;
    const bool col_in = c < box.c1, col_upd = tbdetail::in_interior(g.gy0 + c, g.ny);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t r = R + 4 * lk + v;
      if (!col_in || r >= box.r1) continue;
      const float old = src[r * g.pitch + c];
      const float out = (col_upd && tbdetail::in_interior(g.gx0 + r, g.nx)) ? d[v] : old;
      dst[r * g.pitch + c] = out;
      m = max(m, __float_as_uint(fabsf(out - old)));
    }
  }
  if (resid) tbdetail::wave_max_atomic(m, resid);
}

}  // namespace

void mfma_step(const float* src, float* dst, const StencilGeom& g, const Box& box,
               unsigned* resid, hipStream_t st) {
  if (box.empty()) return;
  dim3 grid(unsigned(ceil_div(box.cols(), 16 * kTileCols)), unsigned(ceil_div(box.rows(), 64)));
  hipLaunchKernelGGL(mfma_kernel, grid, dim3(256), 0, st, src, dst, g, box, resid);
  HIP_CHECK(hipGetLastError());
}

}  // namespace heat::gpu
