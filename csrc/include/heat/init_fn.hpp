// Initial-condition formulas shared by the host (CPU backend, tests) and the
// device init kernel, so both produce bit-identical fields.
//
// Reference: inidat, cuda/cuda_heat.cu:274-280 and
// mpi/mpi_heat_improved_persistent_stat.c:315-321:
//     u[ix][iy] = (float)(ix * (nx-ix-1) * iy * (ny-iy-1));   // int32
// The int32 product overflows for nx = ny >= 432.  RefWrap
// reproduces the wrapped result explicitly with uint32 arithmetic (which is
// what gcc/nvcc emitted for the undefined int overflow), so reference-sized
// grids initialise exactly as the reference binaries did.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define HEAT_HD __host__ __device__
#else
#define HEAT_HD
#endif

namespace heat {

HEAT_HD inline float init_ref_wrap(int64_t ix, int64_t iy, int64_t nx, int64_t ny) {
  // Same evaluation order as the C expression: ((ix*(nx-ix-1))*iy)*(ny-iy-1).
  uint32_t a = uint32_t(ix) * uint32_t(nx - ix - 1);
  a = a * uint32_t(iy);
  a = a * uint32_t(ny - iy - 1);
  return float(int32_t(a));
}

HEAT_HD inline float init_exact(int64_t ix, int64_t iy, int64_t nx, int64_t ny) {
  double v = double(ix) * double(nx - ix - 1) * double(iy) * double(ny - iy - 1);
  return float(v);
}

// splitmix64 finaliser: a counter-based generator, so the value of a cell
// depends only on (seed, gx, gy) and never on the decomposition.
HEAT_HD inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

HEAT_HD inline float init_random(int64_t ix, int64_t iy, uint64_t seed) {
  uint64_t h = mix64(seed * 0xD1B54A32D192ED03ull ^ mix64(uint64_t(ix) * 0x9E3779B97F4A7C15ull ^
                                                           uint64_t(iy)));
  // 24 random mantissa bits -> [0, 1), scaled to a "temperature" in [0, 100).
  return float(h >> 40) * (1.0f / 16777216.0f) * 100.0f;
}

// mode: 0 RefWrap, 1 Exact, 2 Random, 3 Zero (matches heat::InitMode).
HEAT_HD inline float init_value(int mode, int64_t ix, int64_t iy, int64_t nx, int64_t ny,
                                uint64_t seed) {
  if (ix < 0 || iy < 0 || ix >= nx || iy >= ny) return 0.0f;  // outside the plate
  switch (mode) {
    case 0: return init_ref_wrap(ix, iy, nx, ny);
    case 1: return init_exact(ix, iy, nx, ny);
    case 2: return init_random(ix, iy, seed);
    default: return 0.0f;
  }
}

// The canonical fp32 update shared by every backend and kernel variant:
//   u' = u + cx*((s + n) - 2u) + cy*((e + w) - 2u)
// evaluated with a fixed FMA contraction, exactly as written here, so the CPU
// oracle, the naive kernel and the temporally blocked kernel are bitwise
// identical.  (The reference CUDA expression, cuda/cuda_heat.cu:59-65, is the
// same formula; nvcc's default contraction produces this FMA shape.)
HEAT_HD inline float stencil(float c, float n, float s, float w, float e, float cx, float cy) {
  float tx = __builtin_fmaf(-2.0f, c, s + n);
  float ty = __builtin_fmaf(-2.0f, c, e + w);
  return __builtin_fmaf(cy, ty, __builtin_fmaf(cx, tx, c));
}

// The reference MPI program's update (mpi/mpi_heat_improved_persistent_stat.c:
// 168-174): the two neighbour sums are fp32 additions (float + float in C),
// everything else is double because of the 2.0 literal, evaluated left to
// right without contraction, and the result is rounded to fp32 once.
HEAT_HD inline float stencil_mpi(float c, float n, float s, float w, float e, float cx,
                                 float cy) {
#pragma clang fp contract(off)
  const float ns = s + n;
  const float ew = e + w;
  const double dc = double(c);
  const double a = dc + double(cx) * (double(ns) - 2.0 * dc);
  return float(a + double(cy) * (double(ew) - 2.0 * dc));
}

}  // namespace heat
