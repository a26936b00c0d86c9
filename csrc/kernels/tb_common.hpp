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
};

constexpr int kMaxBoxes = 16;

struct TbArgs {
  const float* src;
  float* dst;
  unsigned* resid;
  StencilGeom g;
  int nbox, total_waves;
  TbBox box[kMaxBoxes];
};

__device__ __forceinline__ bool in_interior(int64_t g, int64_t n) { return g >= 1 && g <= n - 2; }

__device__ __forceinline__ void wave_max_atomic(unsigned m, unsigned* resid) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, unsigned(__shfl_xor(int(m), off)));
  if ((threadIdx.x & 63) == 0) atomicMax(resid, m);
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
