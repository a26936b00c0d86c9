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

#include "heat/common.hpp"
#include "heat/init_fn.hpp"
#include "heat/kernels.hpp"

namespace heat::gpu {
namespace {

constexpr int kWave = 64;

__device__ __forceinline__ bool in_interior(int64_t g, int64_t n) { return g >= 1 && g <= n - 2; }

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
__device__ __forceinline__ void wave_max_atomic(unsigned m, unsigned* resid) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = max(m, unsigned(__shfl_xor(int(m), off)));
  if ((threadIdx.x & (kWave - 1)) == 0) atomicMax(resid, m);
}

__global__ __launch_bounds__(256) void naive_kernel(const float* __restrict__ src,
                                                    float* __restrict__ dst, StencilGeom g,
                                                    Box box, unsigned* resid) {
  const int64_t c = box.c0 + int64_t(blockIdx.x) * 64 + threadIdx.x;
  const int64_t r = box.r0 + int64_t(blockIdx.y) * 4 + threadIdx.y;
  unsigned m = 0;
  if (r < box.r1 && c < box.c1) {
    const int64_t i = r * g.pitch + c;
    const float v = src[i];
    float out = v;
    if (in_interior(g.gx0 + r, g.nx) && in_interior(g.gy0 + c, g.ny))
      out = stencil(v, src[i - g.pitch], src[i + g.pitch], src[i - 1], src[i + 1], g.cx, g.cy);
    dst[i] = out;
    m = __float_as_uint(fabsf(out - v));
  }
  if (resid) wave_max_atomic(m, resid);
}

// --------------------------------------------------------------------------
// temporally blocked register-streaming kernel
// --------------------------------------------------------------------------
struct TbBox {
  int64_t r0, r1, c0, c1;
  int nstrips, nchunks, chunk_len, wave_begin;
};

struct TbArgs {
  const float* src;
  float* dst;
  unsigned* resid;
  StencilGeom g;
  int nbox, total_waves;
  TbBox box[5];
};

__device__ __forceinline__ float dpp_from_left(float v) {  // lane l <- lane l-1 (wave_shr:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
}
__device__ __forceinline__ float dpp_from_right(float v) {  // lane l <- lane l+1 (wave_shl:1)
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
}

template <bool EDGE>
struct RowUpdate {
  float cx, cy;
  bool cm0, cm1, cm2, cm3;  // per-column "updatable" masks (EDGE only)
  __device__ __forceinline__ float4 operator()(const float4& a, const float4& b, const float4& c,
                                               bool row_ok) const {
    if (EDGE && !row_ok) return b;
    const float w = dpp_from_left(b.w);
    const float e = dpp_from_right(b.x);
    float4 r;
    r.x = stencil(b.x, a.x, c.x, w, b.y, cx, cy);
    r.y = stencil(b.y, a.y, c.y, b.x, b.z, cx, cy);
    r.z = stencil(b.z, a.z, c.z, b.y, b.w, cx, cy);
    r.w = stencil(b.w, a.w, c.w, b.z, e, cx, cy);
    if (EDGE) {
      r.x = cm0 ? r.x : b.x;
      r.y = cm1 ? r.y : b.y;
      r.z = cm2 ? r.z : b.z;
      r.w = cm3 ? r.w : b.w;
    }
    return r;
  }
};

constexpr int mod3(int v) { return ((v % 3) + 3) % 3; }

template <int K, bool EDGE>
struct TbStream {
  // R[s][slot]: level-s rows in a 3-slot ring (level 0 = input rows).
  float4 R[K][3];
  float4 P[3];  // prefetch ring (rows i+3)
  unsigned m = 0;

  template <int U>
  __device__ __forceinline__ void body(int64_t i, const float* __restrict__ src,
                                       float* __restrict__ dst, int64_t pitch, int64_t last_in,
                                       int64_t rb, int64_t re, int64_t gx0, int64_t nx,
                                       bool store_lane, const RowUpdate<EDGE>& upd,
                                       bool want_resid) {
    R[0][U] = P[U];
    {
      const int64_t nxt = min(i + 3, last_in);
      P[U] = *reinterpret_cast<const float4*>(src + nxt * pitch);
    }
#pragma unroll
    for (int s = 1; s < K; ++s) {
      const bool ok = !EDGE || in_interior(gx0 + (i - s), nx);
      R[s][mod3(U - s)] =
          upd(R[s - 1][mod3(U - s - 1)], R[s - 1][mod3(U - s)], R[s - 1][mod3(U - s + 1)], ok);
    }
    const int64_t ro = i - K;  // output row of this iteration
    const bool ok = !EDGE || in_interior(gx0 + ro, nx);
    const float4& b = R[K - 1][mod3(U - K)];
    const float4 out = upd(R[K - 1][mod3(U - K - 1)], b, R[K - 1][mod3(U - K + 1)], ok);
    if (ro >= rb && ro < re && store_lane) {
      *reinterpret_cast<float4*>(dst + ro * pitch) = out;
      if (want_resid) {
        m = max(m, __float_as_uint(fabsf(out.x - b.x)));
        m = max(m, __float_as_uint(fabsf(out.y - b.y)));
        m = max(m, __float_as_uint(fabsf(out.z - b.z)));
        m = max(m, __float_as_uint(fabsf(out.w - b.w)));
      }
    }
  }

  __device__ __forceinline__ void run(const float* __restrict__ src, float* __restrict__ dst,
                                      int64_t pitch, int64_t rb, int64_t re, int64_t gx0,
                                      int64_t nx, bool store_lane, const RowUpdate<EDGE>& upd,
                                      bool want_resid) {
    // src/dst already offset to this lane's column; rows are absolute local rows.
    const int64_t first_in = rb - K, last_in = re + K - 1;
    const int64_t T = last_in - first_in + 1;
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
      for (int j = 0; j < 3; ++j) R[s][j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 3; ++j)
      P[j] = *reinterpret_cast<const float4*>(src + min(first_in + j, last_in) * pitch);
    for (int64_t t = 0; t < T; t += 3) {
      const int64_t i = first_in + t;
      body<0>(i, src, dst, pitch, last_in, rb, re, gx0, nx, store_lane, upd, want_resid);
      body<1>(i + 1, src, dst, pitch, last_in, rb, re, gx0, nx, store_lane, upd, want_resid);
      body<2>(i + 2, src, dst, pitch, last_in, rb, re, gx0, nx, store_lane, upd, want_resid);
    }
  }
};

template <int K>
__global__ __launch_bounds__(256) void tb_kernel(TbArgs a) {
  constexpr int KK = (K + 3) & ~3;
  constexpr int W = 256 - 2 * KK;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave >= a.total_waves) return;
  int bi = 0;
#pragma unroll
  for (int j = 1; j < 5; ++j)
    if (j < a.nbox && wave >= a.box[j].wave_begin) bi = j;
  const TbBox bx = a.box[bi];
  const int w = wave - bx.wave_begin;
  const int strip = w % bx.nstrips, chunk = w / bx.nstrips;
  const int64_t cbase = bx.c0 + int64_t(strip) * W;
  const int64_t cend = min(cbase + W, bx.c1);
  const int64_t col = cbase - KK + 4 * lane;
  const bool store_lane = col >= cbase && col < cend;
  const int64_t rb = bx.r0 + int64_t(chunk) * bx.chunk_len;
  const int64_t re = min(rb + bx.chunk_len, bx.r1);

  const StencilGeom& g = a.g;
  const float* src = a.src + col;
  float* dst = a.dst + col;
  const bool want_resid = a.resid != nullptr;

  // Wave-uniform fast path: every row and column the wave touches is a
  // global interior cell, so no Dirichlet masking is needed.
  const int64_t gy_lo = g.gy0 + cbase - KK, gy_hi = gy_lo + 255;
  const int64_t gx_lo = g.gx0 + rb - K, gx_hi = g.gx0 + re + K - 1;
  const bool interior = gy_lo >= 1 && gy_hi <= g.ny - 2 && gx_lo >= 1 && gx_hi <= g.nx - 2;
  unsigned m;
  if (interior) {
    RowUpdate<false> upd{g.cx, g.cy, true, true, true, true};
    TbStream<K, false> st;
    st.run(src, dst, g.pitch, rb, re, g.gx0, g.nx, store_lane, upd, want_resid);
    m = st.m;
  } else {
    const int64_t gy = g.gy0 + col;
    RowUpdate<true> upd{g.cx,
                        g.cy,
                        in_interior(gy, g.ny),
                        in_interior(gy + 1, g.ny),
                        in_interior(gy + 2, g.ny),
                        in_interior(gy + 3, g.ny)};
    TbStream<K, true> st;
    st.run(src, dst, g.pitch, rb, re, g.gx0, g.nx, store_lane, upd, want_resid);
    m = st.m;
  }
  if (want_resid) wave_max_atomic(m, a.resid);
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

int grid_1d(int64_t n) { return int(std::min<int64_t>(ceil_div(n, 256), 256 * 16)); }

template <int K>
void launch_tb(TbArgs& args, hipStream_t st) {
  const int blocks = int(ceil_div(args.total_waves, 4));
  hipLaunchKernelGGL(tb_kernel<K>, dim3(blocks), dim3(256), 0, st, args);
}

}  // namespace

bool tb_depth_supported(int k) {
  return (k >= 1 && k <= 8) || k == 10 || k == 12 || k == 16;
}

int tb_strip_width(int k) { return 256 - 2 * int(round_up(k, 4)); }

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

void tb_step(const float* src, float* dst, const StencilGeom& g, const Box* boxes, int nbox,
             int depth, unsigned* resid, hipStream_t st, int waves_target) {
  HEAT_CHECK(tb_depth_supported(depth), "unsupported TB depth %d", depth);
  HEAT_CHECK(nbox >= 0 && nbox <= 5, "nbox=%d", nbox);
  if (waves_target <= 0) waves_target = 2048;
  const int W = tb_strip_width(depth);
  TbArgs args{};
  args.src = src;
  args.dst = dst;
  args.resid = resid;
  args.g = g;
  // Split rows into chunks so the whole launch has about waves_target waves,
  // but never shorter than 4*depth rows (keeps the redundant 2*depth-row
  // halo reads below ~50 %).
  int64_t total_strip_rows = 0;
  for (int b = 0; b < nbox; ++b)
    if (!boxes[b].empty()) total_strip_rows += ceil_div(boxes[b].cols(), W) * boxes[b].rows();
  const int64_t min_len = std::max<int64_t>(4 * depth, 16);
  int64_t len = std::max<int64_t>(min_len, ceil_div(total_strip_rows, waves_target));
  int n = 0, waves = 0;
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
    t.chunk_len = int(std::min<int64_t>(len, B.rows()));
    t.nchunks = int(ceil_div(B.rows(), t.chunk_len));
    t.wave_begin = waves;
    waves += t.nstrips * t.nchunks;
  }
  if (n == 0) return;
  args.nbox = n;
  args.total_waves = waves;
  switch (depth) {
    case 1: launch_tb<1>(args, st); break;
    case 2: launch_tb<2>(args, st); break;
    case 3: launch_tb<3>(args, st); break;
    case 4: launch_tb<4>(args, st); break;
    case 5: launch_tb<5>(args, st); break;
    case 6: launch_tb<6>(args, st); break;
    case 7: launch_tb<7>(args, st); break;
    case 8: launch_tb<8>(args, st); break;
    case 10: launch_tb<10>(args, st); break;
    case 12: launch_tb<12>(args, st); break;
    case 16: launch_tb<16>(args, st); break;
    default: HEAT_CHECK(false, "unsupported TB depth %d", depth);
  }
  HIP_CHECK(hipGetLastError());
}

void pack_box(const float* origin, int64_t pitch, const Box& box, float* buf, hipStream_t st) {
  if (box.empty()) return;
  hipLaunchKernelGGL(pack_kernel, dim3(grid_1d(box.rows() * box.cols())), dim3(256), 0, st,
                     origin, pitch, box, buf);
  HIP_CHECK(hipGetLastError());
}

void unpack_box(const float* buf, float* origin, int64_t pitch, const Box& box, hipStream_t st) {
  if (box.empty()) return;
  hipLaunchKernelGGL(unpack_kernel, dim3(grid_1d(box.rows() * box.cols())), dim3(256), 0, st,
                     buf, origin, pitch, box);
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
