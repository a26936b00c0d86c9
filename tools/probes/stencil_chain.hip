// Issue-rate probe of the TB kernel's arithmetic alone: the ring-3 level
// pipeline of tb_stream.inl (K levels, float4 lanes, DPP east/west, the
// canonical FMA update) on register-resident rows, no memory traffic.
// ILP=1: one strip per wave (the kernel's structure); ILP=2: two independent
// strips interleaved in one wave.  Prints cycles per VALU row-update at the
// nominal clock for 1..4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float from_left(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_right(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ float st(float c, float n, float s, float w, float e, float cx, float cy) {
  float tx = __builtin_fmaf(-2.0f, c, s + n);
  float ty = __builtin_fmaf(-2.0f, c, e + w);
  return __builtin_fmaf(cy, ty, __builtin_fmaf(cx, tx, c));
}
// The update with the center row's lane shifts precomputed (w = row[l-1].w,
// e = row[l+1].x).
__device__ __forceinline__ f4 upd_pre(const f4& a, const f4& b, const f4& c, float w, float e,
                                      float cx, float cy) {
  f4 r;
  r.x = st(b.x, a.x, c.x, w, b.y, cx, cy);
  r.y = st(b.y, a.y, c.y, b.x, b.z, cx, cy);
  r.z = st(b.z, a.z, c.z, b.y, b.w, cx, cy);
  r.w = st(b.w, a.w, c.w, e, b.z, cx, cy);
  return r;
}

template <int VAR>
__device__ __forceinline__ f4 upd(const f4& a, const f4& b, const f4& c, float cx, float cy) {
  f4 r;
  // VAR 0: as the kernel; 1: no DPP (same-lane w/e, wrong math, same op
  // count); 2: coefficients as inline constants (0.5); 3: both.
  float w, e;
  if (VAR & 1) {
    w = b.w;
    e = b.x;
  } else if (VAR & 4) {  // ds_bpermute (LDS crossbar, no LDS memory)
    const int l = threadIdx.x & 63;
    w = __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 63) & 63) << 2, __float_as_int(b.w)));
    e = __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 1) & 63) << 2, __float_as_int(b.x)));
  } else if (VAR & 8) {  // row_shr:1 / row_shl:1 (16-lane rows; row edges wrong)
    w = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(b.w), 0x111, 0xf, 0xf, true));
    e = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(b.x), 0x101, 0xf, 0xf, true));
  } else {
    w = from_left(b.w);
    e = from_right(b.x);
  }
  if (VAR & 2) { cx = 0.5f; cy = 0.5f; }
  if constexpr ((VAR & 32) != 0) {
    // Packed f32 (v_pk_add_f32 / v_pk_fma_f32) on the pairs (x,y), (z,w):
    // the same per-element operations in the same order as st() (bitwise
    // equal; Upd::apply PK in tb_tile_core.hpp, RowUpdate HEAT_TB_PACKED in
    // tb_stream.inl): ~14 VALU per float4 row instead of 24.
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 m2 = {-2.0f, -2.0f}, cx2 = {cx, cx}, cy2 = {cy, cy};
    const f2 b01 = {b.x, b.y}, b23 = {b.z, b.w};
    const f2 ns01 = f2{c.x, c.y} + f2{a.x, a.y}, ns23 = f2{c.z, c.w} + f2{a.z, a.w};
    const f2 ew01 = {b.y + w, b.z + b.x}, ew23 = {b.w + b.y, e + b.z};
    const f2 tx01 = __builtin_elementwise_fma(m2, b01, ns01), tx23 = __builtin_elementwise_fma(m2, b23, ns23);
    const f2 ty01 = __builtin_elementwise_fma(m2, b01, ew01), ty23 = __builtin_elementwise_fma(m2, b23, ew23);
    const f2 r01 = __builtin_elementwise_fma(cy2, ty01, __builtin_elementwise_fma(cx2, tx01, b01));
    const f2 r23 = __builtin_elementwise_fma(cy2, ty23, __builtin_elementwise_fma(cx2, tx23, b23));
    return f4{r01.x, r01.y, r23.x, r23.y};
  }
  r.x = st(b.x, a.x, c.x, w, b.y, cx, cy);
  r.y = st(b.y, a.y, c.y, b.x, b.z, cx, cy);
  r.z = st(b.z, a.z, c.z, b.y, b.w, cx, cy);
  r.w = st(b.w, a.w, c.w, e, b.z, cx, cy);  // e + w order as in the kernel
  return r;
}

template <int K, int ILP, int VAR>
struct Chain {
  f4 R[ILP][K][3];
  template <int U>
  __device__ __forceinline__ void body(f4 in[ILP], float cx, float cy) {
    if constexpr (VAR == 16) {
      // All K center-row lane shifts first (their rows are from the previous
      // iteration), then the K level updates.
#pragma unroll
      for (int p = 0; p < ILP; ++p) {
        float ws[K], es[K];
#pragma unroll
        for (int s = 1; s <= K; ++s) {
          const f4& b = R[p][s - 1][(U - s + 30) % 3];
          ws[s - 1] = from_left(b.w);
          es[s - 1] = from_right(b.x);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the shifts grouped
        R[p][0][U] = in[p];
#pragma unroll
        for (int s = 1; s < K; ++s)
          R[p][s][(U - s + 30) % 3] = upd_pre(R[p][s - 1][(U - s - 1 + 30) % 3], R[p][s - 1][(U - s + 30) % 3],
                                              R[p][s - 1][(U - s + 1 + 30) % 3], ws[s - 1], es[s - 1], cx, cy);
        in[p] = upd_pre(R[p][K - 1][(U - K - 1 + 30) % 3], R[p][K - 1][(U - K + 30) % 3],
                        R[p][K - 1][(U - K + 1 + 30) % 3], ws[K - 1], es[K - 1], cx, cy);
      }
      return;
    }
#pragma unroll
    for (int p = 0; p < ILP; ++p) {
      R[p][0][U] = in[p];
#pragma unroll
      for (int s = 1; s < K; ++s)
        R[p][s][(U - s + 30) % 3] = upd<VAR>(R[p][s - 1][(U - s - 1 + 30) % 3], R[p][s - 1][(U - s + 30) % 3],
                                        R[p][s - 1][(U - s + 1 + 30) % 3], cx, cy);
      in[p] = upd<VAR>(R[p][K - 1][(U - K - 1 + 30) % 3], R[p][K - 1][(U - K + 30) % 3],
                  R[p][K - 1][(U - K + 1 + 30) % 3], cx, cy);
    }
  }
};

template <int K, int ILP, int VAR>
__global__ __launch_bounds__(256) void chain(float* out, int iters, float cx, float cy) {
  Chain<K, ILP, VAR> c;
  f4 in[ILP];
#pragma unroll
  for (int p = 0; p < ILP; ++p) {
    in[p] = f4(float(threadIdx.x + p));
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
      for (int j = 0; j < 3; ++j) c.R[p][s][j] = f4(float(s + j));
  }
  for (int it = 0; it < iters; ++it) {
    c.template body<0>(in, cx, cy);
    c.template body<1>(in, cx, cy);
    c.template body<2>(in, cx, cy);
  }
  float s = 0;
#pragma unroll
  for (int p = 0; p < ILP; ++p) s += in[p].x + in[p].y + in[p].z + in[p].w;
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int K, int ILP, int VAR>
void run(int cus, int clk) {
  float* out;
  CHECK(hipMalloc(&out, 4096));
  const int iters = 400;
  for (int w = 1; w <= 4; ++w) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((chain<K, ILP, VAR>), dim3(cus * w), dim3(256), 0, 0, out, iters, 0.1f, 0.1f);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((chain<K, ILP, VAR>), dim3(cus * w), dim3(256), 0, 0, out, iters, 0.1f, 0.1f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double updates = double(w) * iters * 3 * K * ILP;  // float4 row updates per SIMD
    const double cyc = ms * 1e-3 * clk * 1e3;
    printf("{\"K\": %d, \"ilp\": %d, \"var\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_row_update\": %.1f}\n",
           K, ILP, VAR, w, ms, cyc / updates);
  }
  CHECK(hipFree(out));
}

int main() {
  int cus = 0, clk = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
  run<8, 1, 0>(cus, clk);
  run<8, 1, 1>(cus, clk);
  run<8, 1, 16>(cus, clk);
  // One stage of the depth-12 level-split pipeline (6 levels per wave):
  // DPP shifts, ds_bpermute shifts (the split kernel's), no shifts.
  run<6, 1, 0>(cus, clk);
  run<6, 1, 4>(cus, clk);
  run<6, 1, 1>(cus, clk);
  // Round 6: the packed row update in that stage (ds_bpermute shifts: the
  // split kernel's; DPP; none).
  run<6, 1, 36>(cus, clk);
  run<6, 1, 32>(cus, clk);
  run<6, 1, 33>(cus, clk);
  return 0;
}
