// Cross-lane shift probe for the TB kernel's east/west neighbours (gfx950).
//
// Part A prints, for each lane primitive, which source lane every lane reads
// (input = lane id), so the shift formulas below are checked on hardware.
// Part B runs the ring-3 level pipeline of the TB kernel (as
// tools/probes/stencil_chain.hip) on register-resident rows with the two
// lane shifts of every float4 row update done by MODE:
//   0  wave_shr:1 / wave_shl:1 DPP (the single-wave kernel's form)
//   1  no shift (wrong math, same op count otherwise): the bound
//   2  row_shr:1 / row_shl:1 only (wrong at the 16-lane row edges): bound of 3-6
//   3  west: row_bcast:15 + row_shr:1 (correct), east: wave_shl:1
//   4  west: row_bcast:15 + row_shr:1, east: ds_bpermute
//   5  both ds_bpermute (the level-split kernel's form)
//   6  west: row_bcast:15 + row_shr:1, east: row_shl:1 over a permlane-fixed copy
//   7  both ds_bpermute, issued one iteration early: the shifts of a level's
//      new row are posted right after the next level has consumed the
//      previous ones, so their LDS latency hides behind a whole iteration
//      (compiler-scheduled: it sinks them back next to their uses)
//   8  as 7 with the ds_bpermute issued and waited for in inline asm, so the
//      early issue survives scheduling (waits: lgkmcnt(2K-2), in-order LDS)
// and prints cycles per float4 row update at the nominal clock for 1..4 waves
// per SIMD, plus a correctness flag of the shift formula of each mode.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));              \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int CTRL, int ROWM = 0xf, int BANKM = 0xf, bool BC = true>
__device__ __forceinline__ float dpp(float old, float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROWM, BANKM, BC));
}

// west neighbour value: lane l reads v from lane l-1
template <int MODE>
__device__ __forceinline__ float west(float v) {
  if constexpr (MODE == 0) {
    return dpp<0x138>(0.f, v);
  } else if constexpr (MODE == 1) {
    return v;
  } else if constexpr (MODE == 2) {
    return dpp<0x111>(0.f, v);
  } else if constexpr (MODE == 5) {
    const int l = threadIdx.x & 63;
    return __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 63) & 63) << 2, __float_as_int(v)));
  } else {
    // lanes 16, 32, 48 take lane 15, 31, 47 (row_bcast:15 into bank 0 of rows
    // 1-3), every other lane l-1 within its row (row_shr:1 leaving the row's
    // first lane untouched: bound_ctrl off).
    const float t = dpp<0x142, 0xe, 0x1, false>(v, v);
    return dpp<0x111, 0xf, 0xf, false>(t, v);
  }
}

// east neighbour value: lane l reads v from lane l+1
template <int MODE>
__device__ __forceinline__ float east(float v) {
  if constexpr (MODE == 0 || MODE == 3) {
    return dpp<0x130>(0.f, v);
  } else if constexpr (MODE == 1) {
    return v;
  } else if constexpr (MODE == 2) {
    return dpp<0x101>(0.f, v);
  } else if constexpr (MODE == 4 || MODE == 5) {
    const int l = threadIdx.x & 63;
    return __int_as_float(__builtin_amdgcn_ds_bpermute(((l + 1) & 63) << 2, __float_as_int(v)));
  } else {
    // MODE 6: u = v with each row's lane 0 replaced by the next row's lane 0
    // (lanes 0/16/32 <- 16/32/48 through the two permlane swaps), then
    // row_ror:15 (lane j <- lane j+1 of its row, lane 15 <- the row's lane 0).
    const unsigned x = __float_as_uint(v);
    const auto p16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const auto p32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    const int l = threadIdx.x & 63;
    // p16[1]: row0 <- row1, row2 <- row3 (if the swap is as documented);
    // p32[1]: lanes 0..31 <- 32..63.
    const unsigned u = (l == 16) ? p32[1] : p16[1];
    return dpp<0x12f>(0.f, __uint_as_float(u));
  }
}

__device__ __forceinline__ float st(float c, float n, float s, float w, float e, float cx, float cy) {
  const float tx = __builtin_fmaf(-2.0f, c, s + n);
  const float ty = __builtin_fmaf(-2.0f, c, e + w);
  return __builtin_fmaf(cy, ty, __builtin_fmaf(cx, tx, c));
}

template <int MODE>
__device__ __forceinline__ f4 upd(const f4& a, const f4& b, const f4& c, float cx, float cy) {
  const float w = west<MODE>(b.w);
  const float e = east<MODE>(b.x);
  f4 r;
  r.x = st(b.x, a.x, c.x, w, b.y, cx, cy);
  r.y = st(b.y, a.y, c.y, b.x, b.z, cx, cy);
  r.z = st(b.z, a.z, c.z, b.y, b.w, cx, cy);
  r.w = st(b.w, a.w, c.w, e, b.z, cx, cy);
  return r;
}

__device__ __forceinline__ f4 upd_pre(const f4& a, const f4& b, const f4& c, float w, float e,
                                      float cx, float cy) {
  f4 r;
  r.x = st(b.x, a.x, c.x, w, b.y, cx, cy);
  r.y = st(b.y, a.y, c.y, b.x, b.z, cx, cy);
  r.z = st(b.z, a.z, c.z, b.y, b.w, cx, cy);
  r.w = st(b.w, a.w, c.w, e, b.z, cx, cy);
  return r;
}

template <int K, int MODE>
__global__ __launch_bounds__(256) void chain(float* out, int iters, float cx, float cy) {
  f4 R[K][3];
  f4 in = f4(float(threadIdx.x));
#pragma unroll
  for (int s = 0; s < K; ++s)
#pragma unroll
    for (int j = 0; j < 3; ++j) R[s][j] = f4(float(s + j));
  if constexpr (MODE == 8) {
    // Same schedule as MODE 7; each shifted value is produced by an asm
    // ds_bpermute (opaque to the compiler's waitcnt pass) and read only
    // through an asm s_waitcnt that takes it as an in/out operand, so no
    // use can move above the wait.  2K bpermutes are in flight per
    // iteration; a value is consumed one iteration after issue, when the
    // 2K-2 bpermutes issued after it may still be pending.
    float ws[K], es[K];
#pragma unroll
    for (int s = 0; s < K; ++s) ws[s] = es[s] = float(s);
    const int l = threadIdx.x & 63;
    const int aw = ((l + 63) & 63) << 2, ae = ((l + 1) & 63) << 2;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int U = 0; U < 3; ++U) {
        R[0][U] = in;
#pragma unroll
        for (int s = 1; s <= K; ++s) {
          float w = ws[s - 1], e = es[s - 1];
          // the two shifts of level s-1 were issued 2K-2 LDS ops ago at least
          asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(w), "+v"(e) : "n"(2 * K - 2 > 15 ? 15 : 2 * K - 2));
          f4 r = upd_pre(R[s - 1][(U - s - 1 + 30) % 3], R[s - 1][(U - s + 30) % 3],
                         R[s - 1][(U - s + 1 + 30) % 3], w, e, cx, cy);
          if (s < K) R[s][(U - s + 30) % 3] = r; else in = r;
          const f4& nw = R[s - 1][(U - s + 1 + 30) % 3];
          asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(ws[s - 1]) : "v"(aw), "v"(nw.w));
          asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(es[s - 1]) : "v"(ae), "v"(nw.x));
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float s = in.x + in.y + in.z + in.w + ws[0] + es[0];
    if (s == 1234.5f) out[threadIdx.x] = s;
    return;
  }
  if constexpr (MODE == 7) {
    // ws[s]/es[s]: lane shifts of level s's newest row, consumed by level s+1
    // in the next iteration (level s's row i-s is level s+1's centre row then).
    float ws[K], es[K];
#pragma unroll
    for (int s = 0; s < K; ++s) ws[s] = es[s] = float(s);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int U = 0; U < 3; ++U) {
        R[0][U] = in;
#pragma unroll
        for (int s = 1; s < K; ++s) {
          R[s][(U - s + 30) % 3] = upd_pre(R[s - 1][(U - s - 1 + 30) % 3], R[s - 1][(U - s + 30) % 3],
                                           R[s - 1][(U - s + 1 + 30) % 3], ws[s - 1], es[s - 1], cx, cy);
          // level s-1's newest row (row i-s+1) is the centre of level s next time
          const f4& nw = R[s - 1][(U - s + 1 + 30) % 3];
          ws[s - 1] = west<5>(nw.w);
          es[s - 1] = east<5>(nw.x);
        }
        in = upd_pre(R[K - 1][(U - K - 1 + 30) % 3], R[K - 1][(U - K + 30) % 3],
                     R[K - 1][(U - K + 1 + 30) % 3], ws[K - 1], es[K - 1], cx, cy);
        const f4& nw = R[K - 1][(U - K + 1 + 30) % 3];
        ws[K - 1] = west<5>(nw.w);
        es[K - 1] = east<5>(nw.x);
      }
    }
    const float s = in.x + in.y + in.z + in.w;
    if (s == 1234.5f) out[threadIdx.x] = s;
    return;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int U = 0; U < 3; ++U) {
      R[0][U] = in;
#pragma unroll
      for (int s = 1; s < K; ++s)
        R[s][(U - s + 30) % 3] = upd<MODE>(R[s - 1][(U - s - 1 + 30) % 3], R[s - 1][(U - s + 30) % 3],
                                            R[s - 1][(U - s + 1 + 30) % 3], cx, cy);
      in = upd<MODE>(R[K - 1][(U - K - 1 + 30) % 3], R[K - 1][(U - K + 30) % 3],
                     R[K - 1][(U - K + 1 + 30) % 3], cx, cy);
    }
  }
  const float s = in.x + in.y + in.z + in.w;
  if (s == 1234.5f) out[threadIdx.x] = s;
}

// Part A: lane maps.  out[op*64 + lane] = source lane read (or -1 = own old).
__global__ void lanemap(float* out) {
  const int l = threadIdx.x;
  const float v = float(l);
  const float old = -1.f;
  int k = 0;
  out[k++ * 64 + l] = dpp<0x138, 0xf, 0xf, false>(old, v);  // wave_shr:1
  out[k++ * 64 + l] = dpp<0x130, 0xf, 0xf, false>(old, v);  // wave_shl:1
  out[k++ * 64 + l] = dpp<0x111, 0xf, 0xf, false>(old, v);  // row_shr:1
  out[k++ * 64 + l] = dpp<0x101, 0xf, 0xf, false>(old, v);  // row_shl:1
  out[k++ * 64 + l] = dpp<0x142, 0xe, 0x1, false>(old, v);  // row_bcast:15 rows1-3 bank0
  out[k++ * 64 + l] = dpp<0x12f, 0xf, 0xf, false>(old, v);  // row_ror:15
  {
    const unsigned x = __float_as_uint(v);
    const auto p16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    const auto p32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    out[k++ * 64 + l] = __uint_as_float(p16[0]);
    out[k++ * 64 + l] = __uint_as_float(p16[1]);
    out[k++ * 64 + l] = __uint_as_float(p32[0]);
    out[k++ * 64 + l] = __uint_as_float(p32[1]);
  }
  out[k++ * 64 + l] = west<0>(v);
  out[k++ * 64 + l] = east<0>(v);
  out[k++ * 64 + l] = west<3>(v);
  out[k++ * 64 + l] = east<4>(v);
  out[k++ * 64 + l] = east<6>(v);
}

template <int K, int MODE>
void run(int cus, int clk, float* out) {
  const int iters = 400;
  for (int w = 1; w <= 4; ++w) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL((chain<K, MODE>), dim3(cus * w), dim3(256), 0, 0, out, iters, 0.1f, 0.1f);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((chain<K, MODE>), dim3(cus * w), dim3(256), 0, 0, out, iters, 0.1f, 0.1f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double updates = double(w) * iters * 3 * K;  // float4 row updates per SIMD
    const double cyc = ms * 1e-3 * clk * 1e3;
    printf("{\"probe\": \"chain\", \"K\": %d, \"mode\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
           "\"cycles_per_row_update\": %.1f}\n",
           K, MODE, w, ms, cyc / updates);
    fflush(stdout);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
  }
}

int main() {
  int cus = 0, clk = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
  float* out;
  CHECK(hipMalloc(&out, 64 * 64 * 4));
  CHECK(hipMemset(out, 0, 64 * 64 * 4));
  hipLaunchKernelGGL(lanemap, dim3(1), dim3(64), 0, 0, out);
  CHECK(hipDeviceSynchronize());
  float h[15 * 64];
  CHECK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
  const char* names[] = {"wave_shr1", "wave_shl1", "row_shr1", "row_shl1", "row_bcast15_r1-3_b0",
                         "row_ror15", "p16swap[0]", "p16swap[1]", "p32swap[0]", "p32swap[1]",
                         "west_mode0", "east_mode0", "west_mode3", "east_mode4", "east_mode6"};
  for (int k = 0; k < 15; ++k) {
    printf("{\"probe\": \"lanemap\", \"op\": \"%s\", \"src\": [", names[k]);
    for (int l = 0; l < 64; ++l) printf("%s%d", l ? ", " : "", int(h[k * 64 + l]));
    printf("]}\n");
  }
  fflush(stdout);
  run<8, 0>(cus, clk, out);
  run<8, 1>(cus, clk, out);
  run<8, 2>(cus, clk, out);
  run<8, 3>(cus, clk, out);
  run<8, 4>(cus, clk, out);
  run<8, 5>(cus, clk, out);
  run<8, 6>(cus, clk, out);
  run<8, 7>(cus, clk, out);
  run<8, 8>(cus, clk, out);
  run<6, 8>(cus, clk, out);
  run<12, 8>(cus, clk, out);
  run<4, 7>(cus, clk, out);
  run<6, 7>(cus, clk, out);
  run<12, 0>(cus, clk, out);
  run<12, 1>(cus, clk, out);
  run<12, 5>(cus, clk, out);
  run<12, 7>(cus, clk, out);
  CHECK(hipFree(out));
  return 0;
}
