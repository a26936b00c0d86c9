// VALU issue-rate probe for the stencil's instruction mix (gfx950).
// Each wave runs ITERS iterations of a body of independent instructions on
// NCH accumulator chains; the grid puts W waves on every SIMD.  Prints
// cycles per VALU instruction per SIMD (shader clock from s_memtime deltas
// is not used: wall time x the measured clock is reported instead).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NCH = 16;

template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float a, float b) {
  if constexpr (KIND == 11) asm("v_mov_b32 %0, %1" : "=v"(b) : "s"(b));
  float cf[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) asm volatile("v_mov_b32 %0, %1" : "=v"(cf[q]) : "s"(b));
  float v[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) v[j] = float(threadIdx.x + j);
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 14) {  // DPP add whose result feeds the next instruction
#pragma unroll
      for (int j = 0; j < NCH; j += 2) {
        const float t = v[j] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[(j + 5) % NCH]), 0x138, 0xf, 0xf, true));
        v[j] = __builtin_fmaf(t, -2.0f, v[(j + 1) % NCH]);
      }
      continue;
    }
    if constexpr (KIND == 15) {  // the same ops, DPP results consumed 8 instructions later
      float t[NCH / 2];
#pragma unroll
      for (int j = 0; j < NCH; j += 2)
        t[j / 2] = v[j] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[(j + 5) % NCH]), 0x138, 0xf, 0xf, true));
#pragma unroll
      for (int j = 0; j < NCH; j += 2) v[j] = __builtin_fmaf(t[j / 2], -2.0f, v[(j + 1) % NCH]);
      continue;
    }
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      if constexpr (KIND == 0) {  // v_fmac_f32 (2 VGPR + SGPR)
        v[j] = __builtin_fmaf(v[j], a, b);
      } else if constexpr (KIND == 1) {  // v_add_f32 VGPR+VGPR
        v[j] = v[j] + v[(j + 1) % NCH];
      } else if constexpr (KIND == 2) {  // v_fma_f32 three VGPRs
        v[j] = __builtin_fmaf(v[(j + 3) % NCH], v[(j + 1) % NCH], v[j]);
      } else if constexpr (KIND == 3) {  // v_add_f32_dpp (wave_shr:1)
        v[j] = v[j] + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[(j + 5) % NCH]), 0x138, 0xf, 0xf, false));
      } else if constexpr (KIND == 5) {  // v_fmac_f32 v, s, v (one SGPR operand)
        v[j] = __builtin_fmaf(a, v[(j + 3) % NCH], v[j]);
      } else if constexpr (KIND == 6) {  // v_fmac_f32 v, -2.0, v (inline constant)
        v[j] = __builtin_fmaf(-2.0f, v[(j + 3) % NCH], v[j]);
      } else if constexpr (KIND == 7) {  // v_fma_f32 v, s, v, v (one SGPR, 3 operands)
        v[j] = __builtin_fmaf(a, v[(j + 3) % NCH], v[(j + 7) % NCH]);
      } else if constexpr (KIND == 8) {  // v_fmac_f32 with operands 4 and 8 registers apart
        v[j] = __builtin_fmaf(v[(j + 4) % NCH], v[(j + 8) % NCH], v[j]);
      } else if constexpr (KIND == 9) {  // v_fmac_f32 with operands 1 and 2 registers apart
        v[j] = __builtin_fmaf(v[(j + 1) % NCH], v[(j + 2) % NCH], v[j]);
      } else if constexpr (KIND == 10) {  // v_fma_f32 VOP3, all VGPRs, separate destination
        v[j] = __builtin_fmaf(v[(j + 1) % NCH], v[(j + 2) % NCH], v[(j + 3) % NCH]);
      } else if constexpr (KIND == 11) {  // v_fmac_f32 v, v, v with a VGPR coefficient (cx)
        v[j] = __builtin_fmaf(b, v[(j + 2) % NCH], v[j]);
      } else if constexpr (KIND == 12) {  // v_fmac_f32 v, 0.1 literal, v
        v[j] = __builtin_fmaf(0.1f, v[(j + 2) % NCH], v[j]);
      } else if constexpr (KIND == 13) {  // as 11, 16 chains reading 4 distinct coefficient copies
        v[j] = __builtin_fmaf(cf[j & 3], v[(j + 2) % NCH], v[j]);
      } else if constexpr (KIND == 4) {  // v_pk_fma_f32 (2 lanes per op)
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 x = {v[j], v[(j + 8) % NCH]};
        const f2 y = {a, a}, z = {b, b};
        x = __builtin_elementwise_fma(x, y, z);
        v[j] = x.x;
        v[(j + 8) % NCH] = x.y;
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) s += v[j];
  if (s == 12345.678f) out[threadIdx.x] = s;
}

template <int KIND>
double run(int waves_per_simd, int cus, int iters, float* out) {
  const int blocks = cus * waves_per_simd;  // 256 threads = 1 wave per SIMD
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 0.5f);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 0.5f);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

int main() {
  int cus = 0, clk = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHECK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));  // kHz
  float* out;
  CHECK(hipMalloc(&out, 4096));
  const int iters = 20000;
  const char* names[] = {"v_fma_f32 (v,v,s,s)", "v_add_f32 (v,v)", "v_fmac_f32 (v,v,v)", "v_add_f32_dpp",
                         "v_pk_fma_f32", "v_fmac_f32 (v,s,v)", "v_fmac_f32 (v,-2.0,v)", "v_fma_f32 (v,s,v,v)",
                         "v_fmac_f32 operands +4,+8 regs", "v_fmac_f32 operands +1,+2 regs",
                         "v_fma_f32 (v,v,v,v) VOP3", "v_fmac_f32 (v, vgpr coef, v)",
                         "v_fmac_f32 (v, 0.1 literal, v)", "v_fmac_f32 (v, 4 vgpr coef copies, v)",
                         "dpp add -> dependent fma (8+8 per iter)", "dpp adds then fmas (8+8 per iter)"};
  const int per_body[] = {NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH, NCH};
  for (int kind = 0; kind < 16; ++kind) {
    for (int w : {1, 2, 3, 4}) {
      double ms = 0;
      switch (kind) {
        case 0: ms = run<0>(w, cus, iters, out); break;
        case 1: ms = run<1>(w, cus, iters, out); break;
        case 2: ms = run<2>(w, cus, iters, out); break;
        case 3: ms = run<3>(w, cus, iters, out); break;
        case 4: ms = run<4>(w, cus, iters, out); break;
        case 5: ms = run<5>(w, cus, iters, out); break;
        case 6: ms = run<6>(w, cus, iters, out); break;
        case 7: ms = run<7>(w, cus, iters, out); break;
        case 8: ms = run<8>(w, cus, iters, out); break;
        case 9: ms = run<9>(w, cus, iters, out); break;
        case 10: ms = run<10>(w, cus, iters, out); break;
        case 11: ms = run<11>(w, cus, iters, out); break;
        case 12: ms = run<12>(w, cus, iters, out); break;
        case 13: ms = run<13>(w, cus, iters, out); break;
        case 14: ms = run<14>(w, cus, iters, out); break;
        case 15: ms = run<15>(w, cus, iters, out); break;
      }
      // instructions per SIMD = waves/SIMD x iters x body
      const double instr = double(w) * iters * per_body[kind];
      const double cyc = ms * 1e-3 * clk * 1e3;  // at the nominal max clock
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_instr_at_nominal_clock\": %.2f}\n",
             names[kind], w, ms, cyc / instr);
    }
  }
  return 0;
}
