// Can a halo exchange run concurrently with the interior TB kernel on one
// MI355X?  Single-process probe of the multi-GPU pass schedule at the 8-GPU
// strong-scaling shape (1024 x 8192 slab per rank, K = 8):
//
//   boundary bands (compute stream)  ->  interior || "exchange" (comm stream)
//
// The exchange is proxied by device kernels of the same size as the real one
// (two 8-row padded slabs out and back, as RCCL's p2p kernels would move), so
// it competes for CUs like RCCL does.  Modes:
//   0  serial           exchange, then interior (no overlap)
//   1  two streams      default priorities
//   2  two streams      comm stream at the highest priority
//   3  CU-masked        compute stream without R CUs, comm stream only on them
//   4  sync, m=1        exchange then ONE launch over the whole slab
//   5  sync, m=4        exchange 4K-deep ghosts once per 4 passes; each pass
//                       one launch over the slab grown by the valid ghosts
//
// Build: make probe   Run: build/overlap_probe [R=8] [iters=200] [lx=1024]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "heat/common.hpp"
#include "heat/kernels.hpp"
#include "heat/topology.hpp"

using namespace heat;

static void copy_slab(float* dst, const float* src, size_t n, hipStream_t st) {
  HIP_CHECK(hipMemcpyAsync(dst, src, n * 4, hipMemcpyDeviceToDevice, st));
}

int main(int argc, char** argv) {
  const int reserve = argc > 1 ? std::atoi(argv[1]) : 8;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
  const int64_t lx = argc > 3 ? std::atoll(argv[3]) : 1024, ly = 8192;
  const int K = 8;
  const int M = 4;
  HIP_CHECK(hipSetDevice(0));
  hipDeviceProp_t prop;
  HIP_CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  const Layout L = Layout::make(lx, ly, M * K);
  const size_t elems = size_t(L.rows) * size_t(L.pitch);
  float *base[2], *field[2], *sbuf, *rbuf;
  for (int i = 0; i < 2; ++i) {
    HIP_CHECK(hipMalloc(&base[i], elems * 4));
    field[i] = base[i] + L.hx * L.pitch + L.hy;
    gpu::init_field(field[i], L, 4096, 0, 8192, 8192, 2 /*random*/, 7, nullptr);
  }
  const size_t slab = size_t(M * K) * size_t(L.pitch);
  HIP_CHECK(hipMalloc(&sbuf, 2 * slab * 4));
  HIP_CHECK(hipMalloc(&rbuf, 2 * slab * 4));
  gpu::StencilGeom g;
  g.pitch = L.pitch;
  g.gx0 = 4096;  // an interior slab of the 8192^2 plate: neighbours on both sides
  g.nx = 8192;
  g.ny = 8192;

  int least, greatest;
  HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t comp, comm_lo, comm_hi, comp_m, comm_m;
  HIP_CHECK(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&comm_lo, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithPriority(&comm_hi, hipStreamNonBlocking, greatest));
  std::vector<uint32_t> mask_comp((ncu + 31) / 32, 0), mask_comm((ncu + 31) / 32, 0);
  // Reserve every (ncu/reserve)-th CU, spreading the reserved CUs over XCDs.
  const int stride = reserve > 0 ? ncu / reserve : ncu + 1;
  for (int c = 0; c < ncu; ++c) {
    const bool r = reserve > 0 && c % stride == stride - 1 && c / stride < reserve;
    (r ? mask_comm : mask_comp)[c / 32] |= 1u << (c % 32);
  }
  HIP_CHECK(hipExtStreamCreateWithCUMask(&comp_m, uint32_t(mask_comp.size()), mask_comp.data()));
  HIP_CHECK(hipExtStreamCreateWithCUMask(&comm_m, uint32_t(mask_comm.size()), mask_comm.data()));

  const Box interior{K, lx - K, 0, ly};
  const Box bands[2] = {{0, K, 0, ly}, {lx - K, lx, 0, ly}};
  const int res_waves = gpu::tb_resident_waves(K, -1);
  hipEvent_t ev_bnd, ev_comm, e0, e1;
  HIP_CHECK(hipEventCreateWithFlags(&ev_bnd, hipEventDisableTiming));
  HIP_CHECK(hipEventCreateWithFlags(&ev_comm, hipEventDisableTiming));
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));

  auto exchange = [&](int cur, hipStream_t st, int depth) {
    float* f = field[cur];
    const size_t n = size_t(depth) * size_t(L.pitch);
    copy_slab(sbuf, f - L.hy, n, st);                                   // north send rows
    copy_slab(sbuf + slab, f + (lx - depth) * L.pitch - L.hy, n, st);   // south send rows
    copy_slab(f - depth * L.pitch - L.hy, rbuf, n, st);                 // north ghosts
    copy_slab(f + lx * L.pitch - L.hy, rbuf + slab, n, st);             // south ghosts
  };
  int pass_no = 0;
  auto pass = [&](int mode, int& cur, int waves) {
    hipStream_t cs = mode == 3 ? comp_m : comp;
    hipStream_t ms = mode == 1 ? comm_lo : mode == 3 ? comm_m : comm_hi;
    if (mode == 4 || mode == 5) {
      const int m = mode == 4 ? 1 : M;
      const int j = pass_no++ % m;
      if (j == 0) exchange(cur, cs, m * K);
      const int64_t e = int64_t(m - 1 - j) * K;
      const Box grown{-e, lx + e, 0, ly};
      gpu::tb_step(field[cur], field[cur ^ 1], g, &grown, 1, K, nullptr, cs, waves);
    } else if (mode == 0) {
      exchange(cur, cs, K);
      gpu::tb_step(field[cur], field[cur ^ 1], g, &interior, 1, K, nullptr, cs, waves);
      gpu::tb_step(field[cur], field[cur ^ 1], g, bands, 2, K, nullptr, cs, waves);
    } else {
      HIP_CHECK(hipStreamWaitEvent(cs, ev_comm, 0));
      gpu::tb_step(field[cur], field[cur ^ 1], g, bands, 2, K, nullptr, cs, waves);
      HIP_CHECK(hipEventRecord(ev_bnd, cs));
      gpu::tb_step(field[cur], field[cur ^ 1], g, &interior, 1, K, nullptr, cs, waves);
      HIP_CHECK(hipStreamWaitEvent(ms, ev_bnd, 0));
      exchange(cur ^ 1, ms, K);
      HIP_CHECK(hipEventRecord(ev_comm, ms));
    }
    cur ^= 1;
  };
  const char* names[] = {"serial", "2 streams", "comm high prio", "CU-masked", "sync m=1",
                         "sync m=4"};
  std::printf("{\"ncu\": %d, \"reserve\": %d, \"lx\": %lld, \"ly\": %lld, \"K\": %d, \"resident_waves\": %d}\n",
              ncu, reserve, (long long)lx, (long long)ly, K, res_waves);
  for (int rep = 0; rep < 2; ++rep) {
    for (int mode = 0; mode < 6; ++mode) {
      const int waves = mode == 3 ? res_waves * (ncu - reserve) / ncu : 0;
      int cur = 0;
      HIP_CHECK(hipEventRecord(ev_comm, comm_hi));
      for (int i = 0; i < 10; ++i) pass(mode, cur, waves);
      HIP_CHECK(hipDeviceSynchronize());
      hipStream_t cs = mode == 3 ? comp_m : comp;
      HIP_CHECK(hipEventRecord(e0, cs));
      for (int i = 0; i < iters; ++i) pass(mode, cur, waves);
      HIP_CHECK(hipStreamWaitEvent(cs, ev_comm, 0));
      HIP_CHECK(hipEventRecord(e1, cs));
      HIP_CHECK(hipDeviceSynchronize());
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / iters;
      std::printf("{\"rep\": %d, \"mode\": %d, \"name\": \"%s\", \"us_per_pass\": %.2f, \"gcells_s\": %.1f}\n",
                  rep, mode, names[mode], us, double(lx) * ly * K / us * 1e-3);
    }
  }
  // Components alone.
  {
    int cur = 0;
    HIP_CHECK(hipEventRecord(e0, comp));
    for (int i = 0; i < iters; ++i) exchange(cur, comp, K);
    HIP_CHECK(hipEventRecord(e1, comp));
    HIP_CHECK(hipDeviceSynchronize());
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"name\": \"exchange proxy alone\", \"us\": %.2f}\n", 1e3 * ms / iters);
    HIP_CHECK(hipEventRecord(e0, comp));
    for (int i = 0; i < iters; ++i) {
      gpu::tb_step(field[cur], field[cur ^ 1], g, &interior, 1, K, nullptr, comp, 0);
      cur ^= 1;
    }
    HIP_CHECK(hipEventRecord(e1, comp));
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"name\": \"interior alone\", \"us\": %.2f}\n", 1e3 * ms / iters);
    HIP_CHECK(hipEventRecord(e0, comp));
    for (int i = 0; i < iters; ++i) {
      gpu::tb_step(field[cur], field[cur ^ 1], g, bands, 2, K, nullptr, comp, 0);
      cur ^= 1;
    }
    HIP_CHECK(hipEventRecord(e1, comp));
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"name\": \"bands alone\", \"us\": %.2f}\n", 1e3 * ms / iters);
    const Box full{0, lx, 0, ly};
    HIP_CHECK(hipEventRecord(e0, comp));
    for (int i = 0; i < iters; ++i) {
      gpu::tb_step(field[cur], field[cur ^ 1], g, &full, 1, K, nullptr, comp, 0);
      cur ^= 1;
    }
    HIP_CHECK(hipEventRecord(e1, comp));
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("{\"name\": \"full slab, one launch\", \"us\": %.2f}\n", 1e3 * ms / iters);
  }
  return 0;
}
