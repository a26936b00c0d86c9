// Run-time configuration of a heat-diffusion run.
//
// The reference fixes everything at compile time with -D macros
// (cuda/cuda_heat.cu:7-23, mpi/mpi_heat_improved_persistent_stat.c:7-32,
// mpi/Makefile:1-25).  Here the same knobs are run-time fields; the defaults
// reproduce the reference's source defaults (20x20 grid, cx=cy=0.1,
// eps=1e-3, check interval 20 as in cuda/cuda_heat.cu:16 / mpi/Makefile:8).
#pragma once

#include <cstdint>
#include <string>

namespace heat {

// Initial condition (reference: inidat, cuda/cuda_heat.cu:274-280).
enum class InitMode : int {
  RefWrap = 0,  // ix*(nx-ix-1)*iy*(ny-iy-1) in int32 with two's-complement wrap
                // (bit-identical to what the reference binaries compute)
  Exact = 1,    // the same polynomial evaluated exactly (fp64), then rounded
  Random = 2,   // counter-based hash of (seed, gx, gy) -> [0, 100): independent
                // of the decomposition
  Zero = 3,
};

enum class Backend : int { Cpu = 0, Hip = 1 };

// Stencil kernel family on the GPU.
enum class KernelKind : int {
  Auto = 0,   // temporally blocked streaming kernel (TB) at the tuned depth
  Naive = 1,  // one cell per thread, global loads only (independent oracle)
  TB = 2,     // register-streaming temporally blocked kernel, depth tb_depth
  Lds = 3,    // LDS-staged halo tile, one step per launch (also --numerics mpi)
  Mfma = 4,   // the stencil as banded matmuls on fp32 MFMA, one step per launch
              // (an experiment: not bitwise equal to the others; see mfma.hip)
};

// Reference-compatibility switches.
enum class Compat : int {
  None = 0,  // exactly `steps` updates; check after steps C, 2C, ...; converged <=> max|d| < eps
  Mpi = 1,   // steps+1 updates; check after C, 2C, ...; converged <=> max|d| <= eps
  Cuda = 2,  // steps updates; check after 1, C+1, 2C+1, ...; converged <=> max|d| < eps
};

// How the process grid is formed from the world size.
enum class DecompKind : int {
  Auto = 0,  // 2-D, MPI_Dims_create-compatible (mpi/...c:51-52)
  Rows = 1,  // 1-D slabs along x (contiguous halo rows, no packing)
  Grid2D = 2,
};

// Arithmetic of the update.
enum class Numerics : int {
  Fp32 = 0,  // canonical fp32 FMA expression, heat::stencil (= the reference CUDA
             // kernel's expression under nvcc's default contraction); every kernel
  Mpi = 1,   // the reference MPI program's: fp32 neighbour sums, the rest in
             // double (its 2.0 literal), one rounding to fp32; heat::stencil_mpi.
             // CPU backend and the naive GPU kernel only.
};

// Pass schedule of a multi-rank GPU run (the reference overlaps
// inner-cell compute with MPI_Isend/Irecv).  Measured on MI355X
// (profiles/overlap_probe_r1.md): cross-queue event hops cost ~10 us and
// the boundary bands of a K=8 pass are a latency-bound ~10 us launch, more
// than a 1024x8192 slab's exchange saves by overlapping, so the default is
// the deep-halo synchronous schedule, which instead exchanges m*K-deep
// ghosts once per m passes and computes the shrinking ghost region
// redundantly (one launch per pass, one exchange per m passes).
enum class Schedule : int {
  Auto = 0,      // Sync
  Sync = 1,      // exchange (when ghosts run out) then one launch per pass
  Overlap = 2,   // exchange-first: exchange || interior, then boundary bands
  Pipeline = 3,  // boundary-first: bands, then next exchange || interior
};

struct Params {
  int64_t nx = 20;  // rows (slow index), NXPROB
  int64_t ny = 20;  // columns (contiguous index), NYPROB
  float cx = 0.1f;  // PARMS_CX / parms.cx
  float cy = 0.1f;  // PARMS_CY / parms.cy
  bool converge = false;   // -DCONVERGE
  int check_interval = 20; // CHECK_INTERVAL / STEP
  double eps = 1e-3;       // literal 1e-3 of the reference (a double in mpi/...c:245)
  InitMode init = InitMode::RefWrap;
  uint64_t seed = 0;
  Backend backend = Backend::Cpu;
  KernelKind kernel = KernelKind::Auto;
  int tb_depth = 0;     // 0 = tuned default
  int threads = 0;      // CPU OpenMP threads (0 = runtime default)
  DecompKind decomp = DecompKind::Auto;
  int px = 0, py = 0;   // explicit process grid (0 = derived)
  bool use_graph = true;    // capture step chunks as hipGraphs
  bool overlap = true;      // halo exchange concurrent with interior compute
  Compat compat = Compat::None;
  int device = -1;          // HIP device ordinal (-1 = local rank % device count)
  Schedule schedule = Schedule::Auto;
  int halo_passes = 0;      // passes per exchange with Sync (ghost depth m*K); 0 = auto
  Numerics numerics = Numerics::Fp32;
  bool phase_timing = false;  // per-phase device times in RunStats (runs eagerly)
};

const char* init_mode_name(InitMode m);
const char* kernel_name(KernelKind k);
const char* compat_name(Compat c);
const char* schedule_name(Schedule s);
const char* numerics_name(Numerics n);

}  // namespace heat
