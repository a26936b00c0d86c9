// CPU reference backend (serial / OpenMP).  This is the test oracle and the
// analogue of the reference's MPI/OpenMP loop nests
// (mpi/mpi_heat_improved_persistent_stat.c:162-234, OpenMP pragmas at
// :163-165, :181-183, :210-212).  It evaluates the same FMA expression as the
// GPU kernels (heat::stencil) and is therefore bitwise identical to them.
#pragma once

#include <cstdint>

#include "heat/topology.hpp"

namespace heat::cpu {

struct Geom {
  int64_t pitch = 0;
  int64_t gx0 = 0, gy0 = 0;
  int64_t nx = 0, ny = 0;
  float cx = 0.1f, cy = 0.1f;
  int numerics = 0;  // heat::Numerics
};

void set_threads(int n);
int get_threads();

// Fill every allocated cell of a host field with the initial condition.
void init_field(float* origin, const Layout& L, int64_t gx0, int64_t gy0, int64_t nx, int64_t ny,
                int mode, uint64_t seed);

// One Jacobi step over box; returns max |new-old| over the box (as float;
// NaN if any cell became NaN) when want_resid, else 0.
float step(const float* src, float* dst, const Geom& g, const Box& box, bool want_resid);

void copy_box(const float* src, int64_t src_pitch, float* dst, int64_t dst_pitch, const Box& box);

}  // namespace heat::cpu
