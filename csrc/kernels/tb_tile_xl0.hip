// Workgroup-tile kernels, lane-shift build XL = 0 (both shifts DPP).
#include "tb_tile_kern.hpp"

namespace heat::gpu::tbw {
bool tile_launch_x0(const TbArgs& args, int depth, int rows, int waves, hipStream_t st) {
  return tile_launch_unit<0>(args, depth, rows, waves, st);
}
int tile_occupancy_x0(int rows, int waves) { return tile_occupancy_unit<0>(rows, waves); }
}  // namespace heat::gpu::tbw
