// Workgroup-tile kernels, lane-shift build XL = 1 (both ds_bpermute).
#include "tb_tile_kern.hpp"

namespace heat::gpu::tbw {
bool tile_launch_x1(const TbArgs& args, int depth, int rows, int waves, hipStream_t st) {
  return tile_launch_unit<1>(args, depth, rows, waves, st);
}
int tile_occupancy_x1(int rows, int waves) { return tile_occupancy_unit<1>(rows, waves); }
}  // namespace heat::gpu::tbw
