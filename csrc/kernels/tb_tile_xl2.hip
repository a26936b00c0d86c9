// Workgroup-tile kernels, lane-shift build XL = 2 (mixed: DPP left, ds_bpermute right).
#include "tb_tile_kern.hpp"

namespace heat::gpu::tbw {
bool tile_launch_x2(const TbArgs& args, int depth, int rows, int waves, hipStream_t st) {
  return tile_launch_unit<2>(args, depth, rows, waves, st);
}
int tile_occupancy_x2(int rows, int waves) { return tile_occupancy_unit<2>(rows, waves); }
}  // namespace heat::gpu::tbw
