// Resident workgroup tiles, lane-shift build XL = 1 (both ds_bpermute).
#include "tb_resident_kern.hpp"

namespace heat::gpu::tbw {
bool res_launch_x1(const ResArgs& ra, int rows, int waves, int blocks, hipStream_t st) {
  return res_launch_unit<1>(ra, rows, waves, blocks, st);
}
int res_occupancy_x1(int rows, int waves) { return res_occupancy_unit<1>(rows, waves); }
}  // namespace heat::gpu::tbw
