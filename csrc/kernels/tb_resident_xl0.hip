// Resident workgroup tiles, lane-shift build XL = 0 (both shifts DPP).
#include "tb_resident_kern.hpp"

namespace heat::gpu::tbw {
bool res_launch_x0(const ResArgs& ra, int rows, int waves, int blocks, hipStream_t st) {
  return res_launch_unit<0>(ra, rows, waves, blocks, st);
}
int res_occupancy_x0(int rows, int waves) { return res_occupancy_unit<0>(rows, waves); }
}  // namespace heat::gpu::tbw
