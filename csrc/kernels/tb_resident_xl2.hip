// Resident workgroup tiles, lane-shift build XL = 2 (mixed: DPP left, ds_bpermute right).
#include "tb_resident_kern.hpp"

namespace heat::gpu::tbw {
bool res_launch_x2(const ResArgs& ra, int rows, int waves, int blocks, hipStream_t st) {
  return res_launch_unit<2>(ra, rows, waves, blocks, st);
}
int res_occupancy_x2(int rows, int waves) { return res_occupancy_unit<2>(rows, waves); }
}  // namespace heat::gpu::tbw
