// Workgroup-tile temporally blocked kernel (tb_tile.hip), a header of its own
// so that tile changes rebuild only tb_tile.hip.
#pragma once

#include "tb_common.hpp"

namespace heat::gpu::tbw {  // workgroup tiles, rows of the tile in VGPRs (tb_tile.hip)
bool launch(const tbdetail::TbArgs& args, int depth, int rows, int waves, bool bpermute,
            hipStream_t st);
int occupancy(int rows, int waves, bool bpermute);  // resident blocks per CU (0: not built)
// The lane-shift builds (tb_tile_xl<XL>.hip, compiled in parallel).
bool tile_launch_x0(const tbdetail::TbArgs& args, int depth, int rows, int waves, hipStream_t st);
bool tile_launch_x1(const tbdetail::TbArgs& args, int depth, int rows, int waves, hipStream_t st);
bool tile_launch_x2(const tbdetail::TbArgs& args, int depth, int rows, int waves, hipStream_t st);
int tile_occupancy_x0(int rows, int waves);
int tile_occupancy_x1(int rows, int waves);
int tile_occupancy_x2(int rows, int waves);
// A kTile launch of tb_step (even depth): plans the tiles and launches.
// res_level: the step (1..depth) whose residual goes to resid (0 = depth).
void step(const float* src, float* dst, const StencilGeom& g, const Box* boxes, int nbox, int depth,
          unsigned* resid, int res_level, hipStream_t st, int variant, const TbTuning& tune);

// Issue estimate of one step of a tile launch (shape planning): the row
// updates of the busiest SIMD -- dispatch spreads workgroups over the CUs,
// `occ` at most per CU -- times the cycles per row-update op at that SIMD's
// wave count (2.7 with >= 4 waves, 3.1 with fewer: tools/probes/valu_rate.hip
// and the tile sweeps).  A CU with two tiles where others have one sets the
// pace of the launch (of the whole resident grid, through the neighbour
// waits): 468 tiles of 13 x 8 rows ran 10 % slower than 252 of 12 x 16 on a
// 1024 x 8192 block (profiles/r4_resident.md).
inline double tile_step_estimate(int64_t units, int cus, int occ, int rows, int waves) {
  const int64_t cap = int64_t(cus) * occ;
  const int64_t full = (units - 1) / cap;              // full dispatch rounds
  const int64_t last = units - full * cap;             // tiles of the last round
  const int64_t busiest = (last + cus - 1) / cus;      // tiles on its busiest CU
  auto cost = [&](int64_t tiles) {
    const double wps = double(tiles * waves) / 4.0;    // waves per SIMD
    return wps * rows * (wps >= 4.0 ? 2.7 : 3.1);
  };
  return double(full) * cost(occ) + cost(busiest);
}
}
