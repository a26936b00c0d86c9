// Workgroup-tile temporally blocked kernel (tb_tile.hip), a header of its own
// so that tile changes rebuild only tb_tile.hip.
#pragma once

#include "tb_common.hpp"

namespace heat::gpu::tbw {  // workgroup tiles, rows of the tile in VGPRs (tb_tile.hip)
bool launch(const tbdetail::TbArgs& args, int depth, int rows, int waves, bool bpermute,
            hipStream_t st);
int occupancy(int rows, int waves, bool bpermute);  // resident blocks per CU (0: not built)
// A kTile launch of tb_step (even depth): plans the tiles and launches.
// res_level: the step (1..depth) whose residual goes to resid (0 = depth).
void step(const float* src, float* dst, const StencilGeom& g, const Box* boxes, int nbox, int depth,
          unsigned* resid, int res_level, hipStream_t st, int variant, const TbTuning& tune);
}
