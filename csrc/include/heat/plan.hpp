// Resident-aware planning of the deep-halo depth (host side, no GPU code):
// which passes-per-exchange m keeps every rank's resident span box inside a
// one-dispatch-round resident tile plan of the same shape as its owned
// block's.  Separate from topology.hpp so the kernel units, which include
// that header, do not depend on it.
#pragma once

#include <functional>

#include "heat/topology.hpp"

namespace heat {

// The first box of a resident span after an exchange of H = m * depth deep
// halos: rank b's owned block grown by H - depth rows (columns: rounded down
// to 4) on every side with a neighbour along a decomposed axis, as
// Solver::resident_span tracks ghost validity.
Box span_box(const Cart& cart, const Block& b, int depth, int m);

// A resident tile plan's shape as one int: rows per wave << 8 | waves per
// workgroup (0: the box has no one-round resident plan).
constexpr int res_shape(int rows, int waves) { return rows << 8 | waves; }

// The fewest passes per exchange worth a resident span: a span pays one
// whole-tile load and store, shorter spans lose to m = 8 streaming passes
// (4 x 1 slabs of 8192^2 fit only at m = 2: 4.18 Tcells/s on the 2072-row
// box against the split pipelines' 4.08 on 2216 rows, even once the 4x
// exchanges are paid; profiles/r6_resident_protocol.md).
constexpr int kResMinPasses = 4;

// Resident-aware halo depth (passes per exchange): the largest m in
// [2, mmax] whose H = m * depth fits every rank's extent along the
// decomposed axes and for which every rank's first span box has a one-round
// resident plan of the SAME shape as its owned block's (`shape`); 0 when the
// owned blocks have none or no m >= 2 keeps it.  Large m trades redundant
// ghost compute for fewer exchanges, but a box past its block's plan falls
// to another shape or to the per-pass kernels (round-6 sweeps, one MI355X,
// rank boxes at m-pass spans, per owned cell):
//   8192^2 on 8 x 1: m = 7 (1168 rows, 12 x 16 tiles) 3.72 Tcells/s, m = 8
//     (1192 rows, 14 x 8 two per CU) 3.40;  4 x 2: m = 7 3.88, m = 8 3.36;
//   8192^2 on 2 x 2: m = 5 (4144^2, 20 x 16) 4.73, m = 8 (4180^2, split
//     pipelines) 3.79.
int resident_halo_passes(const Cart& cart, int64_t nx, int64_t ny, int depth, int mmax,
                         const std::function<int(const Box&)>& shape);

// Host-side resident plan of a box at `depth` on an MI355X (`cus` CUs): the
// tile planner's shapes and choice (tb_resident.hip plan_res: the lowest
// tile_step_estimate among the shapes whose tiles are all co-resident) with
// the co-resident workgroups per CU the occupancy API reports for gfx950
// (also RES_SHAPES of parallel/model.py).  `heat --plan` uses it without a
// GPU; the solver asks the device (gpu::tb_resident_shape).
int resident_shape_static(const Box& box, int depth, int cus = 256);

namespace gpu {
// The device planner's shape for a resident launch over `box` (0: none);
// tb_resident.hip.
int tb_resident_shape(const Box& box, int depth, int variant = -1);
}  // namespace gpu

}  // namespace heat
