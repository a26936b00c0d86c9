// Resident-aware planning of the deep-halo depth (host side, no GPU code):
// which passes-per-exchange m keeps every rank's resident span box inside a
// one-dispatch-round resident tile plan.  Separate from topology.hpp so the
// kernel units, which include that header, do not depend on it.
#pragma once

#include <functional>

#include "heat/topology.hpp"

namespace heat {

// The first box of a resident span after an exchange of H = m * depth deep
// halos: rank b's owned block grown by H - depth rows (columns: rounded down
// to 4) on every side with a neighbour along a decomposed axis, as
// Solver::resident_span tracks ghost validity.
Box span_box(const Cart& cart, const Block& b, int depth, int m);

// Resident-aware halo depth (passes per exchange): the largest m in
// [2, mmax] whose H = m * depth fits every rank's extent along the decomposed
// axes and for which every rank's first span box passes `fits`; 0 when the
// owned blocks themselves do not fit or no m >= 2 does.  Large m trades
// redundant ghost compute for fewer exchanges, but a box that no longer has a
// one-round resident plan runs the per-pass kernels: 8192^2 on a 2 x 2 grid
// at m = 8 (4180-cell boxes) ran the split pipelines at 3.9 Tcells/s per
// rank, m = 5 (4144) fits 20 x 16 tiles at ~5.3.
// The fewest passes per exchange worth a resident span (see Solver's m
// choice): shorter spans fall back to m = 8 streaming passes.
constexpr int kResMinPasses = 4;

int resident_halo_passes(const Cart& cart, int64_t nx, int64_t ny, int depth, int mmax,
                         const std::function<bool(const Box&)>& fits);

// Host-side resident fit of a box at `depth` on an MI355X (`cus` CUs): the
// tile planner's shapes (tb_resident.hip plan_res) with their co-resident
// workgroups per CU as the occupancy API reports them for gfx950 (also the
// RES_SHAPES of parallel/model.py).  `heat --plan` uses it without a GPU;
// the solver asks the device (gpu::tb_resident_fits).
bool resident_fits_static(const Box& box, int depth, int cus = 256);

}  // namespace heat
