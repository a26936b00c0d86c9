// Scalar-update build of the temporally blocked kernel (compiled with
// -fno-slp-vectorize, see Makefile): lets the packed and scalar instruction
// selections of the row update be timed against each other in one process.
#include "tb_common.hpp"

#define HEAT_TB_NS tbs
#define HEAT_TB_PACKED 0
// Depth 12 (ring-3 + ramp only): 2/3 the HBM bytes per update of depth 8,
// at 2 waves/SIMD; see tb_depth_supported().
#define HEAT_TB_DEEP 1
#include "tb_stream.inl"
