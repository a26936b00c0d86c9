// Narrow-strip build of the temporally blocked kernel: float2 lanes, 128-column
// strips (scalar row update).  Small blocks (the per-rank slabs of a
// strong-scaled run) get twice the strips, hence twice the chunk length for
// the same number of resident waves, and the halved ring registers allow
// more waves per SIMD; the price is 2x the relative strip overlap.
#include "tb_common.hpp"

#define HEAT_TB_NS tbn
#define HEAT_TB_PACKED 0
#define HEAT_TB_V 2
#include "tb_stream.inl"
