// The packed-update build of the single-wave temporally blocked kernel
// (variants without kScalar): an experiment build (tb_exp.hpp), round 1's
// scalar selection (tb_scalar.hip, -fno-slp-vectorize) is the default.
#include "tb_common.hpp"

#define HEAT_TB_NS tbp
#define HEAT_TB_PACKED 1
#include "tb_stream.inl"
