// Scalar-update build of the temporally blocked kernel (compiled with
// -fno-slp-vectorize, see Makefile): lets the packed and scalar instruction
// selections of the row update be timed against each other in one process.
#include "tb_common.hpp"

#define HEAT_TB_NS tbs
#define HEAT_TB_PACKED 0
#include "tb_stream.inl"
