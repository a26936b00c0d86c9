// Level-split build of the temporally blocked kernel: each (strip, chunk)
// is run by a two-wave pipeline (levels 1..K/2 and K/2+1..K, fed through an
// LDS ring), see tb_split_kernel in tb_stream.inl.  Scalar row update,
// ring-3 + ramp pipeline (the tuned tbs build), east/west lane shifts via
// ds_bpermute instead of DPP, depths 8 and 12.  The default at depth 12.
#include "tb_common.hpp"

#define HEAT_TB_NS tbx
#define HEAT_TB_PACKED 0
#define HEAT_TB_SPLIT 1
#define HEAT_TB_BPERMUTE 1
#include "tb_stream.inl"
