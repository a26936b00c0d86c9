// Chained level-split passes: one launch runs several depth-12 passes of
// the streaming pipelines (tb_split_nt.hip's rows: non-temporal loads;
// write-through sc1 stores) with per-unit flags instead of a grid-wide
// boundary between passes.  See tb_chain_kernel in tb_stream.inl.
#include "tb_common.hpp"

#define HEAT_TB_NS tbc
#define HEAT_TB_PACKED 0
#define HEAT_TB_SPLIT 1
#define HEAT_TB_BPERMUTE 1
#define HEAT_TB_SPLIT_ONLY 1
#define HEAT_TB_NTLOAD 1
#define HEAT_TB_CHAIN 1
#include "tb_stream.inl"
