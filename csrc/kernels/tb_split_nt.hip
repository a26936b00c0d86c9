// Streaming build of the level-split pipelines (tb_split.hip): the input
// rows are loaded and the output rows stored non-temporally.  Taken by
// tb_step (kTbStreamRows) when one pass sweeps more field than the MALL
// holds (8192^2: +3 %, 131072^2: +2 %); fields that fit keep the plain
// build, whose stores the next pass re-reads from the MALL
// (profiles/r5_stores.md).
#include "tb_common.hpp"

#define HEAT_TB_NS tbxn
#define HEAT_TB_PACKED 0
#define HEAT_TB_SPLIT 1
#define HEAT_TB_BPERMUTE 1
#define HEAT_TB_SPLIT_ONLY 1
#define HEAT_TB_NTSTORE 1
#define HEAT_TB_NTLOAD 1
#include "tb_stream.inl"
