// Level-split build with mixed lane shifts (variant bit kShiftMixed): as
// tb_split.hip, but only the east neighbour crosses lanes through the LDS
// crossbar (ds_bpermute, issued up front); the west neighbour is a DPP wave
// shift folded into the e + w add.  Half the LDS-pipe issue of the
// all-ds_bpermute default, at one DPP operand per row update (the mixed form
// the workgroup-tile kernel uses, profiles/r3_tile.md).
#include "tb_common.hpp"

#define HEAT_TB_NS tbxm
#define HEAT_TB_PACKED 0
#define HEAT_TB_SPLIT 1
#define HEAT_TB_BPERMUTE 2
#define HEAT_TB_SPLIT_ONLY 1
#include "tb_stream.inl"
