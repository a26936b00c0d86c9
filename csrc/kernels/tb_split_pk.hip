// Packed-f32 build of the streaming level-split pipelines (tb_split_nt.hip
// with HEAT_TB_PACKED 1): the row update as v_pk_add_f32 / v_pk_fma_f32 on
// the element pairs (x,y), (z,w) -- the same per-element operations in the
// same order as heat::stencil, bitwise equal -- 15.9 instead of 24 VALU per
// float4 row update in one 6-level stage (tools/probes/stencil_chain.hip,
// VAR 36).  The round-6 A/B of the 1-GPU 8192^2 pass (HEAT_TB_SPLIT_PK=1).
#include "tb_common.hpp"

#define HEAT_TB_NS tbxnp
#define HEAT_TB_PACKED 1
#define HEAT_TB_SPLIT 1
#define HEAT_TB_BPERMUTE 1
#define HEAT_TB_SPLIT_ONLY 1
#define HEAT_TB_NTSTORE 1
#define HEAT_TB_NTLOAD 1
#include "tb_stream.inl"
