// Inner-level residual kernels of the level-split build (depth 12, residual
// levels 5..8): a convergence check that falls inside a full-depth pass takes
// its residual at that level instead of cutting the pass (tb_stream.inl,
// TbStream RS; solver plan_passes).  One unit per range of levels so the
// instantiations compile in parallel; same flags as tb_split.hip.
#include "tb_common.hpp"

#define HEAT_TB_NS tbx
#define HEAT_TB_PACKED 0
#define HEAT_TB_SPLIT 1
#define HEAT_TB_BPERMUTE 1
// Streaming rows (non-temporal loads / stores, as tb_split_nt.hip): checked
// runs every 20 steps +0.8 % at 8192^2, +0.5 % on the 2-GPU plate
// (profiles/r5_stores.md).
#define HEAT_TB_NTSTORE 1
#define HEAT_TB_NTLOAD 1
#define HEAT_TB_SPLIT_RL_LO 5
#define HEAT_TB_SPLIT_RL_HI 8
#define HEAT_TB_SPLIT_RL_FN launch_split_rl_b
#include "tb_stream.inl"
