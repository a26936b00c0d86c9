// The experiment kernels: TB builds that measured slower than the defaults
// and are kept for A/Bs and their bitwise tests, built by `make exp` into
// parallel_heat_amd/_lib/libheat_exp.so instead of the product library
// (libheat.so).  Loading libheat_exp.so (Python: HEAT_EXP=1 or
// _native.load_exp(); the CLI: HEAT_EXP=1) registers them here; a launch that
// asks for one without it fails with a message saying so.
//
//   tbp    packed-f32 row update, single-wave pipelines (tb_packed.hip):
//          variants without kScalar
//   tbn    float2 lanes, 128-column strips (tb_narrow.hip): kFloat2
//   tbxm   level-split, mixed DPP / ds_bpermute shifts (tb_split_mixed.hip):
//          kShiftMixed, -0.5 % (profiles/r4_8192_ab.md)
//   tbxnp  level-split streaming rows, packed f32 (tb_split_pk.hip):
//          HEAT_TB_SPLIT_PK=1, 3.67 vs 5.13 Tcells/s (spills 224 B/lane;
//          profiles/r6_split_packed.md)
//   tbc    chained level-split passes (tb_chain.hip): HEAT_TB_CHAIN=1,
//          3.75 vs 5.24 Tcells/s (profiles/r5_chain.md)
#pragma once

#include "tb_common.hpp"

namespace heat::gpu {

struct TbExpKernels {
  bool (*tbp_launch)(const tbdetail::TbArgs&, int depth, int lag, hipStream_t st);
  int (*tbp_occupancy)(int depth, int lag);
  bool (*tbn_launch)(const tbdetail::TbArgs&, int depth, int lag, hipStream_t st);
  int (*tbn_occupancy)(int depth, int lag);
  bool (*tbxm_launch_split)(const tbdetail::TbArgs&, int depth, hipStream_t st);
  int (*tbxm_occupancy_split)(int depth);
  bool (*tbxnp_launch_split)(const tbdetail::TbArgs&, int depth, hipStream_t st);
  int (*tbc_occupancy_chain)(int depth);
  bool (*tbc_launch_chain)(const tbdetail::TbArgs&, int depth, int passes, unsigned* flags,
                           unsigned* done, unsigned* err, hipStream_t st);
};

// The registered table; throws (naming `what`) when libheat_exp.so is not loaded.
const TbExpKernels& tb_exp(const char* what);
bool tb_exp_loaded();

namespace tbxnp {  // packed-f32 streaming level-split pipelines (tb_split_pk.hip)
bool launch_split(const tbdetail::TbArgs& args, int depth, hipStream_t st);
}

}  // namespace heat::gpu

extern "C" void heat_register_exp_kernels(const heat::gpu::TbExpKernels* k);
