// libheat_exp.so's registration of the experiment kernels (tb_exp.hpp) with
// the product library it links against: runs when the library is loaded,
// and again through heat_exp_register() (after an unregistration, e.g. a
// test module that needed them ended).
#include "tb_exp.hpp"

namespace {
const heat::gpu::TbExpKernels* table() {
  using namespace heat::gpu;
  static const TbExpKernels k{&tbp::launch,          &tbp::occupancy,
                              &tbn::launch,          &tbn::occupancy,
                              &tbxm::launch_split,   &tbxm::occupancy_split,
                              &tbxnp::launch_split,  &tbc::occupancy_chain,
                              &tbc::launch_chain};
  return &k;
}
struct Register {
  Register() { heat_register_exp_kernels(table()); }
} reg;
}  // namespace

extern "C" void heat_exp_register(void) { heat_register_exp_kernels(table()); }
