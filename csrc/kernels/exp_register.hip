// libheat_exp.so's registration of the experiment kernels (tb_exp.hpp) with
// the product library it links against: runs when the library is loaded.
#include "tb_exp.hpp"

namespace {
struct Register {
  Register() {
    using namespace heat::gpu;
    static const TbExpKernels k{&tbp::launch,          &tbp::occupancy,
                                &tbn::launch,          &tbn::occupancy,
                                &tbxm::launch_split,   &tbxm::occupancy_split,
                                &tbxnp::launch_split,  &tbc::occupancy_chain,
                                &tbc::launch_chain};
    heat_register_exp_kernels(&k);
  }
} reg;
}  // namespace
