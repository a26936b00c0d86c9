// The per-rank solver: owns the two ping-pong fields of its block, the
// streams/events/graphs of the GPU path, and the halo-exchange schedule.
//
// Reference map:
//   ping-pong buffers            cuda/cuda_heat.cu:177-191, mpi/...c:46, :129, :264  (R22)
//   time loop                    cuda/cuda_heat.cu:204-237, mpi/...c:159-265          (R08, R16)
//   inner/outer overlap          mpi/...c:160-234 (Heat.pdf p.3 Fig. 2)               (PS4)
//   convergence check            cuda/cuda_heat.cu:219-236, mpi/...c:235-262          (R18)
//   gather + output              mpi/...c:270-299, cuda/cuda_heat.cu:242-251          (R19)
//
// MI355X-first execution model:
//   * A "pass" advances k steps: exchange a k-deep halo (RCCL, grouped), then
//     one temporally blocked kernel computes all k steps.  k = tb depth, so
//     there is one exchange per k steps (communication avoiding) instead of
//     one per step as in the reference.
//   * With overlap on, the interior box (whose dependency cone does not
//     reach the ghost ring) runs on the compute stream while the exchange
//     runs on the comm stream; the boundary boxes follow after an event join.
//   * Segments between convergence checks are captured once into a hipGraph
//     per (length, parity) and replayed.
#pragma once

#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <tuple>
#include <vector>

#include "heat/io.hpp"
#include "heat/params.hpp"
#include "heat/topology.hpp"
#include "heat/transport.hpp"

namespace heat {

struct RunStats {
  int64_t steps_done = 0;     // steps advanced by this call
  int64_t total_steps = 0;    // steps completed since initialisation
  bool converged = false;
  int64_t converged_at = -1;  // completed-step count of the converging check
  float last_resid = -1.0f;   // last max|delta| measured (-1 if none)
  double seconds = 0.0;       // synchronised wall time of the call
  int64_t passes = 0;
  int64_t exchanges = 0;
  int64_t checks = 0;
};

class Solver {
 public:
  Solver(const Params& p, std::unique_ptr<Transport> tr);
  ~Solver();
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  // Advance up to `steps` steps.  In converge mode, checks follow the
  // canonical/compat schedule and the call stops at the first converged check.
  RunStats run(int64_t steps);
  // Run the configured number of steps (Params::steps given at construction
  // by the caller; compat=mpi adds one).
  int64_t configured_steps(int64_t steps) const;

  const Params& params() const { return P_; }
  const Cart& cart() const { return cart_; }
  const Block& block() const { return blk_; }
  const Layout& layout() const { return L_; }
  Transport& transport() { return *tr_; }
  int64_t step() const { return step_; }
  int halo() const { return H_; }
  int tb_depth() const { return T_; }
  bool on_gpu() const { return P_.backend == Backend::Hip; }

  // Re-initialise both fields from the initial condition (step := 0).
  void reset();
  // Copy the current owned block to host memory (row pitch in floats).
  void copy_owned(float* host, int64_t host_pitch);
  // Overwrite the owned block (and mark ghosts stale) from host memory.
  void load_owned(const float* host, int64_t host_pitch, int64_t step);
  // Full grid on rank 0 (nx*ny row-major); empty vector on other ranks.
  std::vector<float> gather_root();
  // Inverse of gather_root: rank 0 holds the full nx*ny grid (`full`, ignored
  // elsewhere) and every rank receives its block (the reference's master
  // scatter, mpi/...c:100-127).  Collective.
  void scatter_root(const float* full, int64_t step);
  // Global order-independent checksum (identical on every rank).
  Checksum checksum();
  // Binary output / checkpoint of the current state (all ranks call).
  void write_bin(const std::string& path);
  void read_bin(const std::string& path);
  void synchronize();
  void barrier() { tr_->barrier(); }
  // Device pointer (GPU) or host pointer (CPU) of owned cell (0,0) of the
  // buffer holding the current state.
  float* current() { return field_[cur_]; }

 private:
  struct Plan;  // pass schedule of one segment
  void alloc();
  void free_all();
  void init_fields();
  std::vector<int> pass_depths(int64_t n) const;
  void enqueue_segment(int64_t n, bool resid);
  void enqueue_pass(int k, bool resid);
  void exchange(int buf, int k, hipStream_t st);
  void compute_gpu(int k, bool resid, bool split, int part);
  void compute_cpu(int k, bool resid);
  float finish_resid();
  bool is_check_point(int64_t completed) const;
  bool converged_value(float r) const;
  void reduce_scalars(double* f64, int nf, uint64_t* u64, int nu, float* fmax, int nm);

  Params P_;
  std::unique_ptr<Transport> tr_;
  Cart cart_;
  Block blk_;
  Layout L_;
  int H_ = 1;  // ghost depth (max pass depth)
  int T_ = 1;  // pass depth (TB depth on the GPU)
  bool staged_ = false;  // GPU fields but host-memory transport
  int cur_ = 0;
  int64_t step_ = 0;
  int64_t resid_pending_ = 0;
  float cpu_resid_ = 0.f;
  int64_t stat_passes_ = 0, stat_exchanges_ = 0;

  float* base_[2] = {nullptr, nullptr};
  float* field_[2] = {nullptr, nullptr};
  // Contiguous E/W halo buffers (send W, send E, recv W, recv E).
  float* ew_[4] = {nullptr, nullptr, nullptr, nullptr};
  // Host staging (staged_ mode).
  float* stage_send_[4] = {nullptr, nullptr, nullptr, nullptr};
  float* stage_recv_[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t stage_bytes_ = 0;

  // GPU state.
  hipStream_t s_comp_ = nullptr, s_comm_ = nullptr;
  hipEvent_t ev_ready_ = nullptr, ev_halo_ = nullptr, ev_t0_ = nullptr, ev_t1_ = nullptr;
  unsigned* d_resid_ = nullptr;
  float* h_resid_ = nullptr;
  void* d_scratch_ = nullptr;
  void* d_checksum_ = nullptr;
  struct GraphEntry {
    hipGraphExec_t exec = nullptr;
    int cur_after = 0;
    int64_t passes = 0, exchanges = 0;
  };
  std::map<std::tuple<int64_t, bool, int>, GraphEntry> graphs_;
  bool capturing_ = false;
};

}  // namespace heat
