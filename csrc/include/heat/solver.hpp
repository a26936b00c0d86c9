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
//   * A "pass" advances k steps with one temporally blocked launch (k = tb
//     depth).  Ghosts are H = m*k deep: one exchange (RCCL, grouped) feeds m
//     passes, each of which also recomputes the still-valid part of the ghost
//     ring (communication avoiding: one exchange per m*k steps instead of one
//     per step as in the reference).
//   * Alternative schedules (Params::schedule) overlap the exchange with the
//     interior box on a high-priority comm stream: exchange-first or
//     boundary-first.  Measured slower on MI355X at the strong-scaling shapes
//     (see params.hpp), kept selectable and tested.
//   * Segments between convergence checks are captured once into a hipGraph
//     per (length, parity, ghost state) and replayed; with a host-memory
//     transport (ranks sharing a GPU) the exchange is a host node.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "heat/common.hpp"
#include "heat/io.hpp"
#include "heat/kernels.hpp"
#include "heat/params.hpp"
#include "heat/topology.hpp"
#include "heat/transport.hpp"

namespace heat {

// A run-time error every rank meets at the same point, decided from
// all-reduced or global quantities (a non-finite all-reduced residual): after
// it a rank's queued exchanges were all matched, so the communicator may be
// kept (Solver::run_guarded's "[clean]").  Any other error aborts it.
struct GlobalError : Error {
  using Error::Error;
};

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
  // Per-phase time (Params::phase_timing; device event time on the GPU,
  // summed over launches, so concurrent phases may add up to > seconds).
  double t_exchange = 0.0, t_compute = 0.0, t_reduce = 0.0;
  int64_t resident_passes = 0;  // passes run inside resident-tile launches
  int64_t chained_passes = 0;   // passes run inside chained level-split launches
  // 1: a resident launch of this call gave up a neighbour wait (results
  // invalid; only returned with HEAT_TB_RES_GIVEUP=defer, else run throws).
  int64_t resident_giveups = 0;
};

class Solver {
 public:
  // The transport may be shared by several solvers in turn (one RCCL
  // communicator for all the autotune candidates of a run).
  Solver(const Params& p, std::shared_ptr<Transport> tr);
  ~Solver();
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  // Advance up to `steps` steps.  In converge mode, checks follow the
  // canonical/compat schedule and the call stops at the first converged check.
  // A multi-rank run that throws aborts this rank's communicator first: its
  // queued collectives would otherwise wait for peers forever (and the
  // destructor's device syncs with them).
  RunStats run(int64_t steps);
  // Asynchronous run: enqueues the steps and returns (steps_done set, no
  // timing); the next run() -- run(0) to just complete -- waits for every
  // enqueued step, checks the resident error word and the transport, and
  // reports a give-up.  Back-to-back enqueues keep the device busy across
  // calls (bench.py's timed loop).  Runs that must sync (device-gated
  // checks, phase timing, host-staged exchanges) are synchronous anyway.
  RunStats enqueue(int64_t steps);
  // Seconds per grouped halo exchange of `depth` rows/columns (device time
  // over `iters` back-to-back exchanges, this rank); *max_bytes: the largest
  // message.  Collective.  Feeds the autotune's exchange model.
  double time_exchange(int depth, int iters, int64_t* max_bytes);
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
  Schedule schedule() const { return sched_; }
  int tb_depth() const { return T_; }
  // Default TB depth when neither Params nor HEAT_TB_DEPTH sets one.
  int auto_tb_depth() const;
  bool on_gpu() const { return P_.backend == Backend::Hip; }
  // The temporally blocked kernel runs the passes (else k single-step launches).
  bool tb_kernel() const {
    return on_gpu() && (P_.kernel == KernelKind::Auto || P_.kernel == KernelKind::TB);
  }

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
  // Gives up: aborts the transport (ncclCommAbort) so that this rank and its
  // peers stop waiting on each other; a wait of this solver in progress (on
  // another thread) throws, and the solver is unusable afterwards.  Used by
  // a failing rank of a single-process group and by the watchdog.
  void abort();
  // Device pointer (GPU) or host pointer (CPU) of owned cell (0,0) of the
  // buffer holding the current state.
  float* current() { return field_[cur_]; }

 private:
  // One pass of a segment: k steps; rl in 1..k: a check after the pass's
  // rl-th step (its residual is taken at that level; rl = k: the pass ends at
  // the check), 0: no check.
  struct PassPlan {
    int k = 0;
    int rl = 0;
  };
  // What a gated run needs to restore the state of any check: the pass's
  // first step (relative to its segment in a GraphEntry) and the host state
  // before and after it.
  struct PassRec {
    int64_t step0 = 0;
    int k = 0, rl = 0;
    int cur0 = 0, cur1 = 0;
    int64_t gr1 = 0, gc1 = 0;
    // A pass of a resident span: its position in the span (span = passes
    // from the span's start through this one; cur0 = the span's source
    // buffer) and the span's box growth (er, ec), for replay_check.
    int span = 1;
    int64_t er = 0, ec = 0;
  };
  void alloc();
  void free_all();
  void init_fields();
  std::vector<int> pass_depths(int64_t n) const;
  // Every rank's depth-T launches are small enough for the workgroup-tile
  // kernel (even depths): remainder passes are then split into even parts.
  bool tile_sized() const;
  bool tile_sized_at(int depth) const;
  bool resident_sized() const;
  // Passes for steps [step0, step0+n), cut at every check point (the
  // residual is the last level of its pass).
  std::vector<PassPlan> plan_passes(int64_t step0, int64_t n) const;
  // A check may ride inside a depth-k pass (residual at an inner step).
  bool mid_residual_ok(int k) const;
  void enqueue_segment(const std::vector<PassPlan>& plan);
  void enqueue_pass(int k, int rl);
  // Resident tiles: passes [i, i + n) of the plan in ONE launch whose tiles
  // stay in VGPRs (gpu::tb_resident_step).  resident_span returns n (0: not
  // eligible): same depth, no exchange after the first pass, a check only in
  // the last pass (device-judged runs), and every tile of the first pass's
  // box co-resident.
  int resident_span(const std::vector<PassPlan>& plan, size_t i) const;
  int res_span_max_ = 0;  // HEAT_TB_RES_SPAN (diagnostics; 0: no cap)
  static int device_users(int dev);  // live GPU solvers of this process on dev
  void enqueue_resident(const std::vector<PassPlan>& plan, size_t i0, int n);
  // Chained passes (one-rank runs of the streaming level-split build): the
  // unchecked depth-T_ passes from plan[i] on, run as one launch; false if
  // tb_step's plan did not qualify (chained passes then stay off).
  int chain_span(const std::vector<PassPlan>& plan, size_t i) const;
  bool enqueue_chain(const std::vector<PassPlan>& plan, size_t i0, int n);
  RunStats run_impl(int64_t steps, bool wait);
  RunStats run_guarded(int64_t steps, bool wait);
  void complete_pending();  // run(0) if an enqueue()d run is in flight
  gpu::StencilGeom geom() const;
  void exchange(int buf, int k, hipStream_t st);
  // `st`: the stream to launch on (nullptr = the compute stream).
  void compute_gpu(int k, int rl, bool split, int part, int band = 0, int64_t er = 0,
                   int64_t ec = 0, hipStream_t st = nullptr);
  void compute_cpu(int k, int rl, int64_t er, int64_t ec);
  std::pair<int64_t, int64_t> ensure_ghosts(int k, hipStream_t st);
  float finish_resid();
  // Device waits of the run loop: plain syncs on one rank; with peers, a
  // polling wait with transport error checks and a no-progress timeout
  // (HEAT_WATCHDOG_S, default 300 s, 0 = none), see wait_event.
  void wait_event(hipEvent_t e);
  void sync_watch();
  bool is_check_point(int64_t completed) const;
  int64_t next_check_after(int64_t step) const;
  bool converged_value(float r) const;
  // Device-gated convergence (GPU fields, device or single-rank transport):
  // checks are judged on the device and never block the host.
  // HEAT_HOST_CHECKS=1 forces the host-judged path (A/B diagnostics).
  bool gated() const { return on_gpu() && P_.converge && !staged_ && !host_checks_; }
  void run_segments(int64_t steps, RunStats& s);
  void run_gated(int64_t steps, RunStats& s);
  // State of a converging check that sits inside pass p: its first p.rl
  // steps again from the pass's source buffer.
  void replay_check(const PassRec& p);
  // Launch (capturing on first use) the graph or the eager enqueue of one
  // segment; returns its pass records and check steps relative to step_.
  void launch_segment(const std::vector<PassPlan>& plan, int64_t n, int64_t phase,
                      bool use_graph, std::vector<PassRec>* recs, std::vector<int64_t>* checks);

  void reduce_scalars(double* f64, int nf, uint64_t* u64, int nu, float* fmax, int nm);

  Params P_;
  std::shared_ptr<Transport> tr_;
  Cart cart_;
  Block blk_;
  Layout L_;
  int H_ = 1;  // ghost depth: m * T (m passes per exchange)
  int T_ = 1;  // pass depth (TB depth on the GPU)
  Schedule sched_ = Schedule::Sync;
  bool staged_ = false;  // GPU fields but host-memory transport
  bool host_checks_ = false;
  bool warmed_ = false;    // RCCL connections established outside capture
  bool resident_ = false;  // resident-tile launches enabled for this solver
  bool chain_ = false;     // chained level-split passes (HEAT_TB_CHAIN=1; off by default)
  bool resident_force_ = false;  // HEAT_TB_RESIDENT=2: also with ranks sharing the device
  bool resident_used_ = false;  // one was enqueued in this run (check its error word)
  bool pending_ = false;         // an enqueue()d run not yet completed by run()
  bool defer_giveup_ = false;   // HEAT_TB_RES_GIVEUP=defer: report a give-up, do not throw
  bool inject_giveup_ = false;  // HEAT_TEST_RES_GIVEUP_RANK: fake one give-up (tests)
  float* xbase_[2] = {nullptr, nullptr};  // their exchange fields
  unsigned* d_flags_ = nullptr;           // + per-tile flags and the error word
  unsigned* h_err_ = nullptr;             // pinned copy of the error word
  bool watch_ = false;     // multi-rank GPU run: waits poll with a watchdog
  double watchdog_s_ = 300.0;
  std::atomic<bool> aborted_{false};
  int64_t gr_ = 0, gc_ = 0;  // ghost rows/columns of field_[cur_] at the current level
  bool comm_pending_ = false;  // comm stream has unjoined work
  int cur_ = 0;
  int64_t step_ = 0;
  float cpu_resid_ = 0.f;
  int64_t stat_passes_ = 0, stat_exchanges_ = 0, stat_resident_ = 0, stat_chained_ = 0;

  float* base_[2] = {nullptr, nullptr};
  float* field_[2] = {nullptr, nullptr};
  // Contiguous E/W halo buffers (send W, send E, recv W, recv E).
  float* ew_[4] = {nullptr, nullptr, nullptr, nullptr};
  // Ghost-corner buffers of 2-D grids (send NW NE SW SE, recv NW NE SW SE).
  float* cn_[8] = {};
  // Host staging (staged_ mode), one pair per message of an exchange.
  static constexpr int kMaxMsgs = 8;
  static constexpr size_t kResidentFlagBytes = 16384;  // flags of up to 4096 resident tiles
  static constexpr size_t kResidSpanOffset = 64;      // words: a resident span's residual block
  static constexpr size_t kResidBytes =
      4 * (kResidSpanOffset + size_t(gpu::kTbResidentSlots) * gpu::kTbResidentMaxChecks);
  float* stage_send_[kMaxMsgs] = {};
  float* stage_recv_[kMaxMsgs] = {};
  size_t stage_bytes_ = 0;

  // GPU state.
  hipStream_t s_comp_ = nullptr, s_comm_ = nullptr;
  hipEvent_t ev_ready_ = nullptr, ev_halo_ = nullptr, ev_wait_ = nullptr;
  unsigned* d_resid_ = nullptr;
  float* h_resid_ = nullptr;
  void* d_scratch_ = nullptr;
  void* d_checksum_ = nullptr;
  struct GraphEntry {
    hipGraphExec_t exec = nullptr;
    int cur_after = 0;
    int64_t gr_after = 0, gc_after = 0;
    int64_t passes = 0, exchanges = 0;
    bool resident = false;         // holds a resident-tile launch (check its error word)
    int64_t resident_passes = 0;
    int64_t chained_passes = 0;
    std::vector<PassRec> recs;     // relative to the segment's first step
    std::vector<int64_t> checks;   // check steps (relative), in judge order
  };
  // Key: (steps, check phase or -1, cur, ghost rows, ghost cols).
  std::map<std::tuple<int64_t, int64_t, int, int64_t, int64_t>, GraphEntry> graphs_;
  bool capturing_ = false;
  std::atomic<bool> rccl_graphs_{false};  // a live graph captured RCCL calls (abort())
  // Gated runs: the device gate, two pinned host copies (one per segment
  // parity) and their events; the pass log of the segment being enqueued.
  void* d_gate_ = nullptr;
  void* h_gate_ = nullptr;
  hipEvent_t ev_seg_[2] = {nullptr, nullptr};
  std::vector<PassRec> pass_log_;
  std::vector<int64_t> check_log_;
  bool side_interior_ = false;  // the pass's interior ran on s_comm_ (pipeline under capture)

  // Host-staged exchanges captured into graphs (host nodes): the arguments
  // live as long as the graphs; an error on HIP's callback thread is stored
  // and raised by run() after the next synchronisation.
  struct StagedCall {
    Solver* self = nullptr;
    std::vector<Msg> msgs;
  };
  static void staged_host_fn(void* p);
  void check_staged();
  std::deque<StagedCall> staged_calls_;
  std::mutex staged_mu_;
  std::atomic<bool> staged_failed_{false};
  std::string staged_error_;

  // Phase timing (eager runs only).
  enum Phase { kExchange = 0, kCompute = 1, kReduce = 2 };
  struct Span {
    int phase;
    hipEvent_t a, b;
    double ha, hb;
  };
  class PhaseScope {
   public:
    PhaseScope(Solver* s, int phase, hipStream_t st);
    ~PhaseScope();
   private:
    Solver* s_;
    hipStream_t st_;
    int idx_ = -1;
  };
  hipEvent_t pooled_event();
  void flush_spans();
  double phase_acc_[3] = {0, 0, 0};
  int open_spans_ = 0;
  std::vector<Span> spans_;
  std::vector<hipEvent_t> event_pool_;
  size_t pool_used_ = 0;
  bool timing_ = false;
};

}  // namespace heat
