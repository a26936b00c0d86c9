// Per-rank solver runtime (see solver.hpp for the design and reference map).
#include "heat/solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>

#include "heat/common.hpp"
#include "heat/cpu_backend.hpp"
#include "heat/kernels.hpp"
#include "heat/plan.hpp"
#include "heat/trace.hpp"

namespace heat {
namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int env_int(const char* name, int def) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : def;
}

// Host-side box <-> contiguous copies for the CPU backend's E/W halos.
void host_pack(const float* origin, int64_t pitch, const Box& b, float* buf) {
  for (int64_t r = b.r0; r < b.r1; ++r)
    std::memcpy(buf + (r - b.r0) * b.cols(), origin + r * pitch + b.c0, size_t(b.cols()) * 4);
}
void host_unpack(const float* buf, float* origin, int64_t pitch, const Box& b) {
  for (int64_t r = b.r0; r < b.r1; ++r)
    std::memcpy(origin + r * pitch + b.c0, buf + (r - b.r0) * b.cols(), size_t(b.cols()) * 4);
}

}  // namespace

namespace {
// Solvers of this process per GPU (resident launches need the device alone).
std::mutex g_dev_mu;
std::map<int, int> g_dev_users;
}  // namespace

int Solver::device_users(int dev) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto it = g_dev_users.find(dev);
  return it == g_dev_users.end() ? 0 : it->second;
}

Solver::Solver(const Params& p, std::shared_ptr<Transport> tr)
    : P_(p), tr_(maybe_inject_faults(std::move(tr))) {
  HEAT_CHECK(tr_ != nullptr, "no transport");
  HEAT_CHECK(P_.nx >= 1 && P_.ny >= 1, "grid %lldx%lld", (long long)P_.nx, (long long)P_.ny);
  HEAT_CHECK(P_.check_interval >= 1, "check interval %d", P_.check_interval);
  cart_ = Cart(tr_->world(), P_.decomp, P_.px, P_.py, P_.nx, P_.ny);
  blk_ = make_block(cart_, tr_->rank(), P_.nx, P_.ny);
  if (on_gpu()) {
    // The TB kernel evaluates the canonical fp32 expression only.
    if (P_.numerics != Numerics::Fp32) {
      HEAT_CHECK(P_.kernel != KernelKind::TB && P_.kernel != KernelKind::Mfma,
                 "--numerics %s needs the lds or naive kernel", numerics_name(P_.numerics));
      if (P_.kernel == KernelKind::Auto) P_.kernel = KernelKind::Lds;
    }
    if (!tb_kernel()) {
      T_ = P_.tb_depth > 0 ? P_.tb_depth : 1;
    } else {
      T_ = P_.tb_depth > 0 ? P_.tb_depth : env_int("HEAT_TB_DEPTH", 0);
      if (T_ == 0) T_ = auto_tb_depth();
      HEAT_CHECK(gpu::tb_depth_supported(T_) || (T_ % 2 == 0 && T_ <= 16 && tile_sized_at(T_)),
                 "TB depth %d not supported (1-8 and 12; even depths up to 16 on blocks small "
                 "enough for the workgroup-tile kernel)", T_);
    }
  } else {
    HEAT_CHECK(!tr_->device_memory(), "transport %s needs the GPU backend", tr_->name());
    T_ = P_.tb_depth > 0 ? P_.tb_depth : 1;
    cpu::set_threads(P_.threads);
  }
  // Every decision below is made from global quantities (the smallest block
  // of any rank), so all ranks take the same path and their exchanges match.
  const int world = tr_->world();
  int64_t min_lx = blk_.lx, min_ly = blk_.ly;
  for (int r = 0; r < cart_.world; ++r) {
    const Block b = make_block(cart_, r, P_.nx, P_.ny);
    min_lx = std::min(min_lx, b.lx);
    min_ly = std::min(min_ly, b.ly);
  }
  const int64_t min_ext = std::min(cart_.px > 1 ? min_lx : INT64_MAX, cart_.py > 1 ? min_ly : INT64_MAX);
  sched_ = P_.schedule == Schedule::Auto ? Schedule::Sync : P_.schedule;
  if (!tb_kernel() || world == 1 || !P_.overlap)
    sched_ = Schedule::Sync;
  staged_ = on_gpu() && !tr_->device_memory() && world > 1;
  // Resident tiles for the workgroup-tile shapes (small per-rank blocks):
  // even depths, the synchronous schedule, the automatic variant choice;
  // HEAT_TB_RESIDENT=0 restores one launch per pass.
  // The resident grid must own its device: never with ranks sharing one GPU
  // (loopback threads, or several processes per GPU as in the RCCL
  // rehearsal), where two resident grids could each hold CUs the other's
  // tiles wait for.  Multi-rank runs therefore need a device per rank in
  // sight (device count >= world) and no other solver of this process on
  // the device (resident_span).  HEAT_TB_RESIDENT=2 skips that check (tests
  // whose ranks' grids all fit the one GPU together), 0 disables.
  // The ranks that can share this node's GPUs are the local ones
  // (LOCAL_WORLD_SIZE under torchrun; the whole world otherwise), so a
  // multi-node run with a GPU per local rank still goes resident.
  int ndev = 0;
  if (on_gpu()) {
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    HIP_CHECK(hipSetDevice(P_.device >= 0 ? P_.device : 0));  // occupancy queries below
  }
  const int local_world = std::min(world, std::max(1, env_int("LOCAL_WORLD_SIZE", world)));
  const int res_env = env_int("HEAT_TB_RESIDENT", 1);
  resident_force_ = res_env == 2;
  // Diagnostics: at most this many passes per resident span (a one-GPU
  // plate timed at the span length of an m-pass exchange interval).
  res_span_max_ = env_int("HEAT_TB_RES_SPAN", 0);
  // The halo depth below follows resident fit from global quantities only
  // (every rank must pick the same m: its exchanges pair with its peers');
  // whether this rank's spans then run resident also needs its own device.
  const bool res_shape = on_gpu() && tb_kernel() && T_ >= 4 && T_ % 2 == 0 &&
                         sched_ == Schedule::Sync && !staged_ && gpu::tb_tuning().variant < 0 &&
                         res_env != 0;
  const bool res_ok = res_shape && (world == 1 || ndev >= local_world || resident_force_);
  // Ghost depth H = m*T: with the Sync schedule one exchange feeds m passes,
  // each computing the still-valid part of the ghost ring redundantly.
  int m = 1;
  if (sched_ == Schedule::Sync && world > 1) {
    // m = 8 (H = 64 rows at K = 8, 96 at K = 12): larger m trades a few
    // percent of redundant ghost compute for fewer exchanges, whose
    // latency dominates on small blocks (profiles/halo_passes_r1.md).
    // Unless set, m is resident-aware: when the owned blocks have a
    // one-round resident plan, the largest m <= 8 whose span boxes keep a
    // plan of the same tile shape (8192^2 on 2 x 2 ranks: m = 5, 4144-cell
    // boxes in 20 x 16 tiles, not m = 8 whose 4180-cell boxes ran the split
    // pipelines; on 8 ranks m = 7 keeps the 12 x 16 tiles, m = 8 fell to
    // 14 x 8 ones, -10 % per owned cell; resident_halo_passes, plan.hpp).
    // A span of m passes pays one whole-tile load and store (what a per-pass
    // tile launch pays every pass), so short spans lose their edge: below
    // kResMinPasses the split pipelines at m = 8 are kept.
    m = P_.halo_passes > 0 ? P_.halo_passes : (on_gpu() ? env_int("HEAT_HALO_PASSES", 0) : 1);
    if (m <= 0) {
      m = 8;
      if (res_shape) {
        const int rm = resident_halo_passes(cart_, P_.nx, P_.ny, T_, 8, [&](const Box& b) {
          return gpu::tb_resident_shape(b, T_);
        });
        if (rm >= kResMinPasses) m = rm;
      }
    }
    m = int(std::max<int64_t>(1, std::min<int64_t>(m, min_ext / T_)));
  }
  H_ = m * T_;
  // A rank must own at least H rows/columns along every decomposed axis so
  // that an H-deep halo comes from its direct neighbour only.
  HEAT_CHECK(cart_.px == 1 || blk_.lx >= H_, "block of %lld rows is thinner than halo depth %d",
             (long long)blk_.lx, H_);
  HEAT_CHECK(cart_.py == 1 || blk_.ly >= H_, "block of %lld cols is thinner than halo depth %d",
             (long long)blk_.ly, H_);
  // The boundary-first pipeline needs an interior box off H-deep bands.
  if (sched_ == Schedule::Pipeline &&
      !(min_lx > 2 * int64_t(H_) && round_down(min_ly - H_, 4) > round_up(H_, 4)))
    sched_ = Schedule::Sync;
  L_ = Layout::make(blk_.lx, blk_.ly, H_);
  // Blocks past the tile threshold whose resident grid still fits one
  // dispatch round (the 4-GPU blocks 2048 x 8192 / 4096 x 4096: 20 x 16
  // tiles) go resident too; other large blocks never allocate the exchange
  // fields (two more fields' worth of memory).
  resident_ = res_ok && (tile_sized() || resident_sized());
  // Chained level-split passes (tb_chain.hip, HEAT_TB_CHAIN=1; off by
  // default): one-rank GPU runs of the streaming depth-12 pipelines (large
  // blocks that do not go resident).  Bitwise equal, but 8192^2 ran 3.75 vs
  // 5.24 Tcells/s: the write-through stores the cross-XCD hand-off needs
  // cost ~21 %, and passes that drift apart lose the L2 sharing of the
  // synchronous launches (profiles/r5_chain.md).  Like resident tiles the
  // chained grid must own its device.
  chain_ = on_gpu() && world == 1 && !resident_ && T_ == gpu::kTbDeepDepth && tb_kernel() &&
           sched_ == Schedule::Sync && !staged_ && gpu::tb_tuning().variant < 0 &&
           env_int("HEAT_TB_CHAIN", 0) != 0;
  if (env_int("HEAT_TB_TRACE", 0) != 0)
    std::fprintf(stderr, "[heat solver] rank %d T %d resident %d chain %d sched %d staged %d world %d\n",
                 tr_->rank(), T_, int(resident_), int(chain_), int(sched_), int(staged_), world);
  if (const char* e = std::getenv("HEAT_TB_RES_GIVEUP"); e && std::strcmp(e, "defer") == 0)
    defer_giveup_ = true;
  // Tests: this rank's first run with resident spans reports a give-up.
  inject_giveup_ = resident_ && env_int("HEAT_TEST_RES_GIVEUP_RANK", -1) == tr_->rank();
  host_checks_ = env_int("HEAT_HOST_CHECKS", 0) != 0;
  timing_ = P_.phase_timing || env_int("HEAT_PHASE_TIMING", 0) != 0;
  // Waits on the device poll the transport and give up after this long
  // without completion (multi-rank GPU runs; wait_event).
  watch_ = on_gpu() && world > 1;
  if (const char* w = std::getenv("HEAT_WATCHDOG_S"); w && *w) watchdog_s_ = std::atof(w);
  try {
    alloc();
    init_fields();
  } catch (...) {
    free_all();  // the destructor does not run for a throwing constructor
    throw;
  }
  if (on_gpu()) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    ++g_dev_users[P_.device >= 0 ? P_.device : 0];
  }
}

Solver::~Solver() {
  if (on_gpu()) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    --g_dev_users[P_.device >= 0 ? P_.device : 0];
  }
  free_all();
}

void Solver::alloc() {
  const size_t ew_elems = size_t(blk_.lx) * size_t(H_);
  if (on_gpu()) {
    const int dev = P_.device >= 0 ? P_.device : 0;
    HIP_CHECK(hipSetDevice(dev));
    for (int i = 0; i < 2; ++i) {
      HIP_CHECK(hipMalloc(&base_[i], size_t(L_.bytes())));
      field_[i] = base_[i] + L_.origin();
    }
    if (cart_.py > 1)
      for (auto& b : ew_) HIP_CHECK(hipMalloc(&b, ew_elems * 4));
    if (cart_.px > 1 && cart_.py > 1)
      for (auto& b : cn_) HIP_CHECK(hipMalloc(&b, size_t(H_) * size_t(H_) * 4));
    HIP_CHECK(hipStreamCreateWithFlags(&s_comp_, hipStreamNonBlocking));
    {
      // The comm stream gets the highest priority so RCCL's kernels are
      // dispatched ahead of queued stencil workgroups.
      int least = 0, greatest = 0;
      HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIP_CHECK(hipStreamCreateWithPriority(&s_comm_, hipStreamNonBlocking, greatest));
    }
    HIP_CHECK(hipEventCreateWithFlags(&ev_ready_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_halo_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_wait_, hipEventDisableTiming));
    // Word 0: a pass's residual; from kResidSpanOffset: the residual block of
    // a resident span's checks (slots x checks words).
    HIP_CHECK(hipMalloc(&d_resid_, kResidBytes));
    HIP_CHECK(hipMemset(d_resid_, 0, kResidBytes));
    HIP_CHECK(hipHostMalloc(&h_resid_, 256));
    HIP_CHECK(hipMalloc(&d_scratch_, 4096));
    HIP_CHECK(hipMalloc(&d_checksum_, 256));
    if (resident_ || chain_) {
      if (resident_)
        for (auto& b : xbase_) HIP_CHECK(hipMalloc(&b, size_t(L_.bytes())));
      // Flags, then the error word and the completion counter: zeroed once
      // here, then by the last tile of every launch (tb_resident.hip).
      HIP_CHECK(hipMalloc(&d_flags_, kResidentFlagBytes + 256));
      HIP_CHECK(hipMemset(d_flags_, 0, kResidentFlagBytes + 256));
      HIP_CHECK(hipHostMalloc(&h_err_, 256));
      *h_err_ = 0;
    }
    HIP_CHECK(hipMalloc(&d_gate_, sizeof(gpu::DeviceGate)));
    HIP_CHECK(hipMemset(d_gate_, 0, sizeof(gpu::DeviceGate)));
    HIP_CHECK(hipHostMalloc(&h_gate_, 2 * sizeof(gpu::DeviceGate)));
    std::memset(h_gate_, 0, 2 * sizeof(gpu::DeviceGate));
    for (auto& e : ev_seg_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (staged_) {
      stage_bytes_ = std::max<size_t>(size_t(H_) * size_t(L_.pitch), ew_elems) * 4;
      for (int i = 0; i < kMaxMsgs; ++i) {
        HIP_CHECK(hipHostMalloc(&stage_send_[i], stage_bytes_));
        HIP_CHECK(hipHostMalloc(&stage_recv_[i], stage_bytes_));
      }
    }
  } else {
    for (int i = 0; i < 2; ++i) {
      base_[i] = static_cast<float*>(std::aligned_alloc(256, size_t(round_up(L_.bytes(), 256))));
      HEAT_CHECK(base_[i] != nullptr, "host allocation of %lld bytes failed",
                 (long long)L_.bytes());
      field_[i] = base_[i] + L_.origin();
    }
    if (cart_.py > 1)
      for (auto& b : ew_) {
        b = static_cast<float*>(std::malloc(ew_elems * 4));
        HEAT_CHECK(b != nullptr, "host allocation failed");
      }
    if (cart_.px > 1 && cart_.py > 1)
      for (auto& b : cn_) {
        b = static_cast<float*>(std::malloc(size_t(H_) * size_t(H_) * 4));
        HEAT_CHECK(b != nullptr, "host allocation failed");
      }
  }
}

void Solver::free_all() {
  if (on_gpu() && aborted_) {
    // The transport was aborted with work still queued that may never
    // complete (it waits for a dead peer): leave the device memory and
    // streams to process teardown rather than block here.
    return;
  }
  if (on_gpu()) {
    if (s_comp_) (void)hipStreamSynchronize(s_comp_);
    if (s_comm_) (void)hipStreamSynchronize(s_comm_);
    for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second.exec);
    graphs_.clear();
    staged_calls_.clear();
    for (auto& b : base_)
      if (b) (void)hipFree(b);
    for (auto& b : ew_)
      if (b) (void)hipFree(b);
    for (auto& b : cn_)
      if (b) (void)hipFree(b);
    for (int i = 0; i < kMaxMsgs; ++i) {
      if (stage_send_[i]) (void)hipHostFree(stage_send_[i]);
      if (stage_recv_[i]) (void)hipHostFree(stage_recv_[i]);
    }
    if (d_resid_) (void)hipFree(d_resid_);
    if (h_resid_) (void)hipHostFree(h_resid_);
    if (d_scratch_) (void)hipFree(d_scratch_);
    if (d_checksum_) (void)hipFree(d_checksum_);
    if (d_gate_) (void)hipFree(d_gate_);
    for (auto& b : xbase_)
      if (b) (void)hipFree(b);
    if (d_flags_) (void)hipFree(d_flags_);
    if (h_err_) (void)hipHostFree(h_err_);
    if (h_gate_) (void)hipHostFree(h_gate_);
    for (auto e : {ev_ready_, ev_halo_, ev_wait_, ev_seg_[0], ev_seg_[1]})
      if (e) (void)hipEventDestroy(e);
    for (auto e : event_pool_) (void)hipEventDestroy(e);
    event_pool_.clear();
    if (s_comp_) (void)hipStreamDestroy(s_comp_);
    if (s_comm_) (void)hipStreamDestroy(s_comm_);
  } else {
    for (auto& b : base_) std::free(b);
    for (auto& b : ew_) std::free(b);
    for (auto& b : cn_) std::free(b);
  }
  for (auto& b : base_) b = nullptr;
  for (auto& b : ew_) b = nullptr;
  for (auto& b : cn_) b = nullptr;
  for (int i = 0; i < kMaxMsgs; ++i) stage_send_[i] = stage_recv_[i] = nullptr;
  d_resid_ = nullptr;
  h_resid_ = nullptr;
  d_scratch_ = d_checksum_ = nullptr;
  d_gate_ = h_gate_ = nullptr;
  xbase_[0] = xbase_[1] = nullptr;
  d_flags_ = nullptr;
  h_err_ = nullptr;
  ev_ready_ = ev_halo_ = ev_wait_ = ev_seg_[0] = ev_seg_[1] = nullptr;
  s_comp_ = s_comm_ = nullptr;
}

void Solver::init_fields() {
  TraceRange trace("heat.init");
  const int mode = int(P_.init);
  for (int i = 0; i < 2; ++i) {
    if (on_gpu())
      gpu::init_field(field_[i], L_, blk_.ox, blk_.oy, P_.nx, P_.ny, mode, P_.seed, s_comp_);
    else
      cpu::init_field(field_[i], L_, blk_.ox, blk_.oy, P_.nx, P_.ny, mode, P_.seed);
  }
  if (on_gpu()) HIP_CHECK(hipStreamSynchronize(s_comp_));
  cur_ = 0;
  step_ = 0;
  gr_ = gc_ = 0;
}

void Solver::reset() {
  complete_pending();
  init_fields();
}

int64_t Solver::configured_steps(int64_t steps) const {
  return P_.compat == Compat::Mpi ? steps + 1 : steps;
}

int Solver::auto_tb_depth() const {
  // Depth 12 (2/3 the HBM bytes per update of 8) wins on every per-rank
  // block of an 8192^2 run on 1-8 GPUs once the variant follows the work
  // size (tb_auto_variant: level-split pipelines on large launches, one wave
  // per chunk on small ones): +8 % at 1024 x 8192, +12 % at 2048 x 4096 over
  // the depth-8 / always-split choice of round 1
  // (profiles/tb_block_shapes_r2.md).  Thin blocks keep depth 8 (halo
  // depth, ramp).  Decided from the smallest block of any rank, so every
  // rank picks the same depth.
  if (!gpu::tb_variant_deep(gpu::tb_default_variant(gpu::kTbDeepDepth))) return 8;
  int64_t min_lx = INT64_MAX;
  for (int r = 0; r < cart_.world; ++r) min_lx = std::min(min_lx, make_block(cart_, r, P_.nx, P_.ny).lx);
  const int base = min_lx >= 1024 ? gpu::kTbDeepDepth : 8;
  // Convergence checks on tile-sized blocks: resident spans take a check at
  // any even level of a depth-12 pass (tb_resident_kern.hpp, ACC_MODE 3), so
  // an even interval (20, 50, ...) keeps depth 12 and its spans; round 4
  // forced depth 10 there (checks at pass ends only), -5.6 % per pass on
  // 1024 x 8192.  Odd intervals put every other check at an odd level: a
  // depth dividing the interval keeps those at pass ends.
  if (P_.converge && P_.compat != Compat::Cuda && P_.check_interval % 2 != 0 &&
      P_.check_interval % base != 0 && env_int("HEAT_TB_RESIDENT", 1) != 0) {
    for (int d : {10, 8})
      if (P_.check_interval % d == 0 && tile_sized_at(d)) return d;
  }
  return base;
}

bool Solver::tile_sized() const { return tile_sized_at(T_); }

bool Solver::resident_sized() const {
  // Every rank's owned block has a one-round resident plan at depth T_
  // (spans over deep-halo boxes are checked again, resident_span).
  if (!on_gpu() || !tb_kernel() || T_ < 4 || T_ % 2 != 0) return false;
  for (int r = 0; r < cart_.world; ++r) {
    const Block b = make_block(cart_, r, P_.nx, P_.ny);
    if (!gpu::tb_resident_fits(Box{0, b.lx, 0, b.ly}, T_)) return false;
  }
  return true;
}

bool Solver::tile_sized_at(int depth) const {
  // The same rule as gpu::tb_auto_variant (strip-rows per SIMD of the owned
  // block), decided from the largest block of any rank so that every rank
  // plans the same passes.
  if (!on_gpu() || !tb_kernel()) return false;
  const int64_t W = gpu::tb_strip_width(depth, 4), simds = gpu::tb_simd_count();
  for (int r = 0; r < cart_.world; ++r) {
    const Block b = make_block(cart_, r, P_.nx, P_.ny);
    if (ceil_div(b.ly, W) * b.lx >= int64_t(gpu::tb_tuning().tile_max_srps) * simds) return false;
  }
  return true;
}

std::vector<int> Solver::pass_depths(int64_t n) const {
  std::vector<int> d;
  const bool tb = tb_kernel();
  if (tb && T_ > gpu::kTbMaxDepth) {
    // Deep passes, then the remainder in near-equal passes of at most
    // kTbMaxDepth.  A short remainder (1000 = 83 x 12 + 4, 50 = 4 x 12 + 2)
    // is folded together with the last deep pass: the pass count stays the
    // same and no pass moves the whole field for only a few steps.
    const int64_t q = n / T_;
    int total = int(n % T_);
    d.assign(size_t(q), T_);
    if (total > 0) {
      if (total < gpu::kTbMaxDepth && q >= 1) {
        d.pop_back();
        total += T_;
      }
      const int parts = (total + gpu::kTbMaxDepth - 1) / gpu::kTbMaxDepth;
      if (total % 2 == 0 && tile_sized()) {
        // Even parts where the total allows (a 50-step check period is
        // 12,12,12,8,6, not 12,12,12,7,7): the workgroup-tile kernel of
        // small launches runs steps in pairs, and an odd pass would stream
        // (large launches keep 7,7: a depth-6 streaming pass costs more).
        const int pairs = total / 2;
        for (int i = 0; i < parts; ++i) d.push_back(2 * (pairs / parts + (i < pairs % parts ? 1 : 0)));
      } else {
        for (int i = 0; i < parts; ++i) d.push_back(total / parts + (i < total % parts ? 1 : 0));
      }
    }
    return d;
  }
  while (n > 0) {
    int k = int(std::min<int64_t>(T_, n));
    if (tb)
      while (!gpu::tb_depth_supported(k)) --k;
    d.push_back(k);
    n -= k;
  }
  return d;
}

bool Solver::mid_residual_ok(int k) const {
  // A check inside a pass needs (a) one launch per pass reading a source
  // buffer nothing else writes during the pass (so a converging check can be
  // replayed from it, replay_check) and (b) a kernel that takes the residual
  // at any step: depth-12 TB passes under the automatic variant choice.
  return gated() && tb_kernel() && gpu::tb_mid_residual(k);
}

std::vector<Solver::PassPlan> Solver::plan_passes(int64_t step0, int64_t n) const {
  // Full-depth passes whatever the check phase: a check that falls inside a
  // pass takes its residual at that step (rl < k) of the pass's launch, so
  // checks cost a residual, not a cut pass (was: every check ended a pass,
  // 50 steps = 12,12,12,7,7; 8192^2 checking every 20 steps -12 %,
  // profiles/r3_residual_cost.md).  Where that is not possible (kernels
  // without inner-level residuals, or two checks inside one pass) the pass is
  // cut at the check as before and the rest re-planned.
  // Reference: the check every STEP steps, mpi/...c:235-262,
  // cuda/cuda_heat.cu:219-236.
  std::vector<PassPlan> out;
  int64_t pos = step0;
  const int64_t end = step0 + n;
  std::vector<int> d = pass_depths(n);
  size_t i = 0;
  while (pos < end) {
    HEAT_CHECK(i < d.size(), "pass plan ran out at step %lld of %lld", (long long)pos,
               (long long)end);
    const int k = d[i];
    int64_t c = P_.converge ? next_check_after(pos) : INT64_MAX;
    if (c > pos + k) {  // no check in this pass
      out.push_back({k, 0});
      pos += k;
      ++i;
      continue;
    }
    const bool one = next_check_after(c) > pos + k;
    if (one && (c == pos + k || mid_residual_ok(k))) {
      out.push_back({k, int(c - pos)});
      pos += k;
      ++i;
      continue;
    }
    // Cut at the check, then plan the rest anew.
    const auto cut = pass_depths(c - pos);
    for (size_t j = 0; j < cut.size(); ++j)
      out.push_back({cut[j], j + 1 == cut.size() ? cut[j] : 0});
    pos = c;
    d = pass_depths(end - pos);
    i = 0;
  }
  return out;
}

// ---------------------------------------------------------------------------
// halo exchange
// ---------------------------------------------------------------------------
void Solver::exchange(int buf, int k, hipStream_t st) {
  TraceRange trace("heat.exchange");
  PhaseScope phase(this, kExchange, st);
  float* f = field_[buf];
  const auto& nb = blk_.nbr;
  const int64_t lx = blk_.lx, ly = blk_.ly, pitch = L_.pitch;
  const bool gpu = on_gpu();

  auto do_sendrecv = [&](std::vector<Msg>& msgs) {
    if (msgs.empty()) return;
    if (!staged_) {
      tr_->sendrecv(msgs.data(), int(msgs.size()), st);
      return;
    }
    // GPU fields, host transport: stage through pinned host memory.
    std::vector<Msg> host(msgs.size());
    HEAT_CHECK(int(msgs.size()) <= kMaxMsgs, "%zu messages", msgs.size());
    for (size_t i = 0; i < msgs.size(); ++i) {
      HEAT_CHECK(msgs[i].sbytes <= stage_bytes_ && msgs[i].rbytes <= stage_bytes_, "stage size");
      host[i] = Msg{msgs[i].peer, stage_send_[i], msgs[i].sbytes, stage_recv_[i], msgs[i].rbytes};
      if (msgs[i].sbytes)
        HIP_CHECK(hipMemcpyAsync(stage_send_[i], msgs[i].sbuf, msgs[i].sbytes,
                                 hipMemcpyDeviceToHost, st));
    }
    if (capturing_) {
      // Inside a graph the host-side transfer becomes a host node: HIP runs
      // it on its callback thread, in stream order between the staging
      // copies, every time the graph replays.  This is how the multi-rank
      // graph path (segment graphs keyed by ghost state, deep halos) runs
      // with several processes on ONE GPU, where RCCL refuses two ranks.
      StagedCall& c = staged_calls_.emplace_back();
      c.self = this;
      c.msgs = std::move(host);
      HIP_CHECK(hipLaunchHostFunc(st, &Solver::staged_host_fn, &c));
    } else {
      HIP_CHECK(hipStreamSynchronize(st));
      tr_->sendrecv(host.data(), int(host.size()), st);
    }
    for (size_t i = 0; i < msgs.size(); ++i)
      if (msgs[i].rbytes)
        HIP_CHECK(hipMemcpyAsync(msgs[i].rbuf, stage_recv_[i], msgs[i].rbytes,
                                 hipMemcpyHostToDevice, st));
  };

  // One phase, every message of the exchange in one group (one RCCL
  // latency): packed W/E columns of the owned rows, the N/S neighbours' rows
  // as full padded rows straight into the ghost rows, and on 2-D grids the
  // four k x k ghost corners from the diagonal neighbours, which deep (k > 1)
  // halos need.  A received N/S row also carries the sender's (stale) ghost
  // columns into our corner columns; the corner unpack after the group
  // overwrites them.  (The reference exchanges 1-deep halos, no corners,
  // mpi/mpi_heat_improved_persistent_stat.c:130-161.)
  const Box sw{0, lx, 0, k}, se{0, lx, ly - k, ly}, rw{0, lx, -k, 0}, re{0, lx, ly, ly + k};
  const Box csend[4] = {{0, k, 0, k}, {0, k, ly - k, ly}, {lx - k, lx, 0, k}, {lx - k, lx, ly - k, ly}};
  const Box crecv[4] = {{-k, 0, -k, 0}, {-k, 0, ly, ly + k}, {lx, lx + k, -k, 0}, {lx, lx + k, ly, ly + k}};
  std::vector<Msg> msgs;
  gpu::BoxCopy pk[6], uk[6];
  int np = 0, nu = 0;
  const size_t ew_bytes = size_t(lx) * size_t(k) * 4, c_bytes = size_t(k) * size_t(k) * 4;
  if (nb[West] >= 0) {
    pk[np++] = {sw, ew_[0]};
    uk[nu++] = {rw, ew_[2]};
    msgs.push_back(Msg{nb[West], ew_[0], ew_bytes, ew_[2], ew_bytes});
  }
  if (nb[East] >= 0) {
    pk[np++] = {se, ew_[1]};
    uk[nu++] = {re, ew_[3]};
    msgs.push_back(Msg{nb[East], ew_[1], ew_bytes, ew_[3], ew_bytes});
  }
  for (int d = 0; d < 4; ++d) {
    if (blk_.diag[d] < 0) continue;
    pk[np++] = {csend[d], cn_[d]};
    uk[nu++] = {crecv[d], cn_[4 + d]};
    msgs.push_back(Msg{blk_.diag[d], cn_[d], c_bytes, cn_[4 + d], c_bytes});
  }
  if (nb[North] >= 0 || nb[South] >= 0) {
    const size_t bytes = size_t(k) * size_t(pitch) * 4;
    const int64_t hy = L_.hy;
    if (nb[North] >= 0)
      msgs.push_back(Msg{nb[North], f - hy, bytes, f - k * pitch - hy, bytes});
    if (nb[South] >= 0)
      msgs.push_back(Msg{nb[South], f + (lx - k) * pitch - hy, bytes, f + lx * pitch - hy, bytes});
  }
  if (gpu) {
    gpu::copy_boxes(f, pitch, pk, np, true, st);
  } else {
    for (int i = 0; i < np; ++i) host_pack(f, pitch, pk[i].box, pk[i].buf);
  }
  do_sendrecv(msgs);
  if (gpu) {
    gpu::copy_boxes(f, pitch, uk, nu, false, st);
  } else {
    for (int i = 0; i < nu; ++i) host_unpack(uk[i].buf, f, pitch, uk[i].box);
  }
  ++stat_exchanges_;
}

void Solver::staged_host_fn(void* p) {
  auto* c = static_cast<StagedCall*>(p);
  Solver* self = c->self;
  if (self->staged_failed_.load()) return;  // a failed transport: skip, reported by run()
  try {
    self->tr_->sendrecv(c->msgs.data(), int(c->msgs.size()), nullptr);
  } catch (const std::exception& e) {
    {
      std::lock_guard<std::mutex> lk(self->staged_mu_);
      self->staged_error_ = e.what();
      self->staged_failed_.store(true);
    }
    // Later staged nodes of this rank are skipped, so its peers would wait
    // for messages that never come: let the transport fail them now.
    self->tr_->abort();
  }
}

void Solver::check_staged() {
  if (!staged_failed_.load()) return;
  std::lock_guard<std::mutex> lk(staged_mu_);
  throw_error(__FILE__, __LINE__, "host-staged exchange in a graph failed: " + staged_error_);
}

// ---------------------------------------------------------------------------
// compute
// ---------------------------------------------------------------------------
void Solver::compute_gpu(int k, int rl, bool split, int part, int band, int64_t er,
                         int64_t ec, hipStream_t st) {
  if (!st) st = s_comp_;
  // Host-side enqueue range (interior / boundary bands of the overlap
  // schedules, or the whole pass); the kernels' device time is in the
  // kernel trace.
  TraceRange trace(!split ? "heat.compute" : part == 0 ? "heat.interior" : "heat.boundary");
  PhaseScope phase(this, kCompute, st);
  const float* src = field_[cur_];
  float* dst = field_[cur_ ^ 1];
  const gpu::StencilGeom g = geom();
  unsigned* r = rl > 0 ? d_resid_ : nullptr;
  const int64_t lx = blk_.lx, ly = blk_.ly;
  const auto& nb = blk_.nbr;
  const int waves_target = gpu::tb_tuning().waves;
  // The box of this pass: the owned block grown by (er, ec) into the ghost
  // ring on sides that have a neighbour (deep-halo passes).
  const Box own{nb[North] >= 0 ? -er : 0, lx + (nb[South] >= 0 ? er : 0),
                nb[West] >= 0 ? -ec : 0, ly + (nb[East] >= 0 ? ec : 0)};

  if (!tb_kernel()) {
    // k single steps over shrinking regions (deep halo), ping-ponging.
    for (int j = 0; j < k; ++j) {
      const int64_t e = k - 1 - j;
      Box b{nb[North] >= 0 ? own.r0 - e : 0, own.r1 + (nb[South] >= 0 ? e : 0),
            nb[West] >= 0 ? own.c0 - e : 0, own.c1 + (nb[East] >= 0 ? e : 0)};
      const float* a = field_[cur_];
      float* d = field_[cur_ ^ 1];
      unsigned* rj = j == rl - 1 ? r : nullptr;
      if (P_.kernel == KernelKind::Lds)
        gpu::lds_step(a, d, g, b, rj, st);
      else if (P_.kernel == KernelKind::Mfma)
        gpu::mfma_step(a, d, g, b, rj, st);
      else
        gpu::naive_step(a, d, g, b, rj, st);
      cur_ ^= 1;
    }
    return;
  }

  if (!split) {
    gpu::tb_step(src, dst, g, &own, 1, k, r, st, waves_target, -1, rl);
    return;
  }
  // Boundary bands are `band` >= k deep (k for exchange-first; H for the
  // boundary-first pipeline, whose next exchange sends H rows/columns that
  // the concurrent interior launch must not write).
  if (band < k) band = k;
  const int64_t r0 = nb[North] >= 0 ? band : 0, r1 = nb[South] >= 0 ? lx - band : lx;
  const int64_t c0 = nb[West] >= 0 ? round_up(band, 4) : 0;
  const int64_t c1 = nb[East] >= 0 ? round_down(ly - band, 4) : ly;
  if (part == 0) {
    Box in{r0, r1, c0, c1};
    gpu::tb_step(src, dst, g, &in, 1, k, r, st, waves_target, -1, rl);
  } else {
    Box b[4] = {{0, r0, 0, ly}, {r1, lx, 0, ly}, {r0, r1, 0, c0}, {r0, r1, c1, ly}};
    gpu::tb_step(src, dst, g, b, 4, k, r, st, waves_target, -1, rl);
    // cur_ flips once per pass, after the boundary part.
  }
}

gpu::StencilGeom Solver::geom() const {
  gpu::StencilGeom g;
  g.pitch = L_.pitch;
  g.gx0 = blk_.ox;
  g.gy0 = blk_.oy;
  g.nx = P_.nx;
  g.ny = P_.ny;
  g.cx = P_.cx;
  g.cy = P_.cy;
  g.numerics = int(P_.numerics);
  if (gated()) g.gate = static_cast<const unsigned*>(d_gate_);  // DeviceGate::stop
  return g;
}

int Solver::resident_span(const std::vector<PassPlan>& plan, size_t i) const {
  // Passes of the configured depth, or a run of equal even remainder passes
  // (1000 steps at depth 12 end in 8 + 8: one 2-pass launch instead of two
  // tile launches that each load and store the whole block).
  if (!resident_ || plan[i].k < 4 || plan[i].k % 2 != 0 || plan[i].k > T_) return 0;
  // Checks may end any pass of a span (device-judged runs: each residual goes
  // to its own word, judged in order after the launch; replay_check re-runs
  // the span up to a converging one).
  if (tr_->world() > 1 && !resident_force_ && device_users(P_.device >= 0 ? P_.device : 0) > 1)
    return 0;
  const int k = plan[i].k;
  const bool ns = cart_.px > 1, ew = cart_.py > 1;
  // Ghost validity after the first pass's (possible) exchange, then the
  // bookkeeping of ensure_ghosts pass by pass: the span ends before a pass
  // that would need an exchange.
  int64_t gr = gr_, gc = gc_;
  if ((ns && gr < k) || (ew && gc < k)) gr = gc = H_;
  const Box box{blk_.nbr[North] >= 0 ? -(ns ? gr - k : 0) : 0,
                blk_.lx + (blk_.nbr[South] >= 0 ? (ns ? gr - k : 0) : 0),
                blk_.nbr[West] >= 0 ? -(ew ? round_down(gc - k, 4) : 0) : 0,
                blk_.ly + (blk_.nbr[East] >= 0 ? (ew ? round_down(gc - k, 4) : 0) : 0)};
  int n = 0, nchk = 0;
  for (size_t j = i; j < plan.size(); ++j) {
    if (plan[j].k != k) break;
    // Checks at even levels (the resident kernel's residual bodies: the up
    // steps), device-judged runs only.
    if (plan[j].rl != 0 &&
        (!gated() || plan[j].rl % 2 != 0 || nchk == gpu::kTbResidentMaxChecks))
      break;
    if (n > 0 && ((ns && gr < k) || (ew && gc < k))) break;
    if (res_span_max_ > 0 && n == res_span_max_) break;
    if (ns) gr -= k;
    if (ew) gc = round_down(gc - k, 4);
    ++n;
    if (plan[j].rl != 0) ++nchk;
  }
  if (n < 2 || !gpu::tb_resident_fits(box, k)) return 0;
  return n;
}

void Solver::enqueue_resident(const std::vector<PassPlan>& plan, size_t i0, int n) {
  const int k = plan[i0].k;
  TraceRange trace("heat.resident");
  // The first pass's exchange (if its ghosts ran out) and box; the later
  // passes only shrink the ghost validity (resident_span checked that none
  // of them needs an exchange).  The launch computes the first box in every
  // pass: cells it cannot keep valid lie outside each later pass's box, in
  // ghost columns and rows the bookkeeping already treats as stale.
  const int64_t ex0 = stat_exchanges_;
  const auto ext = ensure_ghosts(k, s_comp_);
  const auto& nb = blk_.nbr;
  const Box box{nb[North] >= 0 ? -ext.first : 0, blk_.lx + (nb[South] >= 0 ? ext.first : 0),
                nb[West] >= 0 ? -ext.second : 0, blk_.ly + (nb[East] >= 0 ? ext.second : 0)};
  for (int j = 1; j < n; ++j) (void)ensure_ghosts(k, s_comp_);
  HEAT_CHECK(stat_exchanges_ - ex0 <= 1, "resident span of %d passes needs an exchange", n);
  const int cur0 = cur_;
  // Always into the other buffer: the source stays intact for replay_check.
  const int out = cur_ ^ 1;
  std::vector<gpu::TbResidentCheck> chk;
  for (int j = 0; j < n; ++j)
    if (plan[i0 + size_t(j)].rl > 0) chk.push_back({j, plan[i0 + size_t(j)].rl});
  {
    PhaseScope phase(this, kCompute, s_comp_);
    gpu::TbResidentBuffers xb;
    xb.base[0] = xbase_[0];
    xb.base[1] = xbase_[1];
    xb.origin = L_.origin();
    xb.bytes = L_.bytes();
    xb.flags = d_flags_;
    xb.max_tiles = int(kResidentFlagBytes / 4);
    xb.err = d_flags_ + kResidentFlagBytes / 4;
    xb.done = xb.err + 1;
    gpu::tb_resident_step(field_[cur_], field_[out], geom(), box, k, n, xb, s_comp_, -1,
                          chk.data(), int(chk.size()), d_resid_ + kResidSpanOffset, blk_.lx,
                          blk_.ly);
  }
  resident_used_ = true;
  if (!chk.empty()) {
    // The span's checks (gated runs only: the judge zeroes the words), one
    // all-reduce and one judge launch for all of them.
    TraceRange trace("heat.allreduce");
    PhaseScope phase(this, kReduce, s_comp_);
    unsigned* rs = d_resid_ + kResidSpanOffset;
    if (tr_->device_memory() && tr_->world() > 1)
      tr_->allreduce_max(reinterpret_cast<float*>(rs),
                         gpu::kTbResidentSlots * gpu::kTbResidentMaxChecks, s_comp_);
    gpu::judge_check(rs, static_cast<gpu::DeviceGate*>(d_gate_), P_.eps, P_.compat == Compat::Mpi,
                     s_comp_, int(chk.size()), gpu::kTbResidentSlots, gpu::kTbResidentMaxChecks);
    for (const auto& c : chk) check_log_.push_back(step_ + int64_t(c.pass) * k + c.step);
  }
  for (int j = 0; j < n; ++j) {
    // Intermediate states live only in registers: a check's pass records the
    // span's source and its offset in the span (replay_check re-runs it).
    PassRec rec;
    rec.step0 = step_ + int64_t(j) * k;
    rec.k = k;
    rec.rl = plan[i0 + size_t(j)].rl;
    rec.cur0 = cur0;
    rec.cur1 = j + 1 == n ? out : -1;  // only the last pass's state is in memory
    rec.gr1 = gr_;
    rec.gc1 = gc_;
    rec.span = j + 1;
    rec.er = ext.first;
    rec.ec = ext.second;
    pass_log_.push_back(rec);
  }
  cur_ = out;
  step_ += int64_t(n) * k;
  stat_passes_ += n;
  stat_resident_ += n;
}

void Solver::compute_cpu(int k, int rl, int64_t er, int64_t ec) {
  TraceRange trace("heat.compute");
  PhaseScope phase(this, kCompute, nullptr);
  cpu::Geom g;
  g.pitch = L_.pitch;
  g.gx0 = blk_.ox;
  g.gy0 = blk_.oy;
  g.nx = P_.nx;
  g.ny = P_.ny;
  g.cx = P_.cx;
  g.cy = P_.cy;
  g.numerics = int(P_.numerics);
  const auto& nb = blk_.nbr;
  for (int j = 0; j < k; ++j) {
    const int64_t e = k - 1 - j;
    Box b{nb[North] >= 0 ? -(er + e) : 0, blk_.lx + (nb[South] >= 0 ? er + e : 0),
          nb[West] >= 0 ? -(ec + e) : 0, blk_.ly + (nb[East] >= 0 ? ec + e : 0)};
    const bool at = j == rl - 1;
    float r = cpu::step(field_[cur_], field_[cur_ ^ 1], g, b, at);
    if (at) cpu_resid_ = r;
    cur_ ^= 1;
  }
}

std::pair<int64_t, int64_t> Solver::ensure_ghosts(int k, hipStream_t st) {
  // gr_/gc_: how many ghost rows/columns of field_[cur_] hold the current
  // time level.  A k-step pass needs k; an exchange refills H.  Invariant:
  // they never exceed the depth of the last exchange of this buffer -- N/S
  // row messages carry the sender's own (stale) ghost columns into our
  // corners, and only the corner unpack of THAT exchange overwrites them up
  // to its depth (the overlap schedule exchanges k < H and then claims 0;
  // tests/test_gpu_loopback.py::test_loopback_deep_halo_chunked mixes depths
  // and short tail segments on 2 x 2 ranks).  The pass
  // then also updates the (valid - k) ghost rows/columns next to the block,
  // which become the valid ghosts of the next level.  Only axes that are
  // decomposed count, so every rank makes the same decision.
  const bool ns = cart_.px > 1, ew = cart_.py > 1;
  if ((ns && gr_ < k) || (ew && gc_ < k)) {
    exchange(cur_, H_, st);
    gr_ = gc_ = H_;
  }
  HEAT_CHECK(gr_ <= H_ && gc_ <= H_, "ghost depth %lld/%lld beyond the exchanged %d",
             (long long)gr_, (long long)gc_, H_);
  // TB boxes start on a float4 column: round the column extension down.
  const bool tb = tb_kernel();
  const int64_t er = ns ? gr_ - k : 0;
  const int64_t ec = ew ? (tb ? round_down(gc_ - k, 4) : gc_ - k) : 0;
  gr_ = er;
  gc_ = ec;
  return {er, ec};
}

void Solver::enqueue_pass(int k, int rl) {
  const auto& nb = blk_.nbr;
  const bool resid = rl > 0;
  // With world > 1 every rank of the (non-periodic) grid has a neighbour.
  const bool multi = tr_->world() > 1;
  PassRec rec;
  rec.step0 = step_;
  rec.k = k;
  rec.rl = rl;
  rec.cur0 = cur_;
  if (on_gpu()) {
    // Gated runs zero the residual word in the judge kernel instead.
    if (resid && !gated()) HIP_CHECK(hipMemsetAsync(d_resid_, 0, 4, s_comp_));
    const bool tb = tb_kernel();
    const int64_t lx = blk_.lx, ly = blk_.ly;
    const int band = sched_ == Schedule::Pipeline ? H_ : k;
    const int64_t ir0 = nb[North] >= 0 ? band : 0, ir1 = nb[South] >= 0 ? lx - band : lx;
    const int64_t ic0 = nb[West] >= 0 ? round_up(band, 4) : 0;
    const int64_t ic1 = nb[East] >= 0 ? round_down(ly - band, 4) : ly;
    const bool interior_ok = ir1 > ir0 && ic1 > ic0;
    // Which work goes on the side stream of the overlap schedules.  Eagerly
    // the exchange does (the high-priority comm stream, so RCCL's kernels
    // are dispatched ahead of queued stencil workgroups).  Under capture a
    // device transport keeps its collectives on the capture's origin stream
    // and the interior kernel forks instead: RCCL called on a forked
    // capturing stream crashes inside the library (RCCL 2.26, measured with
    // tools/rccl_mr_diag.sh), and a graph has the same dependency DAG either
    // way (exchange || interior, then the bands).
    const bool comm_on_side = !(capturing_ && tr_->device_memory());
    side_interior_ = false;
    if (!multi) {
      compute_gpu(k, rl, false, 0);
    } else if (sched_ == Schedule::Pipeline) {
      // Boundary-first: the H-deep ghosts of cur_ were exchanged by the
      // previous pass (or now, if stale).  Compute the H-deep boundary bands,
      // then post the NEXT pass's exchange (its send rows/columns all lie in
      // the bands) concurrent with the interior launch.
      if (gr_ < H_ || gc_ < H_) {
        if (comm_on_side) {
          HIP_CHECK(hipEventRecord(ev_ready_, s_comp_));
          HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
          exchange(cur_, H_, s_comm_);
          HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
          comm_pending_ = true;
        } else {
          exchange(cur_, H_, s_comp_);  // the bands wait for it anyway
        }
      }
      // Only wait on side work posted in this segment: a segment ends by
      // joining the comm stream, and a captured graph may not wait on an
      // event recorded outside its capture.
      if (comm_pending_) HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
      compute_gpu(k, rl, true, 1, band);
      HIP_CHECK(hipEventRecord(ev_ready_, s_comp_));
      if (comm_on_side) {
        // The interior is enqueued before the exchange: the stream semantics
        // are the same (s_comm waits for the bands only), and a host-staged
        // exchange, which blocks the host, then overlaps the interior too.
        compute_gpu(k, rl, true, 0, band);
        HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
        exchange(cur_ ^ 1, H_, s_comm_);
      } else {
        HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
        compute_gpu(k, rl, true, 0, band, 0, 0, s_comm_);
        exchange(cur_ ^ 1, H_, s_comp_);
        side_interior_ = true;
      }
      HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
      comm_pending_ = true;
      gr_ = gc_ = H_;  // for the buffer that becomes cur_ below
    } else if (sched_ == Schedule::Overlap && tb && interior_ok) {
      // Exchange-first: exchange || interior, then the boundary bands.
      HIP_CHECK(hipEventRecord(ev_ready_, s_comp_));
      HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
      if (comm_on_side) {
        exchange(cur_, k, s_comm_);
        HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
        compute_gpu(k, rl, true, 0);
      } else {
        compute_gpu(k, rl, true, 0, 0, 0, 0, s_comm_);
        HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
        exchange(cur_, k, s_comp_);
      }
      HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
      compute_gpu(k, rl, true, 1);
      gr_ = gc_ = 0;
    } else if (sched_ == Schedule::Overlap) {
      exchange(cur_, k, s_comp_);
      compute_gpu(k, rl, false, 0);
      gr_ = gc_ = 0;
    } else {
      // Sync (default): one launch per pass, one exchange per H/k passes.
      const auto ext = ensure_ghosts(k, s_comp_);
      compute_gpu(k, rl, false, 0, 0, ext.first, ext.second);
    }
    if (tb) cur_ ^= 1;
    if (resid) {
      TraceRange trace("heat.allreduce");
      PhaseScope phase(this, kReduce, s_comp_);
      // The residual is complete only once every launch of the pass is:
      // join the interior the pipeline ran on the comm stream (ev_halo_ was
      // recorded right behind it) before the all-reduce reads the word.
      if (side_interior_) HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
      const bool dev = tr_->device_memory();
      if (dev && multi) tr_->allreduce_max(reinterpret_cast<float*>(d_resid_), 1, s_comp_);
      if (gated()) {
        gpu::judge_check(d_resid_, static_cast<gpu::DeviceGate*>(d_gate_), P_.eps,
                         P_.compat == Compat::Mpi, s_comp_);
        check_log_.push_back(step_ + rl);
      } else {
        HIP_CHECK(hipMemcpyAsync(h_resid_, d_resid_, 4, hipMemcpyDeviceToHost, s_comp_));
      }
    }
  } else {
    std::pair<int64_t, int64_t> ext{0, 0};
    if (multi) ext = ensure_ghosts(k, nullptr);
    compute_cpu(k, rl, ext.first, ext.second);
  }
  rec.cur1 = cur_;
  rec.gr1 = gr_;
  rec.gc1 = gc_;
  pass_log_.push_back(rec);
  step_ += k;
  ++stat_passes_;
}

int Solver::chain_span(const std::vector<PassPlan>& plan, size_t i) const {
  if (!chain_ || plan[i].k != T_ || plan[i].rl != 0 || device_users(P_.device >= 0 ? P_.device : 0) > 1)
    return 0;
  int n = 0;
  for (size_t j = i; j < plan.size() && plan[j].k == T_ && plan[j].rl == 0; ++j) ++n;
  return n;
}

bool Solver::enqueue_chain(const std::vector<PassPlan>& plan, size_t i0, int n) {
  const int k = plan[i0].k;
  TraceRange trace("heat.chain");
  const int cur0 = cur_;
  gpu::TbChain ch;
  ch.passes = n;
  ch.flags = d_flags_;
  ch.err = d_flags_ + kResidentFlagBytes / 4;
  ch.done = ch.err + 1;
  ch.max_units = int(kResidentFlagBytes / 4);
  {
    PhaseScope phase(this, kCompute, s_comp_);
    const Box own{0, blk_.lx, 0, blk_.ly};
    gpu::tb_step(field_[cur_], field_[cur_ ^ 1], geom(), &own, 1, k, nullptr, s_comp_,
                 gpu::tb_tuning().waves, -1, 0, &ch);
  }
  if (!ch.chained) {
    chain_ = false;  // this block's plan does not qualify: one launch per pass from now on
    return false;
  }
  resident_used_ = true;  // the give-up word is read after the run (run_impl)
  const int out = (n & 1) ? cur0 ^ 1 : cur0;
  for (int j = 0; j < n; ++j) {
    PassRec rec;
    rec.step0 = step_ + int64_t(j) * k;
    rec.k = k;
    rec.rl = 0;
    rec.cur0 = (cur0 + j) & 1;
    rec.cur1 = (cur0 + j + 1) & 1;
    rec.gr1 = gr_;
    rec.gc1 = gc_;
    pass_log_.push_back(rec);
  }
  cur_ = out;
  step_ += int64_t(n) * k;
  stat_passes_ += n;
  stat_chained_ += n;
  return true;
}

void Solver::enqueue_segment(const std::vector<PassPlan>& plan) {
  for (size_t i = 0; i < plan.size();) {
    if (on_gpu()) {
      const int nc = chain_span(plan, i);
      if (nc >= 2 && enqueue_chain(plan, i, nc)) {
        i += size_t(nc);
        continue;
      }
    }
    const int n = on_gpu() ? resident_span(plan, i) : 0;
    if (n >= 2) {
      enqueue_resident(plan, i, n);
      i += size_t(n);
    } else {
      enqueue_pass(plan[i].k, plan[i].rl);
      ++i;
    }
  }
  if (comm_pending_) {
    // Join the comm stream (the last pass posted the next exchange): a
    // captured graph must end on its origin stream, and the next segment
    // relies on those ghosts.
    HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
    comm_pending_ = false;
  }
}

float Solver::finish_resid() {
  TraceRange trace("heat.residual_wait");
  float r;
  if (on_gpu()) {
    sync_watch();
    check_staged();
    tr_->check();
    std::memcpy(&r, h_resid_, 4);
    if (!tr_->device_memory()) tr_->allreduce_max(&r, 1, nullptr);
  } else {
    PhaseScope phase(this, kReduce, nullptr);
    r = cpu_resid_;
    tr_->allreduce_max(&r, 1, nullptr);
  }
  return r;
}

// ---------------------------------------------------------------------------
// phase timing
// ---------------------------------------------------------------------------
hipEvent_t Solver::pooled_event() {
  if (pool_used_ == event_pool_.size()) {
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    event_pool_.push_back(e);
  }
  return event_pool_[pool_used_++];
}

void Solver::flush_spans() {
  synchronize();
  for (const Span& sp : spans_) {
    double dt = sp.hb - sp.ha;
    if (sp.a) {
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, sp.a, sp.b));
      dt = 1e-3 * double(ms);
    }
    phase_acc_[sp.phase] += dt;
  }
  spans_.clear();
  pool_used_ = 0;
}

Solver::PhaseScope::PhaseScope(Solver* s, int phase, hipStream_t st) : s_(s), st_(st) {
  if (!s_->timing_ || s_->capturing_) return;
  // Bound the event pool on long runs (only between scopes: no open span).
  if (s_->spans_.size() >= 4096 && s_->open_spans_ == 0) s_->flush_spans();
  ++s_->open_spans_;
  Span sp{phase, nullptr, nullptr, now_s(), 0.0};
  if (s_->on_gpu() && st_) {
    sp.a = s_->pooled_event();
    sp.b = s_->pooled_event();
    HIP_CHECK(hipEventRecord(sp.a, st_));
  }
  idx_ = int(s_->spans_.size());
  s_->spans_.push_back(sp);
}

Solver::PhaseScope::~PhaseScope() {
  if (idx_ < 0) return;
  --s_->open_spans_;
  Span& sp = s_->spans_[size_t(idx_)];
  sp.hb = now_s();
  if (sp.b) (void)hipEventRecord(sp.b, st_);
}

bool Solver::is_check_point(int64_t completed) const {
  const int64_t C = P_.check_interval;
  if (P_.compat == Compat::Cuda) return completed >= 1 && (completed - 1) % C == 0;
  return completed >= 1 && completed % C == 0;
}

int64_t Solver::next_check_after(int64_t step) const {
  // Canonical: after steps C, 2C, ...; compat cuda: after steps 1, C+1, 2C+1
  // (cuda/cuda_heat.cu:219 checks at i % 20 == 0, 0-based).
  const int64_t C = P_.check_interval;
  if (P_.compat == Compat::Cuda) return step < 1 ? 1 : ((step - 1) / C + 1) * C + 1;
  return (step / C + 1) * C;
}

bool Solver::converged_value(float r) const {
  // mpi/...c:245 compares the fp32 |delta| against the double 1e-3;
  // cuda/cuda_heat.cu:67 compares in fp32 against 1e-3f.
  if (P_.compat == Compat::Mpi) return double(r) <= P_.eps;
  return r < float(P_.eps);
}

void Solver::launch_segment(const std::vector<PassPlan>& plan, int64_t n, int64_t phase,
                            bool use_graph, std::vector<PassRec>* recs,
                            std::vector<int64_t>* checks) {
  // Records come back relative to the segment's first step.
  const int64_t step_before = step_;
  auto relative = [&](GraphEntry& e) {
    e.recs = std::move(pass_log_);
    e.checks = std::move(check_log_);
    for (auto& r : e.recs) r.step0 -= step_before;
    for (auto& c : e.checks) c -= step_before;
    pass_log_.clear();
    check_log_.clear();
  };
  pass_log_.clear();
  check_log_.clear();
  if (!use_graph) {
    enqueue_segment(plan);
    GraphEntry e;
    relative(e);
    *recs = std::move(e.recs);
    *checks = std::move(e.checks);
    return;
  }
  const auto key = std::make_tuple(n, phase, cur_, gr_, gc_);
  auto it = graphs_.find(key);
  if (it == graphs_.end()) {
    const int64_t p_before = stat_passes_, e_before = stat_exchanges_, r_before = stat_resident_,
                  c_before = stat_chained_;
    const bool res_before = resident_used_;
    resident_used_ = false;
    TraceRange trace_capture("heat.capture");
    hipGraph_t graph;
    HIP_CHECK(hipStreamBeginCapture(s_comp_, hipStreamCaptureModeRelaxed));
    capturing_ = true;
    try {
      enqueue_segment(plan);
    } catch (...) {
      capturing_ = false;
      hipGraph_t g2 = nullptr;
      (void)hipStreamEndCapture(s_comp_, &g2);
      // Release it now: a captured RCCL call holds a reference on the
      // communicator until its graph is destroyed (ncclCommAbort waits).
      if (g2) (void)hipGraphDestroy(g2);
      throw;
    }
    capturing_ = false;
    HIP_CHECK(hipStreamEndCapture(s_comp_, &graph));
    GraphEntry e;
    HIP_CHECK(hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0));
    if (tr_->world() > 1 && std::strcmp(tr_->name(), "rccl") == 0) rccl_graphs_ = true;
    HIP_CHECK(hipGraphDestroy(graph));
    e.cur_after = cur_;
    e.gr_after = gr_;
    e.gc_after = gc_;
    e.passes = stat_passes_ - p_before;
    e.exchanges = stat_exchanges_ - e_before;
    e.resident = resident_used_;
    e.resident_passes = stat_resident_ - r_before;
    e.chained_passes = stat_chained_ - c_before;
    stat_resident_ = r_before;
    stat_chained_ = c_before;
    resident_used_ = res_before;
    relative(e);
    stat_passes_ = p_before;
    stat_exchanges_ = e_before;
    it = graphs_.emplace(key, std::move(e)).first;
  }
  HIP_CHECK(hipGraphLaunch(it->second.exec, s_comp_));
  resident_used_ = resident_used_ || it->second.resident;
  cur_ = it->second.cur_after;
  gr_ = it->second.gr_after;
  gc_ = it->second.gc_after;
  step_ = step_before + n;
  stat_passes_ += it->second.passes;
  stat_exchanges_ += it->second.exchanges;
  stat_resident_ += it->second.resident_passes;
  stat_chained_ += it->second.chained_passes;
  *recs = it->second.recs;
  *checks = it->second.checks;
}

void Solver::run_segments(int64_t steps, RunStats& s) {
  // Host-judged path (CPU backend, host-staged transports): one segment per
  // check, a host round trip per check.
  const bool gpu = on_gpu();
  const bool can_graph = gpu && P_.use_graph && !timing_ &&
                         (tr_->world() == 1 || tr_->graph_capturable() || staged_) &&
                         env_int("HEAT_GRAPH", 1) != 0;
  int64_t remaining = steps;
  std::vector<PassRec> recs;
  std::vector<int64_t> checks;
  while (remaining > 0) {
    int64_t seg = remaining;
    bool resid = false;
    if (P_.converge) {
      const int64_t next = next_check_after(step_);
      if (next - step_ <= remaining) {
        seg = next - step_;
        resid = true;
      }
    }
    const auto d = pass_depths(seg);
    std::vector<PassPlan> plan;
    for (size_t i = 0; i < d.size(); ++i)
      plan.push_back({d[i], resid && i + 1 == d.size() ? d[i] : 0});
    launch_segment(plan, seg, resid ? 0 : -1, can_graph, &recs, &checks);
    remaining -= seg;
    s.steps_done += seg;
    if (resid) {
      const float r = finish_resid();
      ++s.checks;
      s.last_resid = r;
      if (!(r == r) || std::isinf(r))
        throw GlobalError(strprintf("solver.cpp:%d: non-finite residual (%g) at step %lld", __LINE__,
                                    double(r), (long long)step_));
      if (converged_value(r)) {
        s.converged = true;
        s.converged_at = step_;
        break;
      }
    }
  }
}

void Solver::run_gated(int64_t steps, RunStats& s) {
  // Device-judged path: segments of whole check periods are enqueued without
  // waiting on any check (two in flight; the host polls a pinned copy of the
  // gate one segment behind).  After the converging check every stencil
  // launch is a no-op, so the state of that check is its pass's output.
  const bool can_graph = P_.use_graph && !timing_ &&
                         (tr_->world() == 1 || tr_->graph_capturable()) &&
                         env_int("HEAT_GRAPH", 1) != 0;
  const int64_t C = P_.check_interval;
  // ~512 steps per segment, a whole number of check periods: every segment
  // of a run starts at the same check phase (one graph per shape).
  // Segments of a whole number of lcm(C, T) steps where that is at most
  // 1024 (20 and 12: 60-step units; a plain multiple of C left a remainder
  // pair of depth-8 passes in every segment), else of C, about 1024 steps
  // long: a 1000-step run is one segment (one graph, one resident span
  // with up to kTbResidentMaxChecks checks, one judge); ~512-step segments
  // cost the 1024 x 8192 plate 2 % at a check every 100 steps.
  const int64_t L = std::lcm<int64_t>(C, std::max(1, T_));
  const int64_t unit = L <= 1024 ? L : C;
  const int64_t want = std::max(1, env_int("HEAT_SEG_STEPS", 1024));  // A/B knob
  const int64_t seg_cap = unit * std::max<int64_t>(1, (want + unit - 1) / unit);
  auto* gate_h = static_cast<gpu::DeviceGate*>(h_gate_);
  HIP_CHECK(hipMemsetAsync(d_gate_, 0, sizeof(gpu::DeviceGate), s_comp_));
  HIP_CHECK(hipMemsetAsync(d_resid_, 0, 4, s_comp_));
  const int64_t step0 = step_;
  std::vector<PassRec> all_recs;
  std::vector<int64_t> all_checks;
  int64_t remaining = steps, j = 0;
  bool stopped = false;
  while (remaining > 0 && !stopped) {
    const int64_t seg = std::min(remaining, seg_cap);
    const int64_t base = step_;
    const int64_t phase = next_check_after(step_) - step_;
    std::vector<PassRec> recs;
    std::vector<int64_t> checks;
    launch_segment(plan_passes(step_, seg), seg, phase, can_graph, &recs, &checks);
    for (auto& r : recs) {
      r.step0 += base;
      all_recs.push_back(r);
    }
    for (auto c : checks) all_checks.push_back(c + base);
    HIP_CHECK(hipMemcpyAsync(&gate_h[j & 1], d_gate_, sizeof(gpu::DeviceGate),
                             hipMemcpyDeviceToHost, s_comp_));
    HIP_CHECK(hipEventRecord(ev_seg_[j & 1], s_comp_));
    if (j >= 1) {
      wait_event(ev_seg_[(j - 1) & 1]);
      stopped = gate_h[(j - 1) & 1].stop != 0;
    }
    remaining -= seg;
    ++j;
  }
  sync_watch();
  const gpu::DeviceGate gate = gate_h[(j - 1) & 1];
  s.checks = gate.checks;
  if (gate.checks > 0) std::memcpy(&s.last_resid, &gate.last_bits, 4);
  if (!gate.stop) {
    s.steps_done = step_ - step0;
    return;
  }
  HEAT_CHECK(gate.stop_check < all_checks.size(), "gate closed at check %u of %zu",
             gate.stop_check, all_checks.size());
  const int64_t c = all_checks[gate.stop_check];
  const PassRec* p = nullptr;
  for (const auto& r : all_recs)
    if (r.rl > 0 && r.step0 + r.rl == c) p = &r;
  HEAT_CHECK(p != nullptr, "no pass takes the residual of check step %lld", (long long)c);
  // Passes behind the closing check wrote nothing: the state of that check
  // is the output of its pass, or, for a check inside a pass, the pass's
  // first rl steps replayed from its (untouched) source buffer.  Restored
  // before a non-finite residual is reported too, so gather() / save() after
  // the error see the check's state, as on the host-judged path.
  if (p->rl == p->k && p->cur1 >= 0) {
    cur_ = p->cur1;
    gr_ = p->gr1;
    gc_ = p->gc1;
  } else {
    replay_check(*p);
  }
  step_ = c;
  s.steps_done = c - step0;
  if (gate.reason == 2)
    throw GlobalError(strprintf("solver.cpp:%d: non-finite residual (%g) at step %lld", __LINE__,
                                double(s.last_resid), (long long)c));
  s.converged = true;
  s.converged_at = c;
}

void Solver::replay_check(const PassRec& p) {
  // The pass read field_[p.cur0] (owned block plus ghosts valid at least k
  // deep, exchanged or computed before it) and wrote only the other buffer;
  // every later launch was gated off, and later exchanges only re-sent those
  // same frozen states.  Its first rl steps over the owned block alone need
  // rl <= k ghost levels and no exchange: every rank replays locally.
  TraceRange trace("heat.replay_check");
  HEAT_CHECK(tb_kernel(), "replay of an inner-pass check needs the TB kernel");
  HIP_CHECK(hipMemsetAsync(d_gate_, 0, sizeof(unsigned), s_comp_));  // reopen: DeviceGate::stop
  cur_ = p.cur0;
  // A resident span: its first span - 1 passes over the span's (first) box,
  // as the launch ran them, then the check's rl steps.
  for (int j = 0; j + 1 < p.span; ++j) {
    compute_gpu(p.k, 0, false, 0, 0, p.er, p.ec);
    cur_ ^= 1;
  }
  // The check's rl steps as passes tb_step takes (a check at level 9-11 of a
  // depth-12 pass is no depth of its own): rl mod 8 first, then 8-step passes.
  // Each sub-pass covers the box grown by the steps still to come (a multiple
  // of 4, so the column growth is exact and float4-aligned); that needs at
  // most rl <= k valid ghost levels, which the pass itself had.
  const int64_t er0 = p.span > 1 ? p.er : 0, ec0 = p.span > 1 ? p.ec : 0;
  for (int left = p.rl; left > 0;) {
    const int d = gpu::tb_depth_supported(left) ? left : (left % 8 != 0 ? left % 8 : 8);
    left -= d;
    compute_gpu(d, 0, false, 0, 0, std::max<int64_t>(er0, left), std::max<int64_t>(ec0, left));
    cur_ ^= 1;
  }
  gr_ = gc_ = 0;  // the replayed buffer's ghosts are stale
  sync_watch();
}

RunStats Solver::run(int64_t steps) { return run_guarded(steps, true); }

void Solver::complete_pending() {
  // State access after enqueue(): wait for the enqueued steps first.  A
  // deferred resident give-up would otherwise go unseen by a caller that
  // never calls run() again: raise it here.
  if (!pending_) return;
  const RunStats r = run(0);
  HEAT_CHECK(r.resident_giveups == 0,
             "an enqueued run's resident tiles gave up a neighbour wait: the state is invalid");
}

RunStats Solver::enqueue(int64_t steps) { return run_guarded(steps, false); }

RunStats Solver::run_guarded(int64_t steps, bool wait) {
  try {
    return run_impl(steps, wait);
  } catch (const std::exception& e) {
    pending_ = false;
    if (tr_->world() > 1) {
      if (capturing_) {
        // Drop the half-built capture (its stream is unusable otherwise).
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(s_comp_, &g);
        if (g) (void)hipGraphDestroy(g);
        capturing_ = false;
      }
      // A failure of a class every rank meets at the same point (GlobalError:
      // a non-finite all-reduced residual) after which this rank's queued
      // work still completes (every exchange and all-reduce it enqueued was
      // matched, no transport error).  The communicator stays usable; the
      // message says so ("[clean]"), so a caller that agrees with its peers
      // (parallel.tune.autotune) can go on.  Anything else -- a rank-local
      // check included, which may have thrown before an exchange its peers
      // posted -- aborts it so that peers waiting on this rank fail instead
      // of hanging.
      bool clean = false;
      if (dynamic_cast<const GlobalError*>(&e) != nullptr && on_gpu() && !aborted_.load() &&
          !staged_failed_.load()) {
        try {
          sync_watch();
          tr_->check();
          clean = true;
        } catch (...) {
        }
      }
      if (clean) {
        std::fprintf(stderr, "[heat] rank %d: run failed after its queued work completed; "
                             "communicator kept\n", tr_->rank());
        throw Error(std::string("[clean] ") + e.what());
      }
      std::fprintf(stderr, "[heat] rank %d: run failed; aborting\n", tr_->rank());
      abort();
      std::fprintf(stderr, "[heat] rank %d: aborted%s\n", tr_->rank(),
                   rccl_graphs_.load() ? " (communicator left to process exit: live graphs)" : "");
    }
    throw;
  }
}

double Solver::time_exchange(int depth, int iters, int64_t* max_bytes) {
  complete_pending();
  // One grouped exchange phase of `depth` rows / columns (the message list a
  // run's deep-halo exchange sends), timed on the device over `iters`
  // back-to-back phases after one untimed phase (RCCL connections).  A halo
  // exchange of the current buffer is idempotent.  Collective: every rank
  // calls it with the same arguments.  Returns seconds per exchange.
  HEAT_CHECK(on_gpu() && tr_->world() > 1, "time_exchange needs GPU ranks");
  HEAT_CHECK(depth >= 1 && depth <= H_ && iters >= 1, "time_exchange depth %d (halo %d)", depth, H_);
  if (max_bytes) {
    const int64_t ns = (cart_.px > 1) ? int64_t(depth) * L_.pitch * 4 : 0;
    const int64_t ew = (cart_.py > 1) ? blk_.lx * int64_t(depth) * 4 : 0;
    *max_bytes = std::max(ns, ew);
  }
  synchronize();
  exchange(cur_, depth, s_comp_);
  sync_watch();
  hipEvent_t a = pooled_event(), b = pooled_event();
  HIP_CHECK(hipEventRecord(a, s_comp_));
  for (int i = 0; i < iters; ++i) exchange(cur_, depth, s_comp_);
  HIP_CHECK(hipEventRecord(b, s_comp_));
  sync_watch();
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, a, b));
  pool_used_ = 0;
  return 1e-3 * double(ms) / iters;
}

RunStats Solver::run_impl(int64_t steps, bool wait) {
  TraceRange trace("heat.run");
  RunStats s;
  HEAT_CHECK(steps >= 0, "negative step count");
  const int64_t p0 = stat_passes_, e0 = stat_exchanges_, res0 = stat_resident_, ch0 = stat_chained_;
  // An enqueued run (enqueue) still in flight: continue its stream; its
  // error word and transport are checked when this call completes.
  const bool cont = pending_;
  if (!cont) {
    synchronize();
    resident_used_ = false;
  }
  // Only plain GPU runs are asynchronous: gated runs read the device gate
  // on the host, phase timing syncs per phase, host-staged exchanges block.
  if (!on_gpu() || gated() || timing_ || staged_) wait = true;
  const double t0 = now_s();
  const bool gpu = on_gpu();
  if (timing_) {
    spans_.clear();
    pool_used_ = 0;
    phase_acc_[0] = phase_acc_[1] = phase_acc_[2] = 0.0;
  }
  const bool graphs = gpu && P_.use_graph && !timing_ && env_int("HEAT_GRAPH", 1) != 0;
  if (graphs && tr_->world() > 1 && tr_->device_memory() && tr_->graph_capturable() && !warmed_) {
    // Let RCCL establish its connections outside of stream capture.  A halo
    // exchange of the current buffer is idempotent.
    exchange(cur_, H_, s_comp_);
    tr_->allreduce_max(reinterpret_cast<float*>(d_scratch_), 1, s_comp_);
    sync_watch();
    warmed_ = true;
  }
  if (steps > 0) {
    if (gated()) run_gated(steps, s);
    else run_segments(steps, s);
  }
  if (!wait) {
    pending_ = true;
    s.total_steps = step_;
    s.passes = stat_passes_ - p0;
    s.exchanges = stat_exchanges_ - e0;
    s.resident_passes = stat_resident_ - res0;
    s.chained_passes = stat_chained_ - ch0;
    return s;
  }
  pending_ = false;
  unsigned* d_err = resident_used_ ? d_flags_ + kResidentFlagBytes / 4 : nullptr;
  if (d_err) HIP_CHECK(hipMemcpyAsync(h_err_, d_err, 4, hipMemcpyDeviceToHost, s_comp_));
  sync_watch();
  bool gave_up = d_err && *h_err_ != 0;
  if (gave_up) {
    // Clear it for the next launch (the flags and the completion counter
    // were re-zeroed by the last tile, which every tile reaches).
    *h_err_ = 0;
    HIP_CHECK(hipMemsetAsync(d_err, 0, 4, s_comp_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
  }
  if (d_err && inject_giveup_) {  // HEAT_TEST_RES_GIVEUP_RANK (tests)
    inject_giveup_ = false;
    gave_up = true;
  }
  if (gave_up) {
    // A neighbour wait gave up (tiles not co-resident, e.g. another process
    // holds CUs): this run's results are invalid.  All of its exchanges and
    // collectives were matched (the spans make the same transport calls as
    // separate passes), so nothing is left waiting.  Default: throw.  With
    // HEAT_TB_RES_GIVEUP=defer (bench.py, the autotune) the run returns with
    // resident_giveups set and resident spans switched off for this solver,
    // and the caller -- which agrees with its peers -- redoes the work.
    if (!defer_giveup_)
      throw_error(__FILE__, __LINE__,
                  "resident tile launch: a neighbour wait gave up (tiles not co-resident?); "
                  "results are invalid (HEAT_TB_RESIDENT=0 runs one launch per pass)");
    std::fprintf(stderr, "[heat] rank %d: resident tiles gave up a neighbour wait: this run's "
                         "results are invalid; resident spans off for this solver\n", tr_->rank());
    resident_ = false;
    chain_ = false;
    for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second.exec);
    graphs_.clear();
    rccl_graphs_ = false;
    s.resident_giveups = 1;
  }
  check_staged();
  tr_->check();
  s.seconds = now_s() - t0;
  if (timing_) {
    flush_spans();
    s.t_exchange = phase_acc_[kExchange];
    s.t_compute = phase_acc_[kCompute];
    s.t_reduce = phase_acc_[kReduce];
  }
  s.total_steps = step_;
  s.passes = stat_passes_ - p0;
  s.exchanges = stat_exchanges_ - e0;
  s.resident_passes = stat_resident_ - res0;
  s.chained_passes = stat_chained_ - ch0;
  return s;
}

void Solver::wait_event(hipEvent_t e) {
  // The reference's ranks block in MPI_Waitall / MPI_Allreduce
  // (mpi/mpi_heat_improved_persistent_stat.c:177, :255) and hang with a dead
  // peer.  Here a multi-rank GPU wait polls: it spins on hipEventQuery for a
  // few thousand tries (the common case: a segment that is about to end),
  // then sleeps between polls, asks the transport for asynchronous errors
  // every 50 ms (ncclCommGetAsyncError) and gives up after watchdog_s_
  // seconds without completion.  Either way the transport is aborted
  // (ncclCommAbort) and the call throws: a fresh failure exit, no retry.
  if (!watch_) {
    HIP_CHECK(hipEventSynchronize(e));
    return;
  }
  const double t0 = now_s();
  double next_poll = t0 + 0.05;
  for (int spin = 0;; ++spin) {
    if (aborted_.load())
      throw_error(__FILE__, __LINE__, strprintf("rank %d: run aborted", tr_->rank()));
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) HIP_CHECK(q);
    if (spin < 4096) {
      std::this_thread::yield();
      continue;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    const double t = now_s();
    if (t < next_poll) continue;
    next_poll = t + 0.05;
    try {
      check_staged();
      tr_->check();
    } catch (...) {
      abort();
      throw;
    }
    if (watchdog_s_ > 0 && t - t0 > watchdog_s_) {
      abort();
      throw_error(__FILE__, __LINE__,
                  strprintf("rank %d: no progress on the device for %.0f s (HEAT_WATCHDOG_S): a "
                            "peer rank died or hung; transport aborted",
                            tr_->rank(), watchdog_s_));
    }
  }
}

void Solver::sync_watch() {
  if (!watch_) {
    synchronize();
    return;
  }
  HIP_CHECK(hipEventRecord(ev_wait_, s_comm_));
  HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_wait_, 0));
  HIP_CHECK(hipEventRecord(ev_wait_, s_comp_));
  wait_event(ev_wait_);
}

void Solver::abort() {
  // ncclCommAbort waits until every graph that captured an RCCL call is
  // destroyed; such a graph may still be running (waiting for the dead peer)
  // and cannot be destroyed from here.  Then only mark the solver aborted:
  // its waits throw, and the caller ends the process (the CLI exits without
  // destructors; the peers' watchdogs end theirs).
  if (aborted_.exchange(true)) return;
  if (rccl_graphs_.load()) tr_->abandon();
  else tr_->abort();
}

void Solver::synchronize() {
  if (on_gpu()) {
    HIP_CHECK(hipStreamSynchronize(s_comm_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
  }
}

// ---------------------------------------------------------------------------
// state access, gather, checksum, binary I/O
// ---------------------------------------------------------------------------
void Solver::copy_owned(float* host, int64_t host_pitch) {
  complete_pending();
  if (on_gpu()) {
    HIP_CHECK(hipMemcpy2DAsync(host, size_t(host_pitch) * 4, field_[cur_], size_t(L_.pitch) * 4,
                               size_t(blk_.ly) * 4, size_t(blk_.lx), hipMemcpyDeviceToHost,
                               s_comp_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
  } else {
    for (int64_t r = 0; r < blk_.lx; ++r)
      std::memcpy(host + r * host_pitch, field_[cur_] + r * L_.pitch, size_t(blk_.ly) * 4);
  }
}

void Solver::load_owned(const float* host, int64_t host_pitch, int64_t step) {
  complete_pending();
  synchronize();
  for (int b = 0; b < 2; ++b) {
    if (on_gpu()) {
      HIP_CHECK(hipMemcpy2DAsync(field_[b], size_t(L_.pitch) * 4, host, size_t(host_pitch) * 4,
                                 size_t(blk_.ly) * 4, size_t(blk_.lx), hipMemcpyHostToDevice,
                                 s_comp_));
    } else {
      for (int64_t r = 0; r < blk_.lx; ++r)
        std::memcpy(field_[b] + r * L_.pitch, host + r * host_pitch, size_t(blk_.ly) * 4);
    }
  }
  synchronize();
  step_ = step;
  gr_ = gc_ = 0;
}

void Solver::scatter_root(const float* full, int64_t step) {
  complete_pending();
  TraceRange tr("heat.scatter");
  const int rank = tr_->rank(), world = tr_->world();
  const bool dev = tr_->device_memory();
  std::vector<float> mine(static_cast<size_t>(blk_.lx * blk_.ly));
  int64_t max_block = 0;
  for (int r = 0; r < world; ++r) {
    Block b = make_block(cart_, r, P_.nx, P_.ny);
    max_block = std::max(max_block, b.lx * b.ly);
  }
  float* dbuf = nullptr;
  if (dev && world > 1) HIP_CHECK(hipMalloc(&dbuf, size_t(max_block) * 4));
  auto cut = [&](const Block& b, float* dst) {
    for (int64_t r = 0; r < b.lx; ++r)
      std::memcpy(dst + r * b.ly, full + (b.ox + r) * P_.ny + b.oy, size_t(b.ly) * 4);
  };
  if (rank == 0) {
    HEAT_CHECK(full != nullptr, "scatter_root: rank 0 needs the full grid");
    cut(blk_, mine.data());
    std::vector<float> tmp(static_cast<size_t>(max_block));
    for (int r = 1; r < world; ++r) {
      Block b = make_block(cart_, r, P_.nx, P_.ny);
      cut(b, tmp.data());
      const size_t bytes = size_t(b.lx * b.ly) * 4;
      if (dev) {
        HIP_CHECK(hipMemcpyAsync(dbuf, tmp.data(), bytes, hipMemcpyHostToDevice, s_comp_));
        Msg m{r, dbuf, bytes, nullptr, 0};
        tr_->sendrecv(&m, 1, s_comp_);
        HIP_CHECK(hipStreamSynchronize(s_comp_));
      } else {
        Msg m{r, tmp.data(), bytes, nullptr, 0};
        tr_->sendrecv(&m, 1, nullptr);
      }
    }
  } else {
    const size_t bytes = mine.size() * 4;
    if (dev) {
      Msg m{0, nullptr, 0, dbuf, bytes};
      tr_->sendrecv(&m, 1, s_comp_);
      HIP_CHECK(hipMemcpyAsync(mine.data(), dbuf, bytes, hipMemcpyDeviceToHost, s_comp_));
      HIP_CHECK(hipStreamSynchronize(s_comp_));
    } else {
      Msg m{0, nullptr, 0, mine.data(), bytes};
      tr_->sendrecv(&m, 1, nullptr);
    }
  }
  if (dbuf) HIP_CHECK(hipFree(dbuf));
  load_owned(mine.data(), blk_.ly, step);
}

std::vector<float> Solver::gather_root() {
  complete_pending();
  TraceRange trace("heat.gather");
  const int rank = tr_->rank(), world = tr_->world();
  std::vector<float> mine(static_cast<size_t>(blk_.lx * blk_.ly));
  copy_owned(mine.data(), blk_.ly);
  std::vector<float> out;
  const bool dev = tr_->device_memory();
  int64_t max_block = 0;
  for (int r = 0; r < world; ++r) {
    Block b = make_block(cart_, r, P_.nx, P_.ny);
    max_block = std::max(max_block, b.lx * b.ly);
  }
  float* dbuf = nullptr;
  if (dev && world > 1) HIP_CHECK(hipMalloc(&dbuf, size_t(max_block) * 4));
  if (rank == 0) {
    out.assign(size_t(P_.nx * P_.ny), 0.0f);
    auto place = [&](const Block& b, const float* src) {
      for (int64_t r = 0; r < b.lx; ++r)
        std::memcpy(&out[size_t((b.ox + r) * P_.ny + b.oy)], src + r * b.ly, size_t(b.ly) * 4);
    };
    place(blk_, mine.data());
    std::vector<float> tmp(static_cast<size_t>(max_block));
    for (int r = 1; r < world; ++r) {
      Block b = make_block(cart_, r, P_.nx, P_.ny);
      const size_t bytes = size_t(b.lx * b.ly) * 4;
      if (dev) {
        Msg m{r, nullptr, 0, dbuf, bytes};
        tr_->sendrecv(&m, 1, s_comp_);
        HIP_CHECK(hipMemcpyAsync(tmp.data(), dbuf, bytes, hipMemcpyDeviceToHost, s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
      } else {
        Msg m{r, nullptr, 0, tmp.data(), bytes};
        tr_->sendrecv(&m, 1, nullptr);
      }
      place(b, tmp.data());
    }
  } else {
    const size_t bytes = mine.size() * 4;
    if (dev) {
      HIP_CHECK(hipMemcpyAsync(dbuf, mine.data(), bytes, hipMemcpyHostToDevice, s_comp_));
      Msg m{0, dbuf, bytes, nullptr, 0};
      tr_->sendrecv(&m, 1, s_comp_);
      HIP_CHECK(hipStreamSynchronize(s_comp_));
    } else {
      Msg m{0, mine.data(), bytes, nullptr, 0};
      tr_->sendrecv(&m, 1, nullptr);
    }
  }
  if (dbuf) HIP_CHECK(hipFree(dbuf));
  return out;
}

void Solver::reduce_scalars(double* f64, int nf, uint64_t* u64, int nu, float* fmax, int nm) {
  if (tr_->world() == 1) return;
  if (!tr_->device_memory()) {
    if (nf) tr_->allreduce_sum_f64(f64, nf, nullptr);
    if (nu) tr_->allreduce_sum_u64(u64, nu, nullptr);
    if (nm) tr_->allreduce_max(fmax, nm, nullptr);
    return;
  }
  char* d = static_cast<char*>(d_scratch_);
  HIP_CHECK(hipMemcpyAsync(d, f64, size_t(nf) * 8, hipMemcpyHostToDevice, s_comp_));
  HIP_CHECK(hipMemcpyAsync(d + 1024, u64, size_t(nu) * 8, hipMemcpyHostToDevice, s_comp_));
  HIP_CHECK(hipMemcpyAsync(d + 2048, fmax, size_t(nm) * 4, hipMemcpyHostToDevice, s_comp_));
  if (nf) tr_->allreduce_sum_f64(reinterpret_cast<double*>(d), nf, s_comp_);
  if (nu) tr_->allreduce_sum_u64(reinterpret_cast<uint64_t*>(d + 1024), nu, s_comp_);
  if (nm) tr_->allreduce_max(reinterpret_cast<float*>(d + 2048), nm, s_comp_);
  HIP_CHECK(hipMemcpyAsync(f64, d, size_t(nf) * 8, hipMemcpyDeviceToHost, s_comp_));
  HIP_CHECK(hipMemcpyAsync(u64, d + 1024, size_t(nu) * 8, hipMemcpyDeviceToHost, s_comp_));
  HIP_CHECK(hipMemcpyAsync(fmax, d + 2048, size_t(nm) * 4, hipMemcpyDeviceToHost, s_comp_));
  HIP_CHECK(hipStreamSynchronize(s_comp_));
}

Checksum Solver::checksum() {
  complete_pending();
  TraceRange tr("heat.checksum");
  Checksum c;
  if (on_gpu()) {
    // On the device: no host copy of the block (131072^2 grids are 68 GB).
    auto* d = static_cast<gpu::DeviceChecksum*>(d_checksum_);
    gpu::DeviceChecksum h{0, 0.0, 0x7FFFFFFF, int(0x80000000), 0};
    HIP_CHECK(hipMemcpyAsync(d, &h, sizeof h, hipMemcpyHostToDevice, s_comp_));
    gpu::checksum_block(field_[cur_], L_.pitch, blk_.lx, blk_.ly, blk_.ox, blk_.oy, P_.ny, d,
                        s_comp_);
    HIP_CHECK(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, s_comp_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
    c.hash = h.hash;
    c.sum = h.sum;
    c.count = int64_t(h.count);
    c.min = gpu::checksum_key_to_float(h.min_key);
    c.max = gpu::checksum_key_to_float(h.max_key);
  } else {
    std::vector<float> mine(static_cast<size_t>(blk_.lx * blk_.ly));
    copy_owned(mine.data(), blk_.ly);
    c = checksum_block(mine.data(), blk_.ly, blk_.ox, blk_.oy, blk_.lx, blk_.ly, P_.ny);
  }
  double f[1] = {c.sum};
  uint64_t u[2] = {c.hash, uint64_t(c.count)};
  float m[2] = {float(c.max), float(-c.min)};
  reduce_scalars(f, 1, u, 2, m, 2);
  Checksum g;
  g.sum = f[0];
  g.hash = u[0];
  g.count = int64_t(u[1]);
  g.max = m[0];
  g.min = -m[1];
  return g;
}

void Solver::write_bin(const std::string& path) {
  complete_pending();
  TraceRange trace("heat.output");
  // Written as `path`.tmp by every rank, then renamed by rank 0 once all
  // blocks are in: a crash mid-write (a --checkpoint-every run) leaves the
  // previous checkpoint intact.
  const std::string tmp = path + ".tmp";
  if (tr_->rank() == 0) {
    BinHeader h{};
    std::memcpy(h.magic, "HEATF32", 8);
    h.version = 1;
    h.parity = uint32_t(cur_);
    h.nx = P_.nx;
    h.ny = P_.ny;
    h.step = step_;
    h.cx = P_.cx;
    h.cy = P_.cy;
    h.reserved[0] = bin_config_tag(int(P_.compat), int(P_.numerics));
    bin_create(tmp, h);
  }
  tr_->barrier();
  std::vector<float> mine(static_cast<size_t>(blk_.lx * blk_.ly));
  copy_owned(mine.data(), blk_.ly);
  bin_write_block(tmp, P_.nx, P_.ny, blk_.ox, blk_.oy, blk_.lx, blk_.ly, mine.data(), blk_.ly);
  tr_->barrier();
  if (tr_->rank() == 0) bin_commit(tmp, path);
  tr_->barrier();
}

void Solver::read_bin(const std::string& path) {
  complete_pending();
  TraceRange trace("heat.resume");
  BinHeader h = bin_read_header(path);
  HEAT_CHECK(h.nx == P_.nx && h.ny == P_.ny, "checkpoint is %lldx%lld, run is %lldx%lld",
             (long long)h.nx, (long long)h.ny, (long long)P_.nx, (long long)P_.ny);
  // A checkpoint of a different physics or compat mode still loads (the
  // state is just a grid), but the continuation is not the run it came from.
  if (tr_->rank() == 0) {
    if (h.cx != P_.cx || h.cy != P_.cy)
      std::fprintf(stderr, "heat: warning: %s was written with cx=%g cy=%g, this run uses "
                   "cx=%g cy=%g\n", path.c_str(), double(h.cx), double(h.cy), double(P_.cx),
                   double(P_.cy));
    const uint64_t tag = bin_config_tag(int(P_.compat), int(P_.numerics));
    if (h.reserved[0] != 0 && h.reserved[0] != tag)
      std::fprintf(stderr, "heat: warning: %s was written under another --compat/--numerics "
                   "mode (tag %llx, this run %llx)\n", path.c_str(),
                   (unsigned long long)h.reserved[0], (unsigned long long)tag);
  }
  std::vector<float> mine(static_cast<size_t>(blk_.lx * blk_.ly));
  bin_read_block(path, blk_.ox, blk_.oy, blk_.lx, blk_.ly, mine.data(), blk_.ly);
  load_owned(mine.data(), blk_.ly, h.step);
}

}  // namespace heat
