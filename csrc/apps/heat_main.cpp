// `heat` — the standalone command-line entry point.
//
// One binary replaces the reference's compile-time variants
// (cuda_heat, heat_<N>, heat_omp_<N>, heat_con_<N>, heat_con_omp_<N>;
// cuda/Makefile:13-17, mpi/Makefile:12-22): every -D macro is a flag here.
// Multi-process runs read RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR (any
// launcher, e.g. `python -m torch.distributed.run`), use TCP between CPU
// ranks and RCCL between GPU ranks (the RCCL unique id travels over the TCP
// rendezvous).  Output lines reproduce the reference's (mpi/...c:88-96,
// :298-306; cuda/cuda_heat.cu:254-260) under --naming mpi|cuda.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "heat/capi.h"
#include "heat/common.hpp"
#include "heat/plan.hpp"
#include "heat/io.hpp"
#include "heat/solver.hpp"

using namespace heat;

namespace {

void usage() {
  std::printf(
      "usage: heat [options]\n"
      "  --nx N --ny N           grid size (rows x columns)            [20 x 20]\n"
      "  --steps N               time steps                             [10000]\n"
      "  --cx F --cy F           diffusion coefficients                 [0.1 0.1]\n"
      "  --converge              enable the convergence test\n"
      "  --check-interval N      steps between convergence checks       [20]\n"
      "  --eps F                 convergence threshold on max|delta|    [1e-3]\n"
      "  --backend cpu|hip       compute backend                        [hip if a GPU exists]\n"
      "  --threads N             CPU OpenMP threads                     [runtime default]\n"
      "  --kernel auto|tb|lds|mfma|naive  GPU kernel family (auto = tb)  [auto]\n"
      "  --tb-depth K            fused steps per pass (= halo depth)    [8 hip, 1 cpu]\n"
      "  --decomp auto|rows|2d   process grid (auto = MPI_Dims_create)  [auto]\n"
      "  --px P --py Q           explicit process grid\n"
      "  --init ref-wrap|exact|random|zero  initial condition          [ref-wrap]\n"
      "  --seed S                seed for --init random\n"
      "  --out PATH|none         output file                            [per --naming]\n"
      "  --out-format dat|bin|checksum                                  [dat]\n"
      "  --naming plain|mpi|cuda reference-style file names and messages [plain]\n"
      "  --dump-initial          also write the initial grid\n"
      "  --compat none|mpi|cuda  reference step-count/check semantics   [none]\n"
      "  --no-graph --no-overlap disable hipGraph capture / comm overlap\n"
      "  --schedule auto|sync|overlap|pipeline   multi-rank pass schedule [auto=sync]\n"
      "  --halo-passes M         sync schedule: passes per halo exchange [auto]\n"
      "  --numerics fp32|mpi     update arithmetic (mpi = reference MPI double) [fp32]\n"
      "  --checkpoint PATH --checkpoint-every K   periodic binary checkpoints\n"
      "  --resume PATH           start from a binary checkpoint\n"
      "  --transport auto|local|tcp|rccl|loopback inter-rank transport  [auto]\n"
      "  --port P                rendezvous port (default MASTER_PORT+1 or 29600)\n"
      "  --gpus N                one process, N GPU ranks as threads: RCCL (one rank per\n"
      "                          GPU) when N GPUs are visible, else loopback D2D copies\n"
      "  --watchdog S            multi-rank GPU runs: give up (abort the transport, exit 1)\n"
      "                          after S s without device progress [300; 0 = never]\n"
      "  --phase-timing          per-phase times (exchange/compute/reduce) in --json; eager\n"
      "  --plan                  print the per-GPU memory plan (fields + halo buffers, worst\n"
      "                          rank, 288 GB HBM3E check) for --gpus/WORLD_SIZE ranks; exit\n"
      "  --warmup N              N untimed steps first (graph capture), then the initial\n"
      "                          state is restored and the timed run starts     [0]\n"
      "  --json                  print a JSON metrics line\n");
}

int env_i(const char* n, int d) {
  const char* v = std::getenv(n);
  return v && *v ? std::atoi(v) : d;
}

// Command-line options that shape one rank's run (beyond Params).
struct Options {
  int64_t steps = 10000;
  std::string out, out_format = "dat", naming = "plain";
  std::string checkpoint, resume;
  int64_t ckpt_every = 0;
  int64_t warmup = 0;  // untimed steps first (graph capture, first touch), then the state is reset
  bool json = false, dump_initial = false;
};

// The live solvers of a single-process multi-rank run (heat --gpus N): a
// failing rank aborts its peers' solvers (Solver::abort: ncclCommAbort, or
// the communicator abandoned while captured graphs hold it) so that their
// waits on it end and every thread can be joined.  A rank removes its entry
// under the lock before its solver is destroyed, so an abort never runs on a
// solver being destroyed.
struct RankRegistry {
  std::mutex mu;
  std::vector<Solver*> solvers;
  void set(int r, Solver* s) {
    std::lock_guard<std::mutex> lk(mu);
    solvers[size_t(r)] = s;
  }
  void abort_peers(int r) {
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = 0; i < solvers.size(); ++i)
      if (int(i) != r && solvers[i]) solvers[i]->abort();
  }
};

// One rank's whole run: banners, solver, output, reference-style lines.
void run_rank(const Options& o, const Params& P, std::unique_ptr<Transport> tr,
              RankRegistry* reg = nullptr) {
  const int rank = tr->rank(), world = tr->world();
  const bool root = rank == 0;

  // Reference-style banners (mpi/...c:90-96).
  if (root && o.naming == "mpi") {
    std::printf("Starting mpi_heat2D with %d worker tasks.\n", world);
    if (!P.converge)
      std::printf("Grid size: X= %lld  Y= %lld  Time steps= %lld\n", (long long)P.nx,
                  (long long)P.ny, (long long)o.steps);
    else
      std::printf("Grid size: X= %lld  Y= %lld  Time steps= - \n", (long long)P.nx,
                  (long long)P.ny);
    std::fflush(stdout);
  }

  Solver S(P, std::move(tr));
  struct Registered {  // unregistered before S is destroyed (on any exit)
    RankRegistry* reg;
    int r;
    ~Registered() {
      if (reg) reg->set(r, nullptr);
    }
  } registered{reg, rank};
  if (reg) reg->set(rank, &S);
  if (!o.resume.empty()) S.read_bin(o.resume);

  const bool small = P.nx * P.ny <= (int64_t(1) << 24);
  std::string init_path, final_path;
  if (o.naming == "mpi") {
    init_path = "initial_im.dat";
    final_path = "final_im.dat";
  } else if (o.naming == "cuda") {
    // out_cuda_<TPB>_<NB>_<STEPS>.dat with the reference's geometry
    // (THREADS_PER_ROW 32, cuda/cuda_heat.cu:17-21, :245-250).
    const int64_t T = 32;
    const int64_t rb = (P.nx - 2) / T + ((P.nx - 2) % T ? 1 : 0);
    const int64_t cb = (P.ny - 2) / T + ((P.ny - 2) % T ? 1 : 0);
    final_path = strprintf("out_cuda_%lld_%lld_%lld.dat", (long long)(T * T),
                           (long long)(rb * cb), (long long)o.steps);
  } else {
    final_path = small ? "final.dat" : "none";
    init_path = "initial.dat";
  }
  if (!o.out.empty()) final_path = o.out;

  auto emit = [&](const std::string& path) {
    if (path == "none" || path.empty()) return;
    if (o.out_format == "bin") {
      S.write_bin(path);
    } else if (o.out_format == "checksum") {
      Checksum c = S.checksum();
      if (root) {
        FILE* f = std::fopen(path.c_str(), "w");
        HEAT_CHECK(f, "cannot open %s", path.c_str());
        std::fprintf(f,
                     "{\"nx\": %lld, \"ny\": %lld, \"step\": %lld, \"hash\": \"%016llx\", "
                     "\"sum\": %.17g, \"min\": %.9g, \"max\": %.9g, \"count\": %lld}\n",
                     (long long)P.nx, (long long)P.ny, (long long)S.step(),
                     (unsigned long long)c.hash, c.sum, c.min, c.max, (long long)c.count);
        std::fclose(f);
      }
    } else {
      auto g = S.gather_root();
      if (root) write_dat(path, P.nx, P.ny, g.data());
    }
  };
  if (o.warmup > 0) {
    // Untimed warm-up: the segment graphs are captured and the fields
    // touched, then the initial state is restored (the graph cache stays),
    // so the timed run and the output are those of a cold run.
    HEAT_CHECK(o.resume.empty(), "--warmup with --resume");
    (void)S.run(o.warmup);
    S.reset();
  }
  if (o.dump_initial || o.naming == "mpi") emit(init_path);

  const int64_t total = S.configured_steps(o.steps);
  int64_t todo = total - S.step();
  RunStats acc;
  while (todo > 0) {
    const int64_t chunk = o.ckpt_every > 0 ? std::min(o.ckpt_every, todo) : todo;
    RunStats r = S.run(chunk);
    acc.steps_done += r.steps_done;
    acc.seconds += r.seconds;
    acc.passes += r.passes;
    acc.exchanges += r.exchanges;
    acc.checks += r.checks;
    acc.t_exchange += r.t_exchange;
    acc.t_compute += r.t_compute;
    acc.t_reduce += r.t_reduce;
    acc.last_resid = r.last_resid;
    todo -= r.steps_done;
    if (!o.checkpoint.empty() && o.ckpt_every > 0) S.write_bin(o.checkpoint);
    if (r.converged) {
      acc.converged = true;
      acc.converged_at = r.converged_at;
      break;
    }
  }
  emit(final_path);

  if (root) {
    if (P.converge) {
      if (o.naming == "mpi") {
        if (acc.converged) std::printf("Converged after %lld steps\n", (long long)(acc.converged_at - 1));
        else std::printf("Didn't converged\n");
      } else if (o.naming == "cuda") {
        if (acc.converged) std::printf("Converged at %lld steps\n", (long long)(acc.converged_at - 1));
        else std::printf("Did not converge\n");
      } else {
        if (acc.converged) std::printf("Converged after %lld steps\n", (long long)acc.converged_at);
        else std::printf("Did not converge after %lld steps\n", (long long)S.step());
      }
    }
    const double secs = acc.seconds;
    if (o.naming == "cuda") {
      const double ms = secs * 1e3;
      std::printf("Elapsed time: %.3f %ssecs\n", ms / 1000 > 1.0 ? ms / 1000 : ms,
                  ms / 1000 > 1.0 ? "" : "m");
    } else {
      std::printf("Elapsed time %f secs\n", secs);
    }
    const double cells = double(P.nx) * double(P.ny) * double(acc.steps_done);
    if (o.json) {
      const auto& c = S.cart();
      std::printf(
          "{\"nx\": %lld, \"ny\": %lld, \"steps\": %lld, \"steps_done\": %lld, \"ranks\": %d, "
          "\"backend\": \"%s\", \"decomp\": \"%dx%d\", \"tb_depth\": %d, \"seconds\": %.6f, "
          "\"mcells_per_s\": %.3f, \"s_per_1000_iters\": %.6f, \"converged\": %s, "
          "\"converged_at\": %lld, \"last_resid\": %.6g, \"passes\": %lld, \"exchanges\": %lld, "
          "\"transport\": \"%s\", \"schedule\": \"%s\", \"halo\": %d, \"t_exchange\": %.6f, "
          "\"t_compute\": %.6f, \"t_reduce\": %.6f}\n",
          (long long)P.nx, (long long)P.ny, (long long)total, (long long)acc.steps_done, world,
          P.backend == Backend::Hip ? "hip" : "cpu", c.px, c.py, S.tb_depth(), secs,
          secs > 0 ? cells / secs / 1e6 : 0.0,
          acc.steps_done > 0 ? secs * 1000.0 / double(acc.steps_done) : 0.0,
          acc.converged ? "true" : "false", (long long)acc.converged_at, double(acc.last_resid),
          (long long)acc.passes, (long long)acc.exchanges, S.transport().name(),
          schedule_name(S.schedule()), S.halo(), acc.t_exchange, acc.t_compute, acc.t_reduce);
    }
    std::fflush(stdout);
  }
  S.barrier();
}

}  // namespace

int main(int argc, char** argv) {
  Params P;
  Options o;
  std::string transport = "auto";
  int gpus = 0;
  bool backend_set = false;
  bool plan = false;
  int port = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto need = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "-h" || a == "--help") { usage(); return 0; }
    else if (a == "--nx") P.nx = std::atoll(need().c_str());
    else if (a == "--ny") P.ny = std::atoll(need().c_str());
    else if (a == "--steps") o.steps = std::atoll(need().c_str());
    else if (a == "--cx") P.cx = float(std::atof(need().c_str()));
    else if (a == "--cy") P.cy = float(std::atof(need().c_str()));
    else if (a == "--converge") P.converge = true;
    else if (a == "--check-interval") P.check_interval = std::atoi(need().c_str());
    else if (a == "--eps") P.eps = std::atof(need().c_str());
    else if (a == "--numerics") {
      std::string n = need();
      HEAT_CHECK(n == "fp32" || n == "mpi", "--numerics fp32|mpi, got %s", n.c_str());
      P.numerics = n == "mpi" ? Numerics::Mpi : Numerics::Fp32;
    }
    else if (a == "--backend") {
      std::string b = need();
      backend_set = true;
      if (b == "cpu" || b == "serial" || b == "omp") P.backend = Backend::Cpu;
      else if (b == "hip" || b == "gpu") P.backend = Backend::Hip;
      else { std::fprintf(stderr, "bad backend %s\n", b.c_str()); return 2; }
      if (b == "serial") P.threads = 1;
    } else if (a == "--threads") P.threads = std::atoi(need().c_str());
    else if (a == "--kernel") {
      std::string k = need();
      P.kernel = k == "naive" ? KernelKind::Naive
                 : k == "tb"  ? KernelKind::TB
                 : k == "lds" ? KernelKind::Lds
                 : k == "mfma" ? KernelKind::Mfma
                              : KernelKind::Auto;
    } else if (a == "--tb-depth") P.tb_depth = std::atoi(need().c_str());
    else if (a == "--decomp") {
      std::string d = need();
      P.decomp = d == "rows" || d == "1d" ? DecompKind::Rows : d == "2d" ? DecompKind::Grid2D : DecompKind::Auto;
    } else if (a == "--px") P.px = std::atoi(need().c_str());
    else if (a == "--py") P.py = std::atoi(need().c_str());
    else if (a == "--init") {
      std::string m = need();
      P.init = m == "exact" || m == "ref64" ? InitMode::Exact
               : m == "random"              ? InitMode::Random
               : m == "zero"                ? InitMode::Zero
                                            : InitMode::RefWrap;
    } else if (a == "--seed") P.seed = std::strtoull(need().c_str(), nullptr, 10);
    else if (a == "--out") o.out = need();
    else if (a == "--out-format") o.out_format = need();
    else if (a == "--naming") o.naming = need();
    else if (a == "--dump-initial") o.dump_initial = true;
    else if (a == "--compat") {
      std::string c = need();
      P.compat = c == "mpi" ? Compat::Mpi : c == "cuda" ? Compat::Cuda : Compat::None;
    } else if (a == "--no-graph") P.use_graph = false;
    else if (a == "--graph") P.use_graph = true;
    else if (a == "--no-overlap") P.overlap = false;
    else if (a == "--overlap") P.overlap = true;
    else if (a == "--schedule") {
      std::string s = need();
      P.schedule = s == "sync"       ? Schedule::Sync
                   : s == "overlap"  ? Schedule::Overlap
                   : s == "pipeline" ? Schedule::Pipeline
                                     : Schedule::Auto;
    } else if (a == "--halo-passes") P.halo_passes = std::atoi(need().c_str());
    else if (a == "--checkpoint") o.checkpoint = need();
    else if (a == "--checkpoint-every") o.ckpt_every = std::atoll(need().c_str());
    else if (a == "--resume") o.resume = need();
    else if (a == "--transport") transport = need();
    else if (a == "--watchdog") setenv("HEAT_WATCHDOG_S", need().c_str(), 1);
    else if (a == "--port") port = std::atoi(need().c_str());
    else if (a == "--json") o.json = true;
    else if (a == "--warmup") o.warmup = std::atoll(need().c_str());
    else if (a == "--gpus") gpus = std::atoi(need().c_str());
    else if (a == "--phase-timing") P.phase_timing = true;
    else if (a == "--plan") plan = true;
    else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); usage(); return 2; }
  }
  if (o.naming == "mpi" && P.compat == Compat::None) P.compat = Compat::Mpi;
  if (o.naming == "cuda" && P.compat == Compat::None) P.compat = Compat::Cuda;

  if (plan) {
    // Memory plan without allocating: the two fields of
    // every rank's block plus its ghost ring at the deepest halo the solver
    // picks (depth 12 x 8 passes per exchange = 96, or --tb-depth x
    // --halo-passes), E/W and corner halo buffers, the resident tiles'
    // exchange fields on small blocks; the worst rank decides.
    const int ranks = std::max(gpus, env_i("WORLD_SIZE", 1));
    const Cart cart(ranks, P.decomp, P.px, P.py, P.nx, P.ny);
    const int depth = P.tb_depth > 0 ? P.tb_depth : 12;
    // Passes per exchange as the solver picks them (resident-aware unless
    // --halo-passes is given; resident_halo_passes), with the host-side
    // gfx950 resident fit: whether every rank's span box runs as one-round
    // resident tiles.
    auto shape = [&](const Box& b) { return resident_shape_static(b, depth); };
    int m = 1;
    if (ranks > 1) {
      const int rm = resident_halo_passes(cart, P.nx, P.ny, depth, 8, shape);
      m = P.halo_passes > 0 ? P.halo_passes : rm >= kResMinPasses ? rm : 8;
    }
    bool resident = true;
    int res_rows = 0, res_waves = 0;
    for (int r = 0; r < ranks; ++r) {
      const Block b = make_block(cart, r, P.nx, P.ny);
      const int sh = shape(ranks > 1 ? span_box(cart, b, depth, m) : Box{0, b.lx, 0, b.ly});
      resident = resident && sh != 0;
      if (r == 0) res_rows = sh >> 8, res_waves = sh & 255;
    }
    int64_t worst = 0, worst_rank = 0;
    for (int r = 0; r < ranks; ++r) {
      const Block b = make_block(cart, r, P.nx, P.ny);
      int64_t h = int64_t(depth) * m;
      if (cart.px > 1) h = std::min<int64_t>(h, b.lx);
      if (cart.py > 1) h = std::min<int64_t>(h, b.ly);
      const Layout L = Layout::make(b.lx, b.ly, int(std::max<int64_t>(1, h)));
      int64_t bytes = 2 * L.bytes();
      // Resident workgroup tiles (blocks under 64 strip-rows per SIMD on the
      // 1024 SIMDs of an MI355X) add two exchange fields of the same layout.
      const int64_t strip = 256 - 2 * ((depth + 3) / 4 * 4);
      if ((b.ly + strip - 1) / strip * b.lx < 64 * 1024) bytes += 2 * L.bytes();
      if (cart.py > 1) bytes += 4 * b.lx * h * 4;
      if (cart.px > 1 && cart.py > 1) bytes += 8 * h * h * 4;
      if (bytes > worst) worst = bytes, worst_rank = r;
    }
    std::printf("{\"nx\": %lld, \"ny\": %lld, \"ranks\": %d, \"process_grid\": \"%dx%d\", "
                "\"bytes_per_gpu\": %lld, \"gb_per_gpu\": %.3f, \"worst_rank\": %lld, "
                "\"fits_288gb\": %s, \"tb_depth\": %d, \"halo_passes\": %d, \"halo\": %d, "
                "\"resident\": %s, \"resident_tile\": \"%dx%d\"}\n",
                (long long)P.nx, (long long)P.ny, ranks, cart.px, cart.py, (long long)worst,
                double(worst) / 1e9, (long long)worst_rank, worst < int64_t(288e9 * 0.95) ? "true" : "false",
                depth, m, depth * m, resident ? "true" : "false", resident ? res_rows : 0,
                resident ? res_waves : 0);
    return 0;
  }
  const int world = env_i("WORLD_SIZE", 1), rank = env_i("RANK", 0);
  const int local_rank = env_i("LOCAL_RANK", rank);
  const char* maddr = std::getenv("MASTER_ADDR");
  const std::string addr = maddr && *maddr ? maddr : "127.0.0.1";
  if (port == 0) port = env_i("HEAT_PORT", env_i("MASTER_PORT", 29599) + 1);

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  if (!backend_set) P.backend = ndev > 0 ? Backend::Hip : Backend::Cpu;
  if (P.backend == Backend::Hip && ndev == 0) {
    std::fprintf(stderr, "heat: --backend hip requested but no GPU is visible\n");
    return 1;
  }
  if (P.backend == Backend::Hip) P.device = local_rank % ndev;

  if (gpus > 1 && world == 1) {
    // One process, `gpus` ranks as threads, rank r on device r % ndev.  The
    // transport follows heat::choose_group_transport (shared with
    // parallel.group.run_group): RCCL -- one communicator rank per thread and
    // GPU from one unique id, the ncclCommInitAll model of SURVEY R10,
    // graph-captured exchanges -- whenever every rank has a GPU of its own;
    // the loopback transport (D2D / peer copies) only for ranks sharing one.
    if (P.backend != Backend::Hip) {
      std::fprintf(stderr, "heat: --gpus needs the hip backend\n");
      return 2;
    }
    std::vector<int> devs(static_cast<size_t>(gpus));
    for (int r = 0; r < gpus; ++r) devs[size_t(r)] = r % ndev;
    GroupTransport kind;
    try {
      kind = choose_group_transport(transport == "auto" ? "auto" : transport, gpus, devs.data());
    } catch (const std::exception& e) {
      std::fprintf(stderr, "heat: --gpus %d: %s (%d GPUs visible)\n", gpus, e.what(), ndev);
      return 2;
    }
    const bool rccl = kind == GroupTransport::Rccl;
    if (std::getenv("HEAT_VERBOSE"))
      std::fprintf(stderr, "heat: %d ranks as threads on %d GPU(s), transport %s\n", gpus, ndev,
                   group_transport_name(kind));
    unsigned char uid[128] = {0};
    LoopbackHub* hub = nullptr;
    if (rccl)
      rccl_unique_id(uid);
    else
      hub = loopback_hub_create(gpus);
    std::vector<std::thread> threads;
    std::vector<std::string> errors(gpus);
    RankRegistry reg;
    reg.solvers.assign(size_t(gpus), nullptr);
    std::mutex done_mu;
    std::condition_variable done_cv;
    int done = 0;
    bool failed = false;
    for (int r = 0; r < gpus; ++r)
      threads.emplace_back([&, r] {
        try {
          Params Pr = P;
          Pr.device = devs[size_t(r)];
          // ncclCommInitRank blocks until every rank joined: each rank
          // initialises on its own thread, concurrently.
          run_rank(o, Pr,
                   rccl ? make_rccl_transport(r, gpus, uid, Pr.device)
                        : make_loopback_transport(hub, r, Pr.device),
                   &reg);
        } catch (const std::exception& e) {
          {
            // Under the lock: the main thread reads errors[] on the
            // grace-timeout path while other ranks may still be unwinding.
            std::lock_guard<std::mutex> lk(done_mu);
            errors[r] = e.what();
            failed = true;
          }
          // Loopback peers blocked on this rank's messages throw in turn;
          // RCCL peers' solvers are aborted (their watched waits throw).
          if (hub) loopback_hub_fail(hub);
          else reg.abort_peers(r);
        }
        std::lock_guard<std::mutex> lk(done_mu);
        ++done;
        done_cv.notify_all();
      });
    {
      // After a failure every peer gets HEAT_GROUP_ABORT_S (60 s) to unwind;
      // a thread still stuck then (a wait that never polls) ends the process
      // instead of hanging it.
      std::unique_lock<std::mutex> lk(done_mu);
      done_cv.wait(lk, [&] { return done == gpus || failed; });
      if (done < gpus) {
        const double grace = std::getenv("HEAT_GROUP_ABORT_S") ? std::atof(std::getenv("HEAT_GROUP_ABORT_S")) : 60.0;
        if (!done_cv.wait_for(lk, std::chrono::duration<double>(grace), [&] { return done == gpus; })) {
          for (int r = 0; r < gpus; ++r)
            if (!errors[r].empty()) std::fprintf(stderr, "heat: rank %d error: %s\n", r, errors[r].c_str());
          std::fprintf(stderr, "heat: %d of %d ranks did not unwind within %.0f s; exiting\n",
                       gpus - done, gpus, grace);
          std::fflush(stderr);
          std::_Exit(1);
        }
      }
    }
    for (auto& t : threads) t.join();
    if (hub) loopback_hub_destroy(hub);
    // Report the failing rank, not the peers it unblocked.
    int first = -1;
    auto echo = [](const std::string& e) {
      return e.find("a peer rank failed") != std::string::npos ||
             e.find("run aborted") != std::string::npos ||
             e.find("communicator was aborted") != std::string::npos;
    };
    for (int r = 0; r < gpus && first < 0; ++r)
      if (!errors[r].empty() && !echo(errors[r])) first = r;
    for (int r = 0; r < gpus && first < 0; ++r)
      if (!errors[r].empty()) first = r;
    if (first >= 0) {
      std::fprintf(stderr, "heat: rank %d error: %s\n", first, errors[first].c_str());
      return 1;
    }
    return 0;
  }

  try {
    std::unique_ptr<Transport> tr;
    if (world == 1 || transport == "local") {
      tr = make_local_transport();
    } else if (P.backend == Backend::Hip && transport != "tcp") {
      // Rendezvous over TCP, then RCCL.
      unsigned char uid[128] = {0};
      {
        auto boot = make_tcp_transport(rank, world, addr, port);
        if (rank == 0) {
          rccl_unique_id(uid);
          std::vector<Msg> m;
          for (int r = 1; r < world; ++r) m.push_back(Msg{r, uid, 128, nullptr, 0});
          boot->sendrecv(m.data(), int(m.size()), nullptr);
        } else {
          Msg m{0, nullptr, 0, uid, 128};
          boot->sendrecv(&m, 1, nullptr);
        }
        boot->barrier();
      }
      tr = make_rccl_transport(rank, world, uid, P.device);
    } else {
      tr = make_tcp_transport(rank, world, addr, port);
    }
    run_rank(o, P, std::move(tr));
  } catch (const std::exception& e) {
    std::fprintf(stderr, "heat: error: %s\n", e.what());
    std::fflush(stderr);
    // A multi-rank failure (e.g. the watchdog aborted the communicator with
    // work still queued behind a dead peer): leave without running
    // destructors that would wait on that work.
    if (world > 1) std::_Exit(1);
    return 1;
  }
  return 0;
}
