// C ABI (see capi.h).
#include "heat/capi.h"
#include "heat/plan.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstring>
#include <string>
#include <vector>

#include "heat/common.hpp"
#include "heat/cpu_backend.hpp"
#include "heat/init_fn.hpp"
#include "heat/io.hpp"
#include "heat/kernels.hpp"
#include "heat/solver.hpp"

namespace heat {

const char* init_mode_name(InitMode m) {
  switch (m) {
    case InitMode::RefWrap: return "ref-wrap";
    case InitMode::Exact: return "exact";
    case InitMode::Random: return "random";
    case InitMode::Zero: return "zero";
  }
  return "?";
}
const char* kernel_name(KernelKind k) {
  switch (k) {
    case KernelKind::Auto: return "auto";
    case KernelKind::Naive: return "naive";
    case KernelKind::TB: return "tb";
    case KernelKind::Lds: return "lds";
    case KernelKind::Mfma: return "mfma";
  }
  return "?";
}
const char* compat_name(Compat c) {
  switch (c) {
    case Compat::None: return "none";
    case Compat::Mpi: return "mpi";
    case Compat::Cuda: return "cuda";
  }
  return "?";
}

const char* schedule_name(Schedule s) {
  switch (s) {
    case Schedule::Auto: return "auto";
    case Schedule::Sync: return "sync";
    case Schedule::Overlap: return "overlap";
    case Schedule::Pipeline: return "pipeline";
  }
  return "?";
}

const char* numerics_name(Numerics n) {
  switch (n) {
    case Numerics::Fp32: return "fp32";
    case Numerics::Mpi: return "mpi";
  }
  return "?";
}

Params params_from_c(const heat_params* p) {
  Params P;
  P.nx = p->nx;
  P.ny = p->ny;
  P.cx = p->cx;
  P.cy = p->cy;
  P.converge = p->converge != 0;
  P.check_interval = p->check_interval;
  P.eps = p->eps;
  P.init = InitMode(p->init);
  P.seed = p->seed;
  P.backend = Backend(p->backend);
  P.kernel = KernelKind(p->kernel);
  P.tb_depth = p->tb_depth;
  P.threads = p->threads;
  P.decomp = DecompKind(p->decomp);
  P.px = p->px;
  P.py = p->py;
  P.use_graph = p->use_graph != 0;
  P.overlap = p->overlap != 0;
  P.compat = Compat(p->compat);
  P.device = p->device;
  P.schedule = Schedule(p->schedule);
  P.halo_passes = p->halo_passes;
  P.numerics = Numerics(p->numerics);
  P.phase_timing = p->phase_timing != 0;
  return P;
}

}  // namespace heat

struct heat_solver {
  std::unique_ptr<heat::Solver> s;
};

struct heat_transport {
  std::shared_ptr<heat::Transport> t;
  int device = -1;
};

namespace {
thread_local std::string g_err;

template <class F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown error";
  }
  return -1;
}

hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

std::shared_ptr<heat::Transport> make_transport(const heat_comm* c) {
  switch (c ? c->kind : 0) {
    case 0:
      return heat::make_local_transport();
    case 1:
      return heat::make_rccl_transport(c->rank, c->world, c->unique_id, c->device);
    case 2:
      return heat::make_tcp_transport(c->rank, c->world, c->addr ? c->addr : "127.0.0.1", c->port);
    case 3: {
      heat::heat_callbacks cb{};
      cb.ctx = c->ctx;
      cb.rank = c->rank;
      cb.world = c->world;
      cb.sendrecv = reinterpret_cast<int (*)(void*, const heat::heat_msg*, int)>(c->sendrecv);
      cb.allreduce = c->allreduce;
      cb.barrier = c->barrier;
      return heat::make_callback_transport(cb);
    }
    case 4:
      return heat::make_loopback_transport(static_cast<heat::LoopbackHub*>(c->ctx), c->rank,
                                           c->device);
    default:
      HEAT_CHECK(false, "unknown transport kind %d", c->kind);
  }
  return nullptr;
}

heat::gpu::StencilGeom geom(int64_t pitch, int64_t gx0, int64_t gy0, int64_t nx, int64_t ny,
                            float cx, float cy) {
  heat::gpu::StencilGeom g;
  g.pitch = pitch;
  g.gx0 = gx0;
  g.gy0 = gy0;
  g.nx = nx;
  g.ny = ny;
  g.cx = cx;
  g.cy = cy;
  return g;
}
}  // namespace

namespace heat::gpu {
bool tb_exp_loaded();  // stencil.hip (kernels/tb_exp.hpp)
}  // namespace heat::gpu

extern "C" {

const char* heat_last_error(void) { return g_err.c_str(); }
int heat_abi_version(void) { return HEAT_ABI_VERSION; }
const char* heat_build_info(void) {
  return "libheat: gfx950 HIP kernels (naive, tb depths 1-8), RCCL/TCP/callback transports";
}

int heat_rccl_unique_id(uint8_t out[128]) {
  return guard([&] { heat::rccl_unique_id(out); });
}

int heat_device_count(int* n) {
  return guard([&] {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
  });
}

int heat_rccl_self_test(int device, int64_t bytes, int graph, int iters, double* gbps) {
  return guard([&] { *gbps = heat::rccl_self_test(device, size_t(bytes), graph != 0, iters); });
}

int heat_rccl_abort_race_test(int device, int rounds, int* calls) {
  return guard([&] { *calls = heat::rccl_abort_race_test(device, rounds); });
}

int heat_loopback_hub_create(int world, void** out) {
  return guard([&] { *out = heat::loopback_hub_create(world); });
}

int heat_loopback_hub_destroy(void* hub) {
  return guard([&] { heat::loopback_hub_destroy(static_cast<heat::LoopbackHub*>(hub)); });
}

int heat_loopback_hub_fail(void* hub) {
  return guard([&] { heat::loopback_hub_fail(static_cast<heat::LoopbackHub*>(hub)); });
}

int heat_solver_create(const heat_params* p, const heat_comm* c, heat_solver** out) {
  return guard([&] {
    heat::Params P = heat::params_from_c(p);
    std::shared_ptr<heat::Transport> tr = make_transport(c);
    if (P.device < 0 && c && (c->kind == 1 || c->kind == 4)) P.device = c->device;
    auto* h = new heat_solver;
    try {
      h->s = std::make_unique<heat::Solver>(P, std::move(tr));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int heat_transport_create(const heat_comm* c, heat_transport** out) {
  return guard([&] {
    auto* t = new heat_transport;
    try {
      t->t = make_transport(c);
      t->device = c && (c->kind == 1 || c->kind == 4) ? c->device : -1;
    } catch (...) {
      delete t;
      throw;
    }
    *out = t;
  });
}

int heat_transport_destroy(heat_transport* t) {
  return guard([&] { delete t; });
}

int heat_transport_info_get(heat_transport* t, heat_transport_info* out) {
  return guard([&] {
    const heat::TransportInfo i = t->t->info();
    std::memset(out, 0, sizeof *out);
    out->nranks = i.nranks;
    out->device = i.device;
    out->user_rank = i.user_rank;
    std::memcpy(out->bus_id, i.bus_id, sizeof out->bus_id - 1);
    std::strncpy(out->name, t->t->name(), sizeof out->name - 1);
  });
}

int heat_solver_create_shared(const heat_params* p, heat_transport* t, heat_solver** out) {
  return guard([&] {
    HEAT_CHECK(t != nullptr && t->t != nullptr, "null transport");
    heat::Params P = heat::params_from_c(p);
    if (P.device < 0) P.device = t->device;
    auto* h = new heat_solver;
    try {
      h->s = std::make_unique<heat::Solver>(P, t->t);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

int heat_solver_destroy(heat_solver* s) {
  return guard([&] { delete s; });
}

namespace {
void fill_stats(const heat::RunStats& r, heat_run_stats* out) {
  out->steps_done = r.steps_done;
  out->total_steps = r.total_steps;
  out->converged = r.converged;
  out->converged_at = r.converged_at;
  out->last_resid = r.last_resid;
  out->seconds = r.seconds;
  out->t_exchange = r.t_exchange;
  out->t_compute = r.t_compute;
  out->t_reduce = r.t_reduce;
  out->passes = r.passes;
  out->exchanges = r.exchanges;
  out->checks = r.checks;
  out->resident_passes = r.resident_passes;
  out->resident_giveups = r.resident_giveups;
  out->chained_passes = r.chained_passes;
}
}  // namespace

int heat_solver_enqueue(heat_solver* s, int64_t steps, heat_run_stats* out) {
  return guard([&] {
    const heat::RunStats r = s->s->enqueue(steps);
    if (out) fill_stats(r, out);
  });
}

int heat_solver_run(heat_solver* s, int64_t steps, heat_run_stats* out) {
  return guard([&] {
    const heat::RunStats r = s->s->run(steps);
    if (out) fill_stats(r, out);
  });
}

int heat_solver_time_exchange(heat_solver* s, int depth, int iters, double* seconds,
                              int64_t* max_bytes) {
  return guard([&] {
    int64_t b = 0;
    const double t = s->s->time_exchange(depth, iters, &b);
    if (seconds) *seconds = t;
    if (max_bytes) *max_bytes = b;
  });
}

int heat_solver_reset(heat_solver* s) {
  return guard([&] { s->s->reset(); });
}

int heat_solver_info(heat_solver* s, heat_block_info* o) {
  return guard([&] {
    const auto& b = s->s->block();
    const auto& L = s->s->layout();
    const auto& c = s->s->cart();
    o->rank = b.rank;
    o->world = c.world;
    o->px = c.px;
    o->py = c.py;
    o->cx = b.cx;
    o->cy = b.cy;
    o->ox = b.ox;
    o->oy = b.oy;
    o->lx = b.lx;
    o->ly = b.ly;
    for (int i = 0; i < 4; ++i) o->nbr[i] = b.nbr[i];
    o->pitch = L.pitch;
    o->rows = L.rows;
    o->hx = L.hx;
    o->hy = L.hy;
    o->halo = s->s->halo();
    o->tb_depth = s->s->tb_depth();
    o->bytes_per_field = L.bytes();
    o->schedule = int32_t(s->s->schedule());
    o->pad_ = 0;
  });
}

int heat_solver_step(heat_solver* s, int64_t* out) {
  return guard([&] { *out = s->s->step(); });
}

int heat_solver_copy_owned(heat_solver* s, float* host, int64_t host_pitch) {
  return guard([&] { s->s->copy_owned(host, host_pitch); });
}

int heat_solver_load_owned(heat_solver* s, const float* host, int64_t host_pitch, int64_t step) {
  return guard([&] { s->s->load_owned(host, host_pitch, step); });
}

int heat_solver_gather(heat_solver* s, float* host) {
  return guard([&] {
    auto g = s->s->gather_root();
    if (!g.empty() && host) std::memcpy(host, g.data(), g.size() * 4);
  });
}

int heat_solver_checksum(heat_solver* s, heat_checksum* out) {
  return guard([&] {
    auto c = s->s->checksum();
    out->hash = c.hash;
    out->sum = c.sum;
    out->min = c.min;
    out->max = c.max;
    out->count = c.count;
  });
}

int heat_solver_scatter(heat_solver* s, const float* full, int64_t step) {
  return guard([&] { s->s->scatter_root(full, step); });
}

int heat_solver_write_bin(heat_solver* s, const char* path) {
  return guard([&] { s->s->write_bin(path); });
}
int heat_solver_read_bin(heat_solver* s, const char* path) {
  return guard([&] { s->s->read_bin(path); });
}
int heat_solver_barrier(heat_solver* s) {
  return guard([&] { s->s->barrier(); });
}
int heat_solver_current_ptr(heat_solver* s, void** ptr) {
  return guard([&] { *ptr = s->s->current(); });
}

int heat_write_dat(const char* path, int64_t nx, int64_t ny, const float* grid) {
  return guard([&] { heat::write_dat(path, nx, ny, grid); });
}

int heat_format_6_1f(float v, char* out, int cap) {
  return guard([&] {
    std::string s;
    heat::format_6_1f(v, s);
    HEAT_CHECK(int(s.size()) < cap, "buffer too small");
    std::memcpy(out, s.c_str(), s.size() + 1);
  });
}

int heat_dims_create(int nnodes, int ndims, int* dims) {
  return guard([&] {
    auto d = heat::dims_create(nnodes, ndims);
    for (int i = 0; i < ndims; ++i) dims[i] = d[size_t(i)];
  });
}

int heat_block_span(int64_t n, int parts, int index, int64_t* offset, int64_t* size) {
  return guard([&] {
    auto s = heat::block_span(n, parts, index);
    *offset = s.offset;
    *size = s.size;
  });
}

int heat_init_value(int mode, int64_t ix, int64_t iy, int64_t nx, int64_t ny, uint64_t seed,
                    float* out) {
  return guard([&] { *out = heat::init_value(mode, ix, iy, nx, ny, seed); });
}

int heat_cpu_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0, int64_t nx,
                  int64_t ny, float cx, float cy, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                  float* resid) {
  return guard([&] {
    heat::cpu::Geom g;
    g.pitch = pitch;
    g.gx0 = gx0;
    g.gy0 = gy0;
    g.nx = nx;
    g.ny = ny;
    g.cx = cx;
    g.cy = cy;
    float r = heat::cpu::step(src, dst, g, heat::Box{r0, r1, c0, c1}, resid != nullptr);
    if (resid) *resid = r;
  });
}

int heat_op_naive_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                       int64_t nx, int64_t ny, float cx, float cy, int64_t r0, int64_t r1,
                       int64_t c0, int64_t c1, unsigned* resid, void* stream) {
  return guard([&] {
    heat::gpu::naive_step(src, dst, geom(pitch, gx0, gy0, nx, ny, cx, cy),
                          heat::Box{r0, r1, c0, c1}, resid, S(stream));
  });
}

int heat_op_lds_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                     int64_t nx, int64_t ny, float cx, float cy, int64_t r0, int64_t r1,
                     int64_t c0, int64_t c1, unsigned* resid, void* stream, int numerics) {
  return guard([&] {
    auto g = geom(pitch, gx0, gy0, nx, ny, cx, cy);
    g.numerics = numerics;
    heat::gpu::lds_step(src, dst, g, heat::Box{r0, r1, c0, c1}, resid, S(stream));
  });
}

int heat_op_mfma_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                      int64_t nx, int64_t ny, float cx, float cy, int64_t r0, int64_t r1,
                      int64_t c0, int64_t c1, unsigned* resid, void* stream) {
  return guard([&] {
    heat::gpu::mfma_step(src, dst, geom(pitch, gx0, gy0, nx, ny, cx, cy),
                         heat::Box{r0, r1, c0, c1}, resid, S(stream));
  });
}

int heat_op_tb_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                    int64_t nx, int64_t ny, float cx, float cy, const int64_t* boxes, int nbox,
                    int depth, unsigned* resid, void* stream, int waves_target, int variant,
                    int res_level) {
  return guard([&] {
    HEAT_CHECK(nbox >= 1 && nbox <= 5, "nbox %d", nbox);
    heat::Box b[5];
    for (int i = 0; i < nbox; ++i)
      b[i] = heat::Box{boxes[4 * i], boxes[4 * i + 1], boxes[4 * i + 2], boxes[4 * i + 3]};
    heat::gpu::tb_step(src, dst, geom(pitch, gx0, gy0, nx, ny, cx, cy), b, nbox, depth, resid,
                       S(stream), waves_target, variant, res_level);
  });
}

int heat_tb_get_tuning(heat_tb_tuning* out) {
  return guard([&] {
    const heat::gpu::TbTuning t = heat::gpu::tb_tuning();
    std::memset(out, 0, sizeof *out);
    out->variant = t.variant;
    out->rounds = t.rounds;
    out->min_len = t.min_len;
    out->waves = t.waves;
    out->edge_frac = t.edge_frac;
    out->tile_rows = t.tile_rows;
    out->tile_waves = t.tile_waves;
    out->tile_xl = t.tile_xl;
    out->nt = t.nt;
    out->n_weights = int32_t(std::min<size_t>(t.age_weights.size(), 4));
    for (int i = 0; i < out->n_weights; ++i) out->weights[i] = t.age_weights[size_t(i)];
  });
}

int heat_tb_set_tuning(const heat_tb_tuning* in) {
  return guard([&] {
    HEAT_CHECK(in->n_weights >= 0 && in->n_weights <= 4, "%d age weights", in->n_weights);
    HEAT_CHECK(in->edge_frac > 0.0, "edge_frac %g", in->edge_frac);
    heat::gpu::TbTuning t;
    t.variant = in->variant;
    t.rounds = std::max(0, in->rounds);
    t.min_len = std::max(0, in->min_len);
    t.waves = std::max(0, in->waves);
    t.edge_frac = in->edge_frac;
    t.tile_rows = std::max(0, in->tile_rows);
    t.tile_waves = std::max(0, in->tile_waves);
    t.tile_xl = in->tile_xl;
    t.nt = in->nt;
    t.age_weights.assign(in->weights, in->weights + in->n_weights);
    heat::gpu::tb_set_tuning(t);
  });
}

int heat_op_tb_stamps(void* buf, int64_t waves) {
  return guard([&] { heat::gpu::tb_set_stamps(static_cast<unsigned long long*>(buf), waves); });
}

int heat_op_init(float* origin, int64_t lx, int64_t ly, int halo, int64_t gx0, int64_t gy0,
                 int64_t nx, int64_t ny, int mode, uint64_t seed, void* stream) {
  return guard([&] {
    heat::Layout L = heat::Layout::make(lx, ly, halo);
    heat::gpu::init_field(origin, L, gx0, gy0, nx, ny, mode, seed, S(stream));
  });
}

int heat_op_pack(const float* origin, int64_t pitch, int64_t r0, int64_t r1, int64_t c0,
                 int64_t c1, float* buf, void* stream) {
  return guard([&] { heat::gpu::pack_box(origin, pitch, heat::Box{r0, r1, c0, c1}, buf, S(stream)); });
}

int heat_op_unpack(const float* buf, float* origin, int64_t pitch, int64_t r0, int64_t r1,
                   int64_t c0, int64_t c1, void* stream) {
  return guard(
      [&] { heat::gpu::unpack_box(buf, origin, pitch, heat::Box{r0, r1, c0, c1}, S(stream)); });
}

int heat_op_residual(const float* a, const float* b, int64_t pitch, int64_t r0, int64_t r1,
                     int64_t c0, int64_t c1, unsigned* resid, void* stream) {
  return guard([&] {
    heat::gpu::residual_box(a, b, pitch, heat::Box{r0, r1, c0, c1}, resid, S(stream));
  });
}

int heat_layout(int64_t lx, int64_t ly, int halo, int64_t* pitch, int64_t* rows, int* hx,
                int* hy) {
  return guard([&] {
    heat::Layout L = heat::Layout::make(lx, ly, halo);
    *pitch = L.pitch;
    *rows = L.rows;
    *hx = L.hx;
    *hy = L.hy;
  });
}

int heat_tb_supported(int depth) { return heat::gpu::tb_depth_supported(depth) ? 1 : 0; }

int heat_tb_exp_loaded(void) { return heat::gpu::tb_exp_loaded() ? 1 : 0; }

int heat_resident_shape(int64_t rows, int64_t cols, int depth, int device, int32_t* shape) {
  return guard([&] {
    const heat::Box b{0, rows, 0, cols};
    *shape = device ? heat::gpu::tb_resident_shape(b, depth) : heat::resident_shape_static(b, depth);
  });
}

int heat_tb_mid_residual(int depth) { return heat::gpu::tb_mid_residual(depth) ? 1 : 0; }

int heat_group_transport(const char* requested, int world, const int32_t* devices, int32_t* kind) {
  return guard([&] {
    HEAT_CHECK(world >= 1 && devices != nullptr && kind != nullptr, "heat_group_transport: bad args");
    std::vector<int> d(devices, devices + world);
    *kind = int32_t(heat::choose_group_transport(requested ? requested : "auto", world, d.data()));
  });
}

int heat_solver_abort(heat_solver* s) {
  return guard([&] {
    HEAT_CHECK(s && s->s, "null solver");
    s->s->abort();
  });
}

}  // extern "C"
