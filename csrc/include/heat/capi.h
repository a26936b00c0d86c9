/* C ABI of libheat.so — consumed by the Python package (ctypes) and usable
 * from any language.  All functions return 0 on success and -1 on error;
 * heat_last_error() then returns a thread-local message.
 *
 * Two layers:
 *   heat_solver_*  the full per-rank engine (fields, passes, exchange, graphs)
 *   heat_op_*      single kernels on caller-owned device buffers, for tests
 *                  and for composing custom schedules (stream = hipStream_t).
 */
#ifndef HEAT_CAPI_H
#define HEAT_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HEAT_ABI_VERSION 5

typedef struct heat_params {
  int64_t nx, ny;
  float cx, cy;
  int32_t converge, check_interval;
  double eps;
  int32_t init;      /* heat::InitMode */
  uint64_t seed;
  int32_t backend;   /* 0 cpu, 1 hip */
  int32_t kernel;    /* 0 auto, 1 naive, 2 tb */
  int32_t tb_depth;
  int32_t threads;
  int32_t decomp;    /* 0 auto(2-D), 1 rows, 2 grid2d */
  int32_t px, py;
  int32_t use_graph, overlap;
  int32_t compat;    /* 0 none, 1 mpi, 2 cuda */
  int32_t device;
  int32_t schedule;    /* 0 auto, 1 sync, 2 overlap (exchange-first), 3 pipeline */
  int32_t halo_passes; /* sync schedule: passes per exchange (0 = auto) */
  int32_t numerics;    /* 0 fp32 (canonical FMA), 1 mpi (reference MPI double arithmetic) */
  int32_t phase_timing;/* 1: per-phase times in heat_run_stats (disables graphs) */
} heat_params;

/* Transport selection for heat_solver_create. */
typedef struct heat_comm {
  int32_t kind;          /* 0 local, 1 rccl, 2 tcp, 3 callback, 4 loopback (ctx = hub) */
  int32_t rank, world;
  int32_t device;        /* rccl: HIP device */
  uint8_t unique_id[128];/* rccl: ncclUniqueId from heat_rccl_unique_id on rank 0 */
  const char* addr;      /* tcp: rank-0 address */
  int32_t port;          /* tcp: rank-0 port */
  /* callback transport */
  void* ctx;
  int (*sendrecv)(void* ctx, const void* msgs /* heat_msg[n] */, int n);
  int (*allreduce)(void* ctx, void* buf, int count, int dtype);
  int (*barrier)(void* ctx);
} heat_comm;

typedef struct heat_run_stats {
  int64_t steps_done, total_steps;
  int32_t converged;
  int64_t converged_at;
  float last_resid;
  double seconds;
  int64_t passes, exchanges, checks;
  double t_exchange, t_compute, t_reduce; /* seconds per phase (phase_timing) */
  int64_t resident_passes;                /* passes run inside resident-tile launches */
  int64_t resident_giveups;               /* 1: a resident launch gave up (HEAT_TB_RES_GIVEUP=defer) */
  int64_t chained_passes;                 /* passes run inside chained level-split launches */
} heat_run_stats;

typedef struct heat_block_info {
  int32_t rank, world, px, py, cx, cy;
  int64_t ox, oy, lx, ly;
  int32_t nbr[4]; /* north, south, west, east; -1 = none */
  int64_t pitch, rows;
  int32_t hx, hy, halo, tb_depth;
  int64_t bytes_per_field;
  int32_t schedule; /* effective heat::Schedule (1 sync, 2 overlap, 3 pipeline) */
  int32_t pad_;
} heat_block_info;

typedef struct heat_checksum {
  uint64_t hash;
  double sum, min, max;
  int64_t count;
} heat_checksum;

typedef struct heat_solver heat_solver;
typedef struct heat_transport heat_transport;

typedef struct heat_transport_info {
  int32_t nranks;      /* rccl: ncclCommCount; else the world size */
  int32_t device;      /* rccl: ncclCommCuDevice; else -1 */
  int32_t user_rank;   /* rccl: ncclCommUserRank; else the rank */
  char bus_id[32];     /* PCI bus id of `device` ("" if unknown) */
  char name[16];       /* transport name */
} heat_transport_info;

const char* heat_last_error(void);
int heat_abi_version(void);
const char* heat_build_info(void);

int heat_rccl_unique_id(uint8_t out[128]);
int heat_device_count(int* n);

int heat_solver_create(const heat_params* p, const heat_comm* c, heat_solver** out);
/* A transport (e.g. one RCCL communicator) that several solvers use in turn:
 * each solver keeps a reference, so destroying the handle early is safe. */
int heat_transport_create(const heat_comm* c, heat_transport** out);
int heat_transport_destroy(heat_transport* t);
int heat_transport_info_get(heat_transport* t, heat_transport_info* out);
int heat_solver_create_shared(const heat_params* p, heat_transport* t, heat_solver** out);
int heat_solver_destroy(heat_solver* s);
int heat_solver_run(heat_solver* s, int64_t steps, heat_run_stats* out);
/* Asynchronous run (plain GPU runs): enqueue the steps and return; the next
   heat_solver_run (steps 0: just complete) waits for them and checks errors. */
int heat_solver_enqueue(heat_solver* s, int64_t steps, heat_run_stats* out);
/* RCCL on one rank: self send/recv (eager or hipGraph-captured) + all-reduce. */
int heat_rccl_self_test(int device, int64_t bytes, int graph, int iters, double* gbps);
/* RCCL abort while another thread issues calls on the communicator (one-rank
   communicators, `rounds` rounds); *calls = calls completed before the aborts. */
int heat_rccl_abort_race_test(int device, int rounds, int* calls);
/* Loopback transport: ranks are threads of this process sharing one hub. */
int heat_loopback_hub_create(int world, void** out);
int heat_loopback_hub_destroy(void* hub);
/* A rank of the hub failed: peers blocked in an exchange or collective throw. */
int heat_loopback_hub_fail(void* hub);
/* Transport of a single-process multi-rank run (ranks = threads, rank r on
   devices[r]): requested "auto" | "rccl" | "loopback"; *kind = 1 (rccl: every
   rank has a GPU of its own) or 4 (loopback: ranks share a device).  The rule
   of heat::choose_group_transport, shared by `heat --gpus N` and
   parallel.group.run_group. */
int heat_group_transport(const char* requested, int world, const int32_t* devices, int32_t* kind);
/* Give up this rank: abort its transport (ncclCommAbort) so peers stop
   waiting; a wait of the solver on another thread throws.  Thread-safe. */
int heat_solver_abort(heat_solver* s);
/* Seconds per grouped halo exchange of `depth` rows/columns on this rank
   (device time over `iters` exchanges) and its largest message; collective. */
int heat_solver_time_exchange(heat_solver* s, int depth, int iters, double* seconds,
                              int64_t* max_bytes);
/* 1 if the automatic TB variant at `depth` takes a residual at any inner step
   (checks ride inside full-depth passes), else 0. */
int heat_tb_mid_residual(int depth);
int heat_solver_reset(heat_solver* s);
int heat_solver_info(heat_solver* s, heat_block_info* out);
int heat_solver_step(heat_solver* s, int64_t* out);
int heat_solver_copy_owned(heat_solver* s, float* host, int64_t host_pitch);
int heat_solver_load_owned(heat_solver* s, const float* host, int64_t host_pitch, int64_t step);
/* rank 0: host must hold nx*ny floats; other ranks: host may be NULL */
int heat_solver_gather(heat_solver* s, float* host);
int heat_solver_checksum(heat_solver* s, heat_checksum* out);
/* rank 0: full holds nx*ny floats (row-major); other ranks: full may be NULL */
int heat_solver_scatter(heat_solver* s, const float* full, int64_t step);
int heat_solver_write_bin(heat_solver* s, const char* path);
int heat_solver_read_bin(heat_solver* s, const char* path);
int heat_solver_barrier(heat_solver* s);
int heat_solver_current_ptr(heat_solver* s, void** ptr);

/* host utilities */
int heat_write_dat(const char* path, int64_t nx, int64_t ny, const float* grid);
int heat_format_6_1f(float v, char* out, int cap);
int heat_dims_create(int nnodes, int ndims, int* dims);
int heat_block_span(int64_t n, int parts, int index, int64_t* offset, int64_t* size);
int heat_init_value(int mode, int64_t ix, int64_t iy, int64_t nx, int64_t ny, uint64_t seed,
                    float* out);
int heat_cpu_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0, int64_t nx,
                  int64_t ny, float cx, float cy, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                  float* resid /* may be NULL */);

/* device ops (pointers are device pointers to local cell (0,0); stream is a hipStream_t) */
int heat_op_naive_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                       int64_t nx, int64_t ny, float cx, float cy, int64_t r0, int64_t r1,
                       int64_t c0, int64_t c1, unsigned* resid, void* stream);
int heat_op_lds_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                     int64_t nx, int64_t ny, float cx, float cy, int64_t r0, int64_t r1,
                     int64_t c0, int64_t c1, unsigned* resid, void* stream, int numerics);
int heat_op_mfma_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                      int64_t nx, int64_t ny, float cx, float cy, int64_t r0, int64_t r1,
                      int64_t c0, int64_t c1, unsigned* resid, void* stream);
// Diagnostics: per-wave start/end clock stamps of subsequent TB launches
// (4 u64 per wave: start, end at 100 MHz, block, strip<<32|chunk); null = off.
int heat_op_tb_stamps(void* buf, int64_t waves);
int heat_op_tb_step(const float* src, float* dst, int64_t pitch, int64_t gx0, int64_t gy0,
                    int64_t nx, int64_t ny, float cx, float cy, const int64_t* boxes /* nbox*4 */,
                    int nbox, int depth, unsigned* resid, void* stream, int waves_target,
                    int variant /* -1 default; heat::gpu::tbv flags */,
                    int res_level /* residual step 1..depth, 0 = depth */);
/* TB launch-planner knobs (heat::gpu::TbTuning); weights: up to 4 age-group shares;
   tile_rows / tile_waves: rows per wave / waves per workgroup of tile launches
   (0 = planner); tile_xl: tile lane shifts 0 DPP, 1 ds_bpermute, 2 mixed (-1 = default);
   nt: level-split rows non-temporal 1 / plain 0 (-1 = by the bytes a pass sweeps). */
typedef struct heat_tb_tuning {
  int32_t variant, rounds, min_len, waves;
  double edge_frac;
  int32_t n_weights, tile_rows;
  double weights[4];
  int32_t tile_waves, tile_xl;
  int32_t nt, pad_;
} heat_tb_tuning;
int heat_tb_get_tuning(heat_tb_tuning* out);
int heat_tb_set_tuning(const heat_tb_tuning* in);
int heat_op_init(float* origin, int64_t lx, int64_t ly, int halo, int64_t gx0, int64_t gy0,
                 int64_t nx, int64_t ny, int mode, uint64_t seed, void* stream);
int heat_op_pack(const float* origin, int64_t pitch, int64_t r0, int64_t r1, int64_t c0,
                 int64_t c1, float* buf, void* stream);
int heat_op_unpack(const float* buf, float* origin, int64_t pitch, int64_t r0, int64_t r1,
                   int64_t c0, int64_t c1, void* stream);
int heat_op_residual(const float* a, const float* b, int64_t pitch, int64_t r0, int64_t r1,
                     int64_t c0, int64_t c1, unsigned* resid, void* stream);
int heat_layout(int64_t lx, int64_t ly, int halo, int64_t* pitch, int64_t* rows, int* hx,
                int* hy);
int heat_tb_supported(int depth);
/* 1 once libheat_exp.so (the experiment kernels, `make exp`) has registered them. */
int heat_tb_exp_loaded(void);
/* The resident tile plan of a rows x cols box at `depth` as rows << 8 | waves
   (0: none): the device planner (device = 1, needs a GPU) or its host mirror
   (device = 0, what `heat --plan` uses). */
int heat_resident_shape(int64_t rows, int64_t cols, int depth, int device, int32_t* shape);

#ifdef __cplusplus
}
#endif

#endif /* HEAT_CAPI_H */
