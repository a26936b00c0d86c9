// RCCL transport over xGMI (one process per GPU).
//
// Replaces the reference's MPI point-to-point halo exchange and
// MPI_Allreduce (mpi/mpi_heat_improved_persistent_stat.c:130-161, :255).
// All sends/receives of one exchange phase are issued inside one
// ncclGroupStart/End so they progress concurrently over distinct xGMI links
// (on an MI355X node every neighbour pair is one direct hop).  Calls are
// stream-ordered and legal inside hipStreamBeginCapture, so the solver can
// capture whole step chunks, exchanges included, into one hipGraph.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "heat/common.hpp"
#include "heat/transport.hpp"

#define NCCL_CHECK(expr)                                                                       \
  do {                                                                                         \
    ncclResult_t r__ = (expr);                                                                 \
    if (r__ != ncclSuccess)                                                                    \
      ::heat::throw_error(__FILE__, __LINE__, std::string(#expr " -> ") + ncclGetErrorString(r__)); \
  } while (0)

namespace heat {
namespace {

static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");

class RcclTransport final : public Transport {
 public:
  RcclTransport(int rank, int world, const void* uid, int device) : rank_(rank), world_(world) {
    HIP_CHECK(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof id);
    NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
    HIP_CHECK(hipMalloc(&scratch_, 64));
  }
  ~RcclTransport() override {
    if (abandoned_) return;
    if (scratch_) (void)hipFree(scratch_);
    std::lock_guard<std::mutex> lk(mu_);
    if (comm_ && !aborted_.load()) (void)ncclCommDestroy(comm_);
  }
  void abandon() override { abandoned_ = true; }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool device_memory() const override { return true; }
  bool graph_capturable() const override { return true; }

  // Every call holds mu_ (calls are serialised) and is a Call: it announces
  // itself in inflight_, then re-checks aborted_ before touching comm_.
  // abort() may come from another thread (a failing rank of a
  // single-process group, or a solver's watchdog) and frees comm_ in
  // ncclCommAbort; it sets aborted_ first, then looks at inflight_ (both
  // sequentially consistent: either the call sees aborted_ and throws
  // without using comm_, or abort sees the call), so no call STARTS on a
  // freed communicator.
  void sendrecv(const Msg* msgs, int n, hipStream_t st) override {
    if (n == 0) return;
    Call c(*this);
    NCCL_CHECK(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
      const Msg& m = msgs[i];
      if (m.sbytes) NCCL_CHECK(ncclSend(m.sbuf, m.sbytes / 4, ncclFloat, m.peer, comm_, st));
      if (m.rbytes) NCCL_CHECK(ncclRecv(m.rbuf, m.rbytes / 4, ncclFloat, m.peer, comm_, st));
    }
    NCCL_CHECK(ncclGroupEnd());
  }
  void allreduce_max(float* buf, int count, hipStream_t st) override {
    Call c(*this);
    NCCL_CHECK(ncclAllReduce(buf, buf, size_t(count), ncclFloat, ncclMax, comm_, st));
  }
  void allreduce_sum_f64(double* buf, int count, hipStream_t st) override {
    Call c(*this);
    NCCL_CHECK(ncclAllReduce(buf, buf, size_t(count), ncclFloat64, ncclSum, comm_, st));
  }
  void allreduce_sum_u64(uint64_t* buf, int count, hipStream_t st) override {
    Call c(*this);
    NCCL_CHECK(ncclAllReduce(buf, buf, size_t(count), ncclUint64, ncclSum, comm_, st));
  }
  void barrier() override {
    if (world_ == 1) return;
    // A one-element all-reduce on a private stream, then wait for it.
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    {
      Call c(*this);
      NCCL_CHECK(ncclAllReduce(scratch_, scratch_, 1, ncclFloat, ncclMax, comm_, st));
    }
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipStreamDestroy(st));
  }
  void check() override {
    Call c(*this);
    ncclResult_t async = ncclSuccess;
    NCCL_CHECK(ncclCommGetAsyncError(comm_, &async));
    if (async != ncclSuccess && async != ncclInProgress)
      throw_error(__FILE__, __LINE__,
                  std::string("RCCL asynchronous error: ") + ncclGetErrorString(async));
  }
  // ncclCommAbort: RCCL's kernels and proxy threads stop waiting for peers
  // that will never answer; later calls throw.  Idempotent.  Not under mu_:
  // a peer thread of a single-process group can hold it while blocked in
  // ncclGroupEnd waiting for the dead rank, and the abort is what unblocks
  // it (ncclCommAbort is meant to be called from another thread).  Calls
  // already inside RCCL get kAbortGraceMs to leave; one still inside then is
  // blocked in its LAST RCCL call (ncclGroupEnd / ncclAllReduce: the enqueue
  // calls before them do not wait on peers), which the abort ends with an
  // error, so it issues no further call on the freed communicator.
  void abort() override {
    if (aborted_.exchange(true)) return;
    for (int i = 0; i < kAbortGraceMs && inflight_.load() > 0; ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (comm_) (void)ncclCommAbort(comm_);
  }
  const char* name() const override { return "rccl"; }
  TransportInfo info() const override {
    Call c(*this);
    TransportInfo t;
    NCCL_CHECK(ncclCommCount(comm_, &t.nranks));
    NCCL_CHECK(ncclCommCuDevice(comm_, &t.device));
    NCCL_CHECK(ncclCommUserRank(comm_, &t.user_rank));
    if (hipDeviceGetPCIBusId(t.bus_id, int(sizeof t.bus_id), t.device) != hipSuccess)
      t.bus_id[0] = 0;
    return t;
  }

 private:
  static constexpr int kAbortGraceMs = 200;
  // One RCCL call: mu_ held, announced in inflight_, aborted_ re-checked.
  struct Call {
    const RcclTransport& t;
    std::lock_guard<std::mutex> lk;
    explicit Call(const RcclTransport& tr) : t(tr), lk(tr.mu_) {
      t.inflight_.fetch_add(1);
      if (!t.comm_ || t.aborted_.load()) {
        t.inflight_.fetch_sub(1);
        throw_error(__FILE__, __LINE__, "RCCL communicator was aborted");
      }
    }
    ~Call() { t.inflight_.fetch_sub(1); }
  };
  int rank_, world_;
  mutable std::mutex mu_;
  mutable std::atomic<int> inflight_{0};
  std::atomic<bool> abandoned_{false}, aborted_{false};
  ncclComm_t comm_ = nullptr;
  float* scratch_ = nullptr;
};

}  // namespace

std::unique_ptr<Transport> make_rccl_transport(int rank, int world, const void* unique_id,
                                               int device) {
  return std::make_unique<RcclTransport>(rank, world, unique_id, device);
}

double rccl_self_test(int device, size_t bytes, bool graph, int iters) {
  // One-rank communicator; rank 0 sends to and receives from itself inside
  // ncclGroupStart/End, eagerly or as a captured hipGraph, then a max
  // all-reduce.  Checks the bytes and returns the achieved GB/s.
  HIP_CHECK(hipSetDevice(device));
  unsigned char uid[128];
  rccl_unique_id(uid);
  auto tr = make_rccl_transport(0, 1, uid, device);
  const size_t n = std::max<size_t>(bytes / 4, 1);
  float *a = nullptr, *b = nullptr;
  HIP_CHECK(hipMalloc(&a, std::max<size_t>(n * 4, 256)));
  HIP_CHECK(hipMalloc(&b, std::max<size_t>(n * 4, 256)));
  std::vector<float> h(n), back(n);
  for (size_t i = 0; i < n; ++i) h[i] = float(i % 9973) * 0.5f;
  HIP_CHECK(hipMemcpy(a, h.data(), n * 4, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemset(b, 0, n * 4));
  hipStream_t st;
  HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Msg m{0, a, n * 4, b, n * 4};
  hipGraphExec_t exec = nullptr;
  if (graph) {
    tr->sendrecv(&m, 1, st);  // connect outside capture
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipMemset(b, 0, n * 4));
    hipGraph_t g;
    HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    tr->sendrecv(&m, 1, st);
    HIP_CHECK(hipStreamEndCapture(st, &g));
    HIP_CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
  }
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  HIP_CHECK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) {
    if (exec) HIP_CHECK(hipGraphLaunch(exec, st));
    else tr->sendrecv(&m, 1, st);
  }
  HIP_CHECK(hipEventRecord(e1, st));
  HIP_CHECK(hipStreamSynchronize(st));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  tr->check();
  HIP_CHECK(hipMemcpy(back.data(), b, n * 4, hipMemcpyDeviceToHost));
  const bool ok = std::memcmp(back.data(), h.data(), n * 4) == 0;
  // all-reduces on one rank are the identity
  tr->allreduce_max(a, 4, st);
  tr->allreduce_sum_f64(reinterpret_cast<double*>(b), 2, st);
  HIP_CHECK(hipStreamSynchronize(st));
  float first[4];
  HIP_CHECK(hipMemcpy(first, a, sizeof first, hipMemcpyDeviceToHost));
  const bool ok_ar = std::memcmp(first, h.data(), std::min(n, size_t(4)) * 4) == 0;
  if (exec) (void)hipGraphExecDestroy(exec);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipStreamDestroy(st);
  (void)hipFree(a);
  (void)hipFree(b);
  HEAT_CHECK(ok, "RCCL self send/recv delivered wrong bytes");
  HEAT_CHECK(ok_ar, "RCCL all-reduce on one rank changed the data");
  return double(bytes) * iters / (double(ms) * 1e-3) / 1e9;
}

int rccl_abort_race_test(int device, int rounds) {
  // abort() used to free the communicator while another thread
  // could be between its live() check and its next RCCL call.  Each round:
  // a one-rank communicator, a thread issuing self send/recv and all-reduces
  // back to back, an abort from this thread while it runs.  The caller
  // thread must end with "aborted" errors only (no crash, no hang); returns
  // the calls the worker completed over all rounds.
  HIP_CHECK(hipSetDevice(device));
  float* buf = nullptr;
  HIP_CHECK(hipMalloc(&buf, 1 << 16));
  hipStream_t st;
  HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int done_calls = 0;
  for (int r = 0; r < rounds; ++r) {
    unsigned char uid[128];
    rccl_unique_id(uid);
    auto tr = make_rccl_transport(0, 1, uid, device);
    std::atomic<bool> started{false};
    std::string err;
    int calls = 0;
    std::thread worker([&] {
      (void)hipSetDevice(device);
      Msg m{0, buf, 4096, buf + 4096, 4096};
      try {
        for (;;) {
          tr->sendrecv(&m, 1, st);
          tr->allreduce_max(buf + 8192, 16, st);
          ++calls;
          started = true;
        }
      } catch (const std::exception& e) {
        err = e.what();
      }
    });
    while (!started.load()) std::this_thread::sleep_for(std::chrono::microseconds(50));
    std::this_thread::sleep_for(std::chrono::microseconds(200 * (r % 5)));
    tr->abort();
    worker.join();
    (void)hipStreamSynchronize(st);  // an aborted communicator's kernels end with errors
    (void)hipGetLastError();
    HEAT_CHECK(err.find("aborted") != std::string::npos || err.find("RCCL") != std::string::npos,
               "round %d: worker ended with '%s'", r, err.c_str());
    done_calls += calls;
  }
  (void)hipStreamDestroy(st);
  (void)hipFree(buf);
  return done_calls;
}

void rccl_unique_id(void* out128) {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof id);
}

}  // namespace heat
