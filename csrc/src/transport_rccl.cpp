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

#include <cstring>

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
    if (scratch_) (void)hipFree(scratch_);
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool device_memory() const override { return true; }
  bool graph_capturable() const override { return true; }

  void sendrecv(const Msg* msgs, int n, hipStream_t st) override {
    if (n == 0) return;
    NCCL_CHECK(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
      const Msg& m = msgs[i];
      if (m.sbytes) NCCL_CHECK(ncclSend(m.sbuf, m.sbytes / 4, ncclFloat, m.peer, comm_, st));
      if (m.rbytes) NCCL_CHECK(ncclRecv(m.rbuf, m.rbytes / 4, ncclFloat, m.peer, comm_, st));
    }
    NCCL_CHECK(ncclGroupEnd());
  }
  void allreduce_max(float* buf, int count, hipStream_t st) override {
    if (world_ > 1) NCCL_CHECK(ncclAllReduce(buf, buf, size_t(count), ncclFloat, ncclMax, comm_, st));
  }
  void allreduce_sum_f64(double* buf, int count, hipStream_t st) override {
    if (world_ > 1)
      NCCL_CHECK(ncclAllReduce(buf, buf, size_t(count), ncclFloat64, ncclSum, comm_, st));
  }
  void allreduce_sum_u64(uint64_t* buf, int count, hipStream_t st) override {
    if (world_ > 1)
      NCCL_CHECK(ncclAllReduce(buf, buf, size_t(count), ncclUint64, ncclSum, comm_, st));
  }
  void barrier() override {
    if (world_ == 1) return;
    // A one-element all-reduce on a private stream, then wait for it.
    hipStream_t st;
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    NCCL_CHECK(ncclAllReduce(scratch_, scratch_, 1, ncclFloat, ncclMax, comm_, st));
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipStreamDestroy(st));
  }
  void check() override {
    ncclResult_t async = ncclSuccess;
    NCCL_CHECK(ncclCommGetAsyncError(comm_, &async));
    if (async != ncclSuccess && async != ncclInProgress)
      throw_error(__FILE__, __LINE__,
                  std::string("RCCL asynchronous error: ") + ncclGetErrorString(async));
  }
  const char* name() const override { return "rccl"; }

 private:
  int rank_, world_;
  ncclComm_t comm_ = nullptr;
  float* scratch_ = nullptr;
};

}  // namespace

std::unique_ptr<Transport> make_rccl_transport(int rank, int world, const void* unique_id,
                                               int device) {
  return std::make_unique<RcclTransport>(rank, world, unique_id, device);
}

void rccl_unique_id(void* out128) {
  ncclUniqueId id;
  NCCL_CHECK(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, sizeof id);
}

}  // namespace heat
