// Inter-rank transports for halo exchange, residual all-reduce and gather.
//
// The reference does all of this with MPI: persistent
// non-blocking halo sends/receives (mpi/...c:130-161, :177, :263), one
// MPI_Allreduce(LAND) per convergence check (:255) and row-by-row
// scatter/gather through rank 0 (:100-127, :270-297).
//
// Here one process drives one GPU and the transport is pluggable:
//   LocalTransport     world of one (no messages).
//   RcclTransport      RCCL over xGMI: grouped ncclSend/ncclRecv on a comm
//                      stream, ncclAllReduce(max); device buffers,
//                      stream-ordered and hipGraph-capturable.  The unique
//                      id is produced by rank 0 and distributed by the
//                      caller (torch.distributed store or the TCP bootstrap).
//   TcpTransport       host memory over TCP sockets: the CPU multi-process
//                      backend of the standalone `heat` binary (the MPI
//                      program's role) and the RCCL bootstrap.
//   CallbackTransport  host memory; the wire is supplied by the embedding
//                      program (the Python package routes it through
//                      torch.distributed, e.g. gloo on CPU).
//   LoopbackTransport  several ranks as threads of one process, device
//                      memory, stream-ordered D2D/peer copies: tests the
//                      RCCL-shaped path on one GPU; single-process multi-GPU.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace heat {

// One peer exchange: send sbytes from sbuf to `peer` and receive rbytes
// from the same peer into rbuf.  Either side may be empty.
struct Msg {
  int peer = -1;
  const void* sbuf = nullptr;
  size_t sbytes = 0;
  void* rbuf = nullptr;
  size_t rbytes = 0;
};

// What a transport reports about itself (bench JSON, tests): for RCCL the
// communicator's own view (ncclCommCount / ncclCommCuDevice /
// ncclCommUserRank) and the PCI bus id of its device.
struct TransportInfo {
  int nranks = 0;
  int device = -1;
  int user_rank = -1;
  char bus_id[32] = {};
};

class Transport {
 public:
  virtual ~Transport() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // true: buffers are device pointers and operations are ordered on `st`
  // (asynchronous); false: host buffers, operations complete on return.
  virtual bool device_memory() const = 0;
  virtual bool graph_capturable() const { return false; }
  // All messages of one call progress concurrently (grouped).
  virtual void sendrecv(const Msg* msgs, int n, hipStream_t st) = 0;
  // In-place max over ranks of `count` floats.
  virtual void allreduce_max(float* buf, int count, hipStream_t st) = 0;
  // In-place sum over ranks of `count` doubles / uint64 (host or device per device_memory()).
  virtual void allreduce_sum_f64(double* buf, int count, hipStream_t st) = 0;
  virtual void allreduce_sum_u64(uint64_t* buf, int count, hipStream_t st) = 0;
  virtual void barrier() = 0;
  // Throws if the transport has failed asynchronously (e.g. a dead peer).
  virtual void check() {}
  // This rank gives up (e.g. a host-staged exchange failed on HIP's callback
  // thread): make peers blocked on it fail instead of waiting.  TCP shuts its
  // sockets down; the callback transport cannot reach into the embedding
  // runtime, so there a peer waits for that runtime's own timeout (gloo's,
  // bounded in bench.py by its watchdog).
  virtual void abort() {}
  // Give up without ncclCommAbort / ncclCommDestroy: both wait until every
  // graph that captured a call of the communicator is destroyed, and such a
  // graph may still be running, waiting for a dead peer.  The communicator
  // and its resources are left to process exit.
  virtual void abandon() {}
  virtual const char* name() const = 0;
  virtual TransportInfo info() const {
    TransportInfo t;
    t.nranks = world();
    t.user_rank = rank();
    return t;
  }
};

std::unique_ptr<Transport> make_local_transport();

// RCCL: `unique_id` is the 128-byte ncclUniqueId produced by rcclUniqueId()
// on rank 0 and broadcast by the caller.
std::unique_ptr<Transport> make_rccl_transport(int rank, int world, const void* unique_id,
                                               int device);
// Writes a fresh ncclUniqueId (128 bytes) into out.
void rccl_unique_id(void* out128);
// Single-rank RCCL check on `device`: self send/recv of `bytes` (eager or in
// a captured hipGraph) and an all-reduce; throws on wrong data, returns GB/s.
double rccl_self_test(int device, size_t bytes, bool graph, int iters);
// Abort while another thread issues RCCL calls, `rounds` times on a one-rank
// communicator; throws unless every round ends with the caller's calls
// refused ("aborted").  Returns the calls completed before the aborts.
int rccl_abort_race_test(int device, int rounds);

// TCP: rank 0 listens on (addr, port); everyone connects to everyone
// (full mesh, one socket per peer pair).
std::unique_ptr<Transport> make_tcp_transport(int rank, int world, const std::string& addr,
                                              int port);

// Loopback: ranks are host threads of one process sharing a hub; device
// buffers, stream-ordered device-to-device (or peer) copies.
struct LoopbackHub;
LoopbackHub* loopback_hub_create(int world);
void loopback_hub_destroy(LoopbackHub* hub);
// Marks the hub failed: every rank blocked in (or later entering) a loopback
// exchange or collective throws instead of waiting for the failed rank.
void loopback_hub_fail(LoopbackHub* hub);
std::unique_ptr<Transport> make_loopback_transport(LoopbackHub* hub, int rank, int device);

// Callback transport (C ABI so foreign runtimes can implement it).
extern "C" {
struct heat_msg {
  int peer;
  const void* sbuf;
  size_t sbytes;
  void* rbuf;
  size_t rbytes;
};
struct heat_callbacks {
  void* ctx;
  int rank;
  int world;
  // return 0 on success
  int (*sendrecv)(void* ctx, const heat_msg* msgs, int n);
  int (*allreduce)(void* ctx, void* buf, int count, int dtype /*0 f32 max, 1 f64 sum, 2 u64 sum*/);
  int (*barrier)(void* ctx);
};
}
std::unique_ptr<Transport> make_callback_transport(const heat_callbacks& cb);

// Failure injection for tests: with HEAT_TEST_FAIL_AFTER=N in the
// environment, the rank HEAT_TEST_FAIL_RANK (default 1) gets a wrapper that
// throws from its (N+1)-th sendrecv / all-reduce; every other rank (and every
// run without the variable) gets `tr` back unchanged.
std::shared_ptr<Transport> maybe_inject_faults(std::shared_ptr<Transport> tr);

// Transport of a single-process multi-rank run (`heat --gpus N`,
// parallel.group.run_group): ranks are host threads, rank r on devices[r].
// "auto": RCCL whenever every rank has a GPU of its own -- one communicator
// rank per thread from one unique id, the ncclCommInitAll process model of
// SURVEY R10 (mpi/mpi_heat_improved_persistent_stat.c:48-69 is what it
// replaces), hipGraph-capturable -- and the loopback transport (D2D / peer
// copies) only when ranks share a device, which RCCL refuses.  "rccl" /
// "loopback" force one (rccl on shared devices throws).
enum class GroupTransport : int { Rccl = 1, Loopback = 4 };
GroupTransport choose_group_transport(const std::string& requested, int world, const int* devices);
const char* group_transport_name(GroupTransport t);

}  // namespace heat
