// Local (world of one) and callback transports, the fault-injection
// wrapper used by the failure-detection tests, and the transport choice of
// single-process multi-rank runs.
#include <cstdlib>
#include <cstring>
#include <set>

#include "heat/common.hpp"
#include "heat/transport.hpp"

namespace heat {
namespace {

class LocalTransport final : public Transport {
 public:
  int rank() const override { return 0; }
  int world() const override { return 1; }
  bool device_memory() const override { return false; }
  bool graph_capturable() const override { return true; }
  void sendrecv(const Msg*, int n, hipStream_t) override {
    HEAT_CHECK(n == 0, "local transport has no peers (%d messages)", n);
  }
  void allreduce_max(float*, int, hipStream_t) override {}
  void allreduce_sum_f64(double*, int, hipStream_t) override {}
  void allreduce_sum_u64(uint64_t*, int, hipStream_t) override {}
  void barrier() override {}
  const char* name() const override { return "local"; }
};

class CallbackTransport final : public Transport {
 public:
  explicit CallbackTransport(const heat_callbacks& cb) : cb_(cb) {
    HEAT_CHECK(cb.sendrecv && cb.allreduce && cb.barrier, "callback transport: missing callback");
    HEAT_CHECK(cb.world >= 1 && cb.rank >= 0 && cb.rank < cb.world, "rank %d world %d", cb.rank,
               cb.world);
  }
  int rank() const override { return cb_.rank; }
  int world() const override { return cb_.world; }
  bool device_memory() const override { return false; }
  void sendrecv(const Msg* msgs, int n, hipStream_t) override {
    if (n == 0) return;
    std::vector<heat_msg> m(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i)
      m[i] = heat_msg{msgs[i].peer, msgs[i].sbuf, msgs[i].sbytes, msgs[i].rbuf, msgs[i].rbytes};
    HEAT_CHECK(cb_.sendrecv(cb_.ctx, m.data(), n) == 0, "callback sendrecv failed");
  }
  void allreduce_max(float* buf, int count, hipStream_t) override {
    if (cb_.world > 1) HEAT_CHECK(cb_.allreduce(cb_.ctx, buf, count, 0) == 0, "allreduce failed");
  }
  void allreduce_sum_f64(double* buf, int count, hipStream_t) override {
    if (cb_.world > 1) HEAT_CHECK(cb_.allreduce(cb_.ctx, buf, count, 1) == 0, "allreduce failed");
  }
  void allreduce_sum_u64(uint64_t* buf, int count, hipStream_t) override {
    if (cb_.world > 1) HEAT_CHECK(cb_.allreduce(cb_.ctx, buf, count, 2) == 0, "allreduce failed");
  }
  void barrier() override {
    if (cb_.world > 1) HEAT_CHECK(cb_.barrier(cb_.ctx) == 0, "barrier failed");
  }
  const char* name() const override { return "callback"; }

 private:
  heat_callbacks cb_;
};

// Forwards to `inner` and throws from the (after+1)-th message or collective
// call: a rank that dies mid-run (HEAT_TEST_FAIL_AFTER, see
// maybe_inject_faults).  Its peers then wait for messages that never come;
// what they must do is fail within their watchdog instead of hanging
// (Solver::wait_event; the reference's MPI_Allreduce, mpi/...c:255, would
// block forever).
class FaultTransport final : public Transport {
 public:
  FaultTransport(std::shared_ptr<Transport> inner, int64_t after)
      : in_(std::move(inner)), left_(after) {}
  int rank() const override { return in_->rank(); }
  int world() const override { return in_->world(); }
  bool device_memory() const override { return in_->device_memory(); }
  bool graph_capturable() const override { return in_->graph_capturable(); }
  void sendrecv(const Msg* msgs, int n, hipStream_t st) override {
    tick("sendrecv");
    in_->sendrecv(msgs, n, st);
  }
  void allreduce_max(float* buf, int count, hipStream_t st) override {
    tick("allreduce_max");
    in_->allreduce_max(buf, count, st);
  }
  void allreduce_sum_f64(double* buf, int count, hipStream_t st) override {
    tick("allreduce_sum_f64");
    in_->allreduce_sum_f64(buf, count, st);
  }
  void allreduce_sum_u64(uint64_t* buf, int count, hipStream_t st) override {
    tick("allreduce_sum_u64");
    in_->allreduce_sum_u64(buf, count, st);
  }
  void barrier() override { in_->barrier(); }
  void check() override { in_->check(); }
  void abort() override { in_->abort(); }
  void abandon() override { in_->abandon(); }
  const char* name() const override { return in_->name(); }
  TransportInfo info() const override { return in_->info(); }

 private:
  void tick(const char* what) {
    if (left_-- <= 0)
      throw_error(__FILE__, __LINE__,
                  strprintf("injected transport failure on rank %d at %s (HEAT_TEST_FAIL_AFTER)",
                            in_->rank(), what));
  }
  std::shared_ptr<Transport> in_;
  int64_t left_;
};

}  // namespace

std::shared_ptr<Transport> maybe_inject_faults(std::shared_ptr<Transport> tr) {
  const char* after = std::getenv("HEAT_TEST_FAIL_AFTER");
  if (!after || !*after || !tr) return tr;
  const char* rk = std::getenv("HEAT_TEST_FAIL_RANK");
  const int rank = rk && *rk ? std::atoi(rk) : 1;
  if (tr->rank() != rank) return tr;
  return std::make_shared<FaultTransport>(std::move(tr), std::atoll(after));
}

GroupTransport choose_group_transport(const std::string& requested, int world,
                                      const int* devices) {
  HEAT_CHECK(world >= 1 && devices != nullptr, "choose_group_transport: world %d", world);
  std::set<int> seen;
  bool own = true;  // every rank has a device of its own
  for (int r = 0; r < world; ++r) {
    HEAT_CHECK(devices[r] >= 0, "rank %d has no device (%d)", r, devices[r]);
    own = seen.insert(devices[r]).second && own;
  }
  if (requested == "loopback") return GroupTransport::Loopback;
  if (requested == "rccl") {
    HEAT_CHECK(own, "transport rccl needs one GPU per rank (RCCL refuses two ranks on one "
               "device); %d ranks share %zu device(s)", world, seen.size());
    return GroupTransport::Rccl;
  }
  HEAT_CHECK(requested == "auto" || requested.empty(),
             "unknown group transport '%s' (auto, rccl, loopback)", requested.c_str());
  return own && world > 1 ? GroupTransport::Rccl : GroupTransport::Loopback;
}

const char* group_transport_name(GroupTransport t) {
  return t == GroupTransport::Rccl ? "rccl" : "loopback";
}

std::unique_ptr<Transport> make_local_transport() { return std::make_unique<LocalTransport>(); }

std::unique_ptr<Transport> make_callback_transport(const heat_callbacks& cb) {
  return std::make_unique<CallbackTransport>(cb);
}

}  // namespace heat
