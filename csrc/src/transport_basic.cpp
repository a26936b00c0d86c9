// Local (world of one) and callback transports.
#include <cstring>

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

}  // namespace

std::unique_ptr<Transport> make_local_transport() { return std::make_unique<LocalTransport>(); }

std::unique_ptr<Transport> make_callback_transport(const heat_callbacks& cb) {
  return std::make_unique<CallbackTransport>(cb);
}

}  // namespace heat
