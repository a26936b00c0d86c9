// Loopback transport: several ranks in ONE process (one host thread each),
// device buffers, messages moved by stream-ordered device-to-device copies.
//
// Purpose (SURVEY §4 "decomposition invariance (1 GPU)"): RCCL refuses two
// ranks on one device, so this is how the device-memory exchange path of the
// solver (the one RCCL takes: non-staged, comm stream, events, all three pass
// schedules) runs with real concurrency on a single MI355X.  With ranks on
// different devices the copies are peer copies over xGMI, which makes it a
// single-process multi-GPU mode as well.
//
// Semantics of one sendrecv(msgs) on rank A (all host threads do the same
// sequence of calls, so per (src, dst) pair the posts match FIFO):
//   1. post every send: {buffer, bytes, event recorded on A's stream};
//   2. for every receive from P: wait (host) for P's post, make A's stream
//      wait on its event, copy into the receive buffer on A's stream, record
//      a "consumed" event and hand it back;
//   3. make A's stream wait on the "consumed" event of each of A's sends, so
//      A cannot overwrite a send buffer before the peer's copy has run.
// Collectives are host-side (synchronise, reduce under the hub lock, copy
// back); they run at check points only.  Not graph-capturable (events cross
// other threads' captures), so the solver runs these ranks eagerly.
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <vector>

#include "heat/common.hpp"
#include "heat/transport.hpp"

namespace heat {

struct LoopbackHub {
  explicit LoopbackHub(int w) : world(w), box(size_t(w) * size_t(w)) {}

  // Shared by sender and receiver; the events go with the last reference
  // (both sides have enqueued their waits on them by then).
  struct Post {
    const void* buf = nullptr;
    size_t bytes = 0;
    int device = -1;
    hipEvent_t ready = nullptr;
    hipEvent_t consumed = nullptr;
    bool done = false;
    ~Post() {
      if (ready) (void)hipEventDestroy(ready);
      if (consumed) (void)hipEventDestroy(consumed);
    }
  };
  const int world;
  // Set when a rank fails (loopback_hub_fail): every blocked or later wait
  // throws instead of waiting forever for a peer that will never post.
  bool failed = false;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::deque<std::shared_ptr<Post>>> box;  // [src * world + dst]

  // Generation-counted all-reduce / barrier on host values.
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<double> acc_f;
  std::vector<uint64_t> acc_u;
  std::vector<double> result_f;
  std::vector<uint64_t> result_u;

  template <class F>
  void collective(F&& combine_mine, std::unique_lock<std::mutex>& lk) {
    const uint64_t gen = generation;
    combine_mine(arrived == 0);
    if (++arrived == world) {
      result_f = acc_f;
      result_u = acc_u;
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      wait(lk, [&] { return generation != gen; });
    }
  }

  // cv.wait that gives up once a peer rank has failed.
  template <class Pred>
  void wait(std::unique_lock<std::mutex>& lk, Pred pred) {
    cv.wait(lk, [&] { return failed || pred(); });
    if (!pred()) throw_error(__FILE__, __LINE__, "loopback: a peer rank failed");
  }
};

namespace {

class LoopbackTransport final : public Transport {
 public:
  LoopbackTransport(LoopbackHub* hub, int rank, int device) : hub_(hub), rank_(rank), dev_(device) {
    HEAT_CHECK(hub_ != nullptr && rank >= 0 && rank < hub_->world, "loopback rank %d", rank);
    if (dev_ >= 0) HIP_CHECK(hipSetDevice(dev_));
  }
  int rank() const override { return rank_; }
  int world() const override { return hub_->world; }
  bool device_memory() const override { return true; }
  bool graph_capturable() const override { return false; }
  const char* name() const override { return "loopback"; }

  void sendrecv(const Msg* msgs, int n, hipStream_t st) override {
    std::vector<std::shared_ptr<LoopbackHub::Post>> mine;
    {
      std::lock_guard<std::mutex> lk(hub_->mu);
      for (int i = 0; i < n; ++i) {
        if (!msgs[i].sbytes) continue;
        auto p = std::make_shared<LoopbackHub::Post>();
        p->buf = msgs[i].sbuf;
        p->bytes = msgs[i].sbytes;
        p->device = dev_;
        HIP_CHECK(hipEventCreateWithFlags(&p->ready, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(p->ready, st));
        hub_->box[size_t(rank_) * hub_->world + msgs[i].peer].push_back(p);
        mine.push_back(p);
      }
    }
    hub_->cv.notify_all();
    for (int i = 0; i < n; ++i) {
      if (!msgs[i].rbytes) continue;
      std::shared_ptr<LoopbackHub::Post> p;
      {
        std::unique_lock<std::mutex> lk(hub_->mu);
        auto& q = hub_->box[size_t(msgs[i].peer) * hub_->world + rank_];
        hub_->wait(lk, [&] { return !q.empty(); });
        p = q.front();
        q.pop_front();
      }
      HEAT_CHECK(p->bytes == msgs[i].rbytes, "loopback: %zu bytes sent, %zu expected", p->bytes,
                 msgs[i].rbytes);
      if (p->device >= 0 && dev_ >= 0 && p->device != dev_) enable_peer(p->device);
      HIP_CHECK(hipStreamWaitEvent(st, p->ready, 0));
      HIP_CHECK(hipMemcpyAsync(msgs[i].rbuf, p->buf, p->bytes, hipMemcpyDefault, st));
      hipEvent_t consumed;
      HIP_CHECK(hipEventCreateWithFlags(&consumed, hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(consumed, st));
      {
        std::lock_guard<std::mutex> lk(hub_->mu);
        p->consumed = consumed;
        p->done = true;
      }
      hub_->cv.notify_all();
    }
    for (auto& p : mine) {
      {
        std::unique_lock<std::mutex> lk(hub_->mu);
        hub_->wait(lk, [&] { return p->done; });
      }
      HIP_CHECK(hipStreamWaitEvent(st, p->consumed, 0));
    }
  }

  void allreduce_max(float* buf, int count, hipStream_t st) override {
    reduce(buf, count, st, 4, [&](std::vector<double>& acc, const void* v, bool first) {
      const float* f = static_cast<const float*>(v);
      for (int i = 0; i < count; ++i) {
        // NaN-propagating max, as the device residual is (float bits).
        const double x = f[i];
        acc[i] = first ? x : (std::isnan(acc[i]) || std::isnan(x)) ? NAN : std::max(acc[i], x);
      }
    }, [&](const std::vector<double>& r, void* v) {
      float* f = static_cast<float*>(v);
      for (int i = 0; i < count; ++i) f[i] = float(r[i]);
    });
  }
  void allreduce_sum_f64(double* buf, int count, hipStream_t st) override {
    reduce(buf, count, st, 8, [&](std::vector<double>& acc, const void* v, bool first) {
      const double* d = static_cast<const double*>(v);
      for (int i = 0; i < count; ++i) acc[i] = first ? d[i] : acc[i] + d[i];
    }, [&](const std::vector<double>& r, void* v) {
      std::memcpy(v, r.data(), size_t(count) * 8);
    });
  }
  void allreduce_sum_u64(uint64_t* buf, int count, hipStream_t st) override {
    std::vector<uint64_t> h(count);
    sync_copy(h.data(), buf, size_t(count) * 8, st, true);
    std::unique_lock<std::mutex> lk(hub_->mu);
    hub_->collective([&](bool first) {
      if (first) hub_->acc_u.assign(count, 0);
      for (int i = 0; i < count; ++i) hub_->acc_u[i] += h[i];
    }, lk);
    h = hub_->result_u;
    lk.unlock();
    sync_copy(buf, h.data(), size_t(count) * 8, st, false);
  }
  void barrier() override {
    std::unique_lock<std::mutex> lk(hub_->mu);
    hub_->collective([](bool) {}, lk);
  }

 private:
  void enable_peer(int peer) {
    if (peer >= int(peer_on_.size())) peer_on_.resize(size_t(peer) + 1, false);
    if (peer_on_[peer]) return;
    int ok = 0;
    HIP_CHECK(hipDeviceCanAccessPeer(&ok, dev_, peer));
    if (ok) {
      const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_CHECK(e);
      (void)hipGetLastError();
    }
    peer_on_[peer] = true;
  }
  static void sync_copy(void* dst, const void* src, size_t bytes, hipStream_t st, bool d2h) {
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipMemcpy(dst, src, bytes, d2h ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice));
  }
  template <class Combine, class Store>
  void reduce(void* buf, int count, hipStream_t st, size_t esize, Combine combine, Store store) {
    std::vector<char> h(size_t(count) * esize);
    sync_copy(h.data(), buf, h.size(), st, true);
    std::unique_lock<std::mutex> lk(hub_->mu);
    hub_->collective([&](bool first) {
      if (first) hub_->acc_f.assign(count, 0.0);
      combine(hub_->acc_f, h.data(), first);
    }, lk);
    std::vector<double> r = hub_->result_f;
    lk.unlock();
    store(r, h.data());
    sync_copy(buf, h.data(), h.size(), st, false);
  }

  LoopbackHub* hub_;
  int rank_, dev_;
  std::vector<bool> peer_on_;
};

}  // namespace

LoopbackHub* loopback_hub_create(int world) {
  HEAT_CHECK(world >= 1, "loopback world %d", world);
  return new LoopbackHub(world);
}
void loopback_hub_destroy(LoopbackHub* hub) { delete hub; }
void loopback_hub_fail(LoopbackHub* hub) {
  {
    std::lock_guard<std::mutex> lk(hub->mu);
    hub->failed = true;
  }
  hub->cv.notify_all();
}

std::unique_ptr<Transport> make_loopback_transport(LoopbackHub* hub, int rank, int device) {
  return std::make_unique<LoopbackTransport>(hub, rank, device);
}

}  // namespace heat
