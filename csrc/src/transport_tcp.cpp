// TCP transport: host-memory message passing between processes.
//
// This is the CPU multi-process backend of the standalone `heat` binary (the
// role the reference's MPI program plays, mpi/mpi_heat_improved_persistent_stat.c)
// and the rendezvous used to hand the RCCL unique id to every rank when no
// torch.distributed store is available.  Rank 0 listens on (addr, port);
// every rank opens its own listener, rank 0 distributes the address table,
// and the ranks build a full mesh (rank j connects to every i < j).  Each
// sendrecv() call drives all of its sockets with poll() until every byte has
// moved, so the (at most 4) halo messages of a step progress concurrently,
// like the reference's MPI_Startall/MPI_Waitall pairs (:160-161, :177, :263).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <thread>

#include "heat/common.hpp"
#include "heat/transport.hpp"

namespace heat {
namespace {

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

void write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    HEAT_CHECK(k > 0, "tcp send: %s", std::strerror(errno));
    c += k;
    n -= size_t(k);
  }
}

void read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    HEAT_CHECK(k > 0, "tcp recv: %s", k == 0 ? "peer closed" : std::strerror(errno));
    c += k;
    n -= size_t(k);
  }
}

// IPv4 address of a host name or dotted quad ("localhost" from
// torch.distributed.run --standalone included).
in_addr resolve(const std::string& addr) {
  in_addr a{};
  if (inet_pton(AF_INET, addr.c_str(), &a) == 1) return a;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  HEAT_CHECK(getaddrinfo(addr.c_str(), nullptr, &hints, &res) == 0 && res, "cannot resolve %s",
             addr.c_str());
  a = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return a;
}

int listen_on(const std::string& addr, int port, int* bound_port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  HEAT_CHECK(fd >= 0, "socket: %s", std::strerror(errno));
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(uint16_t(port));
  sa.sin_addr = resolve(addr);
  HEAT_CHECK(::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) == 0, "bind %s:%d: %s",
             addr.c_str(), port, std::strerror(errno));
  HEAT_CHECK(::listen(fd, 128) == 0, "listen: %s", std::strerror(errno));
  socklen_t len = sizeof sa;
  getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &len);
  *bound_port = ntohs(sa.sin_port);
  return fd;
}

int connect_to(const std::string& addr, int port, double timeout_s) {
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons(uint16_t(port));
  sa.sin_addr = resolve(addr);
  auto t0 = std::chrono::steady_clock::now();
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    HEAT_CHECK(fd >= 0, "socket: %s", std::strerror(errno));
    if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) == 0) {
      set_nodelay(fd);
      return fd;
    }
    ::close(fd);
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    HEAT_CHECK(el < timeout_s, "connect %s:%d timed out", addr.c_str(), port);
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

struct Endpoint {
  char addr[64];
  int32_t port;
};

class TcpTransport final : public Transport {
 public:
  TcpTransport(int rank, int world, const std::string& addr, int port)
      : rank_(rank), world_(world), fds_(size_t(world), -1) {
    HEAT_CHECK(world >= 1 && rank >= 0 && rank < world, "rank %d world %d", rank, world);
    if (world == 1) return;
    const double timeout = 300.0;
    int my_port = 0;
    int lfd = listen_on(rank == 0 ? addr : addr, rank == 0 ? port : 0, &my_port);
    std::vector<Endpoint> table(static_cast<size_t>(world));
    if (rank == 0) {
      std::snprintf(table[0].addr, sizeof table[0].addr, "%s", addr.c_str());
      table[0].port = my_port;
      // Rendezvous: accept world-1 connections that announce (rank, port).
      for (int i = 1; i < world; ++i) {
        int fd = ::accept(lfd, nullptr, nullptr);
        HEAT_CHECK(fd >= 0, "accept: %s", std::strerror(errno));
        set_nodelay(fd);
        int32_t hello[2];
        read_all(fd, hello, sizeof hello);
        HEAT_CHECK(hello[0] > 0 && hello[0] < world && fds_[size_t(hello[0])] < 0,
                   "bad rendezvous rank %d", hello[0]);
        fds_[size_t(hello[0])] = fd;
        std::snprintf(table[size_t(hello[0])].addr, sizeof table[0].addr, "%s", addr.c_str());
        table[size_t(hello[0])].port = hello[1];
      }
      for (int i = 1; i < world; ++i) write_all(fds_[size_t(i)], table.data(), sizeof(Endpoint) * table.size());
    } else {
      int fd = connect_to(addr, port, timeout);
      int32_t hello[2] = {rank, my_port};
      write_all(fd, hello, sizeof hello);
      read_all(fd, table.data(), sizeof(Endpoint) * table.size());
      fds_[0] = fd;
    }
    // Full mesh among ranks >= 1: j connects to every 0 < i < j, i accepts.
    for (int j = 2; j < world; ++j) {
      for (int i = 1; i < j; ++i) {
        if (rank == j) {
          int fd = connect_to(table[size_t(i)].addr, table[size_t(i)].port, timeout);
          int32_t me = rank;
          write_all(fd, &me, sizeof me);
          fds_[size_t(i)] = fd;
        } else if (rank == i) {
          int fd = ::accept(lfd, nullptr, nullptr);
          HEAT_CHECK(fd >= 0, "accept: %s", std::strerror(errno));
          set_nodelay(fd);
          int32_t who;
          read_all(fd, &who, sizeof who);
          HEAT_CHECK(who > i && who < world && fds_[size_t(who)] < 0, "bad mesh peer %d", who);
          fds_[size_t(who)] = fd;
        }
      }
    }
    ::close(lfd);
    for (int i = 0; i < world; ++i)
      if (i != rank) {
        HEAT_CHECK(fds_[size_t(i)] >= 0, "no connection to rank %d", i);
        ::fcntl(fds_[size_t(i)], F_SETFL, ::fcntl(fds_[size_t(i)], F_GETFL) | O_NONBLOCK);
      }
  }
  void abort() override {
    for (int fd : fds_)
      if (fd >= 0) ::shutdown(fd, SHUT_RDWR);  // peers' reads on these sockets fail at once
  }
  ~TcpTransport() override {
    for (int fd : fds_)
      if (fd >= 0) ::close(fd);
  }
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  bool device_memory() const override { return false; }

  void sendrecv(const Msg* msgs, int n, hipStream_t) override {
    struct Prog {
      int fd;
      const char* s;
      size_t sl;
      char* r;
      size_t rl;
    };
    std::vector<Prog> p;
    for (int i = 0; i < n; ++i) {
      const Msg& m = msgs[i];
      HEAT_CHECK(m.peer >= 0 && m.peer < world_ && m.peer != rank_, "bad peer %d", m.peer);
      for (auto& q : p) HEAT_CHECK(q.fd != fds_[size_t(m.peer)], "duplicate peer %d", m.peer);
      p.push_back({fds_[size_t(m.peer)], static_cast<const char*>(m.sbuf), m.sbytes,
                   static_cast<char*>(m.rbuf), m.rbytes});
    }
    std::vector<pollfd> pf(p.size());
    while (true) {
      size_t active = 0;
      for (size_t i = 0; i < p.size(); ++i) {
        pf[i].fd = p[i].fd;
        pf[i].events = short((p[i].sl ? POLLOUT : 0) | (p[i].rl ? POLLIN : 0));
        pf[i].revents = 0;
        if (pf[i].events) ++active;
      }
      if (!active) break;
      int rc = ::poll(pf.data(), nfds_t(pf.size()), 600000);
      HEAT_CHECK(rc > 0, "tcp poll %s", rc == 0 ? "timed out" : std::strerror(errno));
      for (size_t i = 0; i < p.size(); ++i) {
        if (pf[i].revents & (POLLERR | POLLNVAL))
          HEAT_CHECK(false, "tcp socket error");
        if ((pf[i].revents & POLLOUT) && p[i].sl) {
          ssize_t k = ::send(p[i].fd, p[i].s, p[i].sl, MSG_NOSIGNAL);
          if (k > 0) {
            p[i].s += k;
            p[i].sl -= size_t(k);
          } else {
            HEAT_CHECK(errno == EAGAIN || errno == EINTR, "tcp send: %s", std::strerror(errno));
          }
        }
        if ((pf[i].revents & (POLLIN | POLLHUP)) && p[i].rl) {
          ssize_t k = ::recv(p[i].fd, p[i].r, p[i].rl, 0);
          if (k > 0) {
            p[i].r += k;
            p[i].rl -= size_t(k);
          } else {
            HEAT_CHECK(k < 0 && (errno == EAGAIN || errno == EINTR), "tcp recv: %s",
                       k == 0 ? "peer closed" : std::strerror(errno));
          }
        }
      }
    }
  }

  template <class T, class Op>
  void allreduce(T* buf, int count, Op op) {
    if (world_ == 1 || count == 0) return;
    const size_t bytes = sizeof(T) * size_t(count);
    if (rank_ == 0) {
      std::vector<T> tmp(static_cast<size_t>(count));
      for (int r = 1; r < world_; ++r) {
        Msg m{r, nullptr, 0, tmp.data(), bytes};
        sendrecv(&m, 1, nullptr);
        for (int i = 0; i < count; ++i) buf[i] = op(buf[i], tmp[size_t(i)]);
      }
      std::vector<Msg> ms;
      for (int r = 1; r < world_; ++r) ms.push_back(Msg{r, buf, bytes, nullptr, 0});
      sendrecv(ms.data(), int(ms.size()), nullptr);
    } else {
      Msg up{0, buf, bytes, nullptr, 0};
      sendrecv(&up, 1, nullptr);
      Msg down{0, nullptr, 0, buf, bytes};
      sendrecv(&down, 1, nullptr);
    }
  }

  void allreduce_max(float* buf, int count, hipStream_t) override {
    // NaN-propagating max (a NaN anywhere must stop the run).
    allreduce(buf, count, [](float a, float b) { return (a != a || b != b) ? (a != a ? a : b) : (a > b ? a : b); });
  }
  void allreduce_sum_f64(double* buf, int count, hipStream_t) override {
    allreduce(buf, count, [](double a, double b) { return a + b; });
  }
  void allreduce_sum_u64(uint64_t* buf, int count, hipStream_t) override {
    allreduce(buf, count, [](uint64_t a, uint64_t b) { return a + b; });
  }
  void barrier() override {
    float x = 0.f;
    allreduce_max(&x, 1, nullptr);
  }
  const char* name() const override { return "tcp"; }

 private:
  int rank_, world_;
  std::vector<int> fds_;
};

}  // namespace

std::unique_ptr<Transport> make_tcp_transport(int rank, int world, const std::string& addr,
                                              int port) {
  return std::make_unique<TcpTransport>(rank, world, addr, port);
}

}  // namespace heat
