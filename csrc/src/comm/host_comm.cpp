// HostComm: TCP full-mesh message passing between the ranks of one job (see anx/comm.hpp).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <stdexcept>
#include <thread>

#include "anx/comm.hpp"

namespace anx {

namespace {

int env_int(const char* a, const char* b, int dflt) {
  const char* v = std::getenv(a);
  if (!v || !*v) v = std::getenv(b);
  return (v && *v) ? std::atoi(v) : dflt;
}
std::string env_str(const char* a, const char* b, const char* dflt) {
  const char* v = std::getenv(a);
  if (!v || !*v) v = std::getenv(b);
  return (v && *v) ? std::string(v) : std::string(dflt);
}

[[noreturn]] void die(const std::string& m) { throw std::runtime_error("HostComm: " + m); }

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

sockaddr_in resolve(const std::string& host, int port) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) == 1) return a;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) die("cannot resolve " + host);
  a.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return a;
}

int listen_on(int port, int backlog, int* bound_port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) die("socket");
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) die("bind port " + std::to_string(port));
  if (listen(fd, backlog) != 0) die("listen");
  socklen_t len = sizeof a;
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
  *bound_port = ntohs(a.sin_port);
  return fd;
}

int connect_retry(const sockaddr_in& a, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) die("socket");
    if (connect(fd, reinterpret_cast<const sockaddr*>(&a), sizeof a) == 0) {
      set_nodelay(fd);
      return fd;
    }
    close(fd);
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      die("connect timeout");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

// accept() with a deadline: poll the listening socket first, so a rank that never starts or never
// connects stops the job with a message instead of hanging it (the watchdog only covers wait_all).
int accept_within(int lfd, double timeout_s, const std::string& what, sockaddr_in* peer = nullptr) {
  pollfd pf{lfd, POLLIN, 0};
  const int ms = timeout_s > 0 ? static_cast<int>(timeout_s * 1000) : -1;
  for (;;) {
    const int r = poll(&pf, 1, ms);
    if (r < 0 && errno == EINTR) continue;
    if (r == 0) die(what + " never joined within " + std::to_string(timeout_s) + " s (ANX_COMM_TIMEOUT)");
    if (r < 0) die("poll(accept)");
    break;
  }
  socklen_t plen = sizeof(sockaddr_in);
  const int fd = accept(lfd, reinterpret_cast<sockaddr*>(peer), peer ? &plen : nullptr);
  if (fd < 0) die("accept");
  return fd;
}

// bootstrap reads block at most timeout_s (a peer that connected but never says hello)
void set_recv_timeout(int fd, double timeout_s) {
  if (timeout_s <= 0) return;
  timeval tv{};
  tv.tv_sec = static_cast<time_t>(timeout_s);
  tv.tv_usec = static_cast<suseconds_t>((timeout_s - static_cast<double>(tv.tv_sec)) * 1e6);
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
}

void write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) die("write failed (peer gone?)");
    c += k;
    n -= static_cast<size_t>(k);
  }
}
void read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) die("read failed (peer gone?)");
    c += k;
    n -= static_cast<size_t>(k);
  }
}

}  // namespace

RankInfo rank_info_from_env() {
  RankInfo r;
  r.rank = env_int("ANX_RANK", "RANK", 0);
  r.world = env_int("ANX_WORLD_SIZE", "WORLD_SIZE", 1);
  r.local_rank = env_int("ANX_LOCAL_RANK", "LOCAL_RANK", r.rank);
  r.local_world = env_int("ANX_LOCAL_WORLD_SIZE", "LOCAL_WORLD_SIZE", r.world);
  if (r.local_world < 1 || r.local_world > r.world) r.local_world = r.world;
  r.nnodes = env_int("ANX_NNODES", "GROUP_WORLD_SIZE", (r.world + r.local_world - 1) / r.local_world);
  if (r.nnodes < 1) r.nnodes = 1;
  r.master_addr = env_str("ANX_MASTER_ADDR", "MASTER_ADDR", "127.0.0.1");
  r.master_port = env_int("ANX_MASTER_PORT", "MASTER_PORT", 29555);
  return r;
}

HostComm::HostComm(const RankInfo& ri, double timeout_s)
    : rank_(ri.rank), world_(ri.world), timeout_s_(timeout_s), fd_(ri.world, -1) {
  if (world_ < 1 || rank_ < 0 || rank_ >= world_) die("bad rank/world");
  if (world_ == 1) return;
  int my_port = 0;
  const int lfd = listen_on(rank_ == 0 ? ri.master_port : 0, world_ + 4, &my_port);
  // table[2*r] = IPv4 of rank r as rank 0 sees it (so ranks may live on different nodes),
  // table[2*r+1] = its listen port
  std::vector<uint32_t> table(2 * static_cast<size_t>(world_), 0);
  const sockaddr_in master = resolve(ri.master_addr, ri.master_port);
  table[0] = master.sin_addr.s_addr;
  table[1] = static_cast<uint32_t>(my_port);
  if (rank_ == 0) {
    // star bootstrap: every rank reports (rank, listen port); its address comes from accept()
    for (int i = 1; i < world_; ++i) {
      sockaddr_in peer{};
      const int fd = accept_within(lfd, timeout_s_, std::to_string(world_ - i) + " rank(s) of " +
                                                        std::to_string(world_), &peer);
      set_nodelay(fd);
      set_recv_timeout(fd, timeout_s_);
      int32_t hdr[2];
      read_all(fd, hdr, sizeof hdr);
      if (hdr[0] <= 0 || hdr[0] >= world_ || fd_[hdr[0]] != -1) die("bad hello");
      fd_[hdr[0]] = fd;
      table[2 * hdr[0]] = peer.sin_addr.s_addr;
      table[2 * hdr[0] + 1] = static_cast<uint32_t>(hdr[1]);
    }
    for (int i = 1; i < world_; ++i) write_all(fd_[i], table.data(), table.size() * sizeof(uint32_t));
  } else {
    int fd = connect_retry(master, timeout_s_);
    set_recv_timeout(fd, timeout_s_);
    int32_t hdr[2] = {rank_, my_port};
    write_all(fd, hdr, sizeof hdr);
    read_all(fd, table.data(), table.size() * sizeof(uint32_t));
    fd_[0] = fd;
    // mesh: connect to every lower non-zero rank, then accept every higher rank
    for (int j = 1; j < rank_; ++j) {
      sockaddr_in a = master;
      a.sin_addr.s_addr = table[2 * j];
      a.sin_port = htons(static_cast<uint16_t>(table[2 * j + 1]));
      int c = connect_retry(a, timeout_s_);
      int32_t me = rank_;
      write_all(c, &me, sizeof me);
      fd_[j] = c;
    }
    for (int k = rank_ + 1; k < world_; ++k) {
      const int c = accept_within(lfd, timeout_s_, "a rank above " + std::to_string(rank_));
      set_nodelay(c);
      set_recv_timeout(c, timeout_s_);
      int32_t who = -1;
      read_all(c, &who, sizeof who);
      if (who <= rank_ || who >= world_ || fd_[who] != -1) die("bad mesh hello");
      fd_[who] = c;
    }
  }
  close(lfd);
  for (int i = 0; i < world_; ++i)
    if (fd_[i] >= 0) {
      timeval none{};
      setsockopt(fd_[i], SOL_SOCKET, SO_RCVTIMEO, &none, sizeof none);  // wait_all polls with its own watchdog
      fcntl(fd_[i], F_SETFL, fcntl(fd_[i], F_GETFL) | O_NONBLOCK);
    }
}

HostComm::~HostComm() {
  for (int fd : fd_)
    if (fd >= 0) close(fd);
}

void HostComm::isend(const void* buf, size_t bytes, int dst) {
  if (dst == rank_) die("send to self");
  if (bytes) ops_.push_back({dst, const_cast<char*>(static_cast<const char*>(buf)), bytes, true});
}

void HostComm::irecv(void* buf, size_t bytes, int src) {
  if (src == rank_) die("recv from self");
  if (bytes) ops_.push_back({src, static_cast<char*>(buf), bytes, false});
}

void HostComm::wait_all() {
  // Per peer and direction the queued ops run in FIFO order; all peers/directions progress together.
  std::vector<std::deque<Op*>> sq(world_), rq(world_);
  for (Op& o : ops_) (o.send ? sq : rq)[o.peer].push_back(&o);
  auto last = std::chrono::steady_clock::now();
  for (;;) {
    std::vector<pollfd> pf;
    std::vector<int> peer;
    for (int p = 0; p < world_; ++p) {
      short ev = 0;
      if (!sq[p].empty()) ev |= POLLOUT;
      if (!rq[p].empty()) ev |= POLLIN;
      if (ev) {
        pf.push_back({fd_[p], ev, 0});
        peer.push_back(p);
      }
    }
    if (pf.empty()) break;
    const int n = poll(pf.data(), pf.size(), 1000);
    if (n < 0 && errno != EINTR) abort("poll failed");
    bool progressed = false;
    for (size_t i = 0; i < pf.size(); ++i) {
      const int p = peer[i];
      if (pf[i].revents & (POLLERR | POLLNVAL)) abort("peer " + std::to_string(p) + " socket error");
      if ((pf[i].revents & POLLOUT) && !sq[p].empty()) {
        Op* o = sq[p].front();
        ssize_t k = ::send(fd_[p], o->p, o->left, MSG_NOSIGNAL);
        if (k > 0) {
          o->p += k;
          o->left -= static_cast<size_t>(k);
          progressed = true;
          if (!o->left) sq[p].pop_front();
        } else if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
          abort("send to rank " + std::to_string(p) + " failed");
        }
      }
      if ((pf[i].revents & (POLLIN | POLLHUP)) && !rq[p].empty()) {
        Op* o = rq[p].front();
        ssize_t k = ::recv(fd_[p], o->p, o->left, 0);
        if (k > 0) {
          o->p += k;
          o->left -= static_cast<size_t>(k);
          progressed = true;
          if (!o->left) rq[p].pop_front();
        } else if (k == 0) {
          abort("rank " + std::to_string(p) + " closed the connection");
        } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
          abort("recv from rank " + std::to_string(p) + " failed");
        }
      }
    }
    const auto now = std::chrono::steady_clock::now();
    if (progressed)
      last = now;
    else if (std::chrono::duration<double>(now - last).count() > timeout_s_)
      abort("communication timeout (watchdog)");
  }
  ops_.clear();
}

void HostComm::barrier() {
  if (world_ == 1) return;
  char t = 1;
  std::vector<char> tok(world_, 0);
  if (rank_ == 0) {
    for (int i = 1; i < world_; ++i) irecv(&tok[i], 1, i);
    wait_all();
    for (int i = 1; i < world_; ++i) isend(&t, 1, i);
    wait_all();
  } else {
    send(&t, 1, 0);
    recv(&t, 1, 0);
  }
}

void HostComm::bcast(void* buf, size_t bytes, int root) {
  if (world_ == 1) return;
  if (rank_ == root) {
    for (int i = 0; i < world_; ++i)
      if (i != root) isend(buf, bytes, i);
    wait_all();
  } else {
    recv(buf, bytes, root);
  }
}

void HostComm::allreduce_max(double* v, int n) {
  if (world_ == 1) return;
  if (rank_ == 0) {
    std::vector<double> tmp(static_cast<size_t>(n) * world_);
    for (int i = 1; i < world_; ++i) irecv(tmp.data() + static_cast<size_t>(i) * n, n * sizeof(double), i);
    wait_all();
    for (int i = 1; i < world_; ++i)
      for (int k = 0; k < n; ++k) v[k] = std::max(v[k], tmp[static_cast<size_t>(i) * n + k]);
  } else {
    send(v, n * sizeof(double), 0);
  }
  bcast(v, n * sizeof(double), 0);
}

void HostComm::abort(const std::string& why, int code) {
  std::fprintf(stderr, "[anx rank %d] ABORT: %s\n", rank_, why.c_str());
  std::fflush(stderr);
  for (int& fd : fd_)
    if (fd >= 0) {
      close(fd);
      fd = -1;
    }
  std::_Exit(code);
}

}  // namespace anx
