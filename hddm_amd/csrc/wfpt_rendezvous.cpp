// wfpt_rendezvous.cpp — torch-free exchange of the RCCL unique id (128 bytes)
// between the ranks of one job over TCP (POSIX sockets only).
//
// Rank 0 listens on the address `host` resolves to at `port` (WFPT_COMM_BIND=any:
// the wildcard address of its family instead, for hosts whose name resolves
// to a loopback alias locally, e.g. 127.0.1.1 from /etc/hosts) and sends its
// 128-byte id to each of the nranks - 1 peers that connect; every other rank
// connects (non-blocking, retrying until the deadline: rank 0 may start
// later) and reads the id. A peer identifies itself with a 16-byte hello
// {magic, nranks, rank, token} that rank 0 checks (token: a hash of
// $WFPT_COMM_TOKEN, 0 when unset), so a stray connection or a job with another
// world size or token is rejected instead of silently joining, and
// acknowledges the id with one byte: rank 0 counts a peer as served only after
// its ack (a peer whose read failed reconnects). Each accepted connection gets
// at most kPeerMs for its hello and ack, so a silent client cannot hold the
// rendezvous until the global deadline. Nothing here touches the GPU.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wfpt_amd.h"

int wfpt_rdv_fail(int code, const std::string& msg);  // wfpt_capi.cpp (last-error slot)

namespace {

constexpr uint32_t kMagic = 0x77667074u;  // "wfpt"
constexpr unsigned char kAck = 0x5a;
constexpr int kPeerMs = 2000;  // per-connection budget of rank 0's hello / ack reads
using Clock = std::chrono::steady_clock;

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

int ms_left(Clock::time_point deadline) {
  const auto d = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now());
  return d.count() > 0 ? (int)d.count() : 0;
}

// Reads / writes exactly n bytes before the deadline.
bool io_all(int fd, void* buf, size_t n, bool write, Clock::time_point deadline) {
  char* p = static_cast<char*>(buf);
  size_t done = 0;
  while (done < n) {
    pollfd q{fd, (short)(write ? POLLOUT : POLLIN), 0};
    const int t = ms_left(deadline);
    if (t == 0) return false;
    const int pr = ::poll(&q, 1, t);
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) return false;
    const ssize_t r = write ? ::send(fd, p + done, n - done, MSG_NOSIGNAL)
                            : ::recv(fd, p + done, n - done, 0);
    if (r < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    if (r <= 0) return false;
    done += (size_t)r;
  }
  return true;
}

bool resolve(const char* host, int port, sockaddr_storage* sa, socklen_t* len) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  const std::string ps = std::to_string(port);
  if (::getaddrinfo(host, ps.c_str(), &hints, &res) != 0 || !res) return false;
  std::memcpy(sa, res->ai_addr, res->ai_addrlen);
  *len = res->ai_addrlen;
  ::freeaddrinfo(res);
  return true;
}

// FNV-1a of $WFPT_COMM_TOKEN (0 when unset): the job token of the hello.
uint32_t job_token() {
  const char* t = std::getenv("WFPT_COMM_TOKEN");
  if (!t || !*t) return 0u;
  uint32_t h = 2166136261u;
  for (; *t; ++t) h = (h ^ (unsigned char)*t) * 16777619u;
  return h ? h : 1u;
}

bool bind_any() {
  const char* b = std::getenv("WFPT_COMM_BIND");
  return b && std::strcmp(b, "any") == 0;
}

// The wildcard address of family `fam` at `port` (rank 0's listening socket
// under WFPT_COMM_BIND=any).
socklen_t wildcard(int fam, int port, sockaddr_storage* sa) {
  std::memset(sa, 0, sizeof(*sa));
  if (fam == AF_INET6) {
    auto* s6 = reinterpret_cast<sockaddr_in6*>(sa);
    s6->sin6_family = AF_INET6;
    s6->sin6_addr = in6addr_any;
    s6->sin6_port = htons((uint16_t)port);
    return sizeof(sockaddr_in6);
  }
  auto* s4 = reinterpret_cast<sockaddr_in*>(sa);
  s4->sin_family = AF_INET;
  s4->sin_addr.s_addr = htonl(INADDR_ANY);
  s4->sin_port = htons((uint16_t)port);
  return sizeof(sockaddr_in);
}

// Non-blocking connect polled against the deadline (an unreachable host
// cannot stall the caller past it). Leaves fd non-blocking (io_all polls).
bool connect_by(int fd, const sockaddr_storage& sa, socklen_t len, Clock::time_point deadline) {
  const int fl = ::fcntl(fd, F_GETFL, 0);
  if (fl < 0 || ::fcntl(fd, F_SETFL, fl | O_NONBLOCK) != 0) return false;
  if (::connect(fd, (const sockaddr*)&sa, len) == 0) return true;
  if (errno != EINPROGRESS && errno != EINTR) return false;
  for (;;) {
    pollfd q{fd, POLLOUT, 0};
    const int t = ms_left(deadline);
    if (t == 0) return false;
    const int pr = ::poll(&q, 1, t < 200 ? t : 200);
    if (pr < 0 && errno == EINTR) continue;
    if (pr < 0) return false;
    if (pr == 0) continue;
    int err = 0;
    socklen_t el = sizeof(err);
    if (::getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el) != 0) return false;
    return err == 0;
  }
}

// The address is a loopback one (127/8 or ::1, incl. v4-mapped).
bool is_loopback(const sockaddr_storage& sa) {
  if (sa.ss_family == AF_INET) {
    const uint32_t a = ntohl(reinterpret_cast<const sockaddr_in*>(&sa)->sin_addr.s_addr);
    return (a >> 24) == 127u;
  }
  if (sa.ss_family == AF_INET6) {
    const in6_addr& a = reinterpret_cast<const sockaddr_in6*>(&sa)->sin6_addr;
    if (IN6_IS_ADDR_LOOPBACK(&a)) return true;
    return IN6_IS_ADDR_V4MAPPED(&a) && a.s6_addr[12] == 127;
  }
  return false;
}

// `host` names loopback literally (a single-node job that asked for it).
bool literal_loopback(const char* host) {
  return std::strcmp(host, "localhost") == 0 || std::strncmp(host, "127.", 4) == 0 ||
         std::strcmp(host, "::1") == 0;
}

}  // namespace

extern "C" int wfpt_comm_exchange_id(int nranks, int rank, const char* host, int port,
                                     int timeout_ms, unsigned char id[128]) {
  if (!host || !id || nranks < 1 || rank < 0 || rank >= nranks || port <= 0 || port > 65535)
    return wfpt_rdv_fail(WFPT_ERR_ARG, "wfpt_comm_exchange_id: bad arguments");
  if (nranks == 1) return WFPT_OK;
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 1);
  sockaddr_storage sa{};
  socklen_t slen = 0;
  if (!resolve(host, port, &sa, &slen))
    return wfpt_rdv_fail(WFPT_ERR_COMM, std::string("rendezvous: cannot resolve ") + host);
  if (rank == 0) {
    sockaddr_storage la = sa;
    socklen_t llen = slen;
    if (bind_any()) llen = wildcard(sa.ss_family, port, &la);
    // a host name that resolves to a loopback alias (127.0.1.1 from
    // /etc/hosts) makes rank 0 unreachable for peers on other nodes: say so
    // now, and again in the timeout error, rather than fail silently
    const bool lo_alias = !bind_any() && is_loopback(la) && !literal_loopback(host);
    if (lo_alias)
      std::fprintf(stderr,
                   "wfpt rendezvous: rank 0 listens on a loopback address (%s resolves to one); "
                   "peers on other nodes cannot connect: set WFPT_COMM_BIND=any\n",
                   host);
    Fd ls;
    ls.fd = ::socket(la.ss_family, SOCK_STREAM, 0);
    if (ls.fd < 0) return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: socket() failed");
    const int one = 1;
    (void)::setsockopt(ls.fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(ls.fd, (sockaddr*)&la, llen) != 0 || ::listen(ls.fd, nranks) != 0)
      return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: cannot listen on port " +
                                              std::to_string(port) + " (" + strerror(errno) + ")");
    std::vector<bool> seen(nranks, false);
    for (int got = 0; got < nranks - 1;) {
      pollfd q{ls.fd, POLLIN, 0};
      const int t = ms_left(deadline);
      const int pr = t > 0 ? ::poll(&q, 1, t) : 0;
      if (pr < 0 && errno == EINTR) continue;
      if (pr <= 0)
        return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: timed out with " + std::to_string(got) +
                                                " of " + std::to_string(nranks - 1) +
                                                " peers served" +
                                                (lo_alias ? std::string(" (rank 0 listened on the "
                                                                        "loopback address ") +
                                                                host +
                                                                " resolves to; remote peers need "
                                                                "WFPT_COMM_BIND=any)"
                                                          : std::string()));
      Fd c;
      c.fd = ::accept(ls.fd, nullptr, nullptr);
      if (c.fd < 0) continue;
      const auto peer_deadline = std::min(deadline, Clock::now() + std::chrono::milliseconds(kPeerMs));
      uint32_t hello[4] = {0, 0, 0, 0};
      if (!io_all(c.fd, hello, sizeof(hello), false, peer_deadline)) continue;
      const int pr_rank = (int)hello[2];
      if (hello[0] != kMagic || (int)hello[1] != nranks || pr_rank <= 0 || pr_rank >= nranks ||
          seen[pr_rank] || hello[3] != job_token())
        continue;  // not one of this job's peers: ignored
      unsigned char ack = 0;
      // served only once the peer confirms it holds the id (otherwise it
      // reconnects and is served again)
      if (!io_all(c.fd, id, 128, true, peer_deadline) ||
          !io_all(c.fd, &ack, 1, false, peer_deadline) || ack != kAck)
        continue;
      seen[pr_rank] = true;
      ++got;
    }
    return WFPT_OK;
  }
  for (;;) {
    Fd c;
    c.fd = ::socket(sa.ss_family, SOCK_STREAM, 0);
    if (c.fd < 0) return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: socket() failed");
    if (connect_by(c.fd, sa, slen, deadline)) {
      const uint32_t hello[4] = {kMagic, (uint32_t)nranks, (uint32_t)rank, job_token()};
      unsigned char buf[128];
      unsigned char ack = kAck;
      if (io_all(c.fd, (void*)hello, sizeof(hello), true, deadline) &&
          io_all(c.fd, buf, 128, false, deadline) && io_all(c.fd, &ack, 1, true, deadline)) {
        std::memcpy(id, buf, 128);
        return WFPT_OK;
      }
    }
    if (ms_left(deadline) == 0)
      return wfpt_rdv_fail(WFPT_ERR_COMM, std::string("rendezvous: no id from rank 0 at ") + host +
                                              ":" + std::to_string(port) + " before the deadline");
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}
