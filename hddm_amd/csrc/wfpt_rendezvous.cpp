// wfpt_rendezvous.cpp — torch-free exchange of the RCCL unique id (128 bytes)
// between the ranks of one job over TCP (POSIX sockets only).
//
// Rank 0 listens on (host, port) and sends its 128-byte id to each of the
// nranks - 1 peers that connect; every other rank connects (retrying until
// the deadline: rank 0 may start later) and reads the id. A peer identifies
// itself with a 16-byte hello {magic, nranks, rank} that rank 0 checks, so a
// stray connection or a job with another world size is rejected instead of
// silently joining. Nothing here touches the GPU.
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

#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/wfpt_amd.h"

int wfpt_rdv_fail(int code, const std::string& msg);  // wfpt_capi.cpp (last-error slot)

namespace {

constexpr uint32_t kMagic = 0x77667074u;  // "wfpt"
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
    Fd ls;
    ls.fd = ::socket(sa.ss_family, SOCK_STREAM, 0);
    if (ls.fd < 0) return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: socket() failed");
    const int one = 1;
    (void)::setsockopt(ls.fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(ls.fd, (sockaddr*)&sa, slen) != 0 || ::listen(ls.fd, nranks) != 0)
      return wfpt_rdv_fail(WFPT_ERR_COMM, std::string("rendezvous: cannot listen on ") + host +
                                              ":" + std::to_string(port) + " (" +
                                              strerror(errno) + ")");
    std::vector<bool> seen(nranks, false);
    for (int got = 0; got < nranks - 1;) {
      pollfd q{ls.fd, POLLIN, 0};
      const int t = ms_left(deadline);
      const int pr = t > 0 ? ::poll(&q, 1, t) : 0;
      if (pr < 0 && errno == EINTR) continue;
      if (pr <= 0)
        return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: timed out with " + std::to_string(got) +
                                                " of " + std::to_string(nranks - 1) +
                                                " peers connected");
      Fd c;
      c.fd = ::accept(ls.fd, nullptr, nullptr);
      if (c.fd < 0) continue;
      uint32_t hello[4] = {0, 0, 0, 0};
      if (!io_all(c.fd, hello, sizeof(hello), false, deadline)) continue;
      const int pr_rank = (int)hello[2];
      if (hello[0] != kMagic || (int)hello[1] != nranks || pr_rank <= 0 || pr_rank >= nranks ||
          seen[pr_rank])
        continue;  // not one of this job's peers: ignored
      if (!io_all(c.fd, id, 128, true, deadline))
        return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: sending the id to rank " +
                                                std::to_string(pr_rank) + " failed");
      seen[pr_rank] = true;
      ++got;
    }
    return WFPT_OK;
  }
  for (;;) {
    Fd c;
    c.fd = ::socket(sa.ss_family, SOCK_STREAM, 0);
    if (c.fd < 0) return wfpt_rdv_fail(WFPT_ERR_COMM, "rendezvous: socket() failed");
    if (::connect(c.fd, (sockaddr*)&sa, slen) == 0) {
      const uint32_t hello[4] = {kMagic, (uint32_t)nranks, (uint32_t)rank, 0};
      unsigned char buf[128];
      if (io_all(c.fd, (void*)hello, sizeof(hello), true, deadline) &&
          io_all(c.fd, buf, 128, false, deadline)) {
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
