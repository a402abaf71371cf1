// Minimal blocking TCP framing shared by the rendezvous store and the parameter
// server (csrc/comm/tcp_store.cpp, csrc/ps/param_server.cpp).
//
// Frame: u32 payload_len (little endian) | payload.  Payload starts with a one
// byte opcode; fields are u32-length-prefixed byte strings or fixed-width LE
// integers.  This is the control/PS plane of SURVEY.md §2.6 C6/C7 (TF uses gRPC).
#pragma once
#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdint.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <vector>

#define TDE_API extern "C" __attribute__((visibility("default")))

namespace tde_net {

inline bool send_all(int fd, const void* buf, size_t n) {
  const char* p = (const char*)buf;
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= (size_t)k;
  }
  return true;
}

inline bool recv_all(int fd, void* buf, size_t n) {
  char* p = (char*)buf;
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    if (k == 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

inline bool send_frame(int fd, const std::string& payload) {
  uint32_t n = (uint32_t)payload.size();
  return send_all(fd, &n, 4) && send_all(fd, payload.data(), payload.size());
}

inline bool recv_frame(int fd, std::string* out, size_t max_len = (size_t)1 << 31) {
  uint32_t n = 0;
  if (!recv_all(fd, &n, 4)) return false;
  if (n > max_len) return false;
  out->resize(n);
  return n == 0 || recv_all(fd, &(*out)[0], n);
}

// ---- payload builder / reader
struct Writer {
  std::string s;
  void u8(uint8_t v) { s.push_back((char)v); }
  void u32(uint32_t v) { s.append((const char*)&v, 4); }
  void i64(int64_t v) { s.append((const char*)&v, 8); }
  void f32(float v) { s.append((const char*)&v, 4); }
  void bytes(const void* p, size_t n) {
    u32((uint32_t)n);
    s.append((const char*)p, n);
  }
  void str(const std::string& v) { bytes(v.data(), v.size()); }
};

struct Reader {
  const std::string& s;
  size_t pos = 0;
  bool ok = true;
  explicit Reader(const std::string& str) : s(str) {}
  bool need(size_t n) {
    if (pos + n > s.size()) ok = false;
    return ok;
  }
  uint8_t u8() { return need(1) ? (uint8_t)s[pos++] : 0; }
  uint32_t u32() {
    uint32_t v = 0;
    if (need(4)) { memcpy(&v, s.data() + pos, 4); pos += 4; }
    return v;
  }
  int64_t i64() {
    int64_t v = 0;
    if (need(8)) { memcpy(&v, s.data() + pos, 8); pos += 8; }
    return v;
  }
  float f32() {
    float v = 0;
    if (need(4)) { memcpy(&v, s.data() + pos, 4); pos += 4; }
    return v;
  }
  std::string str() {
    uint32_t n = u32();
    if (!need(n)) return std::string();
    std::string r = s.substr(pos, n);
    pos += n;
    return r;
  }
  const char* view(uint32_t* n_out) {
    uint32_t n = u32();
    *n_out = n;
    if (!need(n)) return nullptr;
    const char* p = s.data() + pos;
    pos += n;
    return p;
  }
};

inline int listen_on(const char* host, int port, int* bound_port) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  addr.sin_addr.s_addr = (host && *host) ? inet_addr(host) : htonl(INADDR_ANY);
  if (::bind(fd, (sockaddr*)&addr, sizeof(addr)) != 0 || ::listen(fd, 256) != 0) {
    ::close(fd);
    return -1;
  }
  socklen_t len = sizeof(addr);
  getsockname(fd, (sockaddr*)&addr, &len);
  if (bound_port) *bound_port = ntohs(addr.sin_port);
  return fd;
}

inline int connect_to(const char* host, int port, int timeout_ms) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  char portstr[16];
  snprintf(portstr, sizeof(portstr), "%d", port);
  while (true) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host, portstr, &hints, &res) == 0 && res) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        return fd;
      }
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
    }
    if (std::chrono::steady_clock::now() >= deadline) return -1;
    usleep(50 * 1000);
  }
}

inline void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

}  // namespace tde_net
