// TCP key-value store: rendezvous, barriers, heartbeats — the control plane that
// plays gRPC's role in the reference's tf.distribute runtime:
//   * MultiWorkerMirroredStrategy bootstrap: the chief publishes the RCCL unique
//     id, workers block on GET until it appears;
//   * barrier(name, n) = ADD + WAIT;
//   * heartbeat(id) / dead(timeout) for failure detection.
// One thread per connection; waits are condition-variable based with timeouts.
#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>

#include "tde_net.h"

namespace {

using Clock = std::chrono::steady_clock;

enum Op : uint8_t {
  kSet = 1, kGet = 2, kAdd = 3, kCheck = 4, kDelete = 5, kWait = 6, kHeartbeat = 7, kDead = 8,
  kNumKeys = 9, kCompareSet = 11, kPing = 12
};

struct StoreServer {
  int lfd = -1;
  int port = 0;
  std::atomic<bool> stop{false};
  std::mutex mu;
  std::condition_variable cv;
  std::map<std::string, std::string> kv;
  std::map<std::string, Clock::time_point> beats;
  std::thread acceptor;
  std::mutex cmu;
  std::set<int> clients;
  std::vector<std::thread> workers;

  bool wait_key(const std::string& k, int timeout_ms, std::unique_lock<std::mutex>& lk) {
    auto pred = [&] { return kv.count(k) > 0 || stop.load(); };
    if (timeout_ms < 0) {
      cv.wait(lk, pred);
    } else if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred)) {
      return false;
    }
    return kv.count(k) > 0;
  }

  void handle(int fd) {
    tde_net::set_nodelay(fd);
    std::string req;
    while (!stop.load() && tde_net::recv_frame(fd, &req)) {
      tde_net::Reader r(req);
      tde_net::Writer w;
      const uint8_t op = r.u8();
      switch (op) {
        case kSet: {
          std::string k = r.str(), v = r.str();
          { std::lock_guard<std::mutex> g(mu); kv[k] = v; }
          cv.notify_all();
          w.u8(0);
          break;
        }
        case kGet:
        case kWait: {
          std::string k = r.str();
          int t = (int)r.u32();
          std::unique_lock<std::mutex> lk(mu);
          bool ok = wait_key(k, t == -1 ? -1 : t, lk);
          w.u8(ok ? 0 : 1);
          if (op == kGet) w.str(ok ? kv[k] : std::string());
          break;
        }
        case kAdd: {
          std::string k = r.str();
          int64_t d = r.i64(), v = 0;
          {
            std::lock_guard<std::mutex> g(mu);
            auto it = kv.find(k);
            if (it != kv.end() && it->second.size() == 8) memcpy(&v, it->second.data(), 8);
            v += d;
            kv[k] = std::string((const char*)&v, 8);
          }
          cv.notify_all();
          w.u8(0);
          w.i64(v);
          break;
        }
        case kCheck: {
          std::string k = r.str();
          std::lock_guard<std::mutex> g(mu);
          w.u8(kv.count(k) ? 1 : 0);
          break;
        }
        case kDelete: {
          std::string k = r.str();
          std::lock_guard<std::mutex> g(mu);
          w.u8(kv.erase(k) ? 1 : 0);
          break;
        }
        case kHeartbeat: {
          std::string id = r.str();
          std::lock_guard<std::mutex> g(mu);
          beats[id] = Clock::now();
          w.u8(0);
          break;
        }
        case kDead: {
          int t = (int)r.u32();
          std::string out;
          auto now = Clock::now();
          std::lock_guard<std::mutex> g(mu);
          for (auto& kvp : beats) {
            if (now - kvp.second > std::chrono::milliseconds(t)) {
              out += kvp.first;
              out.push_back('\n');
            }
          }
          w.u8(0);
          w.str(out);
          break;
        }
        case kNumKeys: {
          std::lock_guard<std::mutex> g(mu);
          w.u8(0);
          w.i64((int64_t)kv.size());
          break;
        }
        case kCompareSet: {
          std::string k = r.str(), expected = r.str(), desired = r.str();
          std::string cur;
          {
            std::lock_guard<std::mutex> g(mu);
            auto it = kv.find(k);
            if ((it == kv.end() && expected.empty()) || (it != kv.end() && it->second == expected)) {
              kv[k] = desired;
              cur = desired;
            } else {
              cur = it == kv.end() ? std::string() : it->second;
            }
          }
          cv.notify_all();
          w.u8(0);
          w.str(cur);
          break;
        }
        case kPing:
          w.u8(0);
          break;
        default:
          w.u8(255);
      }
      if (!r.ok) { w.s.clear(); w.u8(254); }
      if (!tde_net::send_frame(fd, w.s)) break;
    }
    {
      std::lock_guard<std::mutex> g(cmu);
      clients.erase(fd);
    }
    ::close(fd);
  }

  void accept_loop() {
    while (!stop.load()) {
      pollfd p{lfd, POLLIN, 0};
      int rc = ::poll(&p, 1, 100);
      if (rc <= 0) continue;
      int fd = ::accept(lfd, nullptr, nullptr);
      if (fd < 0) continue;
      std::lock_guard<std::mutex> g(cmu);
      clients.insert(fd);
      workers.emplace_back([this, fd] { handle(fd); });
    }
  }

  void shutdown() {
    stop.store(true);
    cv.notify_all();
    if (acceptor.joinable()) acceptor.join();
    {
      std::lock_guard<std::mutex> g(cmu);
      for (int fd : clients) ::shutdown(fd, SHUT_RDWR);
    }
    for (auto& t : workers)
      if (t.joinable()) t.join();
    if (lfd >= 0) ::close(lfd);
    lfd = -1;
  }
};

struct StoreClient {
  int fd = -1;
  std::mutex mu;
  bool call(const tde_net::Writer& w, std::string* resp) {
    std::lock_guard<std::mutex> g(mu);
    return tde_net::send_frame(fd, w.s) && tde_net::recv_frame(fd, resp);
  }
};

}  // namespace

TDE_API void* tde_store_server_start(const char* host, int port, int* bound_port) {
  auto* s = new StoreServer();
  s->lfd = tde_net::listen_on(host, port, &s->port);
  if (s->lfd < 0) {
    delete s;
    return nullptr;
  }
  if (bound_port) *bound_port = s->port;
  s->acceptor = std::thread([s] { s->accept_loop(); });
  return s;
}

TDE_API void tde_store_server_stop(void* h) {
  auto* s = (StoreServer*)h;
  if (!s) return;
  s->shutdown();
  delete s;
}

TDE_API void* tde_store_connect(const char* host, int port, int timeout_ms) {
  int fd = tde_net::connect_to(host, port, timeout_ms);
  if (fd < 0) return nullptr;
  auto* c = new StoreClient();
  c->fd = fd;
  return c;
}

TDE_API void tde_store_close(void* h) {
  auto* c = (StoreClient*)h;
  if (!c) return;
  if (c->fd >= 0) ::close(c->fd);
  delete c;
}

TDE_API int tde_store_set(void* h, const char* key, const void* val, int n) {
  tde_net::Writer w;
  w.u8(kSet);
  w.str(key);
  w.bytes(val, (size_t)n);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  return resp.empty() ? -1 : resp[0];
}

// Returns value length (copied up to cap), -1 on connection error, -2 on timeout.
TDE_API int tde_store_get(void* h, const char* key, void* out, int cap, int timeout_ms) {
  tde_net::Writer w;
  w.u8(kGet);
  w.str(key);
  w.u32((uint32_t)timeout_ms);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  tde_net::Reader r(resp);
  if (r.u8() != 0) return -2;
  std::string v = r.str();
  memcpy(out, v.data(), v.size() < (size_t)cap ? v.size() : (size_t)cap);
  return (int)v.size();
}

TDE_API int tde_store_wait(void* h, const char* key, int timeout_ms) {
  tde_net::Writer w;
  w.u8(kWait);
  w.str(key);
  w.u32((uint32_t)timeout_ms);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  return resp.empty() ? -1 : (resp[0] == 0 ? 0 : -2);
}

TDE_API long long tde_store_add(void* h, const char* key, long long delta) {
  tde_net::Writer w;
  w.u8(kAdd);
  w.str(key);
  w.i64(delta);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return INT64_MIN;
  tde_net::Reader r(resp);
  r.u8();
  return r.i64();
}

TDE_API int tde_store_check(void* h, const char* key) {
  tde_net::Writer w;
  w.u8(kCheck);
  w.str(key);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  return resp.empty() ? -1 : resp[0];
}

TDE_API int tde_store_delete(void* h, const char* key) {
  tde_net::Writer w;
  w.u8(kDelete);
  w.str(key);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  return resp.empty() ? -1 : resp[0];
}

TDE_API int tde_store_heartbeat(void* h, const char* id) {
  tde_net::Writer w;
  w.u8(kHeartbeat);
  w.str(id);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  return 0;
}

// Writes '\n'-separated ids of members silent for > timeout_ms; returns length.
TDE_API int tde_store_dead(void* h, int timeout_ms, char* out, int cap) {
  tde_net::Writer w;
  w.u8(kDead);
  w.u32((uint32_t)timeout_ms);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  tde_net::Reader r(resp);
  r.u8();
  std::string v = r.str();
  memcpy(out, v.data(), v.size() < (size_t)cap ? v.size() : (size_t)cap);
  return (int)v.size();
}

TDE_API long long tde_store_num_keys(void* h) {
  tde_net::Writer w;
  w.u8(kNumKeys);
  std::string resp;
  if (!((StoreClient*)h)->call(w, &resp)) return -1;
  tde_net::Reader r(resp);
  r.u8();
  return r.i64();
}

// Barrier over `world` members: ADD name/count, then wait for name/done.
TDE_API int tde_store_barrier(void* h, const char* name, int world, int timeout_ms) {
  std::string base(name);
  long long n = tde_store_add(h, (base + "/count").c_str(), 1);
  if (n == INT64_MIN) return -1;
  if (n >= world) {
    const char one = 1;
    return tde_store_set(h, (base + "/done").c_str(), &one, 1);
  }
  return tde_store_wait(h, (base + "/done").c_str(), timeout_ms);
}
