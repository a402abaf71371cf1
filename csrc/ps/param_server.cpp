// Parameter-server task for ParameterServerStrategy (SURVEY.md F07, §2.6 C6;
// reference: mnist_keras_distributed.py:242, tf2_mnist_distributed.py:189).
//
// A ps task owns a shard of the variables (round-robin placement by the client,
// like TF's replica_device_setter).  Workers PULL current values and PUSH
// gradients asynchronously; the server applies the update on receipt under a
// per-variable lock (SGD / momentum / Nesterov / Adam, Keras forms; Adam's step count t is the
// variable's own update count, as TF1's async PS applies each variable's Adam update independently).  BN moving statistics are
// updated with MOVING_AVG pushes; the global step is an atomic counter.
// Transport: the length-prefixed TCP framing of tde_net.h (C++ replacement of
// TF's gRPC RecvTensor / variable-update RPCs).
#include <atomic>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>

#include "tde_net.h"

namespace {

enum Op : uint8_t {
  kInit = 1, kPull = 2, kPush = 3, kMovingAvg = 4, kStepAdd = 5, kStepGet = 6, kAssign = 7, kList = 8,
  kSetOpt = 9, kPing = 10, kStats = 11, kStep = 12
};

struct Var {
  std::mutex mu;
  std::vector<float> w, slot, slot2;
  int64_t version = 0;
  int64_t t = 0;   // Adam: updates applied to this variable
};

struct PSServer {
  int lfd = -1, port = 0;
  std::atomic<bool> stop{false};
  std::mutex mu;  // guards the map
  std::map<std::string, std::unique_ptr<Var>> vars;
  std::atomic<int64_t> step{0};          // counter 0: global_step
  std::atomic<int64_t> counters[3]{};     // counters 1..3: tickets etc.
  std::atomic<int64_t> pushes{0}, pulls{0};
  // set by a kSetOpt request on one connection's thread, read by every push handler
  std::atomic<int> kind{0};  // 0 sgd, 1 momentum, 2 nesterov, 3 adam
  std::atomic<float> momentum{0.f};
  std::atomic<float> beta1{0.9f}, beta2{0.999f}, epsilon{1e-7f};
  std::thread acceptor;
  std::mutex cmu;
  std::set<int> clients;
  std::vector<std::thread> workers;

  Var* find(const std::string& n) {
    std::lock_guard<std::mutex> g(mu);
    auto it = vars.find(n);
    return it == vars.end() ? nullptr : it->second.get();
  }

  // Wire payloads sit at arbitrary byte offsets of the request frame: floats are read with memcpy
  // (an unaligned float load is undefined behaviour; found by the UBSan stress run).
  static float wire_f32(const char* p, size_t i) {
    float v;
    memcpy(&v, p + 4 * i, 4);
    return v;
  }

  void apply(Var* v, const char* g, size_t n, float lr) {
    const int k = kind.load();
    const float mom = momentum.load();
    std::lock_guard<std::mutex> lk(v->mu);
    if (n != v->w.size()) return;
    if (k == 0) {
      for (size_t i = 0; i < n; ++i) v->w[i] -= lr * wire_f32(g, i);
    } else if (k == 3) {
      if (v->slot.size() != n) v->slot.assign(n, 0.f);
      if (v->slot2.size() != n) v->slot2.assign(n, 0.f);
      const float b1 = beta1.load(), b2 = beta2.load(), eps = epsilon.load();
      const double t = (double)(++v->t);
      const float lr_t = (float)(lr * std::sqrt(1.0 - std::pow((double)b2, t)) / (1.0 - std::pow((double)b1, t)));
      for (size_t i = 0; i < n; ++i) {
        const float gi = wire_f32(g, i);
        v->slot[i] = b1 * v->slot[i] + (1.f - b1) * gi;
        v->slot2[i] = b2 * v->slot2[i] + (1.f - b2) * gi * gi;
        v->w[i] -= lr_t * v->slot[i] / (std::sqrt(v->slot2[i]) + eps);
      }
    } else {
      if (v->slot.size() != n) v->slot.assign(n, 0.f);
      for (size_t i = 0; i < n; ++i) {
        const float gi = wire_f32(g, i);
        const float nv = mom * v->slot[i] - lr * gi;
        v->slot[i] = nv;
        v->w[i] += (k == 2) ? mom * nv - lr * gi : nv;
      }
    }
    v->version++;
  }

  void handle(int fd) {
    tde_net::set_nodelay(fd);
    std::string req;
    while (!stop.load() && tde_net::recv_frame(fd, &req)) {
      tde_net::Reader r(req);
      tde_net::Writer w;
      const uint8_t op = r.u8();
      switch (op) {
        case kInit: {
          std::string name = r.str();
          uint32_t nb = 0;
          const char* data = r.view(&nb);
          bool created = false;
          {
            std::lock_guard<std::mutex> g(mu);
            auto& slot = vars[name];
            if (!slot) {
              slot.reset(new Var());
              slot->w.resize(nb / 4);
              if (data) memcpy(slot->w.data(), data, nb);
              created = true;
            }
          }
          w.u8(0);
          w.u8(created ? 1 : 0);
          break;
        }
        case kPull: {
          uint32_t k = r.u32();
          w.u8(0);
          for (uint32_t i = 0; i < k && r.ok; ++i) {
            std::string name = r.str();
            Var* v = find(name);
            if (!v) {
              w.s[0] = 2;
              w.bytes(nullptr, 0);
              continue;
            }
            std::lock_guard<std::mutex> lk(v->mu);
            w.bytes(v->w.data(), v->w.size() * 4);
          }
          pulls++;
          break;
        }
        case kPush: {
          float lr = r.f32();
          uint32_t k = r.u32();
          w.u8(0);
          for (uint32_t i = 0; i < k && r.ok; ++i) {
            std::string name = r.str();
            uint32_t nb = 0;
            const char* g = r.view(&nb);
            Var* v = find(name);
            if (!v || !g) {
              w.s[0] = 2;
              continue;
            }
            apply(v, g, nb / 4, lr);
          }
          pushes++;
          break;
        }
        case kMovingAvg: {
          float m = r.f32();
          uint32_t k = r.u32();
          w.u8(0);
          for (uint32_t i = 0; i < k && r.ok; ++i) {
            std::string name = r.str();
            uint32_t nb = 0;
            const char* val = r.view(&nb);
            Var* v = find(name);
            if (!v || !val || nb / 4 != v->w.size()) {
              w.s[0] = 2;
              continue;
            }
            std::lock_guard<std::mutex> lk(v->mu);
            for (size_t j = 0; j < v->w.size(); ++j) v->w[j] = v->w[j] * m + wire_f32(val, j) * (1.f - m);
            v->version++;
          }
          break;
        }
        case kAssign: {
          std::string name = r.str();
          uint32_t nb = 0;
          const char* data = r.view(&nb);
          Var* v = find(name);
          if (!v || nb / 4 != v->w.size()) {
            w.u8(2);
            break;
          }
          std::lock_guard<std::mutex> lk(v->mu);
          memcpy(v->w.data(), data, nb);
          v->version++;
          w.u8(0);
          break;
        }
        case kStepAdd: {
          const uint32_t idx = r.u32();
          int64_t d = r.i64();
          std::atomic<int64_t>& c = idx == 0 ? step : counters[(idx - 1) % 3];
          int64_t nv = c.fetch_add(d) + d;
          w.u8(0);
          w.i64(nv);
          break;
        }
        case kStepGet:
          w.u8(0);
          w.i64(step.load());
          break;
        case kList: {
          std::string out;
          std::lock_guard<std::mutex> g(mu);
          for (auto& kv : vars) {
            out += kv.first;
            out.push_back('\n');
          }
          w.u8(0);
          w.str(out);
          break;
        }
        case kSetOpt: {
          kind.store((int)r.u32());
          momentum.store(r.f32());
          const float b1 = r.f32(), b2 = r.f32(), eps = r.f32();
          if (r.ok) {   // Adam's hyper-parameters (older clients send kind + momentum only)
            beta1.store(b1);
            beta2.store(b2);
            epsilon.store(eps);
          }
          w.u8(0);
          break;
        }
        case kStats:
          w.u8(0);
          w.i64(pushes.load());
          w.i64(pulls.load());
          break;
        case kStep: {
          // One round trip per training step of an async worker (the Estimator's PS loop):
          //   push gradients (SGD/momentum applied on receipt), moving-average pushes of BN statistics,
          //   global-step / ticket counter increments, then pull fresh values of the listed variables
          //   (read AFTER this request's own updates).
          const float lr = r.f32();
          w.u8(0);
          const uint32_t kp = r.u32();
          for (uint32_t i = 0; i < kp && r.ok; ++i) {
            std::string name = r.str();
            uint32_t nb = 0;
            const char* g = r.view(&nb);
            Var* v = find(name);
            if (!v || !g) {
              w.s[0] = 2;
              continue;
            }
            apply(v, g, nb / 4, lr);
          }
          const uint32_t ka = r.u32();
          for (uint32_t i = 0; i < ka && r.ok; ++i) {
            std::string name = r.str();
            const float m = r.f32();
            uint32_t nb = 0;
            const char* val = r.view(&nb);
            Var* v = find(name);
            if (!v || !val || nb / 4 != v->w.size()) {
              w.s[0] = 2;
              continue;
            }
            std::lock_guard<std::mutex> lk(v->mu);
            for (size_t j = 0; j < v->w.size(); ++j) v->w[j] = v->w[j] * m + wire_f32(val, j) * (1.f - m);
            v->version++;
          }
          const int64_t dstep = r.i64(), dticket = r.i64();
          w.i64(dstep ? step.fetch_add(dstep) + dstep : step.load());
          w.i64(dticket ? counters[0].fetch_add(dticket) + dticket : counters[0].load());
          const uint32_t kl = r.u32();
          for (uint32_t i = 0; i < kl && r.ok; ++i) {
            std::string name = r.str();
            Var* v = find(name);
            if (!v) {
              w.s[0] = 2;
              w.bytes(nullptr, 0);
              continue;
            }
            std::lock_guard<std::mutex> lk(v->mu);
            w.bytes(v->w.data(), v->w.size() * 4);
          }
          if (kp) pushes++;
          if (kl) pulls++;
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
      if (::poll(&p, 1, 100) <= 0) continue;
      int fd = ::accept(lfd, nullptr, nullptr);
      if (fd < 0) continue;
      std::lock_guard<std::mutex> g(cmu);
      clients.insert(fd);
      workers.emplace_back([this, fd] { handle(fd); });
    }
  }

  void shutdown() {
    stop.store(true);
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

struct PSClient {
  int fd = -1;
  std::mutex mu;
  bool call(const std::string& req, std::string* resp) {
    std::lock_guard<std::mutex> g(mu);
    return tde_net::send_frame(fd, req) && tde_net::recv_frame(fd, resp);
  }
};

}  // namespace

TDE_API void* tde_ps_server_start(const char* host, int port, int* bound_port) {
  auto* s = new PSServer();
  s->lfd = tde_net::listen_on(host, port, &s->port);
  if (s->lfd < 0) {
    delete s;
    return nullptr;
  }
  if (bound_port) *bound_port = s->port;
  s->acceptor = std::thread([s] { s->accept_loop(); });
  return s;
}

TDE_API void tde_ps_server_stop(void* h) {
  auto* s = (PSServer*)h;
  if (!s) return;
  s->shutdown();
  delete s;
}

TDE_API long long tde_ps_server_step(void* h) { return ((PSServer*)h)->step.load(); }

TDE_API void* tde_ps_connect(const char* host, int port, int timeout_ms) {
  int fd = tde_net::connect_to(host, port, timeout_ms);
  if (fd < 0) return nullptr;
  auto* c = new PSClient();
  c->fd = fd;
  return c;
}

TDE_API void tde_ps_close(void* h) {
  auto* c = (PSClient*)h;
  if (!c) return;
  ::close(c->fd);
  delete c;
}

// Returns 1 if this call created the variable, 0 if it existed, <0 on error.
TDE_API int tde_ps_init(void* h, const char* name, const float* data, long long n) {
  tde_net::Writer w;
  w.u8(kInit);
  w.str(name);
  w.bytes(data, (size_t)n * 4);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp) || resp.size() < 2) return -1;
  return resp[1];
}

// Pull k variables in one round trip into outs[i] (sizes[i] floats each).
TDE_API int tde_ps_pull(void* h, int k, const char** names, float** outs, const long long* sizes) {
  tde_net::Writer w;
  w.u8(kPull);
  w.u32((uint32_t)k);
  for (int i = 0; i < k; ++i) w.str(names[i]);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp)) return -1;
  tde_net::Reader r(resp);
  int st = r.u8();
  for (int i = 0; i < k; ++i) {
    uint32_t nb = 0;
    const char* p = r.view(&nb);
    if (!p || (long long)nb != sizes[i] * 4) return -3;
    memcpy(outs[i], p, nb);
  }
  return st;
}

TDE_API int tde_ps_push(void* h, int k, const char** names, const float** grads, const long long* sizes, float lr) {
  tde_net::Writer w;
  w.u8(kPush);
  w.f32(lr);
  w.u32((uint32_t)k);
  for (int i = 0; i < k; ++i) {
    w.str(names[i]);
    w.bytes(grads[i], (size_t)sizes[i] * 4);
  }
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp) || resp.empty()) return -1;
  return resp[0];
}

TDE_API int tde_ps_moving_avg(void* h, int k, const char** names, const float** vals, const long long* sizes,
                              float momentum) {
  tde_net::Writer w;
  w.u8(kMovingAvg);
  w.f32(momentum);
  w.u32((uint32_t)k);
  for (int i = 0; i < k; ++i) {
    w.str(names[i]);
    w.bytes(vals[i], (size_t)sizes[i] * 4);
  }
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp) || resp.empty()) return -1;
  return resp[0];
}

// One training step's round trip (kStep): push kp gradients, ka moving-average values (per-variable
// momentum), add dstep / dticket to the global-step / ticket counters (returned in *step_out /
// *ticket_out) and pull kl variables into outs[i] (sizes[i] floats).
TDE_API int tde_ps_step(void* h, float lr, int kp, const char** pnames, const float** grads, const long long* psizes,
                        int ka, const char** anames, const float* amoms, const float** avals,
                        const long long* asizes, long long dstep, long long dticket, int kl, const char** lnames,
                        float** outs, const long long* lsizes, long long* step_out, long long* ticket_out) {
  tde_net::Writer w;
  w.u8(kStep);
  w.f32(lr);
  w.u32((uint32_t)kp);
  for (int i = 0; i < kp; ++i) {
    w.str(pnames[i]);
    w.bytes(grads[i], (size_t)psizes[i] * 4);
  }
  w.u32((uint32_t)ka);
  for (int i = 0; i < ka; ++i) {
    w.str(anames[i]);
    w.f32(amoms[i]);
    w.bytes(avals[i], (size_t)asizes[i] * 4);
  }
  w.i64(dstep);
  w.i64(dticket);
  w.u32((uint32_t)kl);
  for (int i = 0; i < kl; ++i) w.str(lnames[i]);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp)) return -1;
  tde_net::Reader r(resp);
  const int st = r.u8();
  const int64_t sv = r.i64(), tv = r.i64();
  if (!r.ok) return -2;
  if (step_out) *step_out = sv;
  if (ticket_out) *ticket_out = tv;
  for (int i = 0; i < kl; ++i) {
    uint32_t nb = 0;
    const char* p = r.view(&nb);
    if (!p || (long long)nb != lsizes[i] * 4) return -3;
    memcpy(outs[i], p, nb);
  }
  return st;
}

TDE_API int tde_ps_assign(void* h, const char* name, const float* data, long long n) {
  tde_net::Writer w;
  w.u8(kAssign);
  w.str(name);
  w.bytes(data, (size_t)n * 4);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp) || resp.empty()) return -1;
  return resp[0];
}

TDE_API long long tde_ps_counter_add(void* h, int idx, long long d) {
  tde_net::Writer w;
  w.u8(kStepAdd);
  w.u32((uint32_t)idx);
  w.i64(d);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp)) return INT64_MIN;
  tde_net::Reader r(resp);
  r.u8();
  return r.i64();
}

TDE_API long long tde_ps_step_add(void* h, long long d) { return tde_ps_counter_add(h, 0, d); }

TDE_API long long tde_ps_step_get(void* h) {
  tde_net::Writer w;
  w.u8(kStepGet);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp)) return INT64_MIN;
  tde_net::Reader r(resp);
  r.u8();
  return r.i64();
}

TDE_API int tde_ps_set_optimizer(void* h, int kind, float momentum, float beta1, float beta2, float epsilon) {
  tde_net::Writer w;
  w.u8(kSetOpt);
  w.u32((uint32_t)kind);
  w.f32(momentum);
  w.f32(beta1);
  w.f32(beta2);
  w.f32(epsilon);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp) || resp.empty()) return -1;
  return resp[0];
}

TDE_API int tde_ps_stats(void* h, long long* pushes, long long* pulls) {
  tde_net::Writer w;
  w.u8(kStats);
  std::string resp;
  if (!((PSClient*)h)->call(w.s, &resp)) return -1;
  tde_net::Reader r(resp);
  r.u8();
  *pushes = r.i64();
  *pulls = r.i64();
  return 0;
}
