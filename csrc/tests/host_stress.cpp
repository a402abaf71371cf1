// Concurrency stress driver for the native host runtime (sanitizer builds of the
// C++ host code).  Built twice by tests/test_sanitizers.py, with -fsanitize=address,undefined and
// with -fsanitize=thread, together with the host sources (csrc/comm/tcp_store.cpp,
// csrc/ps/param_server.cpp, csrc/data/pipeline.cpp, csrc/io/*.cpp), and run: any sanitizer report
// fails the test (halt_on_error), as does a wrong result below.
//
// What runs concurrently (the shapes the framework uses, scaled down):
//   store     8 clients: set / get / wait / add on one shared counter / 3 rounds of barriers /
//             heartbeats / dead-member queries / deletes, then the server stops with clients connected
//   PS        6 workers: pull + push of 3 variables, moving averages, step counter, stats, while the
//             chief re-assigns a variable
//   pipeline  shuffle engine permutation check; row gathers through the thread pool from 2 threads
//   I/O       TensorBundle write + 4 concurrent readers of one handle; event file write + scan
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* tde_store_server_start(const char* host, int port, int* bound_port);
void tde_store_server_stop(void* h);
void* tde_store_connect(const char* host, int port, int timeout_ms);
void tde_store_close(void* h);
int tde_store_set(void* h, const char* key, const void* val, int n);
int tde_store_get(void* h, const char* key, void* out, int cap, int timeout_ms);
int tde_store_wait(void* h, const char* key, int timeout_ms);
long long tde_store_add(void* h, const char* key, long long delta);
int tde_store_check(void* h, const char* key);
int tde_store_delete(void* h, const char* key);
int tde_store_heartbeat(void* h, const char* id);
int tde_store_dead(void* h, int timeout_ms, char* out, int cap);
long long tde_store_num_keys(void* h);
int tde_store_barrier(void* h, const char* name, int world, int timeout_ms);

void* tde_ps_server_start(const char* host, int port, int* bound_port);
void tde_ps_server_stop(void* h);
void* tde_ps_connect(const char* host, int port, int timeout_ms);
void tde_ps_close(void* h);
int tde_ps_init(void* h, const char* name, const float* data, long long n);
int tde_ps_pull(void* h, int k, const char** names, float** outs, const long long* sizes);
int tde_ps_push(void* h, int k, const char** names, const float** grads, const long long* sizes, float lr);
int tde_ps_moving_avg(void* h, int k, const char** names, const float** vals, const long long* sizes, float momentum);
int tde_ps_assign(void* h, const char* name, const float* data, long long n);
long long tde_ps_step_add(void* h, long long d);
long long tde_ps_step_get(void* h);
int tde_ps_stats(void* h, long long* pushes, long long* pulls);

void* tde_shuffle_new(long long cap, unsigned long long seed);
void tde_shuffle_free(void* h);
long long tde_shuffle_feed(void* h, const int64_t* in, long long n, int64_t* out);
long long tde_shuffle_drain(void* h, int64_t* out);
int tde_gather_rows(const void* src, long long row_bytes, long long nsrc, const int64_t* idx, long long n, void* dst,
                    int max_threads);

int tde_bundle_write(const char* prefix, int n, const char** names, const int* dtypes, const int* ranks,
                     const long long* shapes_flat, const void** datas, const long long* nbytes);
void* tde_bundle_open(const char* prefix);
void tde_bundle_close(void* h);
int tde_bundle_count(void* h);
int tde_bundle_read(void* h, const char* name, void* out, long long cap);

void* tde_events_open(const char* path);
int tde_events_write_version(void* h, double wall_time);
int tde_events_write_scalars(void* h, double wall_time, long long step, int n, const char** tags, const float* values);
void tde_events_close(void* h);
long long tde_tfrecord_scan(const char* path, long long want, void* out, long long cap, long long* out_len);
}

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail.fetch_add(1);                                              \
    }                                                                   \
  } while (0)

static void stress_store() {
  int port = 0;
  void* srv = tde_store_server_start("127.0.0.1", 0, &port);
  CHECK(srv != nullptr);
  const int N = 8, ADDS = 200;
  std::vector<std::thread> th;
  std::vector<void*> clients(N);
  for (int i = 0; i < N; ++i) clients[i] = tde_store_connect("127.0.0.1", port, 5000);
  for (int i = 0; i < N; ++i) {
    th.emplace_back([&, i] {
      void* c = clients[i];
      CHECK(c != nullptr);
      char key[64], val[64], out[256];
      snprintf(key, sizeof key, "k/%d", i);
      snprintf(val, sizeof val, "value-%d", i);
      CHECK(tde_store_set(c, key, val, (int)strlen(val)) == 0);
      // read a neighbour's key (waits until it exists)
      snprintf(key, sizeof key, "k/%d", (i + 1) % N);
      const int n = tde_store_get(c, key, out, sizeof out, 5000);
      CHECK(n > 0);
      for (int a = 0; a < ADDS; ++a) tde_store_add(c, "counter", 1);
      for (int round = 0; round < 3; ++round) {
        snprintf(key, sizeof key, "barrier/%d", round);
        CHECK(tde_store_barrier(c, key, N, 10000) == 0);
      }
      snprintf(key, sizeof key, "hb/%d", i);
      CHECK(tde_store_heartbeat(c, key) == 0);
      char dead[1024];
      CHECK(tde_store_dead(c, 60000, dead, sizeof dead) >= 0);
      CHECK(tde_store_check(c, "counter") == 1);
      CHECK(tde_store_num_keys(c) > 0);
      CHECK(tde_store_wait(c, "never", 20) == -2);   // timeout path
    });
  }
  for (auto& t : th) t.join();
  CHECK(tde_store_add(clients[0], "counter", 0) == (long long)N * ADDS);
  CHECK(tde_store_delete(clients[0], "counter") == 1);
  // server stops while clients are still connected; then the clients close
  tde_store_server_stop(srv);
  for (void* c : clients) tde_store_close(c);
}

static void stress_ps() {
  int port = 0;
  void* srv = tde_ps_server_start("127.0.0.1", 0, &port);
  CHECK(srv != nullptr);
  const char* names[3] = {"dense/kernel", "dense/bias", "bn/moving_mean"};
  const long long sizes[3] = {4096, 64, 64};
  void* chief = tde_ps_connect("127.0.0.1", port, 5000);
  std::vector<std::vector<float>> init(3);
  for (int v = 0; v < 3; ++v) {
    init[v].assign((size_t)sizes[v], 1.0f);
    CHECK(tde_ps_init(chief, names[v], init[v].data(), sizes[v]) >= 0);
  }
  const int W = 6, ITERS = 50;
  std::vector<std::thread> th;
  for (int w = 0; w < W; ++w) {
    th.emplace_back([&, w] {
      void* c = tde_ps_connect("127.0.0.1", port, 5000);
      CHECK(c != nullptr);
      std::vector<std::vector<float>> buf(3), grad(3);
      float* outs[3];
      const float* gp[3];
      for (int v = 0; v < 3; ++v) {
        buf[v].resize((size_t)sizes[v]);
        grad[v].assign((size_t)sizes[v], 0.001f * (w + 1));
        outs[v] = buf[v].data();
        gp[v] = grad[v].data();
      }
      for (int it = 0; it < ITERS; ++it) {
        CHECK(tde_ps_pull(c, 3, names, outs, sizes) >= 0);
        CHECK(tde_ps_push(c, 2, names, gp, sizes, 0.01f) >= 0);
        CHECK(tde_ps_moving_avg(c, 1, names + 2, gp + 2, sizes + 2, 0.99f) >= 0);
        tde_ps_step_add(c, 1);
      }
      long long pushes = 0, pulls = 0;
      CHECK(tde_ps_stats(c, &pushes, &pulls) == 0);
      tde_ps_close(c);
    });
  }
  for (int k = 0; k < 20; ++k) CHECK(tde_ps_assign(chief, names[1], init[1].data(), sizes[1]) >= 0);
  for (auto& t : th) t.join();
  CHECK(tde_ps_step_get(chief) == (long long)W * ITERS);
  tde_ps_close(chief);
  tde_ps_server_stop(srv);
}

static void stress_pipeline() {
  const long long n = 10000;
  std::vector<int64_t> in((size_t)n), out((size_t)n + 1000), drained(1000);
  for (long long i = 0; i < n; ++i) in[(size_t)i] = i;
  void* s = tde_shuffle_new(1000, 1234);
  const long long m = tde_shuffle_feed(s, in.data(), n, out.data());
  const long long d = tde_shuffle_drain(s, out.data() + m);
  tde_shuffle_free(s);
  CHECK(m + d == n);
  std::vector<int64_t> seen(out.begin(), out.begin() + (size_t)n);
  std::sort(seen.begin(), seen.end());
  for (long long i = 0; i < n; ++i) CHECK(seen[(size_t)i] == i);
  // gathers large enough to use the pool, from two threads at once
  const long long rows = 4096, row_bytes = 784 * 4;
  std::vector<char> src((size_t)(rows * row_bytes));
  for (size_t i = 0; i < src.size(); ++i) src[i] = (char)(i * 131);
  std::vector<std::thread> th;
  for (int t = 0; t < 2; ++t) {
    th.emplace_back([&, t] {
      std::vector<int64_t> idx((size_t)rows);
      for (long long k = 0; k < rows; ++k) idx[(size_t)k] = (k * 7 + t) % rows;
      std::vector<char> dst((size_t)(rows * row_bytes));
      for (int rep = 0; rep < 5; ++rep)
        CHECK(tde_gather_rows(src.data(), row_bytes, rows, idx.data(), rows, dst.data(), 8) == 0);
      for (long long k = 0; k < rows; k += 97)
        CHECK(memcmp(dst.data() + k * row_bytes, src.data() + idx[(size_t)k] * row_bytes, (size_t)row_bytes) == 0);
      int64_t bad = rows;   // out-of-range index: nothing copied
      CHECK(tde_gather_rows(src.data(), row_bytes, rows, &bad, 1, dst.data(), 1) == -1);
    });
  }
  for (auto& t : th) t.join();
}

static void stress_io(const std::string& dir) {
  const std::string prefix = dir + "/model.ckpt-1";
  std::vector<float> a(1000), b(7);
  std::vector<int64_t> c(3);
  for (size_t i = 0; i < a.size(); ++i) a[i] = (float)i * 0.5f;
  for (size_t i = 0; i < b.size(); ++i) b[i] = -(float)i;
  c = {7, 8, 9};
  const char* names[3] = {"dense/kernel", "dense/bias", "global_step"};
  const int dtypes[3] = {1, 1, 9}, ranks[3] = {2, 1, 1};
  const long long shapes[4] = {10, 100, 7, 3};
  const void* datas[3] = {a.data(), b.data(), c.data()};
  const long long nbytes[3] = {(long long)a.size() * 4, (long long)b.size() * 4, 24};
  CHECK(tde_bundle_write(prefix.c_str(), 3, names, dtypes, ranks, shapes, datas, nbytes) == 0);
  void* h = tde_bundle_open(prefix.c_str());
  CHECK(h != nullptr);
  if (h) {
    CHECK(tde_bundle_count(h) == 3);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t) {
      th.emplace_back([&] {
        std::vector<float> ra(1000);
        for (int rep = 0; rep < 20; ++rep) {
          CHECK(tde_bundle_read(h, "dense/kernel", ra.data(), 4000) == 0);
          CHECK(memcmp(ra.data(), a.data(), 4000) == 0);
        }
        CHECK(tde_bundle_read(h, "missing", ra.data(), 4000) == -1);
      });
    }
    for (auto& t : th) t.join();
    tde_bundle_close(h);
  }
  const std::string ev = dir + "/events.out.tfevents.test";
  void* e = tde_events_open(ev.c_str());
  CHECK(e != nullptr);
  if (e) {
    CHECK(tde_events_write_version(e, 1.0) == 0);
    const char* tags[2] = {"loss", "accuracy"};
    const float vals[2] = {2.3f, 0.1f};
    for (int s = 0; s < 10; ++s) CHECK(tde_events_write_scalars(e, 2.0 + s, s, 2, tags, vals) == 0);
    tde_events_close(e);
    long long len = 0;
    CHECK(tde_tfrecord_scan(ev.c_str(), -1, nullptr, 0, &len) == 11);
  }
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  stress_store();
  stress_ps();
  stress_pipeline();
  stress_io(dir);
  if (g_fail.load()) {
    fprintf(stderr, "host_stress: %d check(s) failed\n", g_fail.load());
    return 1;
  }
  printf("host_stress ok\n");
  return 0;
}
