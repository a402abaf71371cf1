// Native engine of the tf.data-style input pipeline.
//
// The reference's pipelines (distributed_with_keras.py:30 `.cache().shuffle(10000)` batched at the
// global batch :54; mnist_keras_distributed.py:144-145 `.shuffle(1000).repeat().batch(bs)
// .prefetch(100)`) run inside TF's C++ iterators.  Driving them element by element from Python caps
// the host side at ~0.6-0.7 M img/s, a third of what one MI355X consumes on the small CNN, so the
// per-element work lives here instead:
//
//  * Shuffler: TF's shuffle-buffer semantics over streams of int64 element indices — the first
//    `cap` indices fill the buffer, every further index swaps out a uniformly chosen slot (that
//    slot's index is emitted), end of input drains the rest in random order.  xoshiro256** seeded
//    by splitmix64, so a seeded Dataset replays the same order.
//  * tde_gather_rows: batch assembly, dst[k] = src[idx[k]] for fixed-size rows (any dtype), split
//    over persistent pool threads for large batches; called with the GIL released (ctypes), so it overlaps
//    the training loop when the pipeline runs in a prefetch thread.
#include <stdint.h>
#include <string.h>

#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "tde_net.h"

namespace {

struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (auto& w : s) {  // splitmix64
      seed += 0x9E3779B97F4A7C15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      w = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  // uniform in [0, n) (Lemire's multiply-shift; the bias is < n / 2^64)
  uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
};

// Persistent workers for the row gathers (spawning threads per batch costs more than the copy).
// One pool per process: a forked child (multiprocessing workers) builds its own.
class Pool {
 public:
  static Pool& get() {
    static std::mutex mu;
    static Pool* inst = nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!inst || inst->pid_ != getpid()) inst = new Pool();  // a parent's pool has no threads here
    return *inst;
  }
  int workers() const { return (int)th_.size(); }
  // body(t) for t in [0, nt): t = 0 on the caller, the rest on pool threads; returns when all ran
  void run(int nt, const std::function<void(int)>& body) {
    std::lock_guard<std::mutex> serial(run_mu_);
    nt = std::min(nt, workers() + 1);
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = &body;
      njob_ = nt;
      pending_ = nt - 1;
      ++gen_;
    }
    cv_.notify_all();
    body(0);
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  Pool() : pid_(getpid()) {
    const int hw = (int)std::thread::hardware_concurrency();
    const int n = std::max(0, std::min(hw, 8) - 1);
    for (int i = 1; i <= n; ++i) th_.emplace_back([this, i] { loop(i); });
    for (auto& t : th_) t.detach();   // lives for the process
  }
  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= njob_) continue;
        job = job_;
      }
      (*job)(id);
      std::lock_guard<std::mutex> g(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  pid_t pid_;
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int njob_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
};

struct Shuffler {
  std::vector<int64_t> buf;
  size_t cap;
  Rng rng;
  Shuffler(size_t c, uint64_t seed) : cap(c ? c : 1), rng(seed) { buf.reserve(cap); }
};

}  // namespace

TDE_API void* tde_shuffle_new(long long cap, unsigned long long seed) {
  if (cap < 1) cap = 1;
  return new Shuffler((size_t)cap, seed);
}

TDE_API void tde_shuffle_free(void* h) { delete (Shuffler*)h; }

// Feeds n indices; writes the emitted ones to out (capacity >= n) and returns how many.
TDE_API long long tde_shuffle_feed(void* h, const int64_t* in, long long n, int64_t* out) {
  Shuffler& s = *(Shuffler*)h;
  long long k = 0, m = 0;
  while (k < n && s.buf.size() < s.cap) s.buf.push_back(in[k++]);
  const uint64_t sz = s.buf.size();
  for (; k < n; ++k) {
    const uint64_t j = s.rng.below(sz);
    out[m++] = s.buf[j];
    s.buf[j] = in[k];
  }
  return m;
}

// End of input: emits the buffered indices in random order (out capacity >= cap) and empties it.
TDE_API long long tde_shuffle_drain(void* h, int64_t* out) {
  Shuffler& s = *(Shuffler*)h;
  long long m = 0;
  while (!s.buf.empty()) {
    const uint64_t j = s.rng.below(s.buf.size());
    out[m++] = s.buf[j];
    s.buf[j] = s.buf.back();
    s.buf.pop_back();
  }
  return m;
}

TDE_API long long tde_shuffle_size(void* h) { return (long long)((Shuffler*)h)->buf.size(); }

// dst[k, :] = src[idx[k], :] for k < n, rows of row_bytes bytes.  Returns 0, or -1 (nothing
// copied) when an index is outside [0, nsrc).
TDE_API int tde_gather_rows(const void* src, long long row_bytes, long long nsrc, const int64_t* idx,
                        long long n, void* dst, int max_threads) {
  for (long long k = 0; k < n; ++k)
    if (idx[k] < 0 || idx[k] >= nsrc) return -1;
  const char* s = (const char*)src;
  char* d = (char*)dst;
  auto run = [&](long long a, long long b) {
    for (long long k = a; k < b; ++k) memcpy(d + k * row_bytes, s + idx[k] * row_bytes, (size_t)row_bytes);
  };
  // pool threads pay off from ~1 MiB per thread (a wake-up costs 5-25 us; a 128-image MNIST batch
  // is 400 KiB and stays on the calling thread)
  const int nt = (int)std::max<long long>(1, std::min<long long>(max_threads, (n * row_bytes) >> 20));
  if (nt <= 1) {
    run(0, n);
    return 0;
  }
  const long long per = (n + nt - 1) / nt;
  Pool::get().run(nt, [&](int t) { run(std::min(n, t * per), std::min(n, (t + 1) * per)); });
  return 0;
}
