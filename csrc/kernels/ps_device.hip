// Same-node GPU data plane of ParameterServerStrategy (reference
// mnist_keras_distributed.py:242, tf2_mnist_distributed.py:189).
//
// Every ps task owns ONE device window (fine-grained, uncached, IPC-exported) holding ITS shard of the
// variables (round-robin placement, TF's replica_device_setter), sized for that shard on request:
//     [counters: 16 x u64 (0 global_step, 1 step tickets, 2 initialised, 3 pushes) — used in ps 0's]
//     [shard data: trainable variables | their momentum slots (momentum / Nesterov) | BN moving stats]
// Every trainer maps every window (hipIpcOpenMemHandle; same device or a peer over xGMI) and runs its
// whole async exchange as ONE kernel after its backward, over a segment table (one entry per variable:
// window, window offset, local flat offset, length, slot offset), with no host staging and no TCP payload:
//   push    SGD        W[i] += -lr * g[i]                    (system-scope f32 atomics: concurrent trainers
//                                                            lose no update, like the PS's serialised apply)
//           momentum   M[i] := mom*M[i] - lr*g[i] (compare-and-swap), then W[i] += M_new
//           Nesterov   as momentum, then W[i] += mom*M_new - lr*g[i]
//                      (each trainer's slot update is atomic and its weight delta an atomic add: the result
//                       is the serialised Keras update sequence in the order the CASes won)
//           S[j] := m*S[j] + (1-m)*v[j]                     (BN moving statistics, compare-and-swap; v = this
//                                                            trainer's batch statistic recovered from its
//                                                            local update)
//   pull    w[i] = W[i], s[j] = S[j]                        (fresh values, including other trainers' updates)
//   count   global_step += dstep, tickets += dticket in ps 0's counters by the LAST block, after every
//           block's updates on every shard have been performed (system fence + arrival counter), into
//           host-mapped words the host reads after the stream sync — a chief that sees
//           global_step == max_steps sees all of them applied (the TCP plane's "ps 0 last" order).
// The windows live as long as their ps tasks (TF's variables on /job:ps); TCP carries the handles only.
#include "tde_common.h"

#include <string.h>

namespace tde {

constexpr int kPsCounters = 16;
constexpr int kPsMaxShards = 16;

struct PsSeg {        // one variable of one shard (host-built table, device-resident)
  long long woff;     // element offset in the shard's data area
  long long loff;     // element offset in the local flat buffer (w / g, or s / sp / mom for a statistic)
  long long n;
  long long moff;     // momentum slot offset in the shard's data area (< 0: none)
  int win;            // shard (ps task) index
  int state;          // 1: BN moving statistic
};

struct PsDevArgs {
  float* data[kPsMaxShards];   // every window's data area (after its counters)
  unsigned long long* ctr;     // ps 0's counters
  const PsSeg* segs;
  const long long* beg;        // [nseg + 1] element prefix offsets of the segments (device)
  int nseg;
  float* w;                    // local weights (pulled into)
  float* g;                    // local gradients (read, zeroed); null: pull only
  float* s;                    // local state: after this step's forward (push) / pulled into
  float* sp;                   // local copy of the last pulled state (push reads, pull rewrites)
  const float* mom;            // per-element BN momentum (local state layout)
  float lr, mmt;               // learning rate, optimizer momentum
  int kind;                    // 0 SGD, 1 momentum, 2 Nesterov
  long long dstep, dticket;
  unsigned int* done;          // local device word: blocks finished (re-armed by the last)
  long long* out;              // host-mapped [global_step, tickets] after this call
  // pipelined trainer loop (nullable): the step ticket the pushed gradients were computed under; a push
  // whose ticket exceeds `limit` (max_steps) is dropped and advances no counter, so a host that runs a
  // few steps ahead of the tickets it has seen still makes EXACTLY max_steps global updates.  A live
  // push that claims a ticket stores it here for the next step.
  long long* claim;
  long long limit;
};

__device__ __forceinline__ float sys_load(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One flat grid over every element of every segment (`beg`: the segments' element prefix offsets, staged into
// LDS; each thread finds its segment by binary search).  The windows are fine-grained UNCACHED memory, so the
// pushes are performed where the data lives and the pulls read it there: a block only waits for its own
// accesses (s_waitcnt) before it counts its arrival — no cache writeback per block (the previous form
// fenced at system scope in every block of a segment x 64 grid: ~105 us per exchange for Model B).
constexpr int kPsMaxSegsLds = 512;
__global__ __launch_bounds__(256) void ps_dev_step_kernel(PsDevArgs a) {
  const bool live = !(a.claim && a.limit > 0 && *a.claim > a.limit);
  const bool push = a.g != nullptr && live;
  __shared__ long long beg[kPsMaxSegsLds + 1];
  const int nseg = a.nseg;
  if (a.segs) {
    for (int i = threadIdx.x; i <= nseg; i += blockDim.x) beg[i] = a.beg[i];
    __syncthreads();
    const long long total = beg[nseg];
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
      int lo = 0, hi = nseg - 1;   // the segment j with beg[j] <= e < beg[j + 1]
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (beg[mid] <= e) lo = mid;
        else hi = mid - 1;
      }
      const PsSeg sg = a.segs[lo];
      const long long i = e - beg[lo];
      float* const D = a.data[sg.win];
      float* const W = D + sg.woff;
      const long long li = sg.loff + i;
      if (!sg.state) {
        if (push) {
          const float gi = a.g[li];
          if (a.kind == 0) {
            if (gi != 0.f) __hip_atomic_fetch_add(W + i, -a.lr * gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          } else {
            float* const M = D + sg.moff + i;
            float cur = sys_load(M), nv;
            for (;;) {
              nv = a.mmt * cur - a.lr * gi;
              if (__hip_atomic_compare_exchange_strong(M, &cur, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_SYSTEM))
                break;
            }
            const float dw = a.kind == 2 ? a.mmt * nv - a.lr * gi : nv;
            __hip_atomic_fetch_add(W + i, dw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          a.g[li] = 0.f;
        } else if (a.g) {
          a.g[li] = 0.f;   // a dropped push: its gradients are discarded
        }
        a.w[li] = sys_load(W + i);
      } else {
        float val;
        if (push) {
          const float m = a.mom[li];
          // the local forward applied m*old + (1-m)*v to the pulled value old: recover v, apply it to the
          // PS's current value (no lost updates between async trainers)
          const float v = (a.s[li] - m * a.sp[li]) / (1.f - m);
          float cur = sys_load(W + i);
          for (;;) {
            const float nv = cur * m + (1.f - m) * v;
            if (__hip_atomic_compare_exchange_strong(W + i, &cur, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM)) {
              val = nv;
              break;
            }
          }
        } else {
          val = sys_load(W + i);
        }
        a.s[li] = val;
        a.sp[li] = val;
      }
    }
  }
  // every block's window accesses are performed (acknowledged by the uncached memory) before it arrives;
  // the last arrival advances the counters, so every shard's update precedes the global step
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nblk = gridDim.x * gridDim.y;
    const unsigned prev = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == nblk - 1) {
      __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const long long ds = live ? a.dstep : 0, dt = live ? a.dticket : 0;
      const long long gs = (long long)__hip_atomic_fetch_add(a.ctr + 0, (unsigned long long)ds, __ATOMIC_SEQ_CST,
                                                             __HIP_MEMORY_SCOPE_SYSTEM) + ds;
      long long tk = (long long)__hip_atomic_fetch_add(a.ctr + 1, (unsigned long long)dt,
                                                       __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM) + dt;
      if (push) __hip_atomic_fetch_add(a.ctr + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (a.claim) {
        if (live && dt) *a.claim = tk;   // the next step's ticket
        tk = *a.claim;                    // what the host sees: this trainer's ticket for its next step
      }
      if (a.out) {
        a.out[0] = gs;
        a.out[1] = tk;
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
      }
    }
  }
}

// segment-wise copies between the local flat buffers and the windows (initialisation, checkpoint,
// restore): dir 0 local -> windows (momentum slots zeroed), dir 1 windows -> local
struct PsCopyArgs {
  float* data[kPsMaxShards];
  const PsSeg* segs;
  float* w;
  float* s;
  int dir;
};
__global__ __launch_bounds__(256) void ps_dev_copy_kernel(PsCopyArgs a) {
  const PsSeg sg = a.segs[blockIdx.y];
  float* const W = a.data[sg.win] + sg.woff;
  float* const L = (sg.state ? a.s : a.w) + sg.loff;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < sg.n; i += (long long)gridDim.x * blockDim.x) {
    if (a.dir == 0) {
      W[i] = L[i];
      if (!sg.state && sg.moff >= 0) a.data[sg.win][sg.moff + i] = 0.f;
    } else {
      L[i] = W[i];
    }
  }
}

}  // namespace tde

using namespace tde;

TDE_API int tde_psdev_counters() { return kPsCounters; }

// Allocates a zeroed fine-grained (uncached) device window of `bytes` on `device` and its IPC handle.
TDE_API int tde_psdev_alloc(int device, long long bytes, void** window, char* handle_out) {
  if (hipSetDevice(device) != hipSuccess) return -100;
  hipError_t e = hipExtMallocWithFlags(window, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  if ((e = hipMemset(*window, 0, (size_t)bytes)) != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  if ((e = hipIpcGetMemHandle(&h, *window)) != hipSuccess) return (int)e;
  memcpy(handle_out, &h, sizeof(h));
  return (int)hipDeviceSynchronize();
}

TDE_API int tde_psdev_free(void* window) { return window ? (int)hipFree(window) : 0; }

// Host-mapped words the device writes and the host reads without a HIP call.
TDE_API int tde_host_mapped_alloc(long long bytes, void** host, void** dev) {
  hipError_t e = hipHostMalloc(host, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  memset(*host, 0, (size_t)bytes);
  return (int)hipHostGetDevicePointer(dev, *host, 0);
}
TDE_API int tde_host_mapped_free(void* host) { return host ? (int)hipHostFree(host) : 0; }

static int ps_grid_x(long long maxn) {
  long long bx = (maxn + 255) / 256;
  if (bx > 64) bx = 64;
  return bx < 1 ? 1 : (int)bx;
}

static int ps_fill_data(float** data, void* const* windows, int nwin) {
  if (nwin < 1 || nwin > kPsMaxShards) return -1;
  for (int i = 0; i < kPsMaxShards; ++i)
    data[i] = i < nwin && windows[i] ? (float*)((char*)windows[i] + kPsCounters * 8) : nullptr;
  for (int i = 0; i < nwin; ++i)
    if (!windows[i]) return -1;
  return 0;
}

// One async exchange (g != null) or a pull (g == null) over the segment table `segs` (device memory,
// nseg entries; maxn = the largest segment), or, with nseg == 0, a counters-only call; see the header.
// beg: [nseg + 1] device prefix offsets of the segments' element counts (total = beg[nseg], host: `total`).
TDE_API int tde_psdev_step(void* const* windows, int nwin, const void* segs, const void* beg, int nseg, long long total,
                           float* w, float* g, float* s, float* sp, const float* mom, float lr, float mmt, int kind,
                           long long dstep, long long dticket, unsigned int* done, long long* out_dev,
                           long long* claim, long long limit, hipStream_t stream) {
  if (!w || nseg < 0 || (nseg > 0 && (!segs || !beg)) || !done || kind < 0 || kind > 2 || nseg > kPsMaxSegsLds)
    return -1;
  PsDevArgs a;
  if (ps_fill_data(a.data, windows, nwin)) return -1;
  a.ctr = (unsigned long long*)windows[0];
  a.segs = nseg > 0 ? (const PsSeg*)segs : nullptr;
  a.beg = (const long long*)beg;
  a.nseg = nseg;
  a.w = w;
  a.g = g;
  a.s = s;
  a.sp = sp;
  a.mom = mom;
  a.lr = lr;
  a.mmt = mmt;
  a.kind = kind;
  a.dstep = dstep;
  a.dticket = dticket;
  a.done = done;
  a.out = out_dev;
  a.claim = claim;
  a.limit = limit;
  long long nb = nseg > 0 ? (total + 255) / 256 : 1;   // one element per thread (the accesses are latency-bound)
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  ps_dev_step_kernel<<<dim3((unsigned)nb), 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// dir 0: local (w, s) -> windows (momentum slots zeroed); dir 1: windows -> local (w, s).
TDE_API int tde_psdev_copy(void* const* windows, int nwin, const void* segs, int nseg, long long maxn, float* w,
                           float* s, int dir, hipStream_t stream) {
  if (nseg <= 0 || !segs || nseg > 65535) return nseg == 0 ? 0 : -1;
  PsCopyArgs a;
  if (ps_fill_data(a.data, windows, nwin)) return -1;
  a.segs = (const PsSeg*)segs;
  a.w = w;
  a.s = s;
  a.dir = dir;
  ps_dev_copy_kernel<<<dim3(ps_grid_x(maxn), nseg), 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// A window re-armed for a new training session: every byte (counters included: "initialised" = 0) zeroed.
TDE_API int tde_psdev_zero(void* window, long long bytes) {
  hipError_t e = hipMemset(window, 0, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  return (int)hipDeviceSynchronize();
}

// Size of the segment-table entry (the Python side packs the table with numpy).
TDE_API int tde_psdev_seg_bytes() { return (int)sizeof(PsSeg); }

// Counter i of the window := v (host write through hipMemcpy; initialisation / restore only) / read.
TDE_API int tde_psdev_set_counter(void* window, int i, long long v) {
  unsigned long long u = (unsigned long long)v;
  return (int)hipMemcpy((unsigned long long*)window + i, &u, 8, hipMemcpyHostToDevice);
}
TDE_API long long tde_psdev_get_counter(void* window, int i) {
  unsigned long long u = 0;
  if (hipMemcpy(&u, (unsigned long long*)window + i, 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (long long)u;
}
