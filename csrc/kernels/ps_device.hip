// Same-node GPU data plane of ParameterServerStrategy (reference
// mnist_keras_distributed.py:242, tf2_mnist_distributed.py:189).
//
// The ps task owns ONE device window (fine-grained, uncached, IPC-exported): the flat variable buffers
// of the model and the PS counters,
//     [counters: 16 x u64 (0 global_step, 1 step tickets, 2 initialised, 3 pushes)] [W: nw f32] [S: ns f32]
// Every trainer maps it (hipIpcOpenMemHandle; same device or a peer over xGMI) and runs its whole async
// exchange as ONE kernel after its backward, with no host staging and no TCP payload:
//   push    W[i] += -lr * g[i]                 (system-scope f32 atomics: concurrent trainers lose no
//                                               update, like the PS's serialised ApplyGradientDescent)
//           S[j] := m*S[j] + (1-m)*v[j]        (BN moving statistics, compare-and-swap; v = this trainer's
//                                               batch statistic recovered from its local update)
//   pull    w[i] = W[i], s[j] = S[j]           (fresh values, including other trainers' updates)
//   count   global_step += dstep, tickets += dticket by the LAST block, after every block's updates have
//           been performed (system fence + arrival counter), into host-mapped words the host reads after
//           the stream sync — a chief that sees global_step == max_steps sees all of them applied.
// The window lives as long as the ps task (TF's variables on /job:ps); TCP carries the handle only.
#include "tde_common.h"

#include <string.h>

namespace tde {

constexpr int kPsCounters = 16;

struct PsDevArgs {
  unsigned long long* ctr;   // window counters
  float* W;                  // window weights [nw]
  float* S;                  // window state [ns]
  float* w;                  // local weights (pulled into)
  float* g;                  // local gradients (read, zeroed); null: pull only
  long long nw;
  float* s;                  // local state: after this step's forward (push) / pulled into
  float* sp;                 // local copy of the last pulled state (push reads, pull rewrites)
  const float* mom;          // per-element BN momentum [ns]
  long long ns;
  float lr;
  long long dstep, dticket;
  unsigned int* done;        // local device word: blocks finished (re-armed by the last)
  long long* out;            // host-mapped [global_step, tickets] after this call
};

__device__ __forceinline__ float sys_load(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void ps_dev_step_kernel(PsDevArgs a) {
  const bool push = a.g != nullptr;
  const long long n = a.nw + a.ns;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    if (i < a.nw) {
      if (push) {
        const float gi = a.g[i];
        if (gi != 0.f) __hip_atomic_fetch_add(a.W + i, -a.lr * gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        a.g[i] = 0.f;
      }
      a.w[i] = sys_load(a.W + i);
    } else {
      const long long j = i - a.nw;
      float val;
      if (push) {
        const float m = a.mom[j];
        // the local forward applied m*old + (1-m)*v to the pulled value old: recover v, apply it to the PS's
        // current value (no lost updates between async trainers)
        const float v = (a.s[j] - m * a.sp[j]) / (1.f - m);
        float cur = sys_load(a.S + j);
        for (;;) {
          const float nv = cur * m + (1.f - m) * v;
          if (__hip_atomic_compare_exchange_strong(a.S + j, &cur, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_SYSTEM)) {
            val = nv;
            break;
          }
        }
      } else {
        val = sys_load(a.S + j);
      }
      a.s[j] = val;
      a.sp[j] = val;
    }
  }
  // every block's atomics are performed before the last block advances the counters
  __atomic_thread_fence(__ATOMIC_SEQ_CST);   // system scope: drains and orders this thread's accesses
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const unsigned prev = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const long long gs = (long long)__hip_atomic_fetch_add(a.ctr + 0, (unsigned long long)a.dstep, __ATOMIC_SEQ_CST,
                                                             __HIP_MEMORY_SCOPE_SYSTEM) + a.dstep;
      const long long tk = (long long)__hip_atomic_fetch_add(a.ctr + 1, (unsigned long long)a.dticket,
                                                             __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM) + a.dticket;
      if (push) __hip_atomic_fetch_add(a.ctr + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (a.out) {
        a.out[0] = gs;
        a.out[1] = tk;
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
      }
    }
  }
}

// window -> local / local -> window flat copies (initialisation, checkpoint, restore)
__global__ __launch_bounds__(256) void ps_dev_copy_kernel(float* dst, const float* src, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = src[i];
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

// One async exchange (g != null) or a pull (g == null); see the header comment.
TDE_API int tde_psdev_step(void* window, long long nw, long long ns, float* w, float* g, float* s, float* sp,
                           const float* mom, float lr, long long dstep, long long dticket, unsigned int* done,
                           long long* out_dev, hipStream_t stream) {
  if (!window || !w || nw < 0 || ns < 0 || !done || (ns > 0 && (!s || !sp || (g && !mom)))) return -1;
  PsDevArgs a;
  a.ctr = (unsigned long long*)window;
  a.W = (float*)((char*)window + kPsCounters * 8);
  a.S = a.W + nw;
  a.w = w;
  a.g = g;
  a.nw = nw;
  a.s = s;
  a.sp = sp;
  a.mom = mom;
  a.ns = ns;
  a.lr = lr;
  a.dstep = dstep;
  a.dticket = dticket;
  a.done = done;
  a.out = out_dev;
  long long blocks = (nw + ns + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  ps_dev_step_kernel<<<(int)blocks, 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// dir 0: local (w, s) -> window (and counters[0..1] := gstep, tickets when set >= 0, counters[2] := 1);
// dir 1: window -> local (w, s).
TDE_API int tde_psdev_copy(void* window, long long nw, long long ns, float* w, float* s, int dir, hipStream_t stream) {
  float* W = (float*)((char*)window + kPsCounters * 8);
  const long long n1 = nw, n2 = ns;
  if (dir == 0) {
    if (n1) ps_dev_copy_kernel<<<(int)((n1 + 255) / 256 > 1024 ? 1024 : (n1 + 255) / 256), 256, 0, stream>>>(W, w, n1);
    if (n2) ps_dev_copy_kernel<<<(int)((n2 + 255) / 256 > 1024 ? 1024 : (n2 + 255) / 256), 256, 0, stream>>>(W + nw, s, n2);
  } else {
    if (n1) ps_dev_copy_kernel<<<(int)((n1 + 255) / 256 > 1024 ? 1024 : (n1 + 255) / 256), 256, 0, stream>>>(w, W, n1);
    if (n2) ps_dev_copy_kernel<<<(int)((n2 + 255) / 256 > 1024 ? 1024 : (n2 + 255) / 256), 256, 0, stream>>>(s, W + nw, n2);
  }
  TDE_LAUNCH_CHECK();
  return 0;
}

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
