// Single-node gradient all-reduce over xGMI peer memory (one process per GPU).
//
// MI355X nodes are a full xGMI mesh: every GPU has a point-to-point link to each of
// its 7 peers.  A ring all-reduce keeps one outgoing link busy per step and pays
// 2(N-1) latency hops; at the MNIST bucket sizes of the reference models
// (1.0-1.4 MB fp32) that latency, not bandwidth, is the
// step-time cost.  This is the "optional one-shot xGMI P2P all-reduce for small
// buckets" of SURVEY.md §7.1/§7.6, in its two-shot (reduce-scatter + all-gather)
// push form, so every phase drives all N-1 links at once and crosses the fabric
// exactly once:
//
//   phase 1  block c of rank r stores chunk c of every slice s of its gradient
//            straight into rank s's receive area   in[p][r][c]   (remote stores)
//            and raises flag1[p][r][c] on rank s.
//   phase 2  block c of rank s waits for flag1[p][*][c], sums the N contributions
//            of its own slice in rank order 0..N-1 (all reads are LOCAL HBM), and
//            stores the reduced chunk into out[p][s][c] of every rank, raising
//            flag2[p][s][c] there.
//   phase 3  block c of every rank waits for flag2[p][*][c] and copies the reduced
//            chunks back into the gradient bucket — or, in the fused form
//            (tde_xgmi_all_reduce_apply), applies the optimizer to them: every rank
//            updates its fp32 weights (+ slots, + bf16 shadow) from the same reduced
//            sums in the same order and zeroes its gradient, so the separate
//            optimizer launch disappears from the data-parallel step.
//
// Block c only ever waits for block c of its peers, so there is no grid-wide
// barrier; the grid (<= kXgMaxBlocks workgroups) is resident on the 256 CUs at once.
// Every slice is reduced by exactly one rank in a fixed order, so all replicas end
// bit-identical (the DP invariant checked by utils/debug.ReplicaConsistencyCheck).
//
// The shared window of each rank is one IPC-exported allocation:
//   [flags: 2 parities x 2 phases x kXgMaxRanks x kXgMaxBlocks u32] [in: 2 x cap] [out: 2 x cap]
// Flags carry the call's epoch (a device-side counter the call's last finishing block
// advances, so hipGraph replays advance it without the host), never need resetting,
// and the parity double-buffers the areas so call k+1 can start writing while a slow
// peer still copies out call k (a rank can only reach call k+2 after every peer has
// signalled phase 1 of call k+1, i.e. finished call k).  Waits are bounded: a peer
// that never arrives (dead process, broken link) sets the error word (host-mapped
// memory, read by the host with no HIP call) after `timeout_ticks` of the 100 MHz
// wall clock instead of hanging the GPU; check_health() polls it and aborts, like
// ncclCommGetAsyncError.
//
// Memory ordering (MI355X_MICROARCH.md § inter-workgroup visibility, applied at
// system scope).  Producer: payload stores -> every storing wave `s_waitcnt
// vmcnt(0)` -> workgroup barrier -> (cached window only: one system-scope release
// = L2 writeback) -> relaxed system-scope flag store.  The default window is
// fine-grained uncached memory (MTYPE UC), whose stores do not stay in any L2, so
// the release is skipped.  Consumer: ONE lane polls the flags relaxed (with
// s_sleep), then ONE system-scope acquire (L1/L2 invalidate), `s_waitcnt
// vmcnt(0)`, workgroup barrier, plain loads.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "tde_optim.h"
#include "tde_xgmi.h"

namespace tde {

// Workgroup size: 256 threads, or 1024 ("wide") when the whole grid fits one workgroup per CU and no other
// process shares the GPU (tde_xgmi_set_wide).  Every phase is a few dependent memory round trips per loop
// iteration, so a call's time follows the per-thread iteration count: the 2-replica rehearsal ran 82 / 70 /
// 63 / 60.5 us per step at 16 / 32 / 64 / 128 chunks of 256 threads (profiles/r6_xg_wide/).  A 1024-thread
// workgroup holds 4 waves x its VGPRs on every SIMD, so two never share a CU and a co-located process's
// spinning grid could starve it: wide launches are only made when neither can happen.
constexpr int kXgThreads = 256;
constexpr int kXgWideThreads = 1024;

struct XgArgs {
  float* grad;                    // local gradient bucket (in/out), M floats
  char* peer[kXgMaxRanks];        // every rank's window base, mapped in this process
  uint32_t* epoch;                // local device words: [0] calls completed, [1] blocks finished (this call)
  uint32_t* err;                  // host-mapped error word (bit0 phase-1 wait, bit1 phase-2 wait timed out)
  int rank, nranks;
  long long M;                    // elements
  long long L;                    // slice length (multiple of 4 * gridDim.x)
  long long chunk;                // chunk length within a slice (multiple of 4)
  long long cap;                  // elements per area (>= nranks * L)
  long long timeout_ticks;
  // fused optimizer (phase 3): w/m/v flat like grad; shadow[e - sh_lo] = bf16(w[e]) for e in
  // [sh_lo, sh_hi) (sh_lo a multiple of 4), and, when sht != null, sht[c * sht_ld + r] with
  // (r, c) = divmod(e - sh_lo, sh_cols)
  int apply;
  float *w, *m, *v;
  bf16* sh; long long sh_lo, sh_hi;
  bf16* sht; int sh_cols; long long sht_ld;
  const long long* iterations;
  OptHyper h;
  // diagnostics (nullable): per call slot (epoch % trace_calls) and block, kXgTraceWords u64 —
  // [epoch | seen1 << 32, t_start, t_published1, t_phase1_arrived, t_published2, t_phase2_arrived, t_end,
  // info | seen2 << 32] with
  // t = s_memrealtime (100 MHz, one clock for every process on the device) and info = missing source
  // of the phase-1 wait (bits 0-7, 0xff = none) | of the phase-2 wait (8-15) | XCC id (16-23) |
  // HW_ID cu (24-27) | se (28-31); seen1 / seen2 = the flag value a timed-out wait of that phase last read
  unsigned long long* trace;
  int trace_calls;
  // [push_lo, push_hi): bucket elements a producer kernel already stored into the owners' contribution
  // areas (tde_xgmi.h XgPush); phase 1 skips them
  long long push_lo, push_hi;
  // [rep_lo, rep_hi): bucket elements whose gradient is the sum of nrep replicas rep[(g - rep_lo) + r * rep_stride]
  // (the producer's contended atomics spread over replicas); phase 1 sums and zeroes them
  float* rep; int nrep;
  long long rep_lo, rep_hi, rep_stride;
  int acquire;   // force the waits' system-scope acquire on the uncached window (TDE_XGMI_ACQUIRE=1; A/B only)
  int flat;      // phase 3 over (slice, float4) pairs on every thread (gather_apply); TDE_XGMI_FLAT=0: slice by slice
};
constexpr int kXgTraceWords = 8;

__device__ __forceinline__ uint32_t* flag_ptr(char* base, int parity, int phase, int src, int blk) {
  return reinterpret_cast<uint32_t*>(base) + (((parity * 2 + phase) * kXgMaxRanks + src) * kXgMaxBlocks + blk);
}
__device__ __forceinline__ float* area(char* base, int which, int parity, long long cap) {
  return xg_area(base, which, parity, cap);
}

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Makes this block's stores of the phase visible, then raises the phase flag of block
// `blk` on every rank (threads 0..N-1, one flag each).
template <bool UNCACHED>
__device__ __forceinline__ void publish(char* const* peer, int nranks, int parity, int phase, int src, int blk,
                                        uint32_t epoch) {
  drain_stores();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < nranks) {
    if (!UNCACHED) {
      __atomic_thread_fence(__ATOMIC_RELEASE);   // system scope: L2 writeback
      drain_stores();
    }
    __hip_atomic_store(flag_ptr(peer[t], parity, phase, src, blk), epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wave 0 waits until every rank's flag of (parity, phase, blk) equals `epoch`: lane s polls source s, so
// the N flags cost one memory round trip per poll, not N in sequence (with 8 ranks the sequential walk was
// up to 7 extra round trips per phase).  Returns (thread 0) the first source whose flag never arrived, 0xff
// when all did, and in `seen` the value that flag held when the wait gave up (diagnostics: an older epoch
// = never written, a newer one = overwritten early).
// acquire: the cached window (and TDE_XGMI_ACQUIRE=1) drops stale L1/L2 lines after the wait; the default
// uncached window is never held in a cache, so its readers need no invalidation — and one system-scope
// acquire per block per phase (256 per call) was measurable whole-L2 invalidation traffic.
__device__ __forceinline__ uint32_t await(char* base, int parity, int phase, int nranks, int blk, uint32_t epoch,
                                          long long timeout, uint32_t* err, uint32_t bit, uint32_t& seen, bool acquire) {
  uint32_t missing = 0xffu;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const bool mine = lane < nranks;
    const uint32_t* f = flag_ptr(base, parity, phase, mine ? lane : 0, blk);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    bool ok = !mine;
    uint32_t v = epoch;
    unsigned long long pend;
    bool timed_out = false;
    while (true) {
      if (!ok) {
        v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = v == epoch;
      }
      pend = __ballot(!ok);
      if (pend == 0ull) break;
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
        timed_out = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (timed_out) {
      const int first = __ffsll((long long)pend) - 1;
      const uint32_t fv = __shfl(v, first, 64);
      if (lane == 0) {
        missing = (uint32_t)first;
        seen = fv;
        __hip_atomic_fetch_or(err, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (acquire) __atomic_thread_fence(__ATOMIC_ACQUIRE);   // system scope: drop stale L1/L2 lines
    drain_stores();
  }
  __syncthreads();
  return missing;
}

// Payload reads of peer-written window bytes after a flag wait.  On the uncached window the wait drops no cache
// (await's `acquire` is off: there is no L2 copy to invalidate, and 256 system-scope acquires per call were
// measurable), so these reads are `nt` loads (NT = true): `nt` / `sc1` loads bypass the CU's vector L1 and are
// served from L2 / memory (MI355X_MICROARCH.md, inter-workgroup visibility table: "sc1 / sc0 sc1 / nt loads
// bypass L1 only"), so no L1 line left by an earlier call on the same area (areas are reused every second call)
// can be returned stale, whatever the MTYPE of the mapping.  The cached window keeps its acquire and plain loads.
typedef float wf4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 wld4(const float* p, long long i) {
  if constexpr (NT) {
    const wf4 v = __builtin_nontemporal_load(reinterpret_cast<const wf4*>(p) + i);
    return float4{v.x, v.y, v.z, v.w};
  } else {
    return reinterpret_cast<const float4*>(p)[i];
  }
}
template <bool NT>
__device__ __forceinline__ float wld(const float* p, long long i) {
  if constexpr (NT) return __builtin_nontemporal_load(p + i);
  else return p[i];
}

template <bool NT>
__device__ __forceinline__ void copy_chunk(float* dst, const float* src, long long n, bool vec) {
  const int tid = threadIdx.x;
  if (vec) {
    const long long nv = n >> 2;
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (long long i = tid; i < nv; i += (int)blockDim.x) d4[i] = wld4<NT>(src, i);
    for (long long i = (nv << 2) + tid; i < n; i += (int)blockDim.x) dst[i] = wld<NT>(src, i);
  } else {
    for (long long i = tid; i < n; i += (int)blockDim.x) dst[i] = wld<NT>(src, i);
  }
}

__device__ __forceinline__ void shadow_store(const XgArgs& a, long long e, float w) {
  if (e < a.sh_lo || e >= a.sh_hi) return;
  const long long q = e - a.sh_lo;
  const bf16 h = f2bf(w);
  a.sh[q] = h;
  if (a.sht) a.sht[(q % a.sh_cols) * a.sht_ld + q / a.sh_cols] = h;
}

// Optimizer step of the 4 elements e .. e+3 (e % 4 == 0) from their reduced sums gs: w, slots, shadows; grad zeroed.
__device__ __forceinline__ void apply4(const XgArgs& a, float lr_t, long long e, float4 gs) {
  const bool mom = a.h.kind != kOptSGD, adam = a.h.kind == kOptAdam;
  float4 w = *reinterpret_cast<const float4*>(a.w + e);
  float4 m = {0.f, 0.f, 0.f, 0.f}, v = {0.f, 0.f, 0.f, 0.f};
  if (mom) m = *reinterpret_cast<const float4*>(a.m + e);
  if (adam) v = *reinterpret_cast<const float4*>(a.v + e);
  w.x = opt_step(a.h, lr_t, w.x, gs.x, m.x, v.x);
  w.y = opt_step(a.h, lr_t, w.y, gs.y, m.y, v.y);
  w.z = opt_step(a.h, lr_t, w.z, gs.z, m.z, v.z);
  w.w = opt_step(a.h, lr_t, w.w, gs.w, m.w, v.w);
  *reinterpret_cast<float4*>(a.w + e) = w;
  if (mom) *reinterpret_cast<float4*>(a.m + e) = m;
  if (adam) *reinterpret_cast<float4*>(a.v + e) = v;
  *reinterpret_cast<float4*>(a.grad + e) = float4{0.f, 0.f, 0.f, 0.f};
  if (e >= a.sh_lo && e + 4 <= a.sh_hi && !a.sht) {
    *reinterpret_cast<bf16x4*>(a.sh + (e - a.sh_lo)) = bf16x4{f2bf(w.x), f2bf(w.y), f2bf(w.z), f2bf(w.w)};
  } else {
    shadow_store(a, e, w.x);
    shadow_store(a, e + 1, w.y);
    shadow_store(a, e + 2, w.z);
    shadow_store(a, e + 3, w.w);
  }
}
// The same for one element.
__device__ __forceinline__ void apply1(const XgArgs& a, float lr_t, long long e, float g) {
  const bool mom = a.h.kind != kOptSGD, adam = a.h.kind == kOptAdam;
  float m = mom ? a.m[e] : 0.f, v = adam ? a.v[e] : 0.f;
  const float w = opt_step(a.h, lr_t, a.w[e], g, m, v);
  a.w[e] = w;
  if (mom) a.m[e] = m;
  if (adam) a.v[e] = v;
  a.grad[e] = 0.f;
  shadow_store(a, e, w);
}

// Phase 3 of a block: the N reduced slice chunks (slice s: bucket elements s * L + c0 .., window out + s * L + c0)
// back into the bucket, or through the optimizer.  (slice, float4) pairs are dealt over ALL threads — walking the
// slices one after another left all but CH / 4 threads idle per slice (85 of 1024 at N = 8) and cost N dependent
// round trips; each element's operation is unchanged.
template <bool NT>
__device__ __forceinline__ void gather_apply(const XgArgs& a, float lr_t, const float* out, int N, long long L,
                                             long long c0, long long CH, long long M) {
  const long long nv = (CH + 3) >> 2, tot = (long long)N * nv;
  for (long long q = threadIdx.x; q < tot; q += (int)blockDim.x) {
    const int s = (int)(q / nv);
    const long long i = q - (long long)s * nv;
    const long long g0 = (long long)s * L + c0, n = max(0LL, min(CH, M - g0)), e0 = 4 * i;
    if (e0 >= n) continue;
    const float* red = out + (size_t)s * L + c0;
    if (e0 + 4 <= n && (g0 & 3) == 0) {
      const float4 gs = wld4<NT>(red, i);
      if (a.apply) apply4(a, lr_t, g0 + e0, gs);
      else *reinterpret_cast<float4*>(a.grad + g0 + e0) = gs;
    } else {
      for (long long k = e0; k < min(e0 + 4, n); ++k) {
        const float g = wld<NT>(red, k);
        if (a.apply) apply1(a, lr_t, g0 + k, g);
        else a.grad[g0 + k] = g;
      }
    }
  }
}

// Optimizer step on n reduced elements (global index g0..): w, slots, shadows; grad zeroed.  red: window bytes
// (read with wld / wld4, see copy_chunk).
template <bool NT>
__device__ __forceinline__ void apply_chunk(const XgArgs& a, float lr_t, long long g0, const float* red, long long n) {
  const int tid = threadIdx.x;
  const bool mom = a.h.kind != kOptSGD, adam = a.h.kind == kOptAdam;
  long long nv = 0;
  if ((g0 & 3) == 0) {   // area offsets are multiples of 4 elements
    nv = n >> 2;
    for (long long i = tid; i < nv; i += (int)blockDim.x) {
      const long long e = g0 + 4 * i;
      const float4 gs = wld4<NT>(red, i);
      float4 w = *reinterpret_cast<const float4*>(a.w + e);
      float4 m = {0.f, 0.f, 0.f, 0.f}, v = {0.f, 0.f, 0.f, 0.f};
      if (mom) m = *reinterpret_cast<const float4*>(a.m + e);
      if (adam) v = *reinterpret_cast<const float4*>(a.v + e);
      w.x = opt_step(a.h, lr_t, w.x, gs.x, m.x, v.x);
      w.y = opt_step(a.h, lr_t, w.y, gs.y, m.y, v.y);
      w.z = opt_step(a.h, lr_t, w.z, gs.z, m.z, v.z);
      w.w = opt_step(a.h, lr_t, w.w, gs.w, m.w, v.w);
      *reinterpret_cast<float4*>(a.w + e) = w;
      if (mom) *reinterpret_cast<float4*>(a.m + e) = m;
      if (adam) *reinterpret_cast<float4*>(a.v + e) = v;
      *reinterpret_cast<float4*>(a.grad + e) = float4{0.f, 0.f, 0.f, 0.f};
      if (e >= a.sh_lo && e + 4 <= a.sh_hi && !a.sht) {
        *reinterpret_cast<bf16x4*>(a.sh + (e - a.sh_lo)) = bf16x4{f2bf(w.x), f2bf(w.y), f2bf(w.z), f2bf(w.w)};
      } else {
        shadow_store(a, e, w.x);
        shadow_store(a, e + 1, w.y);
        shadow_store(a, e + 2, w.z);
        shadow_store(a, e + 3, w.w);
      }
    }
    nv <<= 2;
  }
  for (long long i = nv + tid; i < n; i += (int)blockDim.x) {
    const long long e = g0 + i;
    float m = mom ? a.m[e] : 0.f, v = adam ? a.v[e] : 0.f;
    const float w = opt_step(a.h, lr_t, a.w[e], wld<NT>(red, i), m, v);
    a.w[e] = w;
    if (mom) a.m[e] = m;
    if (adam) a.v[e] = v;
    a.grad[e] = 0.f;
    shadow_store(a, e, w);
  }
}

// One launch carries the parts of NL ranks (grid.y = local rank): several replicas of one process on
// ONE device (the 1-GPU rehearsal of an N-GPU layout) run their parts in the same grid, so their mutual
// waits never depend on two streams of one device running concurrently.  NL = 1 is the plain one-rank
// launch.  The whole grid is resident at once (<= 8 x 128 workgroups of 256 threads).
constexpr int kXgMaxLocal = 8;
template <int NL>
struct XgLaunch {
  XgArgs r[NL];
};

template <bool UNCACHED, int NL>
__global__ void __launch_bounds__(kXgWideThreads) xgmi_allreduce_kernel(XgLaunch<NL> la) {
  const XgArgs& a = la.r[NL == 1 ? 0 : blockIdx.y];
  const int blk = blockIdx.x, tid = threadIdx.x;
  const uint32_t epoch = a.epoch[0] + 1;
  const int parity = epoch & 1;
  const int N = a.nranks, r = a.rank;
  const long long M = a.M, L = a.L, CH = a.chunk, cap = a.cap;
  const long long c0 = (long long)blk * CH;
  // diagnostics record (thread 0 only)
  unsigned long long* tr = nullptr;
  uint32_t miss1 = 0xffu, miss2 = 0xffu, seen1 = 0u, seen2 = 0u;
  if (a.trace && tid == 0) {
    tr = a.trace + ((size_t)(epoch % (uint32_t)a.trace_calls) * kXgMaxBlocks + blk) * kXgTraceWords;
    tr[0] = epoch;
    tr[1] = __builtin_amdgcn_s_memrealtime();
  }
#define XG_STAMP(i) \
  if (tr) tr[i] = __builtin_amdgcn_s_memrealtime()

  // ---- phase 1: push chunk `blk` of every slice s to rank s (minus the producer-pushed range)
  if (a.flat && a.nrep == 0 && a.push_lo >= a.push_hi) {
    // plain buckets: (slice, float4) pairs over every thread, as phase 3 (gather_apply)
    const long long nv = (CH + 3) >> 2, tot = (long long)N * nv;
    for (long long q = tid; q < tot; q += (int)blockDim.x) {
      const int s = (int)(q / nv);
      const long long i = q - (long long)s * nv;
      const long long g0 = (long long)s * L + c0, n = max(0LL, min(CH, M - g0)), e0 = 4 * i;
      if (e0 >= n) continue;
      float* dst = area(a.peer[s], 0, parity, cap) + (size_t)r * L + c0;
      if (e0 + 4 <= n && (g0 & 3) == 0) {
        *reinterpret_cast<float4*>(dst + e0) = *reinterpret_cast<const float4*>(a.grad + g0 + e0);
      } else {
        for (long long k = e0; k < min(e0 + 4, n); ++k) dst[k] = a.grad[g0 + k];
      }
    }
  } else
  for (int s = 0; s < N; ++s) {
    const long long g0 = (long long)s * L + c0;
    const long long n = max(0LL, min(CH, M - g0));
    float* dst = area(a.peer[s], 0, parity, cap) + (size_t)r * L + c0;
    const long long plo = min(max(a.push_lo - g0, 0LL), n), phi = min(max(a.push_hi - g0, 0LL), n);
    if (a.nrep > 0 && a.rep_lo < g0 + n && a.rep_hi > g0) {
      // a chunk holding replicated elements (the MNIST-CNN conv gradients: a few hundred): element-wise
      for (long long i = tid; i < n; i += (int)blockDim.x) {
        const long long g = g0 + i;
        if (i >= plo && i < phi) continue;
        float v;
        if (g >= a.rep_lo && g < a.rep_hi) {
          // every replica load issued before the first add (one round trip), summed in replica order
          float* q = a.rep + (g - a.rep_lo);
          float rv[kMaxGrep];
#pragma unroll
          for (int k = 0; k < kMaxGrep; ++k) rv[k] = k < a.nrep ? q[k * a.rep_stride] : 0.f;
          v = rv[0];
#pragma unroll
          for (int k = 1; k < kMaxGrep; ++k) v += rv[k];
#pragma unroll
          for (int k = 0; k < kMaxGrep; ++k)
            if (k < a.nrep) q[k * a.rep_stride] = 0.f;
        } else {
          v = a.grad[g];
        }
        dst[i] = v;
      }
    } else if (plo >= phi) {
      copy_chunk<false>(dst, a.grad + g0, n, (g0 & 3) == 0);
    } else {   // [0, plo) and [phi, n) still come from the local bucket
      if (plo > 0) copy_chunk<false>(dst, a.grad + g0, plo, false);
      if (phi < n) copy_chunk<false>(dst + phi, a.grad + g0 + phi, n - phi, false);
    }
  }
  publish<UNCACHED>(a.peer, N, parity, 0, r, blk, epoch);
  XG_STAMP(2);

  // ---- phase 2: reduce own slice chunk from local HBM, push the result to every rank
  miss1 = await(a.peer[r], parity, 0, N, blk, epoch, a.timeout_ticks, a.err, 1u, seen1, !UNCACHED || a.acquire);
  XG_STAMP(3);
  {
    const long long g0 = (long long)r * L + c0;
    const long long n = max(0LL, min(CH, M - g0));
    const float* in = area(a.peer[r], 0, parity, cap) + c0;
    const long long nv = n >> 2;   // area offsets are multiples of 4 elements
    for (long long i = tid; i < nv; i += (int)blockDim.x) {
      float4 acc = wld4<UNCACHED>(in, i);
      for (int s = 1; s < N; ++s) {
        const float4 v = wld4<UNCACHED>(in + (size_t)s * L, i);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      for (int p = 0; p < N; ++p)
        reinterpret_cast<float4*>(area(a.peer[p], 1, parity, cap) + (size_t)r * L + c0)[i] = acc;
    }
    for (long long i = (nv << 2) + tid; i < n; i += (int)blockDim.x) {
      float acc = wld<UNCACHED>(in, i);
      for (int s = 1; s < N; ++s) acc += wld<UNCACHED>(in + (size_t)s * L, i);
      for (int p = 0; p < N; ++p) area(a.peer[p], 1, parity, cap)[(size_t)r * L + c0 + i] = acc;
    }
  }
  publish<UNCACHED>(a.peer, N, parity, 1, r, blk, epoch);
  XG_STAMP(4);

  // ---- phase 3: gather every reduced slice chunk back into the bucket (or apply the update)
  float lr_t = 0.f;
  if (a.apply) lr_t = opt_lr_t(a.h, a.h.kind == kOptAdam ? *a.iterations : 0);
  miss2 = await(a.peer[r], parity, 1, N, blk, epoch, a.timeout_ticks, a.err, 2u, seen2, !UNCACHED || a.acquire);
  XG_STAMP(5);
  const float* out = area(a.peer[r], 1, parity, cap);
  if (a.flat) {
    gather_apply<UNCACHED>(a, lr_t, out, N, L, c0, CH, M);
  } else {
    for (int s = 0; s < N; ++s) {
      const long long g0 = (long long)s * L + c0;
      const long long n = max(0LL, min(CH, M - g0));
      if (a.apply) apply_chunk<UNCACHED>(a, lr_t, g0, out + (size_t)s * L + c0, n);
      else copy_chunk<UNCACHED>(a.grad + g0, out + (size_t)s * L + c0, n, (g0 & 3) == 0);
    }
  }
  if (tr) {
    const uint32_t hw = __builtin_amdgcn_s_getreg(63492);   // hwreg(HW_REG_HW_ID): cu 8-11, se 13-15
    const uint32_t xcc = __builtin_amdgcn_s_getreg(63508);  // hwreg(HW_REG_XCC_ID)
    tr[6] = __builtin_amdgcn_s_memrealtime();
    tr[0] = (unsigned long long)epoch | ((unsigned long long)(miss1 == 0xffu ? 0u : seen1) << 32);
    tr[7] = (unsigned long long)(miss1 | (miss2 << 8) | ((xcc & 0xff) << 16) | (((hw >> 8) & 0xf) << 24) |
                                 (((hw >> 13) & 0x7) << 28)) |
            ((unsigned long long)(miss2 == 0xffu ? 0u : seen2) << 32);
  }
#undef XG_STAMP
  // the last block to finish advances the epoch (every block read it at its start) and re-arms
  // the arrival counter epoch[1] for the next call
  if (tid == 0) {
    const uint32_t arrived = __hip_atomic_fetch_add(&a.epoch[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == gridDim.x - 1) {
      __hip_atomic_store(&a.epoch[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.epoch[0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Slice length for M elements over `nranks` ranks and `nblocks` chunks.
inline long long xg_slice(long long M, int nranks, int nblocks) {
  const long long q = 4LL * nblocks;
  return ((M + nranks - 1) / nranks + q - 1) / q * q;
}

}  // namespace tde

using namespace tde;

// Area capacity (elements) for buckets of up to max_elems elements: nranks * L <=
// max_elems + nranks * 4 * nblocks for every admissible nranks/nblocks.
static long long xg_cap(long long max_elems) {
  return max_elems + (long long)kXgMaxRanks * 4 * kXgMaxBlocks;
}

TDE_API size_t tde_xgmi_window_bytes(long long max_elems) {
  return kXgFlagBytes + 4 * (size_t)xg_cap(max_elems) * sizeof(float);
}
TDE_API int tde_xgmi_max_ranks() { return kXgMaxRanks; }
TDE_API int tde_xgmi_max_blocks() { return kXgMaxBlocks; }
TDE_API int tde_xgmi_ipc_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// Allocates this rank's window (fine-grained / uncached unless `uncached`=0), the
// local epoch word and the host-mapped error word, and returns the window's IPC handle.
TDE_API int tde_xgmi_alloc(int device, long long max_elems, int uncached, void** window, void** epoch, void** err,
                           char* handle_out) {
  if (hipSetDevice(device) != hipSuccess) return -100;
  const size_t bytes = tde_xgmi_window_bytes(max_elems);
  hipError_t e = uncached ? hipExtMallocWithFlags(window, bytes, hipDeviceMallocUncached) : hipMalloc(window, bytes);
  if (e != hipSuccess) return (int)e;
  if ((e = hipMemset(*window, 0, bytes)) != hipSuccess) return (int)e;
  if ((e = hipMalloc(epoch, 2 * sizeof(uint32_t))) != hipSuccess) return (int)e;
  if ((e = hipMemset(*epoch, 0, 2 * sizeof(uint32_t))) != hipSuccess) return (int)e;
  if ((e = hipHostMalloc(err, sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return (int)e;
  *(volatile uint32_t*)*err = 0;
  hipIpcMemHandle_t h;
  if ((e = hipIpcGetMemHandle(&h, *window)) != hipSuccess) return (int)e;
  memcpy(handle_out, &h, sizeof(h));
  return (int)hipDeviceSynchronize();
}

TDE_API int tde_xgmi_open(int device, const char* handle, void** mapped) {
  if (hipSetDevice(device) != hipSuccess) return -100;
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(mapped, h, hipIpcMemLazyEnablePeerAccess);
}

TDE_API int tde_xgmi_close(void* mapped) { return (int)hipIpcCloseMemHandle(mapped); }

// In-process replicas (MirroredStrategy over the GPUs of one process): device `dev` maps the
// memory of device `peer` directly (no IPC), so the windows of the other replicas are plain
// device pointers.  Called for every ordered pair BEFORE the windows are allocated.
// Returns 0 when access is (already) enabled, -5 when the pair has no peer path.
TDE_API int tde_enable_peer_access(int dev, int peer) {
  if (dev == peer) return 0;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, dev, peer) != hipSuccess || !can) return -5;
  if (hipSetDevice(dev) != hipSuccess) return -100;
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();   // clear the sticky "already enabled" status
    return 0;
  }
  return (int)e;
}

TDE_API int tde_xgmi_free(void* window, void* epoch, void* err) {
  hipError_t e1 = window ? hipFree(window) : hipSuccess;
  hipError_t e2 = epoch ? hipFree(epoch) : hipSuccess;
  hipError_t e3 = err ? hipHostFree(err) : hipSuccess;
  return e1 != hipSuccess ? (int)e1 : e2 != hipSuccess ? (int)e2 : (int)e3;
}

// The producer-side descriptor (tde_xgmi.h XgPush) for the next call of a rank: the same slice length
// and area capacity the all-reduce launch computes for a bucket of M elements over nranks x nblocks.
struct TdeXgPush {
  void* peer[kXgMaxRanks];
  const void* epoch;
  long long L, cap, off;
  int rank, nranks;
};
TDE_API int tde_xgmi_push_spec(long long M, long long max_elems, void* const* peers, const void* epoch, int rank,
                               int nranks, int nblocks, long long off, TdeXgPush* out) {
  if (nranks < 1 || nranks > kXgMaxRanks || rank < 0 || rank >= nranks || M < 0 || M > max_elems || !out) return -1;
  nblocks = nblocks < 1 ? 1 : nblocks > kXgMaxBlocks ? kXgMaxBlocks : nblocks;
  memset(out, 0, sizeof(*out));
  for (int i = 0; i < nranks; ++i) out->peer[i] = peers[i];
  out->epoch = epoch;
  out->L = xg_slice(M, nranks, nblocks);
  out->cap = xg_cap(max_elems);
  out->off = off;
  out->rank = rank;
  out->nranks = nranks;
  return out->L * nranks > out->cap ? -3 : 0;
}
static_assert(sizeof(TdeXgPush) == sizeof(XgPush), "TdeXgPush mirrors XgPush");

// Error bits of this rank (host read of the mapped word; no HIP call, never blocks).
TDE_API int tde_xgmi_error(void* err) { return (int)*(volatile uint32_t*)err; }

// Calls completed (synchronous device read; tests/diagnostics only).
TDE_API long long tde_xgmi_epoch(void* epoch) {
  uint32_t h = 0;
  if (hipMemcpy(&h, epoch, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (long long)h;
}

// Fused form: SUM all-reduce of `grad` and the optimizer step of every element on every rank
// (w/m/v flat like grad; shadows as in XgArgs); grad is left zeroed.
struct TdeXgApply {
  int kind;
  float lr, mom, b1, b2, eps;
  float *w, *m, *v;
  const long long* iterations;
  void* sh; long long sh_lo, sh_hi;
  void* sht; int sh_cols; long long sht_ld;
  long long push_lo, push_hi;   // bucket range the step's producer kernel pushed itself (empty: none)
  float* rep; int nrep;         // replicated gradient range (XgArgs::rep; nrep 0: none)
  long long rep_lo, rep_hi, rep_stride;
};

// Diagnostics: trace buffers registered per rank (keyed by the rank's epoch word); every launch
// of that rank then records per-block phase timestamps (XgArgs::trace).
#include <map>
#include <mutex>
static std::mutex g_trace_mu;
static std::map<void*, std::pair<unsigned long long*, int>> g_trace;

TDE_API int tde_xgmi_trace_words() { return kXgTraceWords; }
TDE_API int tde_xgmi_set_trace(void* epoch, void* trace, int calls) {
  std::lock_guard<std::mutex> lk(g_trace_mu);
  if (!trace || calls <= 0) g_trace.erase(epoch);
  else g_trace[epoch] = {(unsigned long long*)trace, calls};
  return 0;
}

static int xg_fill(XgArgs& a, float* grad, long long M, long long max_elems, void* const* peers, void* epoch,
                   void* err, int rank, int nranks, int nblocks, long long timeout_ticks) {
  if (nranks < 1 || nranks > kXgMaxRanks || rank < 0 || rank >= nranks) return -1;
  if (M < 0 || M > max_elems) return -2;
  if (((uintptr_t)grad & 15) != 0) return -4;
  a.grad = grad;
  for (int i = 0; i < nranks; ++i) a.peer[i] = (char*)peers[i];
  a.epoch = (uint32_t*)epoch;
  a.err = (uint32_t*)err;
  a.rank = rank;
  a.nranks = nranks;
  a.M = M;
  a.L = xg_slice(M, nranks, nblocks);
  a.chunk = a.L / nblocks;
  a.cap = xg_cap(max_elems);
  a.timeout_ticks = timeout_ticks;
  static const int force_acquire = [] {
    const char* e = getenv("TDE_XGMI_ACQUIRE");
    return e && atoi(e) != 0 ? 1 : 0;
  }();
  a.acquire = force_acquire;
  static const int flat = [] {
    const char* e = getenv("TDE_XGMI_FLAT");
    return e && *e ? atoi(e) : 1;
  }();
  a.flat = flat;
  {
    std::lock_guard<std::mutex> lk(g_trace_mu);
    auto it = g_trace.find(epoch);
    a.trace = it == g_trace.end() ? nullptr : it->second.first;
    a.trace_calls = it == g_trace.end() ? 0 : it->second.second;
  }
  if (a.L * nranks > a.cap) return -3;   // areas hold nranks slices
  return 0;
}

static int xg_set_apply(XgArgs& a, const TdeXgApply* o) {
  if (!o || !o->w || (o->kind != kOptSGD && !o->m) || (o->kind == kOptAdam && (!o->v || !o->iterations))) return -7;
  if ((((uintptr_t)o->w | (uintptr_t)o->m | (uintptr_t)o->v) & 15) || (o->sh && ((o->sh_lo & 3) || ((uintptr_t)o->sh & 7))))
    return -8;
  if (o->sht && (o->sh_cols <= 0 || !o->sh)) return -9;
  a.apply = 1;
  a.w = o->w;
  a.m = o->m;
  a.v = o->v;
  a.sh = (bf16*)o->sh;
  a.sh_lo = o->sh ? o->sh_lo : 0;
  a.sh_hi = o->sh ? o->sh_hi : 0;
  a.sht = (bf16*)o->sht;
  a.sh_cols = o->sh_cols;
  a.sht_ld = o->sht_ld;
  a.iterations = o->iterations;
  a.h = OptHyper{o->kind, o->lr, o->mom, o->b1, o->b2, o->eps};
  a.push_lo = o->push_lo;
  a.push_hi = o->push_hi;
  if (o->nrep > 1 && (!o->rep || o->nrep > kMaxGrep || o->rep_lo < 0 || o->rep_hi < o->rep_lo ||
                      o->rep_stride < o->rep_hi - o->rep_lo))
    return -10;
  a.rep = o->rep;
  a.nrep = o->nrep > 1 ? o->nrep : 0;
  a.rep_lo = o->rep_lo;
  a.rep_hi = o->rep_hi;
  a.rep_stride = o->rep_stride;
  return 0;
}

static int clamp_blocks(int nblocks) { return nblocks < 1 ? 1 : nblocks > kXgMaxBlocks ? kXgMaxBlocks : nblocks; }

// 0: not set, 1: wide launches allowed, -1: some communicator of this process shares its GPU with another
// process (sticky).  TDE_XGMI_WIDE=0 turns wide launches off (A/B).
static std::atomic<int> g_xg_wide{0};
TDE_API int tde_xgmi_set_wide(int on) {
  if (!on) g_xg_wide.store(-1);
  else {
    int z = 0;
    g_xg_wide.compare_exchange_strong(z, 1);
  }
  return g_xg_wide.load();
}
static int xg_threads(int nloc, int nblocks) {
  static const int env = [] {
    const char* e = getenv("TDE_XGMI_WIDE");
    return e && *e ? atoi(e) : 1;
  }();
  if (!env || g_xg_wide.load() != 1) return kXgThreads;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess)
    return kXgThreads;
  return nloc * nblocks <= cus ? kXgWideThreads : kXgThreads;
}
TDE_API int tde_xgmi_threads(int nloc, int nblocks) { return xg_threads(nloc, clamp_blocks(nblocks)); }

template <int NL>
static int xg_go(const XgLaunch<NL>& la, int nloc, int nblocks, int uncached, hipStream_t stream) {
  const dim3 grid(nblocks, nloc), block(xg_threads(nloc, nblocks));
  if (uncached) hipLaunchKernelGGL((xgmi_allreduce_kernel<true, NL>), grid, block, 0, stream, la);
  else hipLaunchKernelGGL((xgmi_allreduce_kernel<false, NL>), grid, block, 0, stream, la);
  TDE_LAUNCH_CHECK();
  return 0;
}

// In-place SUM all-reduce of `grad` (M fp32 elements, M <= the window's max_elems).
TDE_API int tde_xgmi_all_reduce(float* grad, long long M, long long max_elems, void* const* peers, void* epoch,
                                void* err, int rank, int nranks, int nblocks, int uncached, long long timeout_ticks,
                                hipStream_t stream) {
  nblocks = clamp_blocks(nblocks);
  XgLaunch<1> la;
  memset(&la, 0, sizeof(la));
  const int rc = xg_fill(la.r[0], grad, M, max_elems, peers, epoch, err, rank, nranks, nblocks, timeout_ticks);
  return rc ? rc : xg_go(la, 1, nblocks, uncached, stream);
}

TDE_API int tde_xgmi_all_reduce_apply(float* grad, long long M, long long max_elems, void* const* peers,
                                      void* epoch, void* err, int rank, int nranks, int nblocks, int uncached,
                                      long long timeout_ticks, const TdeXgApply* o, hipStream_t stream) {
  nblocks = clamp_blocks(nblocks);
  XgLaunch<1> la;
  memset(&la, 0, sizeof(la));
  int rc = xg_set_apply(la.r[0], o);
  if (!rc) rc = xg_fill(la.r[0], grad, M, max_elems, peers, epoch, err, rank, nranks, nblocks, timeout_ticks);
  return rc ? rc : xg_go(la, 1, nblocks, uncached, stream);
}

// The parts of the `nloc` local ranks rank0 .. rank0+nloc-1 that share ONE device, in one launch
// (grid.y = local rank).  grads[j] / epochs[j] / errs[j] / peers[j * nranks ...] belong to local rank
// j; specs (nullable: plain all-reduce) holds nloc fused-optimizer descriptors.
TDE_API int tde_xgmi_all_reduce_group(int nloc, float* const* grads, long long M, long long max_elems,
                                      void* const* peers, void* const* epochs, void* const* errs, int rank0,
                                      int nranks, int nblocks, int uncached, long long timeout_ticks,
                                      const TdeXgApply* specs, hipStream_t stream) {
  if (nloc < 1 || nloc > kXgMaxLocal || rank0 < 0 || rank0 + nloc > nranks) return -1;
  nblocks = clamp_blocks(nblocks);
  XgLaunch<kXgMaxLocal> la;
  memset(&la, 0, sizeof(la));
  for (int j = 0; j < nloc; ++j) {
    int rc = specs ? xg_set_apply(la.r[j], specs + j) : 0;
    if (!rc) rc = xg_fill(la.r[j], grads[j], M, max_elems, peers + (size_t)j * nranks, epochs[j], errs[j], rank0 + j,
                          nranks, nblocks, timeout_ticks);
    if (rc) return rc;
  }
  if (nloc == 1) {
    XgLaunch<1> one;
    one.r[0] = la.r[0];
    return xg_go(one, 1, nblocks, uncached, stream);
  }
  return xg_go(la, nloc, nblocks, uncached, stream);
}

// Sizes of the ctypes-mirrored argument structs of this file (tests/test_abi.py checks the Python
// mirrors in ops/kernels.py against them): out = {TdeXgApply, TdeXgPush}.
TDE_API int tde_xgmi_abi_sizes(long long* out, int n) {
  const long long s[] = {(long long)sizeof(TdeXgApply), (long long)sizeof(TdeXgPush)};
  for (int i = 0; i < n && i < 2; ++i) out[i] = s[i];
  return 2;
}
