// Layout of the xGMI all-reduce windows (csrc/comm/xgmi_allreduce.hip), shared with the producer
// kernels that push their gradients straight into them (the fused data-parallel exchange).
//
// The window of each rank is one allocation:
//   [flags: 2 parities x 2 phases x kXgMaxRanks x kXgMaxBlocks u32] [in: 2 x cap] [out: 2 x cap]
// in[parity][src * L + o] holds rank `src`'s contribution to element s * L + o of the bucket, where
// s is the window's owner rank, L the slice length of the call and o < L.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tde {

constexpr int kXgMaxRanks = 8;
constexpr int kXgMaxBlocks = 128;
constexpr size_t kXgFlagWords = 2 * 2 * kXgMaxRanks * kXgMaxBlocks;
constexpr size_t kXgFlagBytes = kXgFlagWords * 4;

// which 0 = in (contributions), 1 = out (reduced slices)
__device__ __forceinline__ float* xg_area(char* base, int which, int parity, long long cap) {
  return reinterpret_cast<float*>(base + kXgFlagBytes) + ((size_t)which * 2 + parity) * (size_t)cap;
}

// A producer kernel (the trunk backward) that writes a contiguous range of the gradient bucket
// straight into the owners' contribution areas of the NEXT all-reduce call instead of into the local
// bucket.  The all-reduce launch that follows on the same stream then skips that range in its push
// phase; its phase-1 flags (raised after this kernel completed, in stream order) cover these stores.
// The next call's parity is read from the rank's completed-calls counter when the producer runs.
struct XgPush {
  char* peer[kXgMaxRanks];     // every rank's window base, mapped in this process (nranks == 0: off)
  const uint32_t* epoch;       // this rank's completed-calls counter
  long long L, cap;            // slice length and area capacity (elements) of the next call
  long long off;               // bucket offset of the producer's element 0
  int rank, nranks;
};

// Stores value v of bucket element g (g = off + local index) into its owner's contribution area.
__device__ __forceinline__ void xg_push_store(const XgPush& p, int parity, long long g, float v) {
  const int s = (int)(g / p.L);
  xg_area(p.peer[s], 0, parity, p.cap)[(size_t)p.rank * p.L + (g - (long long)s * p.L)] = v;
}

// Four consecutive elements g..g+3 (g % 4 == 0, L % 4 == 0: one owner, a 16-byte aligned destination).
__device__ __forceinline__ void xg_push_store4(const XgPush& p, int parity, long long g, float4 v) {
  const int s = (int)(g / p.L);
  *reinterpret_cast<float4*>(xg_area(p.peer[s], 0, parity, p.cap) + (size_t)p.rank * p.L +
                             (g - (long long)s * p.L)) = v;
}

// A pushing wave waits for its stores' acknowledgements before it ends: on an N-GPU node they travel
// over xGMI into peer HBM, and the all-reduce's flag that covers them is raised by the next launch, so
// they must have completed, not merely been issued (the ordering the all-reduce gives its own phase-1
// stores before their flag).
__device__ __forceinline__ void xg_push_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace tde
