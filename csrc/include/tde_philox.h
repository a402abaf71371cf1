// Philox4x32-10 (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11): the
// counter-based generator of every dropout mask in the kernel libraries.  Masks are a pure function of
// (element, step, layer, seed), so they are regenerated in the backward instead of stored, and the
// host twin (tensorflow_distributed_example_amd/ops/philox.py) reproduces them bit for bit.
#pragma once
#include <hip/hip_runtime.h>

namespace tde {

__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const unsigned lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = uint4{hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0};
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Keep scale (0 or 1/(1-rate)) of element e at step `it` of dropout layer `layer`: one Philox block per
// 4 consecutive elements (counter = (e/4, step, layer)), word e%4 compared against 1-rate at 24 bits.
__device__ __forceinline__ float philox_keep(float rate, unsigned long long seed, long long it, int layer,
                                             long long e) {
  const uint2 key{(unsigned)seed, (unsigned)(seed >> 32)};
  const unsigned long long c = (unsigned long long)(e >> 2);
  const uint4 r = philox(uint4{(unsigned)c, (unsigned)(c >> 32), (unsigned)it, (unsigned)layer}, key);
  const int q = (int)(e & 3);
  const unsigned w = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
  const float keep = 1.f - rate;
  return ((w >> 8) * (1.f / 16777216.f) < keep) ? 1.f / keep : 0.f;
}

}  // namespace tde
