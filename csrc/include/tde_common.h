// Shared device/host helpers for the CDNA4 (gfx950) kernel library.
//
// Everything in csrc/kernels is written for MI355X only: 64-lane wavefronts,
// MFMA 16x16x32 bf16 matrix cores, 160 KiB LDS per CU.  Host entry points are
// exported with C linkage (TDE_API) and take raw device pointers plus the
// hipStream_t of the caller, so they can be driven from Python via ctypes and
// captured into hipGraphs (no allocation, no synchronisation inside any entry).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TDE_API extern "C" __attribute__((visibility("default")))

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

namespace tde {

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 v) { return (float)v; }
__device__ __forceinline__ bf16 f2bf(float v) { return (bf16)v; }

// Wave-wide sum over 64 lanes.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// MFMA 16x16x32 bf16 -> f32.  Lane l holds A[row l&15][k 8*(l>>4) .. +7] and
// B[k 8*(l>>4) .. +7][col l&15]; the accumulator holds C[row 4*(l>>4)+r][col l&15].
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// MFMA 32x32x16 bf16 -> f32.  Lane l holds A[row l&31][k 8*(l>>5) .. +7] and
// B[k 8*(l>>5) .. +7][col l&31]; accumulator register r holds
// C[row 8*(r>>2) + 4*(l>>5) + (r&3)][col l&31].
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// 16-byte fragment load with a zero fill outside [0, limit) (limit counted in
// elements along K).  `p` points at element k0 of the row.
__device__ __forceinline__ bf16x8 load_frag(const bf16* p, int k0, int K, bool row_ok) {
  if (row_ok && k0 + 8 <= K) return *reinterpret_cast<const bf16x8*>(p);
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (row_ok && k0 + j < K) ? p[j] : (bf16)0.0f;
  return r;
}

// Reductions over the 16 lanes of a DPP row with DPP modifiers (no LDS
// round trip, unlike __shfl_xor which lowers to ds_bpermute): quad xor1, quad
// xor2, row_half_mirror, row_mirror -> every lane of the row holds the result.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}
__device__ __forceinline__ int row16_min(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  v = min(v, dpp_i<0x141>(v));
  v = min(v, dpp_i<0x140>(v));
  return v;
}
// Sum over the 4 rows of a wave (lanes 0,16,32,48 after a row16 reduction).
__device__ __forceinline__ float rows4_sum(float v) {
  const int x = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(x, 0)) + __int_as_float(__builtin_amdgcn_readlane(x, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(x, 32)) + __int_as_float(__builtin_amdgcn_readlane(x, 48)));
}

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for every
// outstanding global store/atomic of the wave (vmcnt(0)); at MNIST sizes those
// scattered stores cost microseconds, and no wave reads them back in-kernel, so
// the barriers between LDS producer/consumer phases use lgkmcnt(0) + s_barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Diagnostic phase stamps (wall clock, 100 MHz): thread 0 of each workgroup
// records stamps[blockIdx * kMaxStamps + slot]. Only used when a kernel is given
// a non-null stamp buffer (profiling builds/runs); never feeds any output.
constexpr int kMaxStamps = 8;
__device__ __forceinline__ void stamp(long long* st, int slot) {
  if (st && threadIdx.x == 0) {
    const int blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    st[(size_t)blk * kMaxStamps + slot] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

}  // namespace tde

#define TDE_LAUNCH_CHECK() \
  do {                     \
    hipError_t e__ = hipGetLastError(); \
    if (e__ != hipSuccess) return (int)e__; \
  } while (0)
