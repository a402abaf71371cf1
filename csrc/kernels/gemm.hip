// MFMA GEMM for the Dense / im2col paths.
//
//   C[M,N] (f32)  (=|+=)  alpha * A[M,K] . Bt[N,K]^T      (A, Bt bf16, K-contiguous)
//
// Every GEMM the Keras-layout models need is put into this "both operands
// K-contiguous" form by the producers (see tensorflow_distributed_example_amd/
// ops/fused.py): Dense forward uses the optimizer-maintained W^T bf16 shadow,
// dW = X^T G uses the transposed activations written by the producing kernel.
// That keeps every MFMA fragment a single 16-byte load per lane straight from
// global memory (L2-resident operands; no LDS round trip needed at these sizes).
//
// Tile: 256 threads = 4 waves as 2x2, each wave 32x32 = 2x2 MFMA 16x16x32
// fragments -> 64x64 per workgroup.  Split-K over gridDim.z; split results are
// combined with f32 atomics (mode 2) into a pre-zeroed C.
//
// Reference parity: Dense kernels of distributed_with_keras.py:37-38 and
// mnist_keras_distributed.py:103,108.
#include "tde_common.h"

namespace tde {

enum GemmMode { kStore = 0, kAccum = 1, kAtomic = 2 };

template <int MODE, bool EPI>
__global__ __launch_bounds__(256) void gemm_nt_bf16_kernel(
    const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt, int ldb,
    float* __restrict__ C, int ldc, int M, int N, int K, int ksteps_per_split,
    float alpha, const float* __restrict__ bias, int relu, bf16* __restrict__ Cbf,
    int ldcb) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * 64 + wm * 32;
  const int n0 = blockIdx.x * 64 + wn * 32;
  const int kbeg = blockIdx.z * ksteps_per_split * 32;
  const int kend = min(K, kbeg + ksteps_per_split * 32);

  const int fr = lane & 15;        // fragment row (A) / col (B)
  const int fk = (lane >> 4) * 8;  // k offset within the 32-wide step

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ar0 = m0 + fr, ar1 = m0 + 16 + fr;
  const int br0 = n0 + fr, br1 = n0 + 16 + fr;
  const bool a0ok = ar0 < M, a1ok = ar1 < M, b0ok = br0 < N, b1ok = br1 < N;
  const bf16* pa0 = A + (size_t)(a0ok ? ar0 : 0) * lda;
  const bf16* pa1 = A + (size_t)(a1ok ? ar1 : 0) * lda;
  const bf16* pb0 = Bt + (size_t)(b0ok ? br0 : 0) * ldb;
  const bf16* pb1 = Bt + (size_t)(b1ok ? br1 : 0) * ldb;

#pragma unroll 2
  for (int k = kbeg; k < kend; k += 32) {
    const int kk = k + fk;
    bf16x8 a0 = load_frag(pa0 + kk, kk, kend, a0ok);
    bf16x8 a1 = load_frag(pa1 + kk, kk, kend, a1ok);
    bf16x8 b0 = load_frag(pb0 + kk, kk, kend, b0ok);
    bf16x8 b1 = load_frag(pb1 + kk, kk, kend, b1ok);
    acc[0][0] = mfma16(a0, b0, acc[0][0]);
    acc[0][1] = mfma16(a0, b1, acc[0][1]);
    acc[1][0] = mfma16(a1, b0, acc[1][0]);
    acc[1][1] = mfma16(a1, b1, acc[1][1]);
  }

#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + j * 16 + fr;
      if (col >= N) continue;
      float bv = 0.f;
      if (EPI && bias) bv = bias[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= M) continue;
        float v = alpha * acc[i][j][r];
        float* dst = C + (size_t)row * ldc + col;
        if (MODE == kAtomic) {
          atomicAdd(dst, v);
        } else {
          if (MODE == kAccum) v += *dst;
          if (EPI) {
            v += bv;
            if (relu) v = fmaxf(v, 0.f);
            if (Cbf) Cbf[(size_t)row * ldcb + col] = f2bf(v);
          }
          if (C) *dst = v;
        }
      }
    }
  }
}

}  // namespace tde

using namespace tde;

// Pick a split-K factor so that a small-M/N GEMM still spreads over the CUs.
TDE_API int tde_gemm_pick_splits(int M, int N, int K) {
  int tiles = ((M + 63) / 64) * ((N + 63) / 64);
  int ksteps = (K + 31) / 32;
  int splits = 1;
  if (tiles < 128) {
    splits = (192 + tiles - 1) / tiles;
    int max_splits = ksteps / 4 > 0 ? ksteps / 4 : 1;  // >= 4 k-steps per split
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
  }
  return splits;
}

// mode: 0 store, 1 accumulate (C += ...), 2 atomic accumulate (C must be
// pre-zeroed or hold the value to add to; required when splits > 1).
// bias/relu/Cbf: epilogue for mode 0/1 (ignored for atomic mode).
TDE_API int tde_gemm_nt_bf16(const void* A, int lda, const void* Bt, int ldb, float* C,
                             int ldc, int M, int N, int K, float alpha, int mode,
                             int splits, const float* bias, int relu, void* Cbf, int ldcb,
                             hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  if ((lda & 7) || (ldb & 7)) return -1;  // 16-byte fragment loads
  int ksteps = (K + 31) / 32;
  if (splits <= 0) splits = tde_gemm_pick_splits(M, N, K);
  if (splits > ksteps) splits = ksteps;
  if (splits > 1 && mode != kAtomic) return -2;
  int per = (ksteps + splits - 1) / splits;
  splits = (ksteps + per - 1) / per;
  dim3 grid((N + 63) / 64, (M + 63) / 64, splits);
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)Bt;
  bool epi = (bias != nullptr) || relu || (Cbf != nullptr);
  if (mode == kAtomic)
    gemm_nt_bf16_kernel<kAtomic, false><<<grid, 256, 0, stream>>>(
        a, lda, b, ldb, C, ldc, M, N, K, per, alpha, nullptr, 0, nullptr, 0);
  else if (mode == kAccum)
    (epi ? gemm_nt_bf16_kernel<kAccum, true> : gemm_nt_bf16_kernel<kAccum, false>)
        <<<grid, 256, 0, stream>>>(a, lda, b, ldb, C, ldc, M, N, K, per, alpha, bias, relu,
                                   (bf16*)Cbf, ldcb);
  else
    (epi ? gemm_nt_bf16_kernel<kStore, true> : gemm_nt_bf16_kernel<kStore, false>)
        <<<grid, 256, 0, stream>>>(a, lda, b, ldb, C, ldc, M, N, K, per, alpha, bias, relu,
                                   (bf16*)Cbf, ldcb);
  TDE_LAUNCH_CHECK();
  return 0;
}
