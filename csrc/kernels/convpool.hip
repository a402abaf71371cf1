// Fused Conv2D(3x3, VALID, C_in=1, bias, ReLU) + MaxPooling2D(2x2/2) — the
// first two layers of the DWK/TF2M small CNN (distributed_with_keras.py:34-35,
// tf2_mnist_distributed.py:67-68; SURVEY.md §2.5 A1/A2 forward, A11-A13 backward).
//
// C_in = 1 makes the conv a K=9 reduction: far below one MFMA K-step, so this
// is a register-tiled VALU kernel.  One workgroup = one pooled output position
// x 64 images; wave w owns channels [8w, 8w+8) so the filter taps are wave-
// uniform (scalar loads) and each lane (= one image) computes the 2x2 window of
// conv outputs for 8 channels from a 4x4 input patch held in registers.
//
// Outputs, in the layouts the downstream MFMA GEMMs want (both K-contiguous):
//   P   [B, Hp*Wp*C]      bf16  (Flatten order h,w,c — Keras-compatible)
//   Pt  [Hp*Wp*C, ldPt]   bf16  (transposed, for dW = P^T . G)
//   amax[B, Hp*Wp*C]      u8    (window argmax 0..3 of the pre-ReLU value, 0xFF = ReLU inactive)
//
// Backward (per pooled position): dP = G . W1^T for this position's C rows of
// the following Dense kernel is computed in-kernel with MFMA (the Flatten/Dense
// input gradient never round-trips through HBM), routed through the pool argmax
// and the ReLU mask, then reduced into dW[3,3,1,C] and db[C].
#include "tde_common.h"

namespace tde {

__global__ __launch_bounds__(1024) void conv3x3c1_relu_pool_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    bf16* __restrict__ P, bf16* __restrict__ Pt, int ldPt, uint8_t* __restrict__ amax, int B,
    int H, int W, int C, float* __restrict__ zbuf, int zn) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int Wp = (W - 2) / 2, Hp = (H - 2) / 2;
  const int p = blockIdx.x;
  const int py = p / Wp, px = p - py * Wp;
  const int b = blockIdx.y * 64 + lane;
  const int c0 = wave * 8;
  const int K = Hp * Wp * C;

  // Zero-on-the-way: clear the split-K accumulator of the next GEMM.
  if (zbuf) {
    const int nthr = gridDim.x * gridDim.y * blockDim.x;
    const int tid = (blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
    for (int i = tid; i < zn; i += nthr) zbuf[i] = 0.f;
  }

  if (b < B) {
    float patch[16];
    const float* xb = x + (size_t)b * H * W + (2 * py) * W + 2 * px;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float2* row = reinterpret_cast<const float2*>(xb + r * W);
      float2 u = row[0], v = row[1];
      patch[r * 4 + 0] = u.x; patch[r * 4 + 1] = u.y;
      patch[r * 4 + 2] = v.x; patch[r * 4 + 3] = v.y;
    }
    bf16x8 outv;
    uint8_t idxv[8];
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      const int c = c0 + cc;
      float wt[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) wt[t] = w[t * C + c];
      const float bc = bias ? bias[c] : 0.f;
      float best = -3.0e38f;
      int bi = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int dy = q >> 1, dx = q & 1;
        float z = bc;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) z = fmaf(patch[(dy + ky) * 4 + dx + kx], wt[ky * 3 + kx], z);
        if (z > best) { best = z; bi = q; }
      }
      outv[cc] = f2bf(fmaxf(best, 0.f));
      idxv[cc] = best > 0.f ? (uint8_t)bi : (uint8_t)0xFF;
    }
    const size_t off = (size_t)b * K + (size_t)p * C + c0;
    *reinterpret_cast<bf16x8*>(P + off) = outv;
    uint64_t packed = 0;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) packed |= (uint64_t)idxv[cc] << (8 * cc);
    *reinterpret_cast<uint64_t*>(amax + off) = packed;
    if (Pt) {
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) Pt[(size_t)(p * C + c0 + cc) * ldPt + b] = outv[cc];
    }
  } else if (Pt && b < ldPt) {
    // Zero the K-padding columns of the transposed copy.
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) Pt[(size_t)(p * C + c0 + cc) * ldPt + b] = f2bf(0.f);
  }
}

// grid: (Hp*Wp, ceil(B/64)), block 256.
__global__ __launch_bounds__(256) void conv3x3c1_relu_pool_bwd_kernel(
    const float* __restrict__ x, const uint8_t* __restrict__ amax, const bf16* __restrict__ G,
    int ldg, const bf16* __restrict__ W1, int ldw, int Hd, float* __restrict__ dw,
    float* __restrict__ db, int B, int H, int W, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* xs = smem;                 // [64][16]
  float* dps = xs + 64 * 16;        // [64][C]
  float* red = dps + 64 * C;        // [G][C][10]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int Wp = (W - 2) / 2;
  const int p = blockIdx.x;
  const int py = p / Wp, px = p - py * Wp;
  const int b0 = blockIdx.y * 64;
  const int K = ((H - 2) / 2) * Wp * C;

  // Stage the 4x4 input patches of the 64 images.
  {
    const int bl = threadIdx.x >> 2, r = threadIdx.x & 3;
    const int b = b0 + bl;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (b < B) {
      const float2* row = reinterpret_cast<const float2*>(x + (size_t)b * H * W + (2 * py + r) * W + 2 * px);
      float2 u = row[0], t = row[1];
      v = float4{u.x, u.y, t.x, t.y};
    }
    *reinterpret_cast<float4*>(xs + bl * 16 + r * 4) = v;
  }

  // dP[b][c] = sum_j G[b][j] * W1[p*C + c][j]   (MFMA, wave = 16 images).
  {
    const int fr = lane & 15, fk = (lane >> 4) * 8;
    const int brow = b0 + wave * 16 + fr;
    const bool bok = brow < B;
    for (int nt = 0; nt < C / 16; ++nt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const bf16* wrow = W1 + (size_t)(p * C + nt * 16 + fr) * ldw;
      const bf16* grow = G + (size_t)(bok ? brow : 0) * ldg;
      for (int k = 0; k < Hd; k += 32) {
        bf16x8 a = load_frag(grow + k + fk, k + fk, Hd, bok);
        bf16x8 bb = load_frag(wrow + k + fk, k + fk, Hd, true);
        acc = mfma16(a, bb, acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) dps[(wave * 16 + (lane >> 4) * 4 + r) * C + nt * 16 + fr] = acc[r];
    }
  }
  __syncthreads();

  // Route through argmax + ReLU mask and reduce into the 3x3 taps.
  const int ngrp = 256 / C;
  const int c = threadIdx.x % C, g = threadIdx.x / C;
  float acc_w[9], acc_b = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) acc_w[t] = 0.f;
  if (g < ngrp) {
    for (int bl = g; bl < 64; bl += ngrp) {
      const int b = b0 + bl;
      if (b >= B) break;
      const uint8_t id = amax[(size_t)b * K + (size_t)p * C + c];
      if (id == 0xFF) continue;
      const float v = dps[bl * C + c];
      const int dy = id >> 1, dx = id & 1;
      acc_b += v;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc_w[ky * 3 + kx] = fmaf(v, xs[bl * 16 + (dy + ky) * 4 + dx + kx], acc_w[ky * 3 + kx]);
    }
    float* rp = red + (g * C + c) * 10;
#pragma unroll
    for (int t = 0; t < 9; ++t) rp[t] = acc_w[t];
    rp[9] = acc_b;
  }
  __syncthreads();
  for (int o = threadIdx.x; o < C * 10; o += 256) {
    const int cc = o / 10, t = o - cc * 10;
    float s = 0.f;
    for (int gg = 0; gg < ngrp; ++gg) s += red[(gg * C + cc) * 10 + t];
    if (t < 9) atomicAdd(dw + t * C + cc, s);
    else if (db) atomicAdd(db + cc, s);
  }
}

}  // namespace tde

using namespace tde;

TDE_API int tde_conv3x3c1_relu_pool_fwd(const float* x, const float* w, const float* bias,
                                        void* P, void* Pt, int ldPt, uint8_t* amax, int B,
                                        int H, int W, int C, float* zbuf, int zn,
                                        hipStream_t stream) {
  if (C % 8 || C > 128 || (W & 1)) return -1;
  int Hp = (H - 2) / 2, Wp = (W - 2) / 2;
  int by = (B + 63) / 64;
  if (Pt) {
    int byp = (ldPt + 63) / 64;  // cover padding columns too
    if (byp > by) by = byp;
  }
  dim3 grid(Hp * Wp, by);
  conv3x3c1_relu_pool_fwd_kernel<<<grid, (C / 8) * 64, 0, stream>>>(
      x, w, bias, (bf16*)P, (bf16*)Pt, ldPt, amax, B, H, W, C, zbuf, zn);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_conv3x3c1_relu_pool_bwd(const float* x, const uint8_t* amax, const void* G,
                                        int ldg, const void* W1, int ldw, int Hd, float* dw,
                                        float* db, int B, int H, int W, int C,
                                        hipStream_t stream) {
  if (C % 16 || C > 256 || (ldg & 7) || (ldw & 7)) return -1;
  int Hp = (H - 2) / 2, Wp = (W - 2) / 2;
  dim3 grid(Hp * Wp, (B + 63) / 64);
  size_t lds = (64 * 16 + 64 * C + (256 / C) * C * 10) * sizeof(float);
  conv3x3c1_relu_pool_bwd_kernel<<<grid, 256, lds, stream>>>(
      x, amax, (const bf16*)G, ldg, (const bf16*)W1, ldw, Hd, dw, db, B, H, W, C);
  TDE_LAUNCH_CHECK();
  return 0;
}
