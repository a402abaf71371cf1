// Fused classifier head: [bias+ReLU epilogue of the previous Dense] -> Dense ->
// (softmax) -> SparseCategoricalCrossentropy -> accuracy, forward AND backward
// in one launch (TF's SparseSoftmaxCrossEntropyWithLogits is likewise a fused
// fwd+grad op).  SURVEY.md §2.5 A5-A9 / B12-B13; reference lines
// distributed_with_keras.py:37-43, mnist_keras_distributed.py:108-115.
//
// Keras semantics implemented here:
//   * loss reduction AUTO under a strategy = per-replica sum / GLOBAL batch
//     (`scale` = 1/global_batch), so a SUM all-reduce of the gradients gives the
//     mean gradient (SURVEY.md §7.4 "Loss reduction").
//   * Dense(10, activation='softmax') + 'sparse_categorical_crossentropy' is
//     computed from the pre-softmax logits (stable log-softmax, Q5).
//   * 'accuracy' = argmax(first max) == label.
//
// One workgroup = 16 rows, 4 waves.  All three products run on the exact-f32
// MFMA (v_mfma_f32_16x16x4_f32; no bf16 rounding in the loss path):
//   logits[16 x 16]  = h[16 x H] . W2[H x C]          (4 waves x H/16 k-steps, LDS sum)
//   softmax / CE / accuracy in registers on the MFMA C layout (16-lane groups)
//   dW2[H x C]       = h^T . dl                       (wave w: 16-row tiles of H)
//   dH[16 x H]       = dl . W2^T, ReLU mask           (wave w: 16-column tiles of H)
// dH is emitted in bf16 row-major and transposed (K-contiguous for the next
// MFMA GEMMs); bias grads by column sums; parameter grads are f32 atomics.
#include "tde_common.h"

namespace tde {

struct HeadArgs {
  const float* hin; int ldh;          // [B, H] pre-activation input (f32)
  const bf16* hin_b;                  // ... or a bf16 input (the layer-wise plan's activations)
  const float* pre_bias;              // [H] or null
  int pre_relu;
  const float* W2; const float* b2;   // [H, C], [C]
  const int* labels;                  // [B]
  int B, H, C;
  float scale;                        // 1 / global batch
  int compute_grad;
  float* dW2; float* db2; float* dpre_bias;   // += (nullable)
  bf16* G; int ldg; bf16* Gt; int ldgt; float* Gf; int ldgf;
  float* metrics;                     // += {loss_sum, correct, count}
  float* probs; int probs_are_logits; // [B, C] out (nullable)
  float* row_loss;                    // [B] out (nullable)
  float* zero_hin;                    // if set (== hin): rows consumed are zeroed for the next split-K accumulation
  long long* iterations;              // if set: block 0 advances the step counter (Keras optimizer.iterations)
  long long* stamps;                  // diagnostic phase stamps (nullable)
};

constexpr int HR = 16;          // rows per workgroup
constexpr int HMAX = 256;       // max hidden width
constexpr int HST = HMAX + 4;   // LDS row stride of h (floats; +4 breaks bank aliasing)

__device__ __forceinline__ f32x4 mfma_f32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// reductions over the 16 lanes of a lane-group (xor 8,4,2,1 stays inside the group)
__device__ __forceinline__ float g16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float g16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int g16_min_i(int v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ __launch_bounds__(256) void head_xent_kernel(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float hs[HR * HST];   // activated h, f32
  __shared__ float w2s[HMAX * 16];                              // W2 padded to 16 classes
  __shared__ float dls[HR * 16];                                // dlogits
  __shared__ float b2s[16];
  __shared__ int labs[HR];
  __shared__ __attribute__((aligned(16))) float lgp[3 * 64 * 4];  // logits partials of waves 1..3
  stamp(a.stamps, 0);
  const int H = a.H, C = a.C;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int r0 = blockIdx.x * HR;
  if (a.iterations && blockIdx.x == 0 && tid == 0) atomicAdd((unsigned long long*)a.iterations, 1ull);

  // ---- prologue: every global load issued up front into registers (one memory latency,
  // not one per loop trip), then the LDS images (H padded to Hp = 16k with zeros)
  const int Hp = (H + 15) & ~15;
  const int H4 = H / 4, Hp4 = Hp / 4;
  constexpr int NH4 = HR * (HMAX / 4) / 256;  // float4 of h per thread (max)
  constexpr int NW2 = HMAX * 16 / 256;        // W2 elements per thread (max)
  float4 hv[NH4], pb[NH4];
  float wv[NW2];
#pragma unroll
  for (int u = 0; u < NH4; ++u) {
    const int i = tid + u * 256, r = i / Hp4, j4 = (i - r * Hp4) * 4, row = r0 + r;
    hv[u] = float4{0.f, 0.f, 0.f, 0.f};
    pb[u] = float4{0.f, 0.f, 0.f, 0.f};
    if (i < HR * Hp4 && row < a.B && j4 < H) {
      if (a.hin_b) {
        const bf16x4 v = *reinterpret_cast<const bf16x4*>(a.hin_b + (size_t)row * a.ldh + j4);
        hv[u] = float4{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
      } else {
        hv[u] = *reinterpret_cast<const float4*>(a.hin + (size_t)row * a.ldh + j4);
      }
      if (a.pre_bias) pb[u] = *reinterpret_cast<const float4*>(a.pre_bias + j4);
    }
  }
#pragma unroll
  for (int u = 0; u < NW2; ++u) {
    const int i = tid + u * 256, j = i >> 4, c = i & 15;
    wv[u] = (i < Hp * 16 && c < C && j < H) ? a.W2[j * C + c] : 0.f;
  }
  const float bv = (tid < 16 && a.b2 && tid < C) ? a.b2[tid] : 0.f;
  const int lv = (tid < HR && r0 + tid < a.B) ? a.labels[r0 + tid] : 0;
#pragma unroll
  for (int u = 0; u < NH4; ++u) {
    const int i = tid + u * 256, r = i / Hp4, j4 = (i - r * Hp4) * 4;
    if (i < HR * Hp4) {
      float4 v = hv[u];
      v.x += pb[u].x; v.y += pb[u].y; v.z += pb[u].z; v.w += pb[u].w;
      if (a.pre_relu) {
        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
      }
      *reinterpret_cast<float4*>(hs + r * HST + j4) = v;
    }
  }
#pragma unroll
  for (int u = 0; u < NW2; ++u) {
    const int i = tid + u * 256;
    if (i < Hp * 16) w2s[i] = wv[u];
  }
  if (tid < 16) b2s[tid] = bv;
  if (tid < HR) labs[tid] = lv;
  lds_barrier();
  stamp(a.stamps, 1);
  if (a.zero_hin) {
    for (int i = tid; i < HR * H4; i += 256) {
      const int r = i / H4, j4 = (i - r * H4) * 4, row = r0 + r;
      if (row < a.B) *reinterpret_cast<float4*>(a.zero_hin + (size_t)row * a.ldh + j4) = float4{0.f, 0.f, 0.f, 0.f};
    }
  }

  // ---- logits: the Hp/4 k-steps split over the 4 waves (Hp is a multiple of 16), the
  // partial 16x16 tiles summed through LDS -- a 4x shorter dependent MFMA/LDS chain.
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  {
    const int kq = Hp / 4, kb = wave * kq;
    for (int k = kb; k < kb + kq; k += 4) acc = mfma_f32(hs[fr * HST + k + fq], w2s[(k + fq) * 16 + fr], acc);
    if (wave > 0) *reinterpret_cast<f32x4*>(lgp + ((wave - 1) * 64 + lane) * 4) = acc;
  }
  lds_barrier();
  // ---- softmax-CE (wave 0): lane holds logits[4*fq + i][fr]
  if (wave == 0) {
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const f32x4 p = *reinterpret_cast<const f32x4*>(lgp + (w * 64 + lane) * 4);
      acc[0] += p[0]; acc[1] += p[1]; acc[2] += p[2]; acc[3] += p[3];
    }
    float loss_acc = 0.f, corr_acc = 0.f, cnt_acc = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = fq * 4 + i, row = r0 + r;
      const bool valid = row < a.B;
      const bool cv = fr < C;
      const float z = cv ? acc[i] + b2s[fr] : -3.0e38f;
      const float m = row16_max(z);
      const float e = cv ? __expf(z - m) : 0.f;
      const float s = row16_sum(e);
      const float p = e / s;
      const int label = labs[r];
      const int am = row16_min(cv && z == m ? fr : 64);
      const float zl = __shfl(z, (lane & ~15) | (label & 15), 64);
      if (valid) {
        const float l = __logf(s) + m - zl;
        if (fr == 0) {
          loss_acc += l;
          corr_acc += (am == label) ? 1.f : 0.f;
          cnt_acc += 1.f;
          if (a.row_loss) a.row_loss[row] = l;
        }
        if (a.probs && cv) a.probs[(size_t)row * C + fr] = a.probs_are_logits ? z : p;
      }
      dls[r * 16 + fr] = (valid && cv) ? (p - (fr == label ? 1.f : 0.f)) * a.scale : 0.f;
    }
    if (a.metrics) {
      loss_acc = rows4_sum(loss_acc);
      corr_acc = rows4_sum(corr_acc);
      cnt_acc = rows4_sum(cnt_acc);
      if (lane == 0 && cnt_acc > 0.f) {
        atomicAdd(a.metrics + 0, loss_acc);
        atomicAdd(a.metrics + 1, corr_acc);
        atomicAdd(a.metrics + 2, cnt_acc);
      }
    }
  }
  stamp(a.stamps, 2);
  if (!a.compute_grad) return;
  lds_barrier();

  // ---- per wave w: dW2 rows [16w, 16w+16) of H and dH columns [16w, 16w+16)
  for (int t = wave; t < Hp / 16; t += 4) {
    // dW2[j][c] = sum_r h[r][j] * dl[r][c]   (A = h^T tile, B = dl)
    f32x4 gw = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < HR; k += 4) gw = mfma_f32(hs[(k + fq) * HST + t * 16 + fr], dls[(k + fq) * 16 + fr], gw);
    if (a.dW2 && fr < C) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (t * 16 + fq * 4 + i < H) atomicAdd(a.dW2 + (size_t)(t * 16 + fq * 4 + i) * C + fr, gw[i]);
    }
    // dH[r][j] = sum_c dl[r][c] * W2[j][c]   (A = dl, B = W2^T)
    f32x4 gh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 16; k += 4) gh = mfma_f32(dls[fr * 16 + k + fq], w2s[(t * 16 + fr) * 16 + k + fq], gh);
    // lane holds dH[4*fq + i][16t + fr]
    float colsum = 0.f;
    const int j = t * 16 + fr;
    const bool jok = j < H;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = fq * 4 + i, row = r0 + r;
      float v = gh[i];
      if (a.pre_relu && !(hs[r * HST + j] > 0.f)) v = 0.f;
      if (row >= a.B) v = 0.f;
      colsum += v;
      if (row < a.B && jok) {
        if (a.G) a.G[(size_t)row * a.ldg + j] = f2bf(v);
        if (a.Gf) a.Gf[(size_t)row * a.ldgf + j] = v;
      }
      if (a.Gt && jok && row < a.ldgt) a.Gt[(size_t)j * a.ldgt + row] = f2bf(v);
    }
    colsum += __shfl_xor(colsum, 16, 64);
    colsum += __shfl_xor(colsum, 32, 64);
    if (a.dpre_bias && fq == 0 && jok) atomicAdd(a.dpre_bias + j, colsum);
  }
  if (a.db2 && wave == 0) {
    float s = dls[fq * 4 * 16 + fr] + dls[(fq * 4 + 1) * 16 + fr] + dls[(fq * 4 + 2) * 16 + fr] +
              dls[(fq * 4 + 3) * 16 + fr];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (fq == 0 && fr < C) atomicAdd(a.db2 + fr, s);
  }
  stamp(a.stamps, 3);
}

}  // namespace tde

using namespace tde;

TDE_API int tde_head_xent(const float* hin, int ldh, const float* pre_bias, int pre_relu,
                          const float* W2, const float* b2, const int* labels, int B, int H,
                          int C, float scale, int compute_grad, float* dW2, float* db2,
                          float* dpre_bias, void* G, int ldg, void* Gt, int ldgt, float* Gf,
                          int ldgf, float* metrics, float* probs, int probs_are_logits,
                          float* row_loss, int zero_hin, long long* iterations, long long* stamps,
                          int hin_bf16, hipStream_t stream) {
  if (C > 16 || H > HMAX || H % 4 || (ldh & 3)) return -1;
  if (hin_bf16 ? (((uintptr_t)hin & 7) || zero_hin) : (((uintptr_t)hin | (uintptr_t)pre_bias) & 15)) return -2;
  HeadArgs a{hin_bf16 ? nullptr : hin, ldh, hin_bf16 ? (const bf16*)hin : nullptr, pre_bias, pre_relu, W2, b2,
             labels, B, H, C, scale, compute_grad, dW2, db2, dpre_bias, (bf16*)G, ldg, (bf16*)Gt, ldgt, Gf, ldgf,
             metrics, probs, probs_are_logits, row_loss, zero_hin ? const_cast<float*>(hin) : nullptr, iterations,
             stamps};
  int rows = B;
  if (Gt && ldgt > rows) rows = ldgt;
  const int grid = (rows + HR - 1) / HR;
  head_xent_kernel<<<grid, 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}
