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
// The gradient of the preceding Dense's bias+ReLU epilogue (dbias, ReLU mask) is
// produced here too, and dH is emitted in bf16 both row-major and transposed so
// the following MFMA GEMMs read K-contiguous fragments.
#include "tde_common.h"

namespace tde {

struct HeadArgs {
  const float* hin; int ldh;          // [B, H] pre-activation input (f32)
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

constexpr int kHeadRows = 8;

__global__ __launch_bounds__(256) void head_xent_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = a.H, C = a.C, R = kHeadRows;
  float* hs = sm;                 // [R][H]
  float* w2s = hs + R * H;        // [H][C]
  float* lg = w2s + H * C;        // [R][C]
  float* dls = lg + R * C;        // [R][C]
  float* dhs = dls + R * C;       // [R][H]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * R;
  stamp(a.stamps, 0);
  if (a.iterations && blockIdx.x == 0 && tid == 0) atomicAdd((unsigned long long*)a.iterations, 1ull);
  // Prefetch everything this block needs from global memory up front.
  int label_pref = 0;
  if (tid < R && r0 + tid < a.B) label_pref = a.labels[r0 + tid];
  for (int i = tid; i < R * H; i += 256) {
    const int r = i / H, j = i - r * H, row = r0 + r;
    float v = 0.f;
    if (row < a.B) {
      v = a.hin[(size_t)row * a.ldh + j];
      if (a.pre_bias) v += a.pre_bias[j];
      if (a.pre_relu) v = fmaxf(v, 0.f);
    }
    hs[i] = v;
  }
  for (int i = tid; i < H * C; i += 256) w2s[i] = a.W2[i];
  float b2v = 0.f;
  if (tid < C && a.b2) b2v = a.b2[tid];
  int* labs = reinterpret_cast<int*>(dhs);  // scratch until dh is computed
  if (tid < R) labs[tid] = label_pref;
  __shared__ float b2sh[64];
  if (tid < C) b2sh[tid] = b2v;
  lds_barrier();
  stamp(a.stamps, 1);
  if (a.zero_hin) {
    for (int i = tid; i < R * H; i += 256) {
      const int r = i / H, j = i - r * H, row = r0 + r;
      if (row < a.B) a.zero_hin[(size_t)row * a.ldh + j] = 0.f;
    }
  }

  for (int o = tid; o < R * C; o += 256) {
    const int r = o / C, c = o - r * C;
    float s0 = b2sh[c], s1 = 0.f, s2 = 0.f, s3 = 0.f;
    const float* hr = hs + r * H;
    int j = 0;
    for (; j + 4 <= H; j += 4) {
      s0 = fmaf(hr[j], w2s[j * C + c], s0);
      s1 = fmaf(hr[j + 1], w2s[(j + 1) * C + c], s1);
      s2 = fmaf(hr[j + 2], w2s[(j + 2) * C + c], s2);
      s3 = fmaf(hr[j + 3], w2s[(j + 3) * C + c], s3);
    }
    for (; j < H; ++j) s0 = fmaf(hr[j], w2s[j * C + c], s0);
    lg[o] = (s0 + s1) + (s2 + s3);
  }
  lds_barrier();

  float loss_acc = 0.f, corr_acc = 0.f, cnt_acc = 0.f;
  for (int r = wave; r < R; r += 4) {
    const int row = r0 + r;
    const bool valid = row < a.B;
    const float v = lane < C ? lg[r * C + lane] : -3.0e38f;
    const float m = wave_max(v);
    const float e = lane < C ? __expf(v - m) : 0.f;
    const float s = wave_sum(e);
    const float p = e / s;
    const int label = valid ? labs[r] : 0;
    const float lse = __logf(s) + m;
    const unsigned long long mask = __ballot(lane < C && v == m);
    const int am = __ffsll((long long)mask) - 1;
    const float lab_logit = lg[r * C + (label < C ? label : 0)];
    if (valid) {
      const float l = lse - lab_logit;
      loss_acc += l;
      corr_acc += (am == label) ? 1.f : 0.f;
      cnt_acc += 1.f;
      if (lane == 0 && a.row_loss) a.row_loss[row] = l;
      if (a.probs && lane < C) a.probs[(size_t)row * C + lane] = a.probs_are_logits ? v : p;
    }
    if (lane < C) dls[r * C + lane] = valid ? (p - (lane == label ? 1.f : 0.f)) * a.scale : 0.f;
  }
  if (a.metrics && lane == 0 && cnt_acc > 0.f) {
    atomicAdd(a.metrics + 0, loss_acc);
    atomicAdd(a.metrics + 1, corr_acc);
    atomicAdd(a.metrics + 2, cnt_acc);
  }
  stamp(a.stamps, 2);
  if (!a.compute_grad) return;
  lds_barrier();

  // dW2 = h^T . dl ; db2 = sum dl
  if (a.dW2) {
    for (int o = tid; o < H * C; o += 256) {
      const int j = o / C, c = o - j * C;
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < R; ++r) s = fmaf(hs[r * H + j], dls[r * C + c], s);
      atomicAdd(a.dW2 + o, s);
    }
  }
  if (a.db2) {
    for (int c = tid; c < C; c += 256) {
      float s = 0.f;
      for (int r = 0; r < R; ++r) s += dls[r * C + c];
      atomicAdd(a.db2 + c, s);
    }
  }
  // dH = dl . W2^T, through the ReLU mask of the previous epilogue.
  for (int o = tid; o < R * H; o += 256) {
    const int r = o / H, j = o - r * H, row = r0 + r;
    float s = 0.f;
    for (int c = 0; c < C; ++c) s = fmaf(dls[r * C + c], w2s[j * C + c], s);
    if (a.pre_relu && !(hs[o] > 0.f)) s = 0.f;
    dhs[o] = s;
    if (row < a.B) {
      if (a.G) a.G[(size_t)row * a.ldg + j] = f2bf(s);
      if (a.Gf) a.Gf[(size_t)row * a.ldgf + j] = s;
    }
  }
  lds_barrier();
  if (a.Gt) {
    // Transposed copy: consecutive threads walk rows -> coalesced along B.
    for (int o = tid; o < R * H; o += 256) {
      const int j = o / R, r = o - j * R, row = r0 + r;
      if (row < a.ldgt) a.Gt[(size_t)j * a.ldgt + row] = f2bf(row < a.B ? dhs[r * H + j] : 0.f);
    }
  }
  if (a.dpre_bias) {
    for (int j = tid; j < H; j += 256) {
      float s = 0.f;
      for (int r = 0; r < R; ++r) s += dhs[r * H + j];
      atomicAdd(a.dpre_bias + j, s);
    }
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
                          hipStream_t stream) {
  if (C > 64 || H * C > 16384 || H > 2048) return -1;
  HeadArgs a{hin, ldh, pre_bias, pre_relu, W2, b2, labels, B, H, C, scale, compute_grad,
             dW2, db2, dpre_bias, (bf16*)G, ldg, (bf16*)Gt, ldgt, Gf, ldgf, metrics, probs,
             probs_are_logits, row_loss, zero_hin ? const_cast<float*>(hin) : nullptr, iterations, stamps};
  int rows = B;
  if (Gt && ldgt > rows) rows = ldgt;
  int grid = (rows + kHeadRows - 1) / kHeadRows;
  size_t lds = (size_t)(2 * kHeadRows * H + H * C + 2 * kHeadRows * C) * sizeof(float);
  head_xent_kernel<<<grid, 256, lds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}
