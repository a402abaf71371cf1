// Fused training step for small image classifiers whose trunk is per-image: LeNet-5
// (BASELINE.json config 2), dense MLPs (tf2_mnist_distributed.py's CPU plumbing config) and any
// [Conv2D(stride 1, relu) [MaxPooling2D(2)]]* Flatten Dense* head with sparse softmax-CE.
//
// MI355X-first design: at MNIST sizes a whole image's activations (LeNet-5: 8.9K floats) fit in LDS, so
// one workgroup owns one image and runs the forward, the loss and the whole input-gradient chain out
// of LDS, reading weights from L2 — the layer-by-layer plan's ~20 launches with their HBM round trips
// and kernel boundaries become two launches:
//
//   smallnet_step_kernel   grid = batch.  Forward (conv / pool / dense, fp32 FMA), softmax-CE with
//                          (p - onehot) / global_batch into the logits buffer, then the backward in
//                          place (every gradient overwrites the activation it belongs to, masked by
//                          that activation's ReLU), per-image conv weight/bias gradients into `part`,
//                          dense inputs and pre-activation gradients into `rec`.
//   smallnet_wgrad_kernel  batch reductions: conv partials summed over images, dense weight gradients
//                          as X^T G over the batch on the exact-f32 MFMA, bias gradients, metrics; each gradient
//                          element is finished by exactly one thread, which either stores it into the
//                          flat gradient bucket (step mode "plain": all-reduce + optimizer follow) or
//                          applies the optimizer to it right there (step mode "local").
//
// Reference semantics: Keras Conv2D/MaxPooling2D/Dense/SCCE (SURVEY.md §2.5 A1-A14;
// distributed_with_keras.py:33-43, tf2_mnist_distributed.py:66-83); the per-step loss is
// sum(CE) / global_batch (Keras AUTO reduction under a strategy).
#include <cstdlib>
#include <type_traits>

#include "tde_common.h"
#include "tde_optim.h"

namespace tde {

constexpr int kSnMaxLayers = 12;
constexpr int kSnLds = 28 * 1024;  // floats of LDS per workgroup (112 KiB)
constexpr int kSnThreads = 512;
enum { kSnConv = 0, kSnPool = 1, kSnDense = 2 };

// All offsets in floats.  Buffers: `in` / `out` are the layer's input / output activations in LDS;
// after the consumer's backward `out` holds the gradient w.r.t. this layer's output (masked by its
// ReLU), and this layer's backward writes its input gradient into `in` (masked when mask_in).
struct SnLayer {
  int kind, relu, mask_in, need_gin;
  int H, W, C, Ho, Wo, Co;
  int kh, kw, pt, pl;
  int w_off, b_off;    // flat weight offsets (b_off < 0: no bias)
  int in, out, wl;     // LDS offsets: input, output, staged conv kernel (+ bias)
  int part, xo, go;    // conv: offset in the per-image partial record; dense: X / G offsets in `rec`
};
constexpr int kSnLayerInts = sizeof(SnLayer) / sizeof(int);

struct SnArgs {
  SnLayer L[kSnMaxLayers];
  int nl, mode, B, x_stride, in0, n_in0;  // mode 0 train, 1 eval, 2 predict
  int img_H, img_W, img_C, pad_t, pad_l, img_Wp, img_Hp;  // the image lands zero-padded for a same-padded first conv
  const float* w;
  const float* x;
  const int* y;
  float* part;
  int npart, nrec;
  float* rec;
  float* metrics;
  long long* iterations;
  float scale;
  float* probs;
  int probs_softmax;
  long long* stamps;  // optional phase timestamps of workgroup 0 (wall clock, 100 MHz)
  int mfma;           // phases (bit 0 fwd, 1 wgrad, 2 dgrad) of the compile-time-geometry convs on the f32 MFMA
};

template <int CG>
__device__ __forceinline__ void ld_cg(const float* p, float* v) {
  if constexpr (CG == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (CG == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  } else {
    v[0] = p[0];
  }
}

template <int CG>
__device__ __forceinline__ void st_cg(float* p, const float* v) {
  if constexpr (CG == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (CG == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else {
    p[0] = v[0];
  }
}

// The conv loops are LDS-latency bound (a workgroup per image leaves 2 waves per SIMD), so each is
// shaped for independent LDS reads in flight: the (kw, ci) run of a tap row is contiguous in both the
// NHWC input and the HWIO kernel and is walked as one unrolled loop; long reductions are sliced over
// threads and folded with LDS float atomics.
constexpr int kSnScratch = 4096;  // floats of LDS scratch at offset 0 of the layout
constexpr int kSnUnroll = 8;
constexpr int kSnItemsTarget = 1024;

// conv forward: item = (output pixel p, channel group g); pixels fastest, so a wave shares g and its
// kernel reads are LDS broadcasts
template <int CG>
__device__ void sn_conv_fwd(const SnLayer L, float* s) {
  const float* in = s + L.in;
  const float* wl = s + L.wl;
  float* out = s + L.out;
  const int P = L.Ho * L.Wo, ng = L.Co / CG;
  for (int it = threadIdx.x; it < P * ng; it += kSnThreads) {
    const int p = it % P, g = it / P;
    const int oh = p / L.Wo, ow = p - oh * L.Wo;
    float acc[CG], acc2[CG];
    if (L.b_off >= 0) {
      ld_cg<CG>(wl + L.kh * L.kw * L.C * L.Co + g * CG, acc);
    } else {
#pragma unroll
      for (int k = 0; k < CG; ++k) acc[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < CG; ++k) acc2[k] = 0.f;
    const int kh0 = max(0, L.pt - oh), kh1 = min(L.kh, L.H + L.pt - oh);
    const int kw0 = max(0, L.pl - ow), kw1 = min(L.kw, L.W + L.pl - ow);
    const int run = (kw1 - kw0) * L.C;
    for (int kh = kh0; kh < kh1; ++kh) {
      const int ih = oh + kh - L.pt;
      const float* ip = in + (ih * L.W + ow + kw0 - L.pl) * L.C;
      const float* wp = wl + ((kh * L.kw + kw0) * L.C) * L.Co + g * CG;
      int r = 0;
      for (; r + 4 <= run; r += 4) {
        float a[4], wv[4][CG];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u] = ip[r + u];
          ld_cg<CG>(wp + (r + u) * L.Co, wv[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; u += 2) {
#pragma unroll
          for (int k = 0; k < CG; ++k) {
            acc[k] = fmaf(a[u], wv[u][k], acc[k]);
            acc2[k] = fmaf(a[u + 1], wv[u + 1][k], acc2[k]);
          }
        }
      }
      for (; r < run; ++r) {
        float wv[CG];
        ld_cg<CG>(wp + r * L.Co, wv);
#pragma unroll
        for (int k = 0; k < CG; ++k) acc[k] = fmaf(ip[r], wv[k], acc[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < CG; ++k) {
      acc[k] += acc2[k];
      if (L.relu) acc[k] = fmaxf(acc[k], 0.f);
    }
    st_cg<CG>(out + p * L.Co + g * CG, acc);
  }
}

// conv per-image weight (+ bias) gradient: item = (tap-channel t, channel group g, output-row slice);
// t fastest (the output-gradient reads are broadcasts).  With more than one slice the partials meet in
// LDS scratch (float atomics); the bias sums ride along as t = T.
template <int CG>
__device__ void sn_conv_wgrad(const SnLayer L, float* s, float* part) {
  const float* in = s + L.in;
  const float* dz = s + L.out;
  const int T = L.kh * L.kw * L.C, ng = L.Co / CG;
  const int Tb = T + (L.b_off >= 0 ? 1 : 0);
  const int n = Tb * L.Co;
  int S = 1;
  if (n <= kSnScratch) S = max(1, min(L.Ho, kSnItemsTarget / (Tb * ng)));
  float* red = s;  // scratch
  if (S > 1) {
    for (int i = threadIdx.x; i < n; i += kSnThreads) red[i] = 0.f;
    __syncthreads();
  }
  for (int it = threadIdx.x; it < Tb * ng * S; it += kSnThreads) {
    const int t = it % Tb, g = (it / Tb) % ng, sl = it / (Tb * ng);
    float acc[CG], acc2[CG];
#pragma unroll
    for (int k = 0; k < CG; ++k) acc[k] = acc2[k] = 0.f;
    if (t == T) {  // bias: sum of the output gradient over this slice's rows
      const int oh0 = L.Ho * sl / S, oh1 = L.Ho * (sl + 1) / S;
      for (int p = oh0 * L.Wo; p < oh1 * L.Wo; ++p) {
        float d[CG];
        ld_cg<CG>(dz + p * L.Co + g * CG, d);
#pragma unroll
        for (int k = 0; k < CG; ++k) acc[k] += d[k];
      }
    } else {
      const int ci = t % L.C, kk = t / L.C;
      const int kh = kk / L.kw, kw = kk - kh * L.kw;
      const int r0 = max(0, L.pt - kh), r1 = min(L.Ho, L.H + L.pt - kh);
      const int oh0 = max(r0, L.Ho * sl / S), oh1 = min(r1, L.Ho * (sl + 1) / S);
      const int ow0 = max(0, L.pl - kw), ow1 = min(L.Wo, L.W + L.pl - kw);
      for (int oh = oh0; oh < oh1; ++oh) {
        const float* ip = in + ((oh + kh - L.pt) * L.W + kw - L.pl) * L.C + ci;
        const float* dp = dz + oh * L.Wo * L.Co + g * CG;
        int ow = ow0;
        for (; ow + 4 <= ow1; ow += 4) {
          float a[4], d[4][CG];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            a[u] = ip[(ow + u) * L.C];
            ld_cg<CG>(dp + (ow + u) * L.Co, d[u]);
          }
#pragma unroll
          for (int u = 0; u < 4; u += 2) {
#pragma unroll
            for (int k = 0; k < CG; ++k) {
              acc[k] = fmaf(a[u], d[u][k], acc[k]);
              acc2[k] = fmaf(a[u + 1], d[u + 1][k], acc2[k]);
            }
          }
        }
        for (; ow < ow1; ++ow) {
          float d[CG];
          ld_cg<CG>(dp + ow * L.Co, d);
#pragma unroll
          for (int k = 0; k < CG; ++k) acc[k] = fmaf(ip[ow * L.C], d[k], acc[k]);
        }
      }
    }
    const int e = t * L.Co + g * CG;
    if (S > 1) {
#pragma unroll
      for (int k = 0; k < CG; ++k) atomicAdd(&red[e + k], acc[k] + acc2[k]);
    } else {
#pragma unroll
      for (int k = 0; k < CG; ++k) part[L.part + e + k] = acc[k] + acc2[k];
    }
  }
  if (S > 1) {
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kSnThreads) part[L.part + i] = red[i];
  }
}

// conv input gradient, written over the input activation: item = (input pixel q, channel ci), q
// fastest (the kernel reads are broadcasts)
template <int CG>
__device__ void sn_conv_dgrad(const SnLayer L, float* s) {
  float* in = s + L.in;
  const float* dz = s + L.out;
  const float* wl = s + L.wl;
  const int Q = L.H * L.W;
  for (int it = threadIdx.x; it < Q * L.C; it += kSnThreads) {
    const int q = it % Q, ci = it / Q;
    const int ih = q / L.W, iw = q - ih * L.W;
    // output pixels that read input (ih, iw) through tap (kh, kw): oh = ih - kh + pt
    const int kh0 = max(0, ih + L.pt - L.Ho + 1), kh1 = min(L.kh, ih + L.pt + 1);
    const int kw0 = max(0, iw + L.pl - L.Wo + 1), kw1 = min(L.kw, iw + L.pl + 1);
    float acc = 0.f, acc2 = 0.f;
    for (int kh = kh0; kh < kh1; ++kh) {
      const int oh = ih - kh + L.pt;
      for (int kw = kw0; kw < kw1; ++kw) {
        const int ow = iw - kw + L.pl;
        const float* dp = dz + (oh * L.Wo + ow) * L.Co;
        const float* wp = wl + ((kh * L.kw + kw) * L.C + ci) * L.Co;
        int co = 0;
        for (; co + 4 * CG <= L.Co; co += 4 * CG) {
          float d[4][CG], wv[4][CG];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            ld_cg<CG>(dp + co + u * CG, d[u]);
            ld_cg<CG>(wp + co + u * CG, wv[u]);
          }
#pragma unroll
          for (int u = 0; u < 4; u += 2) {
#pragma unroll
            for (int k = 0; k < CG; ++k) {
              acc = fmaf(d[u][k], wv[u][k], acc);
              acc2 = fmaf(d[u + 1][k], wv[u + 1][k], acc2);
            }
          }
        }
        for (; co < L.Co; co += CG) {
          float d[CG], wv[CG];
          ld_cg<CG>(dp + co, d);
          ld_cg<CG>(wp + co, wv);
#pragma unroll
          for (int k = 0; k < CG; ++k) acc = fmaf(d[k], wv[k], acc);
        }
      }
    }
    acc += acc2;
    const int e = q * L.C + ci;
    if (L.mask_in && !(in[e] > 0.f)) acc = 0.f;
    in[e] = acc;
  }
}

// ---------------------------------------------------------------------------------------
// Compile-time-geometry conv phases for the shapes of the zoo models (valid convs; a same-padded first
// conv reads the zero-padded image).  Constant trip counts let every tap / channel loop unroll with
// immediate LDS offsets, so the VALU work is the FMAs instead of runtime-stride address arithmetic
// (the generic phases above spend ~5 VALU instructions per FMA).
constexpr int sn_slices(int Ho, int items) {
  int best = 1;
  for (int d = 1; d <= Ho; ++d)
    if (Ho % d == 0 && items * d <= kSnItemsTarget) best = d;
  return best;
}

template <int CG, int KH, int KW, int C, int Co, int Win, int Ho, int Wo>
__device__ void sn_conv_fwd_c(const SnLayer L, float* s) {
  constexpr int P = Ho * Wo, NG = Co / CG;
  const float* in = s + L.in;
  const float* wl = s + L.wl;
  float* out = s + L.out;
  for (int it = threadIdx.x; it < P * NG; it += kSnThreads) {
    const int p = it % P, g = it / P;
    const int oh = p / Wo, ow = p % Wo;
    const float* ip = in + (oh * Win + ow) * C;
    const float* wp = wl + g * CG;
    float acc[CG], acc2[CG];
    if (L.b_off >= 0) {
      ld_cg<CG>(wl + KH * KW * C * Co + g * CG, acc);
    } else {
#pragma unroll
      for (int k = 0; k < CG; ++k) acc[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < CG; ++k) acc2[k] = 0.f;
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
#pragma unroll
      for (int r = 0; r < KW * C; ++r) {
        const float a = ip[kh * Win * C + r];
        float w[CG];
        ld_cg<CG>(wp + (kh * KW * C + r) * Co, w);
#pragma unroll
        for (int k = 0; k < CG; ++k) {
          if (r & 1) acc2[k] = fmaf(a, w[k], acc2[k]);
          else acc[k] = fmaf(a, w[k], acc[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < CG; ++k) {
      acc[k] += acc2[k];
      if (L.relu) acc[k] = fmaxf(acc[k], 0.f);
    }
    st_cg<CG>(out + p * Co + g * CG, acc);
  }
}

template <int CG, int KH, int KW, int C, int Co, int Win, int Ho, int Wo>
__device__ void sn_conv_wgrad_c(const SnLayer L, float* s, float* part) {
  constexpr int T = KH * KW * C, NG = Co / CG;
  constexpr int S = sn_slices(Ho, T * NG), R = Ho / S;
  static_assert(T * Co + Co <= kSnScratch, "scratch");
  const float* in = s + L.in;
  const float* dz = s + L.out;
  float* red = s;
  constexpr int n = T * Co + Co;
  for (int i = threadIdx.x; i < n; i += kSnThreads) red[i] = 0.f;
  __syncthreads();
  for (int it = threadIdx.x; it < T * NG * S; it += kSnThreads) {
    const int t = it % T, g = (it / T) % NG, sl = it / (T * NG);
    const int ci = t % C, kk = t / C;
    const int kh = kk / KW, kw = kk % KW;
    const float* ip = in + ((sl * R + kh) * Win + kw) * C + ci;
    const float* dp = dz + sl * R * Wo * Co + g * CG;
    float acc[CG], acc2[CG];
#pragma unroll
    for (int k = 0; k < CG; ++k) acc[k] = acc2[k] = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
      for (int ow = 0; ow < Wo; ++ow) {
        const float a = ip[(r * Win + ow) * C];
        float d[CG];
        ld_cg<CG>(dp + (r * Wo + ow) * Co, d);
#pragma unroll
        for (int k = 0; k < CG; ++k) {
          if (ow & 1) acc2[k] = fmaf(a, d[k], acc2[k]);
          else acc[k] = fmaf(a, d[k], acc[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < CG; ++k) atomicAdd(&red[t * Co + g * CG + k], acc[k] + acc2[k]);
  }
  if (L.b_off >= 0) {  // bias: column sums of the output gradient, sliced over rows
    for (int it = threadIdx.x; it < NG * Ho; it += kSnThreads) {
      const int g = it % NG, oh = it / NG;
      float acc[CG];
#pragma unroll
      for (int k = 0; k < CG; ++k) acc[k] = 0.f;
#pragma unroll
      for (int ow = 0; ow < Wo; ++ow) {
        float d[CG];
        ld_cg<CG>(dz + (oh * Wo + ow) * Co + g * CG, d);
#pragma unroll
        for (int k = 0; k < CG; ++k) acc[k] += d[k];
      }
#pragma unroll
      for (int k = 0; k < CG; ++k) atomicAdd(&red[T * Co + g * CG + k], acc[k]);
    }
  }
  __syncthreads();
  const int nw = L.b_off >= 0 ? n : T * Co;
  for (int i = threadIdx.x; i < nw; i += kSnThreads) part[L.part + i] = red[i];
}

template <int CG, int KH, int KW, int C, int Co, int Win, int Hin, int Ho, int Wo>
__device__ void sn_conv_dgrad_c(const SnLayer L, float* s) {
  constexpr int Q = Hin * Win;
  float* in = s + L.in;
  const float* dz = s + L.out;
  const float* wl = s + L.wl;
  for (int it = threadIdx.x; it < Q * C; it += kSnThreads) {
    const int q = it % Q, ci = it / Q;
    const int ih = q / Win, iw = q % Win;
    float acc = 0.f, acc2 = 0.f;
#pragma unroll
    for (int kh = 0; kh < KH; ++kh) {
      const int oh = ih - kh;
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) {
        const int ow = iw - kw;
        if ((unsigned)oh < (unsigned)Ho && (unsigned)ow < (unsigned)Wo) {
          const float* dp = dz + (oh * Wo + ow) * Co;
          const float* wp = wl + ((kh * KW + kw) * C + ci) * Co;
#pragma unroll
          for (int co = 0; co < Co; co += CG) {
            float d[CG], w[CG];
            ld_cg<CG>(dp + co, d);
            ld_cg<CG>(wp + co, w);
#pragma unroll
            for (int k = 0; k < CG; ++k) {
              if ((co / CG) & 1) acc2 = fmaf(d[k], w[k], acc2);
              else acc = fmaf(d[k], w[k], acc);
            }
          }
        }
      }
    }
    acc += acc2;
    const int e = q * C + ci;
    if (L.mask_in && !(in[e] > 0.f)) acc = 0.f;
    in[e] = acc;
  }
}

// ---------------------------------------------------------------------------------------
// The same compile-time-geometry conv phases on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32; lane l
// holds A[l & 15][k] and B[k][l & 15] for k = 4 step + (l >> 4), and D rows 4 (l >> 4) + i of column
// l & 15): the per-image convolution as three GEMM forms read straight out of the LDS activations —
//   forward  out[p][co]  = sum_k in_col[p][k] W[k][co],           k = (kh, kw, ci)
//   wgrad    dW[t][co]   = sum_p in_col[p][t] dz[p][co],           t = (kh, kw, ci); row t = T is all
//                          ones, so the same tile also sums the bias gradient; K (pixels) sliced over
//                          waves when the tiles are few, slices summed in order (deterministic)
//   dgrad    din[q][ci]  = sum_k dz_col[q][k] W[(kh, kw, ci)][co], k = (kh, kw, co), zero outside the
//                          output
// Items (M tile, N tile[, slice]) over the 8 waves.  TDE_SN_MFMA (bit mask: 1 forward, 2 weight
// gradient, 4 input gradient; default 3) selects them, 0 keeps the VALU forms above: the MFMA input
// gradient measured slower than the VALU one on LeNet-5 (13 M tiles of a 6-channel output on 8 waves),
// so it is opt-in.  Only the forward K loop is unrolled: unrolling the others pushed the whole step
// kernel past 256 VGPRs into scratch spills.
constexpr int kSnWaves = kSnThreads / 64;

__device__ __forceinline__ f32x4 sn_mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int KH, int KW, int C, int Co, int Win, int Ho, int Wo>
__device__ void sn_conv_fwd_m(const SnLayer L, float* s) {
  constexpr int P = Ho * Wo, K = KH * KW * C, KS = (K + 3) / 4, MT = (P + 15) / 16, NT = (Co + 15) / 16;
  const float* in = s + L.in;
  const float* wl = s + L.wl;
  float* out = s + L.out;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  for (int item = wave; item < MT * NT; item += kSnWaves) {
    const int mt = item / NT, nt = item - mt * NT;
    const int p = min(mt * 16 + fr, P - 1), oh = p / Wo, ow = p - oh * Wo;
    const float* ip = in + (oh * Win + ow) * C;
    const int co = nt * 16 + fr;
    const bool cok = co < Co;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 4 * ks + fq, kc = min(k, K - 1);
      const int kh = kc / (KW * C), r = kc - kh * (KW * C);
      const float av = k < K ? ip[kh * Win * C + r] : 0.f;
      const float bv = (k < K && cok) ? wl[kc * Co + co] : 0.f;
      acc = sn_mfma4(av, bv, acc);
    }
    if (cok) {
      const float bias = L.b_off >= 0 ? wl[K * Co + co] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pr = mt * 16 + 4 * fq + i;
        float v = acc[i] + bias;
        if (L.relu) v = fmaxf(v, 0.f);
        if (pr < P) out[pr * Co + co] = v;
      }
    }
  }
}

template <int KH, int KW, int C, int Co, int Win, int Ho, int Wo>
__device__ void sn_conv_wgrad_m(const SnLayer L, float* s, float* part) {
  constexpr int T = KH * KW * C, T1 = T + 1, P = Ho * Wo, PS = (P + 3) / 4;
  constexpr int MT = (T1 + 15) / 16, NT = (Co + 15) / 16;
  constexpr int S0 = kSnWaves / (MT * NT) > 0 ? kSnWaves / (MT * NT) : 1;
  constexpr int S = S0 * T1 * Co <= kSnScratch ? S0 : 1;
  static_assert(T1 * Co <= kSnScratch, "scratch");
  const float* in = s + L.in;
  const float* dz = s + L.out;
  float* red = s;   // [S][T + 1][Co]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  for (int item = wave; item < MT * NT * S; item += kSnWaves) {
    const int sl = item / (MT * NT), rest = item - sl * (MT * NT), mt = rest / NT, nt = rest - mt * NT;
    const int t = mt * 16 + fr, tc = min(t, T - 1);
    const int kk = tc / C, ci = tc - kk * C, kh = kk / KW, kw = kk - kh * KW;
    const float* ip = in + (kh * Win + kw) * C + ci;
    const int co = nt * 16 + fr;
    const bool cok = co < Co;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int s0 = PS * sl / S, s1 = PS * (sl + 1) / S;
#pragma unroll 1
    for (int ks = s0; ks < s1; ++ks) {
      const int p = 4 * ks + fq, pc = min(p, P - 1);
      const int oh = pc / Wo, ow = pc - oh * Wo;
      const bool pok = p < P;
      const float av = !pok || t > T ? 0.f : (t == T ? 1.f : ip[(oh * Win + ow) * C]);
      const float bv = (pok && cok) ? dz[pc * Co + co] : 0.f;
      acc = sn_mfma4(av, bv, acc);
    }
    if (cok) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tr = mt * 16 + 4 * fq + i;
        if (tr <= T) red[(sl * T1 + tr) * Co + co] = acc[i];
      }
    }
  }
  __syncthreads();
  const int nw = L.b_off >= 0 ? T1 * Co : T * Co;
  for (int e = threadIdx.x; e < nw; e += kSnThreads) {
    float v = red[e];
#pragma unroll
    for (int sl = 1; sl < S; ++sl) v += red[sl * T1 * Co + e];
    part[L.part + e] = v;
  }
}

template <int KH, int KW, int C, int Co, int Win, int Hin, int Ho, int Wo>
__device__ void sn_conv_dgrad_m(const SnLayer L, float* s) {
  // two M tiles per item share every B fragment (the weights depend only on k and ci): half the weight
  // reads per MFMA and two independent accumulator chains per wave
  constexpr int Q = Hin * Win, K = KH * KW * Co, KS = (K + 3) / 4, MT = (Q + 15) / 16, NT = (C + 15) / 16;
  constexpr int MP = (MT + 1) / 2;
  float* in = s + L.in;
  const float* dz = s + L.out;
  const float* wl = s + L.wl;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  for (int item = wave; item < MP * NT; item += kSnWaves) {
    const int mp = item / NT, nt = item - mp * NT;
    int ih[2], iw[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = min((2 * mp + h) * 16 + fr, Q - 1);
      ih[h] = q / Win;
      iw[h] = q - ih[h] * Win;
    }
    const int ci = nt * 16 + fr;
    const bool cok = ci < C;
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll 1
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 4 * ks + fq, kc = min(k, K - 1);
      const int tap = kc / Co, co = kc - tap * Co, kh = tap / KW, kw = tap - kh * KW;
      const float bv = (k < K && cok) ? wl[(tap * C + min(ci, C - 1)) * Co + co] : 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int oh = ih[h] - kh, ow = iw[h] - kw;
        const bool ok = k < K && (unsigned)oh < (unsigned)Ho && (unsigned)ow < (unsigned)Wo;
        acc[h] = sn_mfma4(ok ? dz[(oh * Wo + ow) * Co + co] : 0.f, bv, acc[h]);
      }
    }
    if (cok) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qr = (2 * mp + h) * 16 + 4 * fq + i;
          if (qr < Q) {
            const int e = qr * C + ci;
            float v = acc[h][i];
            if (L.mask_in && !(in[e] > 0.f)) v = 0.f;
            in[e] = v;
          }
        }
    }
  }
}

// (KH, KW, C, Co, input H, input W): LeNet-5's two convs (the first on the 32x32 zero-padded image)
// and the DWK small CNN's conv
#define SN_FAST_GEOS(X) \
  X(5, 5, 1, 6, 32, 32)   \
  X(5, 5, 6, 16, 14, 14)  \
  X(3, 3, 1, 32, 28, 28)

// phase 0 forward, 1 weight gradient, 2 input gradient; false when the geometry is not compiled in
__device__ __forceinline__ bool sn_conv_fast(int phase, const SnLayer L, float* s, float* part, int mfma) {
  if (L.pt != 0 || L.pl != 0) return false;
#define SN_FAST_CASE(KH_, KW_, C_, CO_, H_, W_)                                                              \
  if (L.kh == KH_ && L.kw == KW_ && L.C == C_ && L.Co == CO_ && L.H == H_ && L.W == W_) {                    \
    constexpr int CG = (CO_ % 4 == 0) ? 4 : ((CO_ % 2 == 0) ? 2 : 1);                                        \
    constexpr int HO = H_ - KH_ + 1, WO = W_ - KW_ + 1;                                                      \
    if (mfma & (1 << phase)) {                                                                               \
      if (phase == 0) sn_conv_fwd_m<KH_, KW_, C_, CO_, W_, HO, WO>(L, s);                                    \
      else if (phase == 1) sn_conv_wgrad_m<KH_, KW_, C_, CO_, W_, HO, WO>(L, s, part);                       \
      else sn_conv_dgrad_m<KH_, KW_, C_, CO_, W_, H_, HO, WO>(L, s);                                         \
      return true;                                                                                           \
    }                                                                                                        \
    if (phase == 0) sn_conv_fwd_c<CG, KH_, KW_, C_, CO_, W_, HO, WO>(L, s);                                  \
    else if (phase == 1) sn_conv_wgrad_c<CG, KH_, KW_, C_, CO_, W_, HO, WO>(L, s, part);                     \
    else sn_conv_dgrad_c<CG, KH_, KW_, C_, CO_, W_, H_, HO, WO>(L, s);                                       \
    return true;                                                                                             \
  }
  SN_FAST_GEOS(SN_FAST_CASE)
#undef SN_FAST_CASE
  return false;
}

// ---------------------------------------------------------------------------------------
__device__ void sn_pool_fwd(const SnLayer L, float* s) {
  const float* in = s + L.in;
  float* out = s + L.out;
  const int n = L.Ho * L.Wo * L.C;
  for (int it = threadIdx.x; it < n; it += kSnThreads) {
    const int c = it % L.C, pw = (it / L.C) % L.Wo, ph = it / (L.C * L.Wo);
    const float* p = in + ((2 * ph) * L.W + 2 * pw) * L.C + c;
    out[it] = fmaxf(fmaxf(p[0], p[L.C]), fmaxf(p[L.W * L.C], p[L.W * L.C + L.C]));
  }
}

// gradient routed to the first maximum of each window (scan order), written over the window
__device__ void sn_pool_bwd(const SnLayer L, float* s) {
  float* in = s + L.in;
  const float* g = s + L.out;
  const int n = L.Ho * L.Wo * L.C;
  for (int it = threadIdx.x; it < n; it += kSnThreads) {
    const int c = it % L.C, pw = (it / L.C) % L.Wo, ph = it / (L.C * L.Wo);
    float* p = in + ((2 * ph) * L.W + 2 * pw) * L.C + c;
    const int o[4] = {0, L.C, L.W * L.C, L.W * L.C + L.C};
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p[o[k]];
    int am = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (v[k] > v[am]) am = k;
    const float gv = (L.mask_in && !(v[am] > 0.f)) ? 0.f : g[it];
#pragma unroll
    for (int k = 0; k < 4; ++k) p[o[k]] = k == am ? gv : 0.f;
  }
  if (L.H != 2 * L.Ho || L.W != 2 * L.Wo) {  // odd edge rows / columns feed no window
    for (int it = threadIdx.x; it < L.H * L.W * L.C; it += kSnThreads) {
      const int hw = it / L.C, h = hw / L.W, w = hw - h * L.W;
      if (h >= 2 * L.Ho || w >= 2 * L.Wo) in[it] = 0.f;
    }
  }
}

// ---------------------------------------------------------------------------------------
// dense forward.  W rows come from L2 (every image re-reads them), so the loop is shaped for loads in
// flight, not FLOPs: a thread owns 4 adjacent outputs (one float4 of a W row) and a slice of the inputs,
// 16 independent row loads are issued before their FMAs, and the S slices are summed through LDS.

__device__ void sn_dense_fwd(const SnLayer L, float* s, const float* w, float* scratch, float* rec, bool train) {
  const float* in = s + L.in;
  float* out = s + L.out;
  const int In = L.C, Co = L.Co, T = kSnThreads;
  if (train)
    for (int i = threadIdx.x; i < In; i += T) rec[L.xo + i] = in[i];
  const float* W = w + L.w_off;
  const bool v4 = (Co & 3) == 0 && (L.w_off & 3) == 0;
  const int cg = v4 ? 4 : 1, ng = Co / cg;
  int S = max(1, min(T / max(ng, 1), In));
  S = min(S, kSnScratch / Co);
  const int g = threadIdx.x % ng, sl = threadIdx.x / ng;
  if (sl < S && threadIdx.x < ng * S) {
    const int i0 = (int)((long long)In * sl / S), i1 = (int)((long long)In * (sl + 1) / S);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (v4) {
      const float* wp = W + g * 4;
      int i = i0;
      for (; i + kSnUnroll <= i1; i += kSnUnroll) {
        float4 wv[kSnUnroll];
#pragma unroll
        for (int u = 0; u < kSnUnroll; ++u) wv[u] = *reinterpret_cast<const float4*>(wp + (long long)(i + u) * Co);
#pragma unroll
        for (int u = 0; u < kSnUnroll; ++u) {
          const float a = in[i + u];
          acc[0] = fmaf(a, wv[u].x, acc[0]);
          acc[1] = fmaf(a, wv[u].y, acc[1]);
          acc[2] = fmaf(a, wv[u].z, acc[2]);
          acc[3] = fmaf(a, wv[u].w, acc[3]);
        }
      }
      for (; i < i1; ++i) {
        const float4 wv = *reinterpret_cast<const float4*>(wp + (long long)i * Co);
        const float a = in[i];
        acc[0] = fmaf(a, wv.x, acc[0]);
        acc[1] = fmaf(a, wv.y, acc[1]);
        acc[2] = fmaf(a, wv.z, acc[2]);
        acc[3] = fmaf(a, wv.w, acc[3]);
      }
    } else {
      int i = i0;
      for (; i + kSnUnroll <= i1; i += kSnUnroll) {
        float wv[kSnUnroll];
#pragma unroll
        for (int u = 0; u < kSnUnroll; ++u) wv[u] = W[(long long)(i + u) * Co + g];
#pragma unroll
        for (int u = 0; u < kSnUnroll; ++u) acc[0] = fmaf(in[i + u], wv[u], acc[0]);
      }
      for (; i < i1; ++i) acc[0] = fmaf(in[i], W[(long long)i * Co + g], acc[0]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < cg) scratch[sl * Co + g * cg + k] = acc[k];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < Co; j += T) {
    float acc = L.b_off >= 0 ? w[L.b_off + j] : 0.f;
    for (int k = 0; k < S; ++k) acc += scratch[k * Co + j];
    out[j] = L.relu ? fmaxf(acc, 0.f) : acc;
  }
}

// dense backward: the pre-activation gradient (in `out`) to `rec`, the input gradient over `in`
// (a thread per input row; the row's float4s are issued together)
__device__ void sn_dense_bwd(const SnLayer L, float* s, const float* w, float* rec) {
  float* in = s + L.in;
  const float* dz = s + L.out;
  const int In = L.C, Co = L.Co;
  for (int j = threadIdx.x; j < Co; j += kSnThreads) rec[L.go + j] = dz[j];
  if (!L.need_gin) return;
  const float* W = w + L.w_off;
  const bool v4 = (Co & 3) == 0 && (L.w_off & 3) == 0;
  for (int i = threadIdx.x; i < In; i += kSnThreads) {
    const float* wr = W + (long long)i * Co;
    float acc = 0.f;
    if (v4) {
      int j = 0;
      for (; j + 4 * kSnUnroll <= Co; j += 4 * kSnUnroll) {
        float4 wv[kSnUnroll];
#pragma unroll
        for (int u = 0; u < kSnUnroll; ++u) wv[u] = *reinterpret_cast<const float4*>(wr + j + 4 * u);
#pragma unroll
        for (int u = 0; u < kSnUnroll; ++u) {
          const int jj = j + 4 * u;
          acc = fmaf(wv[u].x, dz[jj], acc);
          acc = fmaf(wv[u].y, dz[jj + 1], acc);
          acc = fmaf(wv[u].z, dz[jj + 2], acc);
          acc = fmaf(wv[u].w, dz[jj + 3], acc);
        }
      }
      float4 wv[kSnUnroll];
      const int nrem = (Co - j) >> 2;
#pragma unroll
      for (int u = 0; u < kSnUnroll; ++u)
        if (u < nrem) wv[u] = *reinterpret_cast<const float4*>(wr + j + 4 * u);
#pragma unroll
      for (int u = 0; u < kSnUnroll; ++u) {
        if (u < nrem) {
          const int jj = j + 4 * u;
          acc = fmaf(wv[u].x, dz[jj], acc);
          acc = fmaf(wv[u].y, dz[jj + 1], acc);
          acc = fmaf(wv[u].z, dz[jj + 2], acc);
          acc = fmaf(wv[u].w, dz[jj + 3], acc);
        }
      }
    } else {
      for (int j = 0; j < Co; ++j) acc = fmaf(wr[j], dz[j], acc);
    }
    if (L.mask_in && !(in[i] > 0.f)) acc = 0.f;
    in[i] = acc;
  }
}

template <typename F>
__device__ __forceinline__ void sn_by_cg(int Co, F&& f) {
  if ((Co & 3) == 0) f(std::integral_constant<int, 4>{});
  else if ((Co & 1) == 0) f(std::integral_constant<int, 2>{});
  else f(std::integral_constant<int, 1>{});
}

__global__ __launch_bounds__(kSnThreads) void smallnet_step_kernel(SnArgs a) {
  __shared__ __attribute__((aligned(16))) float s[kSnLds];
  const int b = blockIdx.x;
  const bool train = a.mode == 0;
  float* scratch = s;  // [kSnScratch] dense slice partials
  // the image and every conv kernel (+ bias) into LDS
  const float* xb = a.x + (long long)b * a.x_stride;
  if (a.img_Hp == a.img_H && a.img_Wp == a.img_W) {
    for (int i = threadIdx.x; i < a.n_in0; i += kSnThreads) s[a.in0 + i] = xb[i];
  } else {
    const int n = a.img_Hp * a.img_Wp * a.img_C;
    for (int i = threadIdx.x; i < n; i += kSnThreads) {
      const int c = i % a.img_C, q = i / a.img_C;
      const int h = q / a.img_Wp - a.pad_t, w = q % a.img_Wp - a.pad_l;
      s[a.in0 + i] = (h >= 0 && h < a.img_H && w >= 0 && w < a.img_W) ? xb[(h * a.img_W + w) * a.img_C + c] : 0.f;
    }
  }
  for (int l = 0; l < a.nl; ++l) {
    const SnLayer L = a.L[l];
    if (L.kind != kSnConv) continue;
    const int nw = L.kh * L.kw * L.C * L.Co;
    for (int i = threadIdx.x; i < nw; i += kSnThreads) s[L.wl + i] = a.w[L.w_off + i];
    if (L.b_off >= 0)
      for (int i = threadIdx.x; i < L.Co; i += kSnThreads) s[L.wl + nw + i] = a.w[L.b_off + i];
  }
  if (train && b == 0 && threadIdx.x == 0) a.iterations[0] += 1;
  __syncthreads();
  int ns = 0;
  auto stamp = [&]() {
    if (a.stamps && b == 0 && threadIdx.x == 0) a.stamps[ns] = wall_clock64();
    ++ns;
  };
  stamp();
  float* rec = a.rec + (long long)b * a.nrec;
  for (int l = 0; l < a.nl; ++l) {
    const SnLayer L = a.L[l];
    if (L.kind == kSnConv) {
      if (!sn_conv_fast(0, L, s, nullptr, a.mfma)) sn_by_cg(L.Co, [&](auto cg) { sn_conv_fwd<decltype(cg)::value>(L, s); });
    } else if (L.kind == kSnPool) {
      sn_pool_fwd(L, s);
    } else {
      sn_dense_fwd(L, s, a.w, scratch, rec, train);
    }
    __syncthreads();
    stamp();
  }
  // softmax cross-entropy on the last layer's logits (one wave)
  const SnLayer H = a.L[a.nl - 1];
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    float* lg = s + H.out;
    const int C = H.Co;
    float mx = -INFINITY;
    int am = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      if (lg[c] > mx) {
        mx = lg[c];
        am = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oi = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oi < am)) {
        mx = om;
        am = oi;
      }
    }
    float se = 0.f;
    for (int c = lane; c < C; c += 64) se += __expf(lg[c] - mx);
    se = wave_sum(se);
    const int y = a.y ? a.y[b] : 0;
    const float ly = (y >= 0 && y < C) ? lg[y] : mx;
    const float loss = mx + __logf(se) - ly;
    const float corr = am == y ? 1.f : 0.f;
    const float inv = 1.f / se;
    // every lane has read lg[y] above before any lane overwrites the logits below
    __builtin_amdgcn_wave_barrier();
    for (int c = lane; c < C; c += 64) {
      const float p = __expf(lg[c] - mx) * inv;
      if (train) lg[c] = (p - (c == y ? 1.f : 0.f)) * a.scale;
      if (a.mode == 2 && a.probs) a.probs[(long long)b * C + c] = a.probs_softmax ? p : lg[c];
    }
    if (lane == 0) {
      if (train) {
        rec[a.nrec - 2] = loss;
        rec[a.nrec - 1] = corr;
      } else if (a.mode == 1 && a.metrics) {
        atomicAdd(&a.metrics[0], loss);
        atomicAdd(&a.metrics[1], corr);
        atomicAdd(&a.metrics[2], 1.f);
      }
    }
  }
  if (!train) return;
  __syncthreads();
  stamp();
  float* part = a.part + (long long)b * a.npart;
  for (int l = a.nl - 1; l >= 0; --l) {
    const SnLayer L = a.L[l];
    if (L.kind == kSnConv) {
      if (!sn_conv_fast(1, L, s, part, a.mfma))
        sn_by_cg(L.Co, [&](auto cg) { sn_conv_wgrad<decltype(cg)::value>(L, s, part); });
      __syncthreads();  // the weight gradient reads the input the input gradient overwrites
      stamp();
      if (L.need_gin && !sn_conv_fast(2, L, s, nullptr, a.mfma))
        sn_by_cg(L.Co, [&](auto cg) { sn_conv_dgrad<decltype(cg)::value>(L, s); });
    } else if (L.kind == kSnPool) {
      sn_pool_bwd(L, s);
    } else {
      sn_dense_bwd(L, s, a.w, rec);
    }
    __syncthreads();
    stamp();
  }
}

// ---------------------------------------------------------------------------------------
// batch reductions + gradient commit / optimizer apply
struct SnRange {
  int part_lo, n, flat_off;
};
struct SnDense {
  int In, Co, xo, go, w_off, b_off, blk0, nblk;
};
constexpr int kSnStrip = 16;   // dense weight rows per workgroup (one MFMA row tile)
constexpr int kSnColTiles = 4; // 16-column tiles per workgroup (one per wave)

struct SnWgradArgs {
  SnRange r[2 * kSnMaxLayers];
  SnDense d[kSnMaxLayers];
  int nr, nd, conv_blk0, conv_nblk, B, npart, nrec, apply;
  const float* part;
  const float* rec;
  float* w;
  float* g;
  float* m;
  float* v;
  const long long* iterations;
  float* metrics;
  OptHyper h;
};

__device__ __forceinline__ void sn_commit(const SnWgradArgs& a, int e, float grad, float lr_t) {
  if (!a.apply) {
    a.g[e] = grad;
    return;
  }
  float m = a.h.kind != kOptSGD ? a.m[e] : 0.f;
  float v = a.h.kind == kOptAdam ? a.v[e] : 0.f;
  a.w[e] = opt_step(a.h, lr_t, a.w[e], grad, m, v);
  if (a.h.kind != kOptSGD) a.m[e] = m;
  if (a.h.kind == kOptAdam) a.v[e] = v;
}


__global__ __launch_bounds__(256) void smallnet_wgrad_kernel(SnWgradArgs a) {
  __shared__ float red[8][33];
  const int blk = blockIdx.x, tid = threadIdx.x;
  const float lr_t = a.apply ? opt_lr_t(a.h, *a.iterations) : 0.f;
  if (blk == 0) {  // metrics: loss sum, correct, count
    float ls = 0.f, cs = 0.f;
    for (int b = tid; b < a.B; b += 256) {
      ls += a.rec[(long long)b * a.nrec + a.nrec - 2];
      cs += a.rec[(long long)b * a.nrec + a.nrec - 1];
    }
    ls = wave_sum(ls);
    cs = wave_sum(cs);
    if ((tid & 63) == 0) {
      red[0][tid >> 6] = ls;
      red[1][tid >> 6] = cs;
    }
    __syncthreads();
    if (tid == 0 && a.metrics) {
      atomicAdd(&a.metrics[0], red[0][0] + red[0][1] + red[0][2] + red[0][3]);
      atomicAdd(&a.metrics[1], red[1][0] + red[1][1] + red[1][2] + red[1][3]);
      atomicAdd(&a.metrics[2], (float)a.B);
    }
    return;
  }
  if (blk < a.conv_blk0 + a.conv_nblk) {  // conv partials: 32 parameters x 8 image slices
    const int pp = tid & 31, sl = tid >> 5;
    const int p = (blk - a.conv_blk0) * 32 + pp;
    float acc = 0.f;
    if (p < a.npart) {
#pragma unroll 16
      for (int b = sl; b < a.B; b += 8) acc += a.part[(long long)b * a.npart + p];
    }
    red[sl][pp] = acc;
    __syncthreads();
    if (sl == 0 && p < a.npart) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += red[k][pp];
      for (int r = 0; r < a.nr; ++r) {
        if (p >= a.r[r].part_lo && p < a.r[r].part_lo + a.r[r].n) {
          sn_commit(a, a.r[r].flat_off + p - a.r[r].part_lo, sum, lr_t);
          break;
        }
      }
    }
    return;
  }
  // dense weight gradients dW[i][j] = sum_b X[b][i] G[b][j] on the exact-f32 MFMA: workgroup = a
  // 16-row strip x up to 4 column tiles of 16 (wave w = column tile), 4 images per MFMA step, every
  // operand read straight from the per-image records (lane (fr, fq) takes X[b][i0 + fr] and G[b][j0 + fr]
  // of image b = 4s + fq: the A / B fragment layout of v_mfma_f32_16x16x4_f32), the images summed in
  // order (deterministic); the strip at i0 = 0 also sums the bias gradient (an MFMA against ones).
  int k = 0;
  while (k + 1 < a.nd && blk >= a.d[k + 1].blk0) ++k;
  const SnDense D = a.d[k];
  const int nct = (D.Co + 15) >> 4, ncg = (nct + kSnColTiles - 1) / kSnColTiles;
  const int lb = blk - D.blk0, strip = lb / ncg, cgp = lb - strip * ncg;
  const int lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int jt = cgp * kSnColTiles + wave;
  if (jt >= nct) return;   // no workgroup barrier below
  const int i0 = strip * kSnStrip, j0 = jt * 16;
  const float* X = a.rec + D.xo + min(i0 + fr, D.In - 1);
  const float* G = a.rec + D.go + min(j0 + fr, D.Co - 1);
  const bool bias = i0 == 0 && D.b_off >= 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accb = {0.f, 0.f, 0.f, 0.f};
  for (int b0 = 0; b0 < a.B; b0 += 64) {
    float xv[16], gv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const long long b = min(b0 + 4 * s + fq, a.B - 1);
      xv[s] = X[b * a.nrec];
      gv[s] = G[b * a.nrec];
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bool ok = b0 + 4 * s + fq < a.B;
      const float g = ok ? gv[s] : 0.f;
      acc = sn_mfma4(ok ? xv[s] : 0.f, g, acc);
      if (bias) accb = sn_mfma4(1.f, g, accb);
    }
  }
  // lane (fr, fq) holds rows 4 fq + ii of column j0 + fr
  if (j0 + fr < D.Co) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = i0 + 4 * fq + ii;
      if (i < D.In) sn_commit(a, D.w_off + i * D.Co + j0 + fr, acc[ii], lr_t);
    }
    if (bias && fq == 0) sn_commit(a, D.b_off + j0 + fr, accb[0], lr_t);
  }
}

}  // namespace tde

using namespace tde;

TDE_API int tde_smallnet_limits(int* out) {
  out[0] = kSnMaxLayers;
  out[1] = kSnLds;
  out[2] = kSnScratch;
  out[3] = kSnLayerInts;
  return 0;
}

// layers: nl x kSnLayerInts int32 (SnLayer field order).  mode 0 train (part / rec written,
// iterations += 1), 1 eval (metrics += loss, correct, count), 2 predict (probs).
TDE_API int tde_smallnet_step(const int* layers, int nl, int mode, int B, const float* w, const float* x,
                              int x_stride, int in0, int n_in0, const int* img, const int* y, float* part, int npart,
                              float* rec,
                              int nrec, float* metrics, long long* iterations, float scale, float* probs,
                              int probs_softmax, long long* stamps, hipStream_t stream) {
  if (nl < 1 || nl > kSnMaxLayers || B <= 0) return -1;
  if (mode == 0 && (!part || !rec || !iterations || nrec < 2)) return -2;
  SnArgs a{};
  for (int l = 0; l < nl; ++l) {
    int* f = reinterpret_cast<int*>(&a.L[l]);
    for (int k = 0; k < kSnLayerInts; ++k) f[k] = layers[l * kSnLayerInts + k];
    const SnLayer L = a.L[l];
    if (L.kind == kSnDense && L.Co > kSnThreads && mode == 0) return -3;
    if (L.in < 0 || L.out < 0 || L.in >= kSnLds || L.out >= kSnLds) return -4;
  }
  if (a.L[nl - 1].kind != kSnDense) return -5;
  a.nl = nl;
  a.mode = mode;
  a.B = B;
  a.x_stride = x_stride;
  a.in0 = in0;
  a.n_in0 = n_in0;
  a.img_H = img[0];
  a.img_W = img[1];
  a.img_C = img[2];
  a.pad_t = img[3];
  a.pad_l = img[4];
  a.img_Hp = img[5];
  a.img_Wp = img[6];
  if ((long long)a.img_Hp * a.img_Wp * a.img_C > kSnLds || a.img_Hp < a.img_H + a.pad_t || a.img_Wp < a.img_W + a.pad_l)
    return -6;
  a.w = w;
  a.x = x;
  a.y = y;
  a.part = part;
  a.npart = npart;
  a.nrec = nrec;
  a.rec = rec;
  a.metrics = metrics;
  a.iterations = iterations;
  a.scale = scale;
  a.probs = probs;
  a.probs_softmax = probs_softmax;
  a.stamps = stamps;
  static const int mfma = [] {
    const char* e = getenv("TDE_SN_MFMA");   // bit mask of MFMA conv phases; 0 = VALU forms only
    return e ? atoi(e) : 3;
  }();
  a.mfma = mfma;
  smallnet_step_kernel<<<B, kSnThreads, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// ranges: nr x {part_lo, n, flat_off}; dense: nd x {In, Co, xo, go, w_off, b_off, blk0, nblk}.
// Grid: block 0 metrics, then conv_nblk conv blocks, then the dense blocks.  apply = 0 stores the
// gradients into g; apply = 1 applies the optimizer (kind, lr, mom, b1, b2, eps) to w / m / v.
TDE_API int tde_smallnet_wgrad(const int* ranges, int nr, const int* dense, int nd, int conv_nblk, int B,
                               const float* part, int npart, const float* rec, int nrec, float* w, float* g, float* m,
                               float* v, const long long* iterations, float* metrics, int apply, int kind, float lr,
                               float mom, float b1, float b2, float eps, hipStream_t stream) {
  if (nr > 2 * kSnMaxLayers || nd > kSnMaxLayers || B <= 0) return -1;
  if (apply && (!iterations || (kind != kOptSGD && !m) || (kind == kOptAdam && !v))) return -2;
  if (!apply && !g) return -2;
  SnWgradArgs a{};
  for (int r = 0; r < nr; ++r) a.r[r] = SnRange{ranges[3 * r], ranges[3 * r + 1], ranges[3 * r + 2]};
  int nblk = 1 + conv_nblk;
  for (int k = 0; k < nd; ++k) {
    const int* f = dense + 8 * k;
    a.d[k] = SnDense{f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7]};
    if (a.d[k].Co > 256 || a.d[k].blk0 != nblk) return -3;
    nblk += a.d[k].nblk;
  }
  a.nr = nr;
  a.nd = nd;
  a.conv_blk0 = 1;
  a.conv_nblk = conv_nblk;
  a.B = B;
  a.npart = npart;
  a.nrec = nrec;
  a.apply = apply;
  a.part = part;
  a.rec = rec;
  a.w = w;
  a.g = g;
  a.m = m;
  a.v = v;
  a.iterations = iterations;
  a.metrics = metrics;
  a.h = OptHyper{kind, lr, mom, b1, b2, eps};
  smallnet_wgrad_kernel<<<nblk, 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}
