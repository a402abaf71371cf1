// Fused float32 training step of the BN-CNN family — Model B of mnist_keras_distributed.py:79-109
// (== tf2_mnist_distributed.py:105-135):
//   [Reshape] · (Conv2D(no bias) · BatchNormalization · ReLU) x L · Flatten ·
//   Dense(no bias) · BatchNormalization · ReLU · [Dropout] · Dense(+bias)[softmax] + SCCE
// in the reference's precision: every GEMM-shaped product on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32), statistics in f32/f64, no bf16 anywhere.
//
// BatchNormalization needs batch-wide statistics between layers, so the step is a short chain of
// launches whose boundaries ARE the statistics exchanges (one per BN, forward and backward); each
// launch applies the previous layer's BN + ReLU while it stages its input, so no activation is
// ever written in normalised form:
//   conv_fwd x L   stage relu(BN(z_prev)) (the BN finalised from the producer's per-workgroup
//                  (mean, M2) partials, Chan-combined in f64) -> implicit-GEMM conv -> raw z,
//                  this layer's statistics partials
//   dense_fwd      relu(BN(z_L)) flattened . W_dense -> h (split-K f32 atomics)
//   head           ONE workgroup: the dense BN statistics over the batch, ReLU, Philox dropout,
//                  Dense head (MFMA), softmax-CE / accuracy, and the head + dropout + ReLU + BN
//                  backward down to dL/dh; head / BN gradients
//   dense_bwd      dW_dense = A^T . dh and dA = dh . W^T -> g_L = dA * relu mask, BN_L backward
//                  partial sums (sum g, sum g*xhat)
//   conv_bwd x L   dZ = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) on load; roles per image:
//                  input gradient per stride class (only the taps that hit that class) -> g of the
//                  previous layer + its partial sums; weight gradient partials per image
//   reduce         per-image weight-gradient partials -> the flat gradient bucket (fixed order:
//                  deterministic, no atomics)
// Gradients land in the replica's flat fp32 bucket (one all-reduce for data parallelism), then the
// multi-tensor optimizer kernel applies them.
#include "tde_common.h"

namespace tde {
namespace bncnn {

constexpr int NTH = 256;   // threads of every workgroup except the head's

struct Geo {   // NHWC input [B][H][W][C], HWIO kernel [kh][kw][C][Co], NHWC output [B][Ho][Wo][Co]
  int H, W, C, Ho, Wo, Co, kh, kw, sh, sw, pt, pl;
};

// The BatchNormalization (+ ReLU) that follows a layer, C channels.
enum { kBnNone = 0, kBnTrain = 1, kBnMoving = 2, kBnBatch = 3, kBnSaved = 4 };
struct Bn {
  int mode;        // kBnNone: raw values (the image); kBnTrain: batch statistics + saved + moving update;
                   // kBnMoving: moving statistics; kBnBatch: batch statistics, no update (learning phase 1
                   // in evaluation, Q4); kBnSaved: the statistics the forward saved (backward)
  int C;
  const float* pmean; const float* pm2; const float* pn; int npart;   // statistics partials [npart][C], [npart]
  const float* gamma; const float* beta;
  float eps, momentum, bessel;
  float* mmean; float* mvar;
  float* saved;    // [2][C] mean, rstd
};

// Backward partial sums of a BN: g = dL/d(BN output, pre-ReLU); sums of g and g*xhat per channel.
struct BnBwd {
  const float* psg; const float* psgx; int npart;   // [npart][C]
  float* dbeta; float* dgamma;                        // flat gradient bucket views (nullable)
};

// Per-channel scale / shift of the forward BN (y = x*sc + sh, then ReLU) and mean / rstd, into LDS
// (st: 4*C floats: sc, sh, mean, rstd).  red: 2*NTH doubles of LDS.  Block `writer` stores the
// saved statistics and the moving-average update (training).  Ends with a barrier.
__device__ void bn_prepare(const Bn& bn, float* st, double* red, bool writer) {
  const int C = bn.C, t = threadIdx.x;
  float* sc = st;
  float* sh = st + C;
  float* mu = st + 2 * C;
  float* rs = st + 3 * C;
  if (bn.mode == kBnNone) {
    for (int c = t; c < C; c += NTH) {
      sc[c] = 1.f; sh[c] = 0.f; mu[c] = 0.f; rs[c] = 1.f;
    }
    __syncthreads();
    return;
  }
  if (bn.mode == kBnMoving || bn.mode == kBnSaved) {
    for (int c = t; c < C; c += NTH) {
      float mean, rstd;
      if (bn.mode == kBnMoving) {
        mean = bn.mmean[c];
        rstd = rsqrtf(bn.mvar[c] + bn.eps);
      } else {
        mean = bn.saved[c];
        rstd = bn.saved[C + c];
      }
      const float g = bn.gamma ? bn.gamma[c] : 1.f;
      sc[c] = g * rstd;
      sh[c] = (bn.beta ? bn.beta[c] : 0.f) - mean * g * rstd;
      mu[c] = mean;
      rs[c] = rstd;
    }
    __syncthreads();
    return;
  }
  // batch statistics from the producer's per-workgroup (count, mean, M2): Chan's parallel combination
  // in two f64 passes (total mean; then sum of M2_w + n_w (mean_w - mean)^2), NTH/C threads per channel
  const int G = NTH / C, c = t % C, j = t / C;
  double s = 0.0, n = 0.0;
  if (j < G) {
    for (int w = j; w < bn.npart; w += G) {
      const double nw = bn.pn[w];
      s += nw * (double)bn.pmean[(size_t)w * C + c];
      n += nw;
    }
  }
  red[t] = s;
  red[NTH + t] = n;
  __syncthreads();
  double S = 0.0, N = 0.0;
  if (j < G) {
    for (int q = 0; q < G; ++q) {
      S += red[q * C + c];
      N += red[NTH + q * C + c];
    }
  }
  const double mean = N > 0.0 ? S / N : 0.0;
  __syncthreads();
  double m2 = 0.0;
  if (j < G) {
    for (int w = j; w < bn.npart; w += G) {
      const double d = (double)bn.pmean[(size_t)w * C + c] - mean;
      m2 += (double)bn.pm2[(size_t)w * C + c] + (double)bn.pn[w] * d * d;
    }
  }
  red[t] = m2;
  __syncthreads();
  if (t < C) {
    double M2 = 0.0;
    for (int q = 0; q < G; ++q) M2 += red[q * C + t];
    const float var = N > 0.0 ? (float)(M2 / N) : 0.f;
    const float rstd = (float)(1.0 / sqrt((double)var + (double)bn.eps));
    const float g = bn.gamma ? bn.gamma[t] : 1.f;
    sc[t] = g * rstd;
    sh[t] = (bn.beta ? bn.beta[t] : 0.f) - (float)mean * g * rstd;
    mu[t] = (float)mean;
    rs[t] = rstd;
    if (writer && bn.mode == kBnTrain) {
      bn.saved[t] = (float)mean;
      bn.saved[C + t] = rstd;
      if (bn.mmean) {
        bn.mmean[t] = bn.mmean[t] * bn.momentum + (float)mean * (1.f - bn.momentum);
        bn.mvar[t] = bn.mvar[t] * bn.momentum + var * bn.bessel * (1.f - bn.momentum);
      }
    }
  }
  __syncthreads();
}

// Sums of a BN's backward partials -> k[c] = sum g, k[C + c] = sum g*xhat (LDS, 2*C floats);
// block `writer` stores dbeta / dgamma.  Ends with a barrier.
__device__ void bnbwd_prepare(const BnBwd& bb, int C, float* k, double* red, bool writer) {
  const int t = threadIdx.x, G = NTH / C, c = t % C, j = t / C;
  double s1 = 0.0, s2 = 0.0;
  if (j < G) {
    for (int w = j; w < bb.npart; w += G) {
      s1 += bb.psg[(size_t)w * C + c];
      s2 += bb.psgx[(size_t)w * C + c];
    }
  }
  red[t] = s1;
  red[NTH + t] = s2;
  __syncthreads();
  if (t < C) {
    double a = 0.0, b = 0.0;
    for (int q = 0; q < G; ++q) {
      a += red[q * C + t];
      b += red[NTH + q * C + t];
    }
    k[t] = (float)a;
    k[C + t] = (float)b;
    if (writer) {
      if (bb.dbeta) bb.dbeta[t] = (float)a;
      if (bb.dgamma) bb.dgamma[t] = (float)b;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Input image of one sample, BN + ReLU applied (st from bn_prepare; bn_mode kBnNone: raw), into the
// zero-padded LDS image Xs [(Hp)][(Wp)][C] (the image at offset (pt, pl)); only padded rows
// [r0, r1) are written (the rows a workgroup's output pixels read).
__device__ void stage_image(const Geo& g, const float* in, int b, int bn_mode, const float* st, float* Xs, int Wp,
                            int r0, int r1) {
  const int C = g.C;
  const float* sc = st;
  const float* sh = st + C;
  const int n = (r1 - r0) * Wp * C;
  const float* img = in + (size_t)b * g.H * g.W * C;
  for (int e = threadIdx.x; e < n; e += NTH) {
    const int c = e % C, pix = e / C;
    const int y = r0 + pix / Wp, x = pix % Wp;
    const int iy = y - g.pt, ix = x - g.pl;
    float v = 0.f;
    if (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W) {
      v = img[((size_t)iy * g.W + ix) * C + c];
      if (bn_mode != kBnNone) v = fmaxf(fmaf(v, sc[c], sh[c]), 0.f);
    }
    Xs[(size_t)y * Wp * C + (size_t)x * C + c] = v;
  }
}

// ------------------------------------------------------------------------------------------------
// Forward conv: grid (B, nchunk); each workgroup = one image x a chunk of 16-pixel output tiles.
// Wave w: K part kp = w % KS (of KS), tile group tg = w / KS owning TPW consecutive tiles; NT tiles of
// 16 output channels.  Partial sums of the KS K parts are combined through LDS.
struct ConvFwdArgs {
  Geo g;
  int B;
  const float* in;
  Bn bn;                     // BN + ReLU of the input (kBnNone for the image)
  const float* w;
  float* z;
  float *pmean, *pm2, *pn;   // this layer's statistics partials (nullable: no statistics needed)
  int nchunk, Hp, Wp, Kp;
  float* zero; long long nzero;   // a buffer zeroed cooperatively by the grid (the dense accumulator)
};

struct ConvFwdLds {
  int xs, ws, koff, st, red, acc, sts, total;
};
template <int TPW, int NT, int KS>
__host__ __device__ ConvFwdLds conv_fwd_lds(int Hp, int Wp, int C, int Kp) {
  ConvFwdLds L;
  int o = 0;
  L.red = o; o += 2 * NTH * 8;
  L.xs = o; o += ((Hp * Wp * C + 3) & ~3) * 4;
  L.ws = o; o += Kp * NT * 16 * 4;
  L.koff = o; o += Kp * 4;
  L.st = o; o += 4 * ((C + 3) & ~3) * 4;
  L.acc = o; o += (KS - 1) * (4 / KS) * TPW * NT * 256 * 4;
  L.sts = o; o += (4 + 1) * NT * 16 * 4;
  L.total = o;
  return L;
}

template <int TPW, int NT, int KS>
__global__ __launch_bounds__(NTH) void conv_fwd_kernel(ConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const Geo g = a.g;
  const ConvFwdLds L = conv_fwd_lds<TPW, NT, KS>(a.Hp, a.Wp, g.C, a.Kp);
  double* red = reinterpret_cast<double*>(sm + L.red);
  float* Xs = reinterpret_cast<float*>(sm + L.xs);
  float* Ws = reinterpret_cast<float*>(sm + L.ws);
  int* koff = reinterpret_cast<int*>(sm + L.koff);
  float* st = reinterpret_cast<float*>(sm + L.st);
  float* accs = reinterpret_cast<float*>(sm + L.acc);
  float* sts = reinterpret_cast<float*>(sm + L.sts);
  constexpr int NTP = NT * 16, MTW = (4 / KS) * TPW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x, chunk = blockIdx.y;
  const int Wp = a.Wp, C = g.C, Co = g.Co, K = g.kh * g.kw * C, Kp = a.Kp;
  const int M = g.Ho * g.Wo;

  if (a.zero) {
    const long long nb = (long long)gridDim.x * gridDim.y, me = (long long)blockIdx.y * gridDim.x + blockIdx.x;
    const long long per = (a.nzero + nb - 1) / nb;
    for (long long i = me * per + tid; i < min(a.nzero, (me + 1) * per); i += NTH) a.zero[i] = 0.f;
  }
  bn_prepare(a.bn, st, red, b == 0 && chunk == 0);
  // padded input rows of this chunk's output pixels
  const int m0 = chunk * MTW * 16, m1 = min(M, m0 + MTW * 16);
  const int r0 = (m0 / g.Wo) * g.sh, r1 = ((m1 - 1) / g.Wo) * g.sh + g.kh;
  stage_image(g, a.in, b, a.bn.mode, st, Xs, Wp, r0, r1);
  for (int e = tid; e < Kp * NTP; e += NTH) {
    const int k = e / NTP, n = e - k * NTP;
    Ws[e] = (k < K && n < Co) ? a.w[(size_t)k * Co + n] : 0.f;
  }
  for (int k = tid; k < Kp; k += NTH) {
    int off = 0;
    if (k < K) {
      const int ci = k % C, t = k / C, kx = t % g.kw, ky = t / g.kw;
      off = (ky * Wp + kx) * C + ci;
    }
    koff[k] = off;
  }
  __syncthreads();

  const int kp = wave % KS, tg = wave / KS;
  const int tile0 = chunk * MTW + tg * TPW;
  int pb[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int m = (tile0 + j) * 16 + fr;
    const int oh = m / g.Wo, ow = m - oh * g.Wo;
    pb[j] = m < M ? (oh * g.sh * Wp + ow * g.sw) * C : r0 * Wp * C;
  }
  f32x4 acc[TPW][NT];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int steps = Kp / 4;
  for (int s = kp; s < steps; s += KS) {
    const int k = 4 * s + fq;
    const int off = koff[k];
    float bv[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) bv[n] = Ws[k * NTP + n * 16 + fr];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const float av = Xs[pb[j] + off];
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[j][n] = mfma4(av, bv[n], acc[j][n]);
    }
  }
  if (KS > 1) {
    if (kp > 0) {
#pragma unroll
      for (int j = 0; j < TPW; ++j)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          *reinterpret_cast<f32x4*>(accs + ((((kp - 1) * (4 / KS) + tg) * TPW + j) * NT + n) * 256 + lane * 4) =
              acc[j][n];
    }
    __syncthreads();
    if (kp == 0) {
      for (int q = 1; q < KS; ++q)
#pragma unroll
        for (int j = 0; j < TPW; ++j)
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            const f32x4 v =
                *reinterpret_cast<const f32x4*>(accs + ((((q - 1) * (4 / KS) + tg) * TPW + j) * NT + n) * 256 + lane * 4);
            acc[j][n] += v;
          }
    }
  }
  // ---- epilogue: raw z, then this chunk's per-channel (mean, M2)
  float* zb = a.z + (size_t)b * M * Co;
  float csum[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) csum[n] = 0.f;
  if (kp == 0) {
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (tile0 + j) * 16 + fq * 4 + r;
        if (m >= m1) continue;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const int co = n * 16 + fr;
          if (co < Co) zb[(size_t)m * Co + co] = acc[j][n][r];
          csum[n] += acc[j][n][r];
        }
      }
  }
  if (!a.pmean) return;
  const int wg = b * a.nchunk + chunk;
  const float cnt = (float)(m1 - m0);
  float* mean_s = sts + 4 * NTP;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    float v = csum[n];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (fq == 0) sts[wave * NTP + n * 16 + fr] = kp == 0 ? v : 0.f;
  }
  __syncthreads();
  if (tid < NTP) mean_s[tid] = (sts[tid] + sts[NTP + tid] + sts[2 * NTP + tid] + sts[3 * NTP + tid]) / cnt;
  __syncthreads();
#pragma unroll
  for (int n = 0; n < NT; ++n) csum[n] = 0.f;
  if (kp == 0) {
#pragma unroll
    for (int j = 0; j < TPW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (tile0 + j) * 16 + fq * 4 + r;
        if (m >= m1) continue;
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const float d = acc[j][n][r] - mean_s[n * 16 + fr];
          csum[n] += d * d;
        }
      }
  }
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    float v = csum[n];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (fq == 0) sts[wave * NTP + n * 16 + fr] = kp == 0 ? v : 0.f;
  }
  __syncthreads();
  if (tid < Co) {
    a.pmean[(size_t)wg * Co + tid] = mean_s[tid];
    a.pm2[(size_t)wg * Co + tid] = sts[tid] + sts[NTP + tid] + sts[2 * NTP + tid] + sts[3 * NTP + tid];
  }
  if (tid == 0) a.pn[wg] = cnt;
}

// ------------------------------------------------------------------------------------------------
// Dense forward: h[B][Dp] += relu(BN(in))[B][K] . W[K][D]; grid (Dp/16, K chunks, row blocks of 64).
// Wave w = 16-row tile w of the block; K chunk staged in LDS with the BN + ReLU applied.
struct DenseFwdArgs {
  int B, K, D, Dp, kc, lda;
  const float* in;           // [B][K], channel of feature k = k % bn.C
  Bn bn;
  const float* w;            // [K][D]
  float* h;                  // [B][Dp] (+=)
};

__global__ __launch_bounds__(NTH) void dense_fwd_kernel(DenseFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  double* red = reinterpret_cast<double*>(sm);
  float* st = reinterpret_cast<float*>(sm + 2 * NTH * 8);
  float* As = st + 4 * ((a.bn.C + 3) & ~3);          // [64][lda]
  float* Bs = As + 64 * a.lda;                         // [kc][16]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int nt = blockIdx.x, k0 = blockIdx.y * a.kc, b0 = blockIdx.z * 64;
  const int kn = min(a.kc, a.K - k0), C = a.bn.C;
  bn_prepare(a.bn, st, red, nt == 0 && blockIdx.y == 0 && blockIdx.z == 0);
  const float* sc = st;
  const float* sh = st + C;
  for (int e = tid; e < 64 * a.kc; e += NTH) {
    const int r = e / a.kc, kk = e - r * a.kc;
    float v = 0.f;
    if (kk < kn && b0 + r < a.B) {
      const int k = k0 + kk, c = k % C;
      v = fmaxf(fmaf(a.in[(size_t)(b0 + r) * a.K + k], sc[c], sh[c]), 0.f);
    }
    As[r * a.lda + kk] = v;
  }
  for (int e = tid; e < a.kc * 16; e += NTH) {
    const int kk = e >> 4, n = e & 15, col = nt * 16 + n;
    Bs[e] = (kk < kn && col < a.D) ? a.w[(size_t)(k0 + kk) * a.D + col] : 0.f;
  }
  __syncthreads();
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* Ar = As + (wave * 16 + fr) * a.lda;
  for (int s = 0; s < a.kc / 4; ++s) {
    const int k = 4 * s + fq;
    acc = mfma4(Ar[k], Bs[k * 16 + fr], acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = b0 + wave * 16 + fq * 4 + r;
    if (row < a.B) atomicAdd(a.h + (size_t)row * a.Dp + nt * 16 + fr, acc[r]);
  }
}

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based: the dropout mask is a function of (element, step, layer))
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
__device__ __forceinline__ float keep_scale(float rate, unsigned long long seed, long long it, int layer, long long e) {
  const uint2 key{(unsigned)seed, (unsigned)(seed >> 32)};
  const unsigned long long c = (unsigned long long)(e >> 2);
  const uint4 r = philox(uint4{(unsigned)c, (unsigned)(c >> 32), (unsigned)it, (unsigned)layer}, key);
  const int q = (int)(e & 3);
  const unsigned w = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
  const float keep = 1.f - rate;
  return ((w >> 8) * (1.f / 16777216.f) < keep) ? 1.f / keep : 0.f;
}

// ------------------------------------------------------------------------------------------------
// Head: ONE workgroup of 1024 threads.  h [B][Dp] -> BN (batch statistics over the B rows, or moving)
// -> ReLU -> dropout -> Dense(D -> NC) + bias -> softmax-CE / accuracy; training: the head gradients,
// and the dropout / ReLU / BN backward down to dL/dh.  Row blocks of 64.
struct HeadArgs {
  int B, D, Dp, NC, mode;          // mode 0 train, 1 eval (metrics), 2 predict
  const float* h;
  Bn bn;                            // C = D (mode kBnTrain / kBnMoving / kBnBatch)
  float rate; unsigned long long seed; const long long* iter; int layer_id, drop_on;
  const float* wh; const float* bh;
  const int* labels; float scale;
  float* metrics;
  float* out; int out_softmax;      // predict: [B][NC] probabilities (softmax head) or logits
  float *dwh, *dbh, *dbeta, *dgamma;
  float* dh;                        // [B][Dp]: dL/dh (holds the pre-ReLU gradient g until the last pass)
};
constexpr int kHeadThreads = 1024;
constexpr int kHeadMaxDp = 240;          // <= 15 feature tiles: wave 15 keeps the bias gradient
constexpr int HLD = kHeadMaxDp + 4;   // LDS row stride of the row-block tile
struct HeadLdsMap {
  int mu, rs, sc, sh, sg, sgx, whs, bhs, as, part, dl, lab, red, total;
};
__host__ __device__ constexpr HeadLdsMap head_lds() {
  HeadLdsMap L{};
  int o = 0;
  L.mu = o; o += kHeadMaxDp * 4;
  L.rs = o; o += kHeadMaxDp * 4;
  L.sc = o; o += kHeadMaxDp * 4;
  L.sh = o; o += kHeadMaxDp * 4;
  L.sg = o; o += kHeadMaxDp * 4;
  L.sgx = o; o += kHeadMaxDp * 4;
  L.whs = o; o += kHeadMaxDp * 16 * 4;     // [Dp][16]
  L.bhs = o; o += 16 * 4;
  L.as = o; o += 64 * HLD * 4;             // post-dropout activations of the row block
  L.part = o; o += 12 * 64 * 4 * 4;        // logits partials
  L.dl = o; o += 64 * 16 * 4;              // dlogits
  L.lab = o; o += 64 * 4;
  L.red = o; o += 4 * 256 * 8;             // f64 [4][256]: 4 threads per feature, f = tid & 255
  L.total = o;
  return L;
}

__global__ __launch_bounds__(kHeadThreads) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  constexpr HeadLdsMap L = head_lds();
  float* mu = reinterpret_cast<float*>(sm + L.mu);
  float* rs = reinterpret_cast<float*>(sm + L.rs);
  float* sc = reinterpret_cast<float*>(sm + L.sc);
  float* sh = reinterpret_cast<float*>(sm + L.sh);
  float* sg = reinterpret_cast<float*>(sm + L.sg);
  float* sgx = reinterpret_cast<float*>(sm + L.sgx);
  float* whs = reinterpret_cast<float*>(sm + L.whs);
  float* bhs = reinterpret_cast<float*>(sm + L.bhs);
  float* as = reinterpret_cast<float*>(sm + L.as);
  float* part = reinterpret_cast<float*>(sm + L.part);
  float* dls = reinterpret_cast<float*>(sm + L.dl);
  int* labs = reinterpret_cast<int*>(sm + L.lab);
  double* red = reinterpret_cast<double*>(sm + L.red);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int B = a.B, D = a.D, Dp = a.Dp, NC = a.NC;
  const bool train = a.mode == 0;
  const long long it = a.iter ? *a.iter : 0;

  // ---- BN statistics of h over the batch (4 threads per feature, two f64 passes), or moving statistics
  {
    const int f = tid & 255, q = tid >> 8;
    const bool batch = a.bn.mode == kBnTrain || a.bn.mode == kBnBatch;
    if (batch) {
      double s = 0.0;
      if (f < D)
        for (int b = q; b < B; b += 4) s += a.h[(size_t)b * Dp + f];
      red[q * 256 + f] = s;
      __syncthreads();
      const double mean = (red[f] + red[256 + f] + red[512 + f] + red[768 + f]) / B;
      __syncthreads();
      double m2 = 0.0;
      if (f < D)
        for (int b = q; b < B; b += 4) {
          const double d = a.h[(size_t)b * Dp + f] - mean;
          m2 += d * d;
        }
      red[q * 256 + f] = m2;
      __syncthreads();
      if (q == 0 && f < D) {
        const double M2 = red[f] + red[256 + f] + red[512 + f] + red[768 + f];
        const float var = (float)(M2 / B);
        const float rstd = (float)(1.0 / sqrt((double)var + (double)a.bn.eps));
        mu[f] = (float)mean;
        rs[f] = rstd;
        if (a.bn.mode == kBnTrain) {
          a.bn.saved[f] = (float)mean;
          a.bn.saved[D + f] = rstd;
          a.bn.mmean[f] = a.bn.mmean[f] * a.bn.momentum + (float)mean * (1.f - a.bn.momentum);
          a.bn.mvar[f] = a.bn.mvar[f] * a.bn.momentum + var * a.bn.bessel * (1.f - a.bn.momentum);
        }
      }
    } else if (q == 0 && f < D) {
      mu[f] = a.bn.mmean[f];
      rs[f] = rsqrtf(a.bn.mvar[f] + a.bn.eps);
    }
    __syncthreads();
    if (q == 0 && f < Dp) {
      const float g = (f < D && a.bn.gamma) ? a.bn.gamma[f] : 1.f;
      sc[f] = f < D ? g * rs[f] : 0.f;
      sh[f] = f < D ? (a.bn.beta ? a.bn.beta[f] : 0.f) - mu[f] * g * rs[f] : 0.f;
      sg[f] = 0.f;
      sgx[f] = 0.f;
    }
  }
  for (int e = tid; e < Dp * 16; e += kHeadThreads) {
    const int f = e >> 4, c = e & 15;
    whs[e] = (f < D && c < NC) ? a.wh[(size_t)f * NC + c] : 0.f;
  }
  if (tid < 16) bhs[tid] = tid < NC ? a.bh[tid] : 0.f;
  __syncthreads();

  const int ksteps = Dp / 16;   // per K quarter: Dp/4 features = Dp/16 steps of 4
  f32x4 gw = {0.f, 0.f, 0.f, 0.f};   // dWh tile of waves 0..Dp/16-1
  float gb = 0.f, la = 0.f, ca = 0.f, na = 0.f;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int nb = min(64, B - b0);
    // ---- row block: post-dropout activation
    for (int e = tid; e < 64 * Dp; e += kHeadThreads) {
      const int r = e / Dp, f = e - r * Dp;
      float v = 0.f;
      if (r < nb && f < D) {
        const float x = a.h[(size_t)(b0 + r) * Dp + f];
        v = fmaxf(fmaf(x, sc[f], sh[f]), 0.f);
        if (a.drop_on) v *= keep_scale(a.rate, a.seed, it, a.layer_id, (long long)(b0 + r) * D + f);
      }
      as[r * HLD + f] = v;
    }
    if (tid < 64) labs[tid] = (tid < nb && a.labels) ? a.labels[b0 + tid] : 0;
    __syncthreads();
    // ---- logits [64][16] = as . Wh: wave = (row tile rt = w & 3, K quarter kq = w >> 2)
    f32x4 lg = {0.f, 0.f, 0.f, 0.f};
    {
      const int rt = wave & 3, kq = wave >> 2;
      for (int s = 0; s < ksteps; ++s) {
        const int k = kq * (Dp / 4) + 4 * s + fq;
        lg = mfma4(as[(rt * 16 + fr) * HLD + k], whs[k * 16 + fr], lg);
      }
      if (kq > 0) *reinterpret_cast<f32x4*>(part + (((kq - 1) * 4 + rt) * 64 + lane) * 4) = lg;
    }
    __syncthreads();
    if (wave < 4) {
      const int rt = wave;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const f32x4 pv = *reinterpret_cast<const f32x4*>(part + ((q * 4 + rt) * 64 + lane) * 4);
        lg += pv;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rt * 16 + fq * 4 + i;
        const bool valid = r < nb, cv = fr < NC;
        const float z = cv ? lg[i] + bhs[fr] : -3.0e38f;
        const float m = row16_max(z);
        const float ex = cv ? __expf(z - m) : 0.f;
        const float s = row16_sum(ex);
        const float pr = ex / s;
        const int label = labs[r];
        const int amx = row16_min(cv && z == m ? fr : 64);
        const float zl = __shfl(z, (lane & ~15) | (label & 15), 64);
        if (valid && fr == 0) {
          la += __logf(s) + m - zl;
          ca += (amx == label) ? 1.f : 0.f;
          na += 1.f;
        }
        if (a.mode == 2 && valid && cv) a.out[(size_t)(b0 + r) * NC + fr] = a.out_softmax ? pr : z;
        dls[r * 16 + fr] = (train && valid && cv) ? (pr - (fr == label ? 1.f : 0.f)) * a.scale : 0.f;
      }
    }
    __syncthreads();
    if (train) {
      // dWh tile (features w*16.., classes) += as^T . dl; wave ksteps*4..: dbh
      if (wave < Dp / 16) {
        for (int s = 0; s < 16; ++s) {
          const int r = 4 * s + fq;
          gw = mfma4(as[r * HLD + wave * 16 + fr], dls[r * 16 + fr], gw);
        }
      } else if (wave == 15) {
        for (int r = fq; r < 64; r += 4) gb += dls[r * 16 + fr];
      }
      // g = dl . Wh^T, dropout, ReLU mask -> dh buffer (pre-BN-backward), sums of g and g*xhat
      const int ntile = Dp / 16;
      for (int t = wave; t < 4 * ntile; t += 16) {
        const int mt = t / ntile, nt = t - mt * ntile;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int c = 4 * s + fq;
          acc = mfma4(dls[(mt * 16 + fr) * 16 + c], whs[(nt * 16 + fr) * 16 + c], acc);
        }
        // lane holds g[row mt*16 + 4fq + i][feature nt*16 + fr]
        const int f = nt * 16 + fr;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = mt * 16 + fq * 4 + i;
          float gval = 0.f, xh = 0.f;
          if (r < nb && f < D) {
            const float act = as[r * HLD + f];
            // act > 0 <=> ReLU passed AND dropout kept; the kept scale is 1/keep
            if (act > 0.f) gval = a.drop_on ? acc[i] * (1.f / (1.f - a.rate)) : acc[i];
            a.dh[(size_t)(b0 + r) * Dp + f] = gval;
            xh = (a.h[(size_t)(b0 + r) * Dp + f] - mu[f]) * rs[f];
          }
          s1 += gval;
          s2 += gval * xh;
        }
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (fq == 0 && f < D) {
          atomicAdd(sg + f, s1);
          atomicAdd(sgx + f, s2);
        }
      }
    }
    __syncthreads();
  }
  // ---- metrics
  if (wave < 4) {
    la = rows4_sum(la);
    ca = rows4_sum(ca);
    na = rows4_sum(na);
    if (a.metrics && lane == 0 && na > 0.f) {
      atomicAdd(a.metrics + 0, la);
      atomicAdd(a.metrics + 1, ca);
      atomicAdd(a.metrics + 2, na);
    }
  }
  if (!train) return;
  // ---- head gradients
  if (wave < Dp / 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = wave * 16 + fq * 4 + i;
      if (f < D && fr < NC) a.dwh[(size_t)f * NC + fr] = gw[i];
    }
  } else if (wave == 15) {
    gb += __shfl_xor(gb, 16, 64);
    gb += __shfl_xor(gb, 32, 64);
    if (fq == 0 && fr < NC) a.dbh[fr] = gb;
  }
  __syncthreads();   // the g stores of every wave are complete and visible to the workgroup
  if (tid < D) {
    if (a.dbeta) a.dbeta[tid] = sg[tid];
    if (a.dgamma) a.dgamma[tid] = sgx[tid];
  }
  // ---- dL/dh = gamma * rstd * (g - mean(g) - xhat * mean(g * xhat))
  const float invB = 1.f / (float)B;
  for (int e = tid; e < B * D; e += kHeadThreads) {
    const int r = e / D, f = e - r * D;
    const float g = a.dh[(size_t)r * Dp + f];
    const float xh = (a.h[(size_t)r * Dp + f] - mu[f]) * rs[f];
    const float gm = a.bn.gamma ? a.bn.gamma[f] : 1.f;
    a.dh[(size_t)r * Dp + f] = gm * rs[f] * (g - sg[f] * invB - xh * sgx[f] * invB);
  }
}

// ------------------------------------------------------------------------------------------------
// Dense backward: grid (ceil(K/16), 2).  role 0: dW[k-tile][0..D) = relu(BN(in))^T . dh;
// role 1: dA = dh . W^T for the k-tile -> g = dA * relu mask of the input BN, the input BN's backward
// partial sums (per k-tile workgroup, per channel).  Row blocks of 64 (dh staged per block).
struct DenseBwdArgs {
  int B, K, D, Dp, ldh;
  const float* in; Bn bn;           // the input layer's raw output and its BN (kBnSaved)
  const float* w;                   // [K][D]
  const float* dh;                  // [B][Dp]
  float* dw;                        // [K][D] (gradient bucket)
  float* g;                         // [B][K]
  float *psg, *psgx;                // [gridDim.x][C]
};

__global__ __launch_bounds__(NTH) void dense_bwd_kernel(DenseBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int C = a.bn.C, CP = (C + 3) & ~3;
  double* red = reinterpret_cast<double*>(sm);
  float* st = reinterpret_cast<float*>(sm + 2 * NTH * 8);
  float* dhs = st + 4 * CP;                   // [64][ldh]
  float* tile = dhs + 64 * a.ldh;             // role 0: A^T block [64][17]; role 1: W rows [16][ldh]
  float* csum = tile + 16 * a.ldh;            // [2][CP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int kt = blockIdx.x, role = blockIdx.y, K = a.K, D = a.D, Dp = a.Dp;
  bn_prepare(a.bn, st, red, false);
  const float* sc = st;
  const float* sh = st + C;
  const float* mu = st + 2 * C;
  const float* rs = st + 3 * C;
  const int ntile = Dp / 16;
  if (role == 0) {
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int b0 = 0; b0 < a.B; b0 += 64) {
      const int nb = min(64, a.B - b0);
      __syncthreads();
      for (int e = tid; e < 64 * Dp; e += NTH) {
        const int r = e / Dp, n = e - r * Dp;
        dhs[r * a.ldh + n] = r < nb ? a.dh[(size_t)(b0 + r) * Dp + n] : 0.f;
      }
      for (int e = tid; e < 64 * 16; e += NTH) {
        const int r = e >> 4, kk = e & 15, k = kt * 16 + kk;
        float v = 0.f;
        if (r < nb && k < K) {
          const int c = k % C;
          v = fmaxf(fmaf(a.in[(size_t)(b0 + r) * K + k], sc[c], sh[c]), 0.f);
        }
        tile[r * 17 + kk] = v;
      }
      __syncthreads();
      for (int s = 0; s < 16; ++s) {
        const int r = 4 * s + fq;
        const float av = tile[r * 17 + fr];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int nt = wave + 4 * j;
          if (nt < ntile) acc[j] = mfma4(av, dhs[r * a.ldh + nt * 16 + fr], acc[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nt = wave + 4 * j;
      if (nt >= ntile) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = kt * 16 + fq * 4 + i, n = nt * 16 + fr;
        if (k < K && n < D) a.dw[(size_t)k * D + n] = acc[j][i];
      }
    }
    return;
  }
  // role 1
  for (int e = tid; e < 16 * Dp; e += NTH) {
    const int kk = e / Dp, n = e - kk * Dp, k = kt * 16 + kk;
    tile[kk * a.ldh + n] = (k < K && n < D) ? a.w[(size_t)k * D + n] : 0.f;
  }
  for (int c = tid; c < 2 * CP; c += NTH) csum[c] = 0.f;
  const int k = kt * 16 + fr;
  const int ck = k % C;
  float s1 = 0.f, s2 = 0.f;
  for (int b0 = 0; b0 < a.B; b0 += 64) {
    const int nb = min(64, a.B - b0);
    __syncthreads();
    for (int e = tid; e < 64 * Dp; e += NTH) {
      const int r = e / Dp, n = e - r * Dp;
      dhs[r * a.ldh + n] = r < nb ? a.dh[(size_t)(b0 + r) * Dp + n] : 0.f;
    }
    __syncthreads();
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < Dp / 4; ++s) {
      const int n = 4 * s + fq;
      acc = mfma4(dhs[(wave * 16 + fr) * a.ldh + n], tile[fr * a.ldh + n], acc);
    }
    // lane: dA[row wave*16 + 4fq + i][feature kt*16 + fr]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wave * 16 + fq * 4 + i;
      if (r < nb && k < K) {
        const float x = a.in[(size_t)(b0 + r) * K + k];
        const float pre = fmaf(x, sc[ck], sh[ck]);
        const float gv = pre > 0.f ? acc[i] : 0.f;
        a.g[(size_t)(b0 + r) * K + k] = gv;
        s1 += gv;
        s2 += gv * (x - mu[ck]) * rs[ck];
      }
    }
  }
  s1 += __shfl_xor(s1, 16, 64);
  s1 += __shfl_xor(s1, 32, 64);
  s2 += __shfl_xor(s2, 16, 64);
  s2 += __shfl_xor(s2, 32, 64);
  __syncthreads();
  if (fq == 0 && k < K) {
    atomicAdd(csum + ck, s1);
    atomicAdd(csum + CP + ck, s2);
  }
  __syncthreads();
  for (int c = tid; c < C; c += NTH) {
    a.psg[(size_t)kt * C + c] = csum[c];
    a.psgx[(size_t)kt * C + c] = csum[CP + c];
  }
}

// ------------------------------------------------------------------------------------------------
// Conv backward: grid (B, n_dg + n_wg).  Prologue of every role: this layer's BN backward sums
// (from the consumer's partials) and dZ = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) of the image
// into a zero-bordered LDS grid.
//   dgrad role y < n_dg: stride class (ry, rx) = (y / dg_chunks) of the input pixels, chunk of its
//     16-pixel tiles; K = the taps that hit that class x Co; -> g of the previous layer's BN output
//     (ReLU mask applied) + that BN's backward partial sums (per workgroup, per channel)
//   wgrad role: a chunk of 16-row tiles of dW (rows = (kh, kw, ci)); K = the image's output pixels;
//     the input image staged with the previous BN + ReLU as in the forward -> per-image partial dW.
struct ConvBwdArgs {
  Geo g;
  int B;
  const float* z; Bn bn; BnBwd bb; const float* gout; float count;   // this layer (count = B*Ho*Wo)
  const float* w;
  const float* in; Bn bn_in; float* gin; float *psg_in, *psgx_in;     // the input side
  float* dwpart;                     // [B][K][Co]
  int n_dg, n_wg, dg_chunks, Ph, Pw, Hd, Wd, Hp, Wp, TPW_dg, TPW_wg;
};

struct ConvBwdLds {
  int red, st, stin, kk, dz, xs, wc, koff, ptab, csum, total;
};
__host__ __device__ inline ConvBwdLds conv_bwd_lds(const Geo& g, int Hd, int Wd, int Hp, int Wp) {
  ConvBwdLds L{};
  const int CoP = (g.Co + 3) & ~3, CP = (g.C + 3) & ~3;
  const int K = g.kh * g.kw * g.C, Kp = (K + 15) & ~15;
  const int ntah = (g.kh + g.sh - 1) / g.sh, ntaw = (g.kw + g.sw - 1) / g.sw;
  const int Kc = ((ntah * ntaw * g.Co + 3) & ~3);
  int o = 0;
  L.red = o; o += 2 * NTH * 8;
  L.st = o; o += 4 * CoP * 4;
  L.stin = o; o += 4 * CP * 4;
  L.kk = o; o += 2 * CoP * 4;
  L.dz = o; o += (Hd * Wd * g.Co + 16) * 4;
  L.xs = o; o += ((Hp * Wp * g.C + 3) & ~3) * 4;
  L.wc = o; o += Kc * ((g.C + 15) & ~15) * 4;
  L.koff = o; o += (Kp > Kc ? Kp : Kc) * 4;
  L.ptab = o; o += 2 * ((g.Ho * g.Wo + 3) & ~3) * 4;
  L.csum = o; o += 2 * CP * 4;
  L.total = o;
  return L;
}

__global__ __launch_bounds__(NTH) void conv_bwd_kernel(ConvBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const Geo g = a.g;
  const ConvBwdLds L = conv_bwd_lds(g, a.Hd, a.Wd, a.Hp, a.Wp);
  double* red = reinterpret_cast<double*>(sm + L.red);
  float* st = reinterpret_cast<float*>(sm + L.st);
  float* stin = reinterpret_cast<float*>(sm + L.stin);
  float* kks = reinterpret_cast<float*>(sm + L.kk);
  float* dz = reinterpret_cast<float*>(sm + L.dz);
  float* Xs = reinterpret_cast<float*>(sm + L.xs);
  float* Wc = reinterpret_cast<float*>(sm + L.wc);
  int* koff = reinterpret_cast<int*>(sm + L.koff);
  int* ptab = reinterpret_cast<int*>(sm + L.ptab);
  float* csum = reinterpret_cast<float*>(sm + L.csum);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x, y = blockIdx.y;
  const int C = g.C, Co = g.Co, Mo = g.Ho * g.Wo, K = g.kh * g.kw * C;
  const int Wd = a.Wd;
  const bool writer = b == 0 && y == 0;

  bn_prepare(a.bn, st, red, false);
  bnbwd_prepare(a.bb, Co, kks, red, writer);
  // dZ of this image into the bordered grid (borders stay zero)
  {
    const float* mu = st + 2 * Co;
    const float* rs = st + 3 * Co;
    const float inv = 1.f / a.count;
    const int nd = a.Hd * Wd * Co;
    for (int e = tid; e < nd + 16; e += NTH) dz[e] = 0.f;
    __syncthreads();
    const float* gz = a.gout + (size_t)b * Mo * Co;
    const float* zz = a.z + (size_t)b * Mo * Co;
    for (int e = tid; e < Mo * Co; e += NTH) {
      const int co = e % Co, p = e / Co, oh = p / g.Wo, ow = p - oh * g.Wo;
      const float xh = (zz[e] - mu[co]) * rs[co];
      const float gm = a.bn.gamma ? a.bn.gamma[co] : 1.f;
      const float v = gm * rs[co] * (gz[e] - kks[co] * inv - xh * kks[Co + co] * inv);
      dz[((oh + a.Ph) * Wd + ow + a.Pw) * Co + co] = v;
    }
  }
  bn_prepare(a.bn_in, stin, red, false);   // (barrier: dz complete)

  if (y < a.n_dg) {
    // ---------------- input gradient of one stride class
    const int cls = y / a.dg_chunks, chunk = y - cls * a.dg_chunks;
    const int ry = cls / g.sw, rx = cls - ry * g.sw;
    // input rows / cols of the class: (i + pt) % sh == ry
    const int ih0 = ((ry - g.pt) % g.sh + g.sh) % g.sh, iw0 = ((rx - g.pl) % g.sw + g.sw) % g.sw;
    const int Hc = ih0 < g.H ? (g.H - ih0 + g.sh - 1) / g.sh : 0;
    const int Wc_ = iw0 < g.W ? (g.W - iw0 + g.sw - 1) / g.sw : 0;
    const int Mc = Hc * Wc_;
    const int nth = (g.kh - ry + g.sh - 1) / g.sh, ntw = (g.kw - rx + g.sw - 1) / g.sw;
    const int Kc = nth * ntw * Co, Kcp = (Kc + 3) & ~3;
    const int CP16 = (C + 15) & ~15;
    for (int e = tid; e < Kcp * CP16; e += NTH) {
      const int kk = e / CP16, ci = e - kk * CP16;
      float v = 0.f;
      if (kk < Kc && ci < C) {
        const int co = kk % Co, t = kk / Co, jw = t % ntw, jh = t / ntw;
        const int ky = ry + g.sh * jh, kx = rx + g.sw * jw;
        v = a.w[(((size_t)ky * g.kw + kx) * C + ci) * Co + co];
      }
      Wc[e] = v;
    }
    for (int kk = tid; kk < Kcp; kk += NTH) {
      int off = 0;
      if (kk < Kc) {
        const int co = kk % Co, t = kk / Co, jw = t % ntw, jh = t / ntw;
        off = (-jh * Wd - jw) * Co + co;
      }
      koff[kk] = off;
    }
    for (int c = tid; c < 2 * ((C + 3) & ~3); c += NTH) csum[c] = 0.f;
    __syncthreads();
    const int TPW = a.TPW_dg;
    const int NTc = CP16 / 16;
    const int CPad = (C + 3) & ~3;
    float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
    for (int j = 0; j < TPW; ++j) {
      const int tile = (chunk * 4 + wave) * TPW + j;
      const int m = tile * 16 + fr;
      const int mc = m < Mc ? m : 0;
      const int ih = ih0 + (mc / Wc_) * g.sh, iw = iw0 + (mc % Wc_) * g.sw;
      const int ohb = (ih + g.pt - ry) / g.sh, owb = (iw + g.pl - rx) / g.sw;
      const int base = ((ohb + a.Ph) * Wd + owb + a.Pw) * Co;
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      for (int s = 0; s < Kcp / 4; ++s) {
        const int kk = 4 * s + fq;
        const float av = dz[base + koff[kk]];
#pragma unroll
        for (int n = 0; n < 2; ++n)
          if (n < NTc) acc[n] = mfma4(av, Wc[kk * CP16 + n * 16 + fr], acc[n]);
      }
      // lane: dA[class pixel tile*16 + 4fq + i][ci = n*16 + fr] -> g_in (ReLU mask of the input BN)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mm = tile * 16 + fq * 4 + i;
        if (mm >= Mc) continue;
        const int ih2 = ih0 + (mm / Wc_) * g.sh, iw2 = iw0 + (mm % Wc_) * g.sw;
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int ci = n * 16 + fr;
          if (n >= NTc || ci >= C) continue;
          const size_t e = (((size_t)b * g.H + ih2) * g.W + iw2) * C + ci;
          const float x = a.in[e];
          const float pre = fmaf(x, stin[ci], stin[C + ci]);
          const float gv = pre > 0.f ? acc[n][i] : 0.f;
          a.gin[e] = gv;
          s1[n] += gv;
          s2[n] += gv * (x - stin[2 * C + ci]) * stin[3 * C + ci];
        }
      }
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      float v1 = s1[n], v2 = s2[n];
      v1 += __shfl_xor(v1, 16, 64);
      v1 += __shfl_xor(v1, 32, 64);
      v2 += __shfl_xor(v2, 16, 64);
      v2 += __shfl_xor(v2, 32, 64);
      const int ci = n * 16 + fr;
      if (fq == 0 && n < NTc && ci < C) {
        atomicAdd(csum + ci, v1);
        atomicAdd(csum + CPad + ci, v2);
      }
    }
    __syncthreads();
    const int wg = b * a.n_dg + y;
    for (int c = tid; c < C; c += NTH) {
      a.psg_in[(size_t)wg * C + c] = csum[c];
      a.psgx_in[(size_t)wg * C + c] = csum[CPad + c];
    }
    return;
  }
  // ---------------- weight gradient partial of this image: rows (kh, kw, ci) tiles of this chunk
  const int chunk = y - a.n_dg;
  const int TPW = a.TPW_wg;
  const int Kp = (K + 15) & ~15;
  const int Wp = a.Wp;
  stage_image(g, a.in, b, a.bn_in.mode, stin, Xs, Wp, 0, a.Hp);
  for (int k = tid; k < Kp; k += NTH) {
    int off = 0;
    if (k < K) {
      const int ci = k % C, t = k / C, kx = t % g.kw, ky = t / g.kw;
      off = (ky * Wp + kx) * C + ci;
    }
    koff[k] = off;
  }
  for (int p = tid; p < ((Mo + 3) & ~3); p += NTH) {
    const int pc = p < Mo ? p : 0;
    const int oh = pc / g.Wo, ow = pc - oh * g.Wo;
    ptab[2 * p] = (oh * g.sh * Wp + ow * g.sw) * C;
    ptab[2 * p + 1] = p < Mo ? ((oh + a.Ph) * Wd + ow + a.Pw) * Co : -1;
  }
  __syncthreads();
  const int NTo = (Co + 15) / 16;
  for (int j = 0; j < TPW; ++j) {
    const int tile = (chunk * 4 + wave) * TPW + j;
    if (tile * 16 >= K) break;
    const int off = koff[tile * 16 + fr];
    f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    for (int s = 0; s < (Mo + 3) / 4; ++s) {
      const int p = 4 * s + fq;
      const int pb = ptab[2 * p], pz = ptab[2 * p + 1];
      const float av = Xs[pb + off];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        if (n >= NTo) continue;
        const float bv = pz >= 0 ? dz[pz + n * 16 + fr] : 0.f;
        acc[n] = mfma4(av, bv, acc[n]);
      }
    }
    float* dst = a.dwpart + (size_t)b * K * Co;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = tile * 16 + fq * 4 + i;
      if (k >= K) continue;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int co = n * 16 + fr;
        if (n < NTo && co < Co) dst[(size_t)k * Co + co] = acc[n][i];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Per-image weight-gradient partials -> the flat gradient bucket, summed in image order.
constexpr int kMaxRed = 4;
struct ReduceArgs {
  int n, B;
  const float* part[kMaxRed];
  float* out[kMaxRed];
  long long len[kMaxRed];
};
__global__ __launch_bounds__(NTH) void reduce_kernel(ReduceArgs a) {
  long long e = (long long)blockIdx.x * NTH + threadIdx.x;
  for (int j = 0; j < a.n; ++j) {
    if (e < a.len[j]) {
      float s = 0.f;
      for (int b = 0; b < a.B; ++b) s += a.part[j][(size_t)b * a.len[j] + e];
      a.out[j][e] = s;
      return;
    }
    e -= a.len[j];
  }
}

}  // namespace bncnn
}  // namespace tde

using namespace tde;
using namespace tde::bncnn;

// ---- host entry points (ctypes).  Geometry / BN descriptors are passed as flat C structs.
struct TdeBnGeo { int H, W, C, Ho, Wo, Co, kh, kw, sh, sw, pt, pl; };
struct TdeBn {
  int mode, C;
  const float *pmean, *pm2, *pn; int npart;
  const float *gamma, *beta;
  float eps, momentum, bessel;
  float *mmean, *mvar, *saved;
};
static Geo geo_of(const TdeBnGeo* g) { return Geo{g->H, g->W, g->C, g->Ho, g->Wo, g->Co, g->kh, g->kw, g->sh, g->sw, g->pt, g->pl}; }
static Bn bn_of(const TdeBn* b) {
  return Bn{b->mode, b->C, b->pmean, b->pm2, b->pn, b->npart, b->gamma, b->beta, b->eps, b->momentum, b->bessel,
            b->mmean, b->mvar, b->saved};
}
static bool bn_ok(const TdeBn* b) {
  if (!b || b->C < 1 || b->C > NTH) return false;
  if ((b->mode == kBnTrain || b->mode == kBnBatch) && (!b->pmean || !b->pm2 || !b->pn || b->npart < 1)) return false;
  if (b->mode == kBnTrain && !b->saved) return false;
  if (b->mode == kBnMoving && (!b->mmean || !b->mvar)) return false;
  if (b->mode == kBnSaved && !b->saved) return false;
  return b->mode >= kBnNone && b->mode <= kBnSaved;
}

template <typename F>
static void set_lds(F* f, int bytes) {
  (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// tiles-per-wave / N tiles / K split of the forward conv, chosen by the host (see bncnn_conv_fwd)
#define TDE_CONV_FWD_CFG(X) X(4, 1, 1) X(2, 1, 1) X(1, 1, 1) X(1, 2, 4) X(1, 1, 4) X(2, 2, 1) X(1, 2, 1)

TDE_API int tde_bncnn_conv_fwd_lds(const TdeBnGeo* gg, int tpw, int nt, int ks) {
  const Geo g = geo_of(gg);
  const int Hp = (g.Ho - 1) * g.sh + g.kh, Wp = (g.Wo - 1) * g.sw + g.kw;
  const int K = g.kh * g.kw * g.C, steps = (K + 3) / 4, Kp = ((steps + ks - 1) / ks) * ks * 4;
#define X(T, N, S) if (tpw == T && nt == N && ks == S) return conv_fwd_lds<T, N, S>(Hp, Wp, g.C, Kp).total;
  TDE_CONV_FWD_CFG(X)
#undef X
  return -1;
}

// z = conv(relu(BN_in(in))); statistics partials of this layer (nullable).  zero/nzero: a buffer the
// grid zeroes.  Returns <0 on an unsupported configuration.
TDE_API int tde_bncnn_conv_fwd(const TdeBnGeo* gg, int B, const float* in, const TdeBn* bn_in, const float* w, float* z,
                               float* pmean, float* pm2, float* pn, int tpw, int nt, int ks, float* zero,
                               long long nzero, hipStream_t stream) {
  const Geo g = geo_of(gg);
  if (!bn_ok(bn_in) || bn_in->C != g.C || B < 1 || g.Co > nt * 16 || g.Co < 1) return -1;
  if (bn_in->mode == kBnSaved) return -2;
  const int Hp = (g.Ho - 1) * g.sh + g.kh, Wp = (g.Wo - 1) * g.sw + g.kw;
  const int K = g.kh * g.kw * g.C, steps = (K + 3) / 4, Kp = ((steps + ks - 1) / ks) * ks * 4;
  const int M = g.Ho * g.Wo, MTW = (4 / ks) * tpw, nchunk = ((M + 15) / 16 + MTW - 1) / MTW;
  ConvFwdArgs a{g, B, in, bn_of(bn_in), w, z, pmean, pm2, pn, nchunk, Hp, Wp, Kp, zero, nzero};
  const int lds = tde_bncnn_conv_fwd_lds(gg, tpw, nt, ks);
  if (lds < 0 || lds > 160 * 1024) return -3;
  const dim3 grid(B, nchunk);
#define X(T, N, S)                                                          \
  if (tpw == T && nt == N && ks == S) {                                    \
    set_lds(conv_fwd_kernel<T, N, S>, lds);                                \
    conv_fwd_kernel<T, N, S><<<grid, NTH, lds, stream>>>(a);               \
    TDE_LAUNCH_CHECK();                                                    \
    return nchunk;                                                         \
  }
  TDE_CONV_FWD_CFG(X)
#undef X
  return -4;
}

TDE_API int tde_bncnn_dense_fwd(int B, int K, int D, int Dp, int kc, const float* in, const TdeBn* bn, const float* w,
                                float* h, hipStream_t stream) {
  if (!bn_ok(bn) || bn->mode == kBnSaved || bn->mode == kBnNone || (kc & 3) || kc < 4 || (Dp & 15) || Dp < D)
    return -1;
  const int lda = kc + ((2 - kc % 32) + 32) % 32;   // lda = 2 (mod 32): the 32-lane halves hit 32 banks
  const int lds = 2 * NTH * 8 + 4 * ((bn->C + 3) & ~3) * 4 + 64 * lda * 4 + kc * 16 * 4;
  if (lds > 160 * 1024) return -3;
  DenseFwdArgs a{B, K, D, Dp, kc, lda, in, bn_of(bn), w, h};
  set_lds(dense_fwd_kernel, lds);
  dense_fwd_kernel<<<dim3(Dp / 16, (K + kc - 1) / kc, (B + 63) / 64), NTH, lds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_bncnn_head(int B, int D, int Dp, int NC, int mode, const float* h, const TdeBn* bn, float rate,
                           unsigned long long seed, const long long* iter, int layer_id, int drop_on, const float* wh,
                           const float* bh, const int* labels, float scale, float* metrics, float* out, int out_softmax,
                           float* dwh, float* dbh, float* dbeta, float* dgamma, float* dh, hipStream_t stream) {
  // the head computes its BN statistics itself (no partials): check the fields it uses
  if (!bn || bn->C != D || D > kHeadMaxDp || Dp > kHeadMaxDp || (Dp & 15) || Dp < D || NC < 1 || NC > 16) return -1;
  if (!(bn->mode == kBnTrain || bn->mode == kBnMoving || bn->mode == kBnBatch)) return -2;
  if ((bn->mode == kBnTrain && !bn->saved) || ((bn->mode == kBnTrain || bn->mode == kBnMoving) && (!bn->mmean || !bn->mvar)))
    return -2;
  if (mode == 0 && (!dwh || !dbh || !dh || !labels || bn->mode != kBnTrain)) return -3;
  if (mode == 2 && !out) return -4;
  if (drop_on && !(rate > 0.f && rate < 1.f)) return -5;
  HeadArgs a{B, D, Dp, NC, mode, h, bn_of(bn), rate, seed, iter, layer_id, drop_on, wh, bh, labels, scale, metrics,
             out, out_softmax, dwh, dbh, dbeta, dgamma, dh};
  constexpr int lds = head_lds().total;
  static_assert(lds <= 160 * 1024, "head LDS");
  set_lds(head_kernel, lds);
  head_kernel<<<1, kHeadThreads, lds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_bncnn_dense_bwd(int B, int K, int D, int Dp, const float* in, const TdeBn* bn, const float* w,
                                const float* dh, float* dw, float* g, float* psg, float* psgx, hipStream_t stream) {
  if (!bn_ok(bn) || bn->mode != kBnSaved || (Dp & 15) || Dp < D || Dp > 256) return -1;
  const int ldh = Dp + 4;
  const int CP = (bn->C + 3) & ~3;
  const int lds = 2 * NTH * 8 + 4 * CP * 4 + 64 * ldh * 4 + 16 * ldh * 4 + 2 * CP * 4;
  if (64 * 17 > 16 * ldh || lds > 160 * 1024) return -3;
  DenseBwdArgs a{B, K, D, Dp, ldh, in, bn_of(bn), w, dh, dw, g, psg, psgx};
  set_lds(dense_bwd_kernel, lds);
  dense_bwd_kernel<<<dim3((K + 15) / 16, 2), NTH, lds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return (K + 15) / 16;
}

struct TdeBnBwd {
  const float *psg, *psgx; int npart;
  float *dbeta, *dgamma;
};

// Geometry of the backward grid (bordered dZ, dgrad roles) for the host to size buffers:
// out = {n_dg, n_wg, dg_chunks, Ph, Pw, Hd, Wd, Hp, Wp, TPW_dg, TPW_wg, lds}
TDE_API int tde_bncnn_conv_bwd_plan(const TdeBnGeo* gg, int dgrad, int* out) {
  const Geo g = geo_of(gg);
  const int K = g.kh * g.kw * g.C;
  const int nth = (g.kh + g.sh - 1) / g.sh, ntw = (g.kw + g.sw - 1) / g.sw;
  const int Ph = dgrad ? nth + 1 : 0, Pw = dgrad ? ntw + 1 : 0;
  // bottom / right margin: the largest base row (H-1+pt)/sh must stay inside the bordered grid
  const int Hd = g.Ho + 2 * Ph + (dgrad ? ((g.H - 1 + g.pt) / g.sh - (g.Ho - 1)) : 0);
  const int Wd = g.Wo + 2 * Pw + (dgrad ? ((g.W - 1 + g.pl) / g.sw - (g.Wo - 1)) : 0);
  const int Hp = (g.Ho - 1) * g.sh + g.kh, Wp = (g.Wo - 1) * g.sw + g.kw;
  // dgrad: classes x chunks of 4 waves x TPW tiles
  const int classes = g.sh * g.sw;
  const int Mc_max = ((g.H + g.sh - 1) / g.sh) * ((g.W + g.sw - 1) / g.sw);
  const int tiles_c = (Mc_max + 15) / 16;
  const int TPW_dg = tiles_c >= 16 ? 2 : 1;
  const int dg_chunks = (tiles_c + 4 * TPW_dg - 1) / (4 * TPW_dg);
  const int n_dg = dgrad ? classes * dg_chunks : 0;
  const int tiles_w = (K + 15) / 16;
  const int TPW_wg = tiles_w >= 32 ? 2 : 1;
  const int n_wg = (tiles_w + 4 * TPW_wg - 1) / (4 * TPW_wg);
  const ConvBwdLds L = conv_bwd_lds(g, Hd, Wd, Hp, Wp);
  const int v[12] = {n_dg, n_wg, dg_chunks, Ph, Pw, Hd, Wd, Hp, Wp, TPW_dg, TPW_wg, L.total};
  for (int i = 0; i < 12; ++i) out[i] = v[i];
  return (L.total > 160 * 1024 || g.Co > 32 || g.C > 32) ? -1 : 0;
}

TDE_API int tde_bncnn_conv_bwd(const TdeBnGeo* gg, int B, const float* z, const TdeBn* bn, const TdeBnBwd* bb,
                               const float* gout, const float* w, const float* in, const TdeBn* bn_in, float* gin,
                               float* psg_in, float* psgx_in, float* dwpart, int dgrad, hipStream_t stream) {
  const Geo g = geo_of(gg);
  int p[12];
  if (tde_bncnn_conv_bwd_plan(gg, dgrad, p) != 0) return -1;
  if (!bn_ok(bn) || bn->mode != kBnSaved || bn->C != g.Co || !bb || bb->npart < 1) return -2;
  if (!bn_ok(bn_in) || bn_in->C != g.C || !(bn_in->mode == kBnSaved || bn_in->mode == kBnNone)) return -3;
  if (dgrad && (!gin || !psg_in || !psgx_in || bn_in->mode != kBnSaved)) return -4;
  ConvBwdArgs a{};
  a.g = g;
  a.B = B;
  a.z = z;
  a.bn = bn_of(bn);
  a.bb = BnBwd{bb->psg, bb->psgx, bb->npart, bb->dbeta, bb->dgamma};
  a.gout = gout;
  a.count = (float)((double)B * g.Ho * g.Wo);
  a.w = w;
  a.in = in;
  a.bn_in = bn_of(bn_in);
  a.gin = gin;
  a.psg_in = psg_in;
  a.psgx_in = psgx_in;
  a.dwpart = dwpart;
  a.n_dg = p[0];
  a.n_wg = p[1];
  a.dg_chunks = p[2];
  a.Ph = p[3];
  a.Pw = p[4];
  a.Hd = p[5];
  a.Wd = p[6];
  a.Hp = p[7];
  a.Wp = p[8];
  a.TPW_dg = p[9];
  a.TPW_wg = p[10];
  set_lds(conv_bwd_kernel, p[11]);
  conv_bwd_kernel<<<dim3(B, a.n_dg + a.n_wg), NTH, p[11], stream>>>(a);
  TDE_LAUNCH_CHECK();
  return a.n_dg;   // the number of input-BN partials per image
}

TDE_API int tde_bncnn_reduce(int n, int B, const float* const* part, float* const* out, const long long* len,
                             hipStream_t stream) {
  if (n < 1 || n > kMaxRed || B < 1) return -1;
  ReduceArgs a{};
  a.n = n;
  a.B = B;
  long long tot = 0;
  for (int j = 0; j < n; ++j) {
    a.part[j] = part[j];
    a.out[j] = out[j];
    a.len[j] = len[j];
    tot += len[j];
  }
  reduce_kernel<<<(unsigned)((tot + NTH - 1) / NTH), NTH, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}
