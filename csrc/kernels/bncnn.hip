// Fused float32 training step of the BN-CNN family — Model B of mnist_keras_distributed.py:79-109
// (== tf2_mnist_distributed.py:105-135):
//   [Reshape] · (Conv2D(no bias) · BatchNormalization · ReLU) x L · Flatten ·
//   Dense(no bias) · BatchNormalization · ReLU · [Dropout] · Dense(+bias)[softmax] + SCCE
// in the reference's precision: every GEMM-shaped product on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32), batch statistics accumulated in f64, no bf16 anywhere.
//
// BatchNormalization needs batch-wide statistics between layers, so the step is a chain of launches
// whose boundaries ARE the statistics exchanges (one per BN each way); every launch applies the
// previous layer's BN + ReLU while it stages its input, so no normalised activation is stored:
//   conv_fwd x L   one image per workgroup: relu(BN(z_prev)) and the weights staged in LDS ->
//                  implicit-GEMM conv -> raw z + this BN's sums (sum, sum of squares: f64)
//   dense_fwd      relu(BN(z_L)) . W_dense -> per-K-chunk partials of h (summed in a fixed order)
//   head_fwd/bwd   per 16-feature tile: the dense BN statistics, ReLU, Philox dropout, the Dense head,
//                  softmax-CE / accuracy, and the head + dropout + ReLU + BN backward down to dL/dh
//   dense_bwd      per 32-feature K tile: dW_dense = A^T . dh and dA = dh . W^T -> g_L (ReLU mask) and
//                  BN_L's backward sums (sum g, sum g*xhat)
//   conv_bwd x L   one image per workgroup: dZ = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) in LDS;
//                  input gradient per stride class (only the taps that hit that class) -> g of the
//                  previous layer + its BN backward sums; the image's weight-gradient partial
//   reduce         per-image weight-gradient partials -> the flat gradient bucket in image order
// Statistics sums travel as per-workgroup partials ([producer workgroup][2][C] f64, plain stores) that
// the consumer sums in a fixed order: no atomics, no zeroing, and the whole step is deterministic.
//
// Latency is the budget at MNIST sizes: a dependent round trip to data another XCD just wrote costs
// ~2 us, an MFMA pass over a whole image well under that.  So the conv / dense launches run 1024-thread
// workgroups (one per CU) that issue EVERY global load they need in one batch into registers (the
// statistics sums included), then work out of LDS: one round trip per launch.
// Gradients land in the replica's flat fp32 bucket (one all-reduce for data parallelism), then the
// multi-tensor optimizer kernel applies them.
#include "tde_common.h"
#include "tde_philox.h"
#include "tde_xgmi.h"
#include "tde_optim.h"

namespace tde {
namespace bncnn {

constexpr int NTH = 256;    // head / reduce workgroups
constexpr int NTB = 1024;   // conv / dense workgroups: 16 waves
constexpr int kUAct = 5, kUW = 11, kUImg = 5;   // prefetch registers per thread (x NTB elements)
constexpr int kMaxCls = 4;                       // stride classes of the input gradient (strides <= 2)

struct Geo {   // NHWC input [B][H][W][C], HWIO kernel [kh][kw][C][Co], NHWC output [B][Ho][Wo][Co]
  int H, W, C, Ho, Wo, Co, kh, kw, sh, sw, pt, pl;
};

// The BatchNormalization (+ ReLU) after a layer, C channels.
enum { kBnNone = 0, kBnTrain = 1, kBnMoving = 2, kBnBatch = 3, kBnSaved = 4 };
struct Bn {
  int mode;        // kBnNone: raw values (the image); kBnTrain: batch statistics + saved + moving update;
                   // kBnMoving: moving statistics; kBnBatch: batch statistics, no update (learning phase 1
                   // in evaluation, Q4); kBnSaved: the statistics the forward saved (backward)
  int C;
  const double* acc; int npart; double count;   // batch statistics: [npart][2][C] partial sums, sums of squares
  const float* gamma; const float* beta;
  float eps, momentum, bessel;
  float* mmean; float* mvar;
  float* saved;    // [2][C] mean, rstd
};

// Backward sums of a BN: g = dL/d(BN output, pre-ReLU); acc = [npart][2][C] partial sum g, sum g*xhat.
struct BnBwd {
  const double* acc; int npart;
  float* dbeta; float* dgamma;   // flat gradient bucket views (nullable)
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- one-batch prefetch: element i = tid + u * NTB of an n-element source into registers (clamped
// addresses, so every load of the batch is issued without a branch), stored to LDS later
template <int U>
struct Pf {
  float v[U];
};
template <int U, typename LD>
__device__ __forceinline__ void pf_load(Pf<U>& p, int n, LD ld) {
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (u * NTB < n) p.v[u] = ld(min((int)threadIdx.x + u * NTB, n - 1));
}
template <int U, typename ST>
__device__ __forceinline__ void pf_store(const Pf<U>& p, int n, ST st) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = threadIdx.x + u * NTB;
    if (i < n) st(i, p.v[u]);
  }
}

// Linear id of this workgroup: its row in a [npart][2][C] partial-statistics buffer.
__device__ __forceinline__ int wg_id() {
  return (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
}

// red[q] = sum over p < np of red[p * Q + q] (q < Q), in a fixed order with a short dependent chain:
// G groups of threads each sum every G-th part, then one thread per q sums the G group sums.  Ends with
// a barrier.  (A single thread per q walking all np parts in LDS was a ~85-long serial chain of LDS
// reads and f64 adds: ~3 us of every conv / dense launch's prologue.)
__device__ void parts_to_slots(double* red, int np, int Q) {
  const int t = threadIdx.x, G = min(16, (int)blockDim.x / Q);
  double S = 0.0;
  if (t < G * Q) {
    const int g = t / Q, q = t - g * Q;
    for (int p = g; p < np; p += G) S += red[p * Q + q];
  }
  lds_barrier();
  if (t < G * Q) red[t] = S;
  lds_barrier();
  double T = 0.0;
  if (t < Q)
    for (int g = 0; g < G; ++g) T += red[g * Q + t];
  lds_barrier();
  if (t < Q) red[t] = T;
  lds_barrier();
}

// red[q] = sum over the npart partials acc[p][q], q < Q (Q <= blockDim), in a fixed order (thread
// (part, q) sums p = part, part + np, ...; then the parts in order); red: blockDim doubles of LDS.
// Ends with a barrier.  U loads per thread are in flight at once: a launch whose partials need more than
// U * np of them per slot pays one more cross-XCD round trip (~2 us) per U.
template <int U = 8>
__device__ void slot_sums(const double* acc, int npart, int Q, double* red) {
  const int t = threadIdx.x, np = blockDim.x / Q, q = t % Q, part = t / Q;
  double s = 0.0;
  if (part < np) {
    for (int j0 = part; j0 < npart; j0 += U * np) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * np;
        v[u] = j < npart ? acc[j * Q + q] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) s += v[u];
    }
    red[t] = s;
  }
  lds_barrier();
  parts_to_slots(red, np, Q);
}

// Per-channel scale / shift of the forward BN (y = x*sc + sh, then ReLU) and mean / rstd into LDS
// (st: 4*C floats: sc, sh, mean, rstd).  Block `writer` stores the saved statistics and the
// moving-average update (training).  red: blockDim doubles of LDS (batch modes).  Ends with a barrier.
template <int U = 8>
__device__ void bn_prepare(const Bn& bn, float* st, bool writer, double* red) {
  const int C = bn.C;
  const bool batch = bn.mode == kBnTrain || bn.mode == kBnBatch;
  // gamma / beta (and the writer's moving averages) of channel threadIdx.x are issued with the
  // statistics partials, not after their reduction: one global round trip in the prologue, not two
  const int c0 = threadIdx.x;
  float g0 = 1.f, b0 = 0.f, mm0 = 0.f, mv0 = 0.f;
  if (c0 < C && bn.mode != kBnNone) {
    if (bn.gamma) g0 = bn.gamma[c0];
    if (bn.beta) b0 = bn.beta[c0];
  }
  if (c0 < C && writer && bn.mode == kBnTrain && bn.mmean) {
    mm0 = bn.mmean[c0];
    mv0 = bn.mvar[c0];
  }
  if (batch) slot_sums<U>(bn.acc, bn.npart, 2 * C, red);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const bool first = c == c0;
    float mean = 0.f, rstd = 1.f, var = 0.f;
    if (bn.mode == kBnMoving) {
      mean = bn.mmean[c];
      rstd = rsqrtf(bn.mvar[c] + bn.eps);
    } else if (bn.mode == kBnSaved) {
      mean = bn.saved[c];
      rstd = bn.saved[C + c];
    } else if (batch) {
      // E[x^2] - E[x]^2 over f64 sums of f32 values: ~1e-16 * (mean/std)^2 relative on the variance
      const double m = red[c] / bn.count;
      const double v = fmax(red[C + c] / bn.count - m * m, 0.0);
      mean = (float)m;
      var = (float)v;
      rstd = (float)(1.0 / sqrt(v + (double)bn.eps));
    }
    float sc = 1.f, sh = 0.f;
    if (bn.mode != kBnNone) {
      const float g = first ? g0 : (bn.gamma ? bn.gamma[c] : 1.f);
      sc = g * rstd;
      sh = (first ? b0 : (bn.beta ? bn.beta[c] : 0.f)) - mean * sc;
    }
    st[c] = sc;
    st[C + c] = sh;
    st[2 * C + c] = mean;
    st[3 * C + c] = rstd;
    if (writer && bn.mode == kBnTrain) {
      bn.saved[c] = mean;
      bn.saved[C + c] = rstd;
      if (bn.mmean) {
        const float om = first ? mm0 : bn.mmean[c], ov = first ? mv0 : bn.mvar[c];
        bn.mmean[c] = om * bn.momentum + mean * (1.f - bn.momentum);
        bn.mvar[c] = ov * bn.momentum + var * bn.bessel * (1.f - bn.momentum);
      }
    }
  }
  lds_barrier();
}

// Per-wave column statistics (lanes fq == 0 after the cross-fq shuffles hold column fr of N tile n)
// -> cs[wave][stat][32] -> this workgroup's partial row acc[wg][stat][C], the 16 waves summed in a
// fixed order.
__device__ __forceinline__ void wave_cols_to_slot(const double (&s1)[2], const double (&s2)[2], double* cs,
                                                  double* acc, int C) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    double x1 = s1[n], x2 = s2[n];
    x1 += __shfl_xor(x1, 16, 64);
    x1 += __shfl_xor(x1, 32, 64);
    x2 += __shfl_xor(x2, 16, 64);
    x2 += __shfl_xor(x2, 32, 64);
    if (fq == 0) {
      cs[(wave * 2 + 0) * 32 + n * 16 + fr] = x1;
      cs[(wave * 2 + 1) * 32 + n * 16 + fr] = x2;
    }
  }
  lds_barrier();
  if (tid < 2 * C) {
    const int j = tid / C, c = tid - j * C;
    double S = 0.0;
    for (int w = 0; w < 16; ++w) S += cs[(w * 2 + j) * 32 + c];
    acc[(size_t)wg_id() * 2 * C + j * C + c] = S;
  }
}

// Fast integer division for the staging index math: q = floor(i / d) for 0 <= i < 2^21 from a
// host-rounded reciprocal ((i + 0.5) / d lies >= 0.5 / d away from the next integer, far more than
// the f32 rounding of the product).
struct Dv {
  int d;
  float r;
};
__device__ __forceinline__ int dq(int i, Dv v) { return (int)(((float)i + 0.5f) * v.r); }

// Backward conv geometry (see conv_bwd_kernel); the forward also stages the input-gradient weights.
constexpr int kMaxDgNT = 4;   // input-gradient N tiles: classes x C <= 64
struct ConvBwdP {
  Geo g;
  int K, Mo, Hp, Wp, Hd, Wd, Ph, Pw, zslot, dgrad, nco;
  // input gradient (depth-to-space)
  int nth, ntw, Kd, Kdp, ncls, NC, NP, nnt, obh0, obw0, Nbw, Md, mtd, ksd, spd, n_dg_items;
  // weight gradient
  int wg_tiles, wg_split, wg_spp, Kw16, n_wg_items;
  int wgather;   // the class-stacked weights fit the registers (a forward-staged copy can be used)
  Dv dC, dCo, dW, dWo, dWd, dWp, dkw, dntw, dNbw, dNP, dsh, dsw;
  int o_red, o_cs, o_st, o_stin, o_kk, o_dz, o_role;
  int o_xs, o_kow, o_ptab, o_part;           // weight-gradient role
  int o_xr, o_wb, o_kod, o_partd;            // input-gradient role
  int lds;
};
// Source of element i of the class-stacked [Kdp][NP] input-gradient weights: the HWIO index of
// (ky, kx, ci, co), or -1 in the holes (padding rows / columns, taps past the kernel).
__device__ __forceinline__ int wstack_src(const ConvBwdP& P, int i) {
  const Geo& g = P.g;
  const int kk = dq(i, P.dNP), n = i - kk * P.NP;
  const int t = dq(kk, P.dCo), co = kk - t * g.Co, jh = dq(t, P.dntw), jw = t - jh * P.ntw;
  const int cl = dq(n, P.dC), ci = n - cl * g.C, ry = dq(cl, P.dsw), rx = cl - ry * g.sw;
  const int ky = ry + g.sh * jh, kx = rx + g.sw * jw;
  if (kk >= P.Kd || n >= P.NC || ky >= g.kh || kx >= g.kw) return -1;
  return ((ky * g.kw + kx) * g.C + ci) * g.Co + co;
}

// ------------------------------------------------------------------------------------------------
// Forward conv: grid (B, msplit): workgroup (b, h) = image b, output tiles [h * mtw, (h+1) * mtw)
// (two workgroups per image keep all 256 CUs busy at B = 128).  Work items (16-pixel output tile,
// 16-channel N tile, K part) over the 16 waves; K parts (strided K steps) summed through LDS in a fixed
// order.
struct ConvFwdP {
  Geo g;
  int K, M, Hp, Wp, nct, ks, spp, Kpad, mt, mtw, msplit;
  Dv dC, dCo, dW, dWo, dWp, dkw, dNTP;
  int o_red, o_cs, o_st, o_xs, o_ws, o_koff, o_part, lds;
};
struct ConvFwdArgs {
  ConvFwdP p;
  int B;
  const float* in;
  Bn bn;                     // BN + ReLU of the input (kBnNone for the image)
  const float* w;
  float* z;
  double* acc;               // this layer's BN partial sums [msplit * B][2][Co] (nullable: no statistics)
  long long* stamps;         // diagnostic phase clock (tde_bncnn_stamps), nullable
  long long* inc_iter;       // training, first layer: the step counter this step advances (nullable)
  float* wstack;             // training, layers with an input gradient: the class-stacked weights of this
  ConvBwdP sp;               // step's backward (layout of sp), written here once (nullable)
};

__global__ __launch_bounds__(NTB) void conv_fwd_kernel(ConvFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const ConvFwdP& P = a.p;
  const Geo& g = P.g;
  double* red = reinterpret_cast<double*>(sm + P.o_red);
  double* cs = reinterpret_cast<double*>(sm + P.o_cs);
  float* st = reinterpret_cast<float*>(sm + P.o_st);
  float* Xs = reinterpret_cast<float*>(sm + P.o_xs);
  float* Ws = reinterpret_cast<float*>(sm + P.o_ws);
  int* koff = reinterpret_cast<int*>(sm + P.o_koff);
  float* part = reinterpret_cast<float*>(sm + P.o_part);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x, C = g.C, Co = g.Co, K = P.K, M = P.M, NTP = P.nct * 16, Wp = P.Wp;
  stamp(a.stamps, 0);
  // the step counter (Keras optimizer.iterations: the dropout seed and Adam's t) advances at the start
  // of a training step; no other launch of the step writes it, later ones read it
  if (a.inc_iter && b == 0 && blockIdx.y == 0 && tid == 0) *a.inc_iter += 1;
  // ---- one batch of global loads: the image and the weights (the BN sums join in bn_prepare)
  const int nimg = g.H * g.W * C, nw = K * Co;
  const float* img = a.in + (size_t)b * nimg;
  Pf<kUImg> pi;
  Pf<kUW> pw;
  pf_load(pi, nimg, [&](int i) { return img[i]; });
  pf_load(pw, nw, [&](int i) { return a.w[i]; });
  // this step's class-stacked input-gradient weights (the weights do not change until the step's
  // optimizer update): element wid * NTB + tid, one per thread of the first workgroups
  const int wsi = (blockIdx.y * gridDim.x + b) * NTB + tid;
  const bool wst = a.wstack && wsi < a.sp.Kdp * a.sp.NP;
  float wsv = 0.f;
  if (wst) {
    const int src = wstack_src(a.sp, wsi);
    wsv = a.w[max(src, 0)];
    if (src < 0) wsv = 0.f;
  }
  // LDS the registers do not cover: image border, weight padding, im2col offsets
  for (int i = tid; i < P.Hp * Wp; i += NTB) {
    const int y = dq(i, P.dWp), x = i - y * Wp, iy = y - g.pt, ix = x - g.pl;
    if (iy < 0 || iy >= g.H || ix < 0 || ix >= g.W)
      for (int c = 0; c < C; ++c) Xs[i * C + c] = 0.f;
  }
  for (int i = tid; i < P.Kpad * NTP; i += NTB) {
    const int k = dq(i, P.dNTP), col = i - k * NTP;
    if (k >= K || col >= Co) Ws[i] = 0.f;
  }
  for (int k = tid; k < P.Kpad; k += NTB) {
    int off = 0;
    if (k < K) {
      const int t = dq(k, P.dC), ci = k - t * C, ky = dq(t, P.dkw), kx = t - ky * g.kw;
      off = (ky * Wp + kx) * C + ci;
    }
    koff[k] = off;
  }
  bn_prepare(a.bn, st, b == 0 && blockIdx.y == 0, red);
  stamp(a.stamps, 1);
  {
    const float* sc = st;
    const float* sh = st + C;
    const bool raw = a.bn.mode == kBnNone;
    pf_store(pi, nimg, [&](int i, float v) {
      const int pix = dq(i, P.dC), c = i - pix * C, y = dq(pix, P.dW), x = pix - y * g.W;
      Xs[((y + g.pt) * Wp + x + g.pl) * C + c] = raw ? v : fmaxf(fmaf(v, sc[c], sh[c]), 0.f);
    });
    pf_store(pw, nw, [&](int i, float v) {
      const int k = dq(i, P.dCo), co = i - k * Co;
      Ws[k * NTP + co] = v;
    });
  }
  if (wst) a.wstack[wsi] = wsv;
  lds_barrier();
  stamp(a.stamps, 2);
  // ---- MFMA work items over this workgroup's output tiles
  const int mt0 = blockIdx.y * P.mtw, mtn = min(P.mtw, P.mt - mt0);
  const int ntile = mtn * P.nct, nitems = ntile * P.ks;
  for (int item = wave; item < nitems; item += 16) {
    const int kp = item % P.ks, t = item / P.ks, n = t % P.nct, mtile = mt0 + t / P.nct;
    const int m = min(mtile * 16 + fr, M - 1);
    const int oh = dq(m, P.dWo), ow = m - oh * g.Wo;
    const int pb = (oh * g.sh * Wp + ow * g.sw) * C;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i0 = 0; i0 < P.spp; i0 += 4) {
      int ko[4];
      float bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = 4 * (kp + (i0 + u) * P.ks) + fq;
        ko[u] = koff[k];
        bv[u] = Ws[k * NTP + n * 16 + fr];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = mfma4(Xs[pb + ko[u]], bv[u], acc);
    }
    *reinterpret_cast<f32x4*>(part + ((size_t)(kp * ntile + t) * 64 + lane) * 4) = acc;
  }
  lds_barrier();
  stamp(a.stamps, 3);
  // ---- epilogue: the K parts summed in order; raw z; this layer's BN sums
  float* zb = a.z + (size_t)b * M * Co;
  double s1[2] = {0.0, 0.0}, s2[2] = {0.0, 0.0};
  for (int t = wave; t < ntile; t += 16) {
    const int n = t % P.nct, mtile = mt0 + t / P.nct;
    f32x4 v = *reinterpret_cast<const f32x4*>(part + ((size_t)t * 64 + lane) * 4);
    for (int kp = 1; kp < P.ks; ++kp) v += *reinterpret_cast<const f32x4*>(part + ((size_t)(kp * ntile + t) * 64 + lane) * 4);
    const int co = n * 16 + fr;
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mtile * 16 + fq * 4 + i;
      if (m < M && co < Co) {
        zb[(size_t)m * Co + co] = v[i];
        t1 += v[i];
        t2 += (double)v[i] * v[i];
      }
    }
    if (n == 0) {
      s1[0] += t1;
      s2[0] += t2;
    } else {
      s1[1] += t1;
      s2[1] += t2;
    }
  }
  if (a.acc) wave_cols_to_slot(s1, s2, cs, a.acc, Co);
  stamp(a.stamps, 4);
}

// ------------------------------------------------------------------------------------------------
// Philox4x32-10: tde_philox.h (counter-based: masks are regenerated, never stored)
// The keep scales of the 4 elements e0 .. e0+3 (e0 % 4 == 0): one Philox call (the same values as
// keep_scale of each element).
__device__ __forceinline__ float4 keep_scale4(float rate, unsigned long long seed, long long it, int layer, long long e0) {
  const uint2 key{(unsigned)seed, (unsigned)(seed >> 32)};
  const unsigned long long c = (unsigned long long)(e0 >> 2);
  const uint4 r = philox(uint4{(unsigned)c, (unsigned)(c >> 32), (unsigned)it, (unsigned)layer}, key);
  const float keep = 1.f - rate, inv = 1.f / keep;
  auto f = [&](unsigned w) { return ((w >> 8) * (1.f / 16777216.f) < keep) ? inv : 0.f; };
  return float4{f(r.x), f(r.y), f(r.z), f(r.w)};
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
// Dense forward: h = relu(BN(in)) . W_dense; grid (Dp/16 column tiles, ceil(B/16) row tiles).  One
// 16x16 output tile per workgroup over the full K: wave w takes K range [w*kw, (w+1)*kw) with its MFMA
// operands loaded straight from global into registers (no LDS staging), the 16 partial tiles summed in
// LDS in wave order (deterministic).  Also the dense BN's statistics partials of the tile (per column:
// sum, sum of squares over its 16 rows, f64) -> hstat[row tile][2][Dp].
constexpr int kDS = 24;   // K steps per wave (K <= 16 * 4 * kDS = 1536)
struct DenseFwdArgs {
  int B, K, D, Dp, kw;
  Dv dC;
  const float* in;           // [B][K], channel of feature k = k % bn.C
  Bn bn;
  const float* w;            // [K][D]
  float* h;                  // [B][Dp]
  double* hstat;             // [ceil(B/16)][2][Dp]
  long long* stamps;
  // training with dropout and the head folded into the dense backward (nullable): the dropout keep flags of
  // this workgroup's 16 x 16 tile in MFMA output layout, keep[(row tile * Dp/16 + column tile) * 64 + lane] =
  // 4 bytes (rows 4 fq + i, column fr; 1 = kept), the masks keep_scale draws for the head
  unsigned* keep;
  float rate; unsigned long long seed; const long long* iter; int layer_id;
};

// V4 (K % 4 == 0, kw % 16 == 0): the A operand as one float4 load per 4 MFMA steps.  Lane (fr, fq)
// loads in[row][k0 + 16s + 4fq .. +3] and MFMA j of the group contracts k = k0 + 16s + 4fq + j over
// fq: a permutation of the K order that the B operand (W rows k) follows, so the product is the same.
template <bool V4>
__global__ __launch_bounds__(NTB) void dense_fwd_kernel(DenseFwdArgs a) {
  __shared__ double red[NTB];
  __shared__ float st[4 * 32];
  __shared__ float part[16][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int c0 = blockIdx.x * 16, r0 = blockIdx.y * 16, K = a.K;
  const int k0 = wave * a.kw;
  const int row = min(r0 + fr, a.B - 1), col = min(c0 + fr, a.D - 1);
  stamp(a.stamps, 0);
  float av[kDS], bv[kDS];
  if (V4) {
    const float* ar = a.in + (size_t)row * K;
#pragma unroll
    for (int s4 = 0; s4 < kDS / 4; ++s4)
      if (16 * s4 < a.kw) {
        const int kb = min(k0 + 16 * s4 + 4 * fq, K - 4);
        const float4 v = *reinterpret_cast<const float4*>(ar + kb);
        av[4 * s4 + 0] = v.x;
        av[4 * s4 + 1] = v.y;
        av[4 * s4 + 2] = v.z;
        av[4 * s4 + 3] = v.w;
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[4 * s4 + j] = a.w[(size_t)min(k0 + 16 * s4 + 4 * fq + j, K - 1) * a.D + col];
      }
  } else {
#pragma unroll
    for (int s = 0; s < kDS; ++s)
      if (4 * s < a.kw) {
        const int k = min(k0 + 4 * s + fq, K - 1);
        av[s] = a.in[(size_t)row * K + k];
        bv[s] = a.w[(size_t)k * a.D + col];
      }
  }
  // 13 loads in flight: the last conv's 256 partials of 2 x 24 slots (21 parts per slot) in one round
  // trip (8: two); 16 spills at this kernel's 128-VGPR budget
  bn_prepare<13>(a.bn, st, blockIdx.x == 0 && blockIdx.y == 0, red);
  stamp(a.stamps, 1);
  const float* sc = st;
  const float* sh = st + a.bn.C;
  const bool rok = r0 + fr < a.B, cok = c0 + fr < a.D;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kDS; ++s)
    if (4 * s < a.kw) {
      // V4: element j = s & 3 of group s >> 2; else step s, lane fq
      const int k = V4 ? k0 + 16 * (s >> 2) + 4 * fq + (s & 3) : k0 + 4 * s + fq;
      const int c = k - dq(k, a.dC) * a.bn.C;
      const bool kok = k < K && k - k0 < a.kw;
      const float x = (kok && rok) ? fmaxf(fmaf(av[s], sc[c], sh[c]), 0.f) : 0.f;
      acc = mfma4(x, (kok && cok) ? bv[s] : 0.f, acc);
    }
  *reinterpret_cast<f32x4*>(&part[wave][lane * 4]) = acc;
  lds_barrier();
  stamp(a.stamps, 2);
  if (wave == 0) {
    f32x4 v = acc;
    for (int w = 1; w < 16; ++w) v += *reinterpret_cast<const f32x4*>(&part[w][lane * 4]);
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + fq * 4 + i;
      if (r < a.B) {
        a.h[(size_t)r * a.Dp + c0 + fr] = v[i];
        s1 += v[i];
        s2 += (double)v[i] * v[i];
      }
    }
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (fq == 0) {
      a.hstat[((size_t)blockIdx.y * 2 + 0) * a.Dp + c0 + fr] = s1;
      a.hstat[((size_t)blockIdx.y * 2 + 1) * a.Dp + c0 + fr] = s2;
    }
    if (a.keep) {
      const long long it = *a.iter;
      unsigned w = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + fq * 4 + i;
        const bool k = r < a.B && c0 + fr < a.D &&
                       keep_scale(a.rate, a.seed, it, a.layer_id, (long long)r * a.D + c0 + fr) != 0.f;
        w |= (k ? 1u : 0u) << (8 * i);
      }
      a.keep[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 64 + lane] = w;
    }
  }
  stamp(a.stamps, 3);
}


// ------------------------------------------------------------------------------------------------
// Head: grid ceil(B/16), one 16-row tile per workgroup (all Dp features):
//   the dense BN statistics (fixed-order sum of dense_fwd's row-tile partials, or the moving ones),
//   ReLU, Philox dropout, Dense head (MFMA), softmax-CE / accuracy / prediction; training: the row
//   tile's partials of dWh, dbh (summed by the reduce launch), g = dl . Wh^T through the dropout / ReLU
//   masks, and the dense BN's backward partial sums (sum g, sum g*xhat per feature) -> dense_bwd
//   finishes dL/dh = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) while it stages it.
constexpr int kHeadMaxDp = 256;
constexpr int NTHH = 1024;                   // head workgroups: 16 waves share the elementwise work
constexpr int kHU = kHeadMaxDp * 16 / NTHH;  // h / g elements per thread
constexpr int kHLD = kHeadMaxDp + 4;         // LDS row stride of the activation tile
struct HeadArgs {
  int B, D, Dp, NC, mode, nrt;       // mode 0 train, 1 eval (metrics), 2 predict; nrt = row tiles
  Dv dDp;
  const float* h;                    // [B][Dp]
  const double* hstat;               // [nrt][2][Dp]
  Bn bn;                             // C = D (mode kBnTrain / kBnMoving / kBnBatch)
  float rate; unsigned long long seed; const long long* iter; int layer_id, drop_on;
  const float* wh; const float* bh;
  const int* labels; float scale;
  float* metrics;
  float* out; int out_softmax;       // predict: [B][NC] probabilities (softmax head) or logits
  float* dwh_part;                   // [nrt][D][NC]
  float* dbh_part;                   // [nrt][NC]
  float* g;                          // [B][Dp]  dL/d(BN output) through the masks
  double* gstat;                     // [nrt][2][Dp]
  long long* stamps;
};

__global__ __launch_bounds__(NTHH) void head_kernel(HeadArgs a) {
  __shared__ float mu[kHeadMaxDp], rs[kHeadMaxDp], sc[kHeadMaxDp], sh[kHeadMaxDp];
  __shared__ float As[16 * kHLD], Xh[16 * kHLD];
  __shared__ float whs[kHeadMaxDp * 17];   // [feature][class], row stride 17 (conflict-free column reads)
  __shared__ float lgp[4][256];
  __shared__ float dls[16 * 17];           // row stride 17
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int B = a.B, D = a.D, Dp = a.Dp, NC = a.NC, rt = blockIdx.x, r0 = rt * 16;
  const bool train = a.mode == 0, lead = rt == 0;
  const bool batch = a.bn.mode == kBnTrain || a.bn.mode == kBnBatch;
  const long long it = a.iter ? *a.iter : 0;
  stamp(a.stamps, 0);
  // ---- one batch of loads: the row tile of h, the statistics partials of feature tid, Wh
  float hv[kHU];
#pragma unroll
  for (int u = 0; u < kHU; ++u) {
    const int e = tid + u * NTHH;
    if (u * NTHH < 16 * Dp) hv[u] = a.h[(size_t)r0 * Dp + min(e, (B - r0) * Dp - 1)];   // rows contiguous
  }
  float wv[kHU];
#pragma unroll
  for (int u = 0; u < kHU; ++u) {
    const int e = tid + u * NTHH, f = e >> 4, c = e & 15;
    if (u * NTHH < 16 * Dp) wv[u] = (f < D && c < NC) ? a.wh[(size_t)min(f, D - 1) * NC + min(c, NC - 1)] : 0.f;
  }
  const int f = tid;
  // gamma / beta of feature f, the head bias and wave 0's labels join the batch (no later round trip)
  const float gm = (f < D && a.bn.gamma) ? a.bn.gamma[f] : 1.f;
  const float bt = (f < D && a.bn.beta) ? a.bn.beta[f] : 0.f;
  const bool upd = f < D && ((lead && a.bn.mode == kBnTrain) || !batch);
  const float om = upd ? a.bn.mmean[f] : 0.f, ov = upd ? a.bn.mvar[f] : 1.f;
  float bias = 0.f;
  int lab[4] = {0, 0, 0, 0};
  if (wave == 0) {
    if (fr < NC) bias = a.bh[fr];
    if (a.labels) {
#pragma unroll
      for (int i = 0; i < 4; ++i) lab[i] = a.labels[min(r0 + fq * 4 + i, B - 1)];
    }
  }
  double S = 0.0, S2 = 0.0;
  if (f < D && batch) {
    for (int p0 = 0; p0 < a.nrt; p0 += 8) {
      double v1[8], v2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = min(p0 + u, a.nrt - 1);
        v1[u] = a.hstat[((size_t)p * 2 + 0) * Dp + f];
        v2[u] = a.hstat[((size_t)p * 2 + 1) * Dp + f];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (p0 + u < a.nrt) {
          S += v1[u];
          S2 += v2[u];
        }
    }
  }
  if (f < Dp) {
    float mean = 0.f, rstd = 1.f;
    if (f < D) {
      if (batch) {
        const double m = S / B, v = fmax(S2 / B - m * m, 0.0);
        mean = (float)m;
        rstd = (float)(1.0 / sqrt(v + (double)a.bn.eps));
        if (lead && a.bn.mode == kBnTrain) {
          a.bn.saved[f] = mean;
          a.bn.saved[D + f] = rstd;
          a.bn.mmean[f] = om * a.bn.momentum + mean * (1.f - a.bn.momentum);
          a.bn.mvar[f] = ov * a.bn.momentum + (float)v * a.bn.bessel * (1.f - a.bn.momentum);
        }
      } else {
        mean = om;
        rstd = rsqrtf(ov + a.bn.eps);
      }
    }
    mu[f] = mean;
    rs[f] = rstd;
    sc[f] = f < D ? gm * rstd : 0.f;
    sh[f] = f < D ? bt - mean * gm * rstd : 0.f;
  }
  lds_barrier();
  stamp(a.stamps, 1);
  // ---- activation / xhat tiles, Wh.  With D % 4 == 0 the dropout masks are made 4 features at a time
  // (one Philox call per 4 consecutive elements, D-indexed, so the same masks as element by element)
  const bool quad = a.drop_on && (D & 3) == 0;
#pragma unroll
  for (int u = 0; u < kHU; ++u) {
    const int e = tid + u * NTHH;
    if (e < 16 * Dp) {
      const int r = dq(e, a.dDp), ff = e - r * Dp;
      float act = 0.f, xh = 0.f;
      if (r0 + r < B && ff < D) {
        xh = (hv[u] - mu[ff]) * rs[ff];
        act = fmaxf(fmaf(hv[u], sc[ff], sh[ff]), 0.f);
        if (a.drop_on && !quad) act *= keep_scale(a.rate, a.seed, it, a.layer_id, (long long)(r0 + r) * D + ff);
      }
      As[r * kHLD + ff] = act;
      Xh[r * kHLD + ff] = xh;
    }
    if (e < 16 * Dp) whs[(e >> 4) * 17 + (e & 15)] = wv[u];
  }
  if (quad) {
    lds_barrier();
    for (int q = tid; q < 4 * D; q += NTHH) {   // 16 rows x D/4 groups
      const int r = q / (D >> 2), f0 = 4 * (q - r * (D >> 2));
      if (r0 + r >= B) continue;
      const float4 k = keep_scale4(a.rate, a.seed, it, a.layer_id, (long long)(r0 + r) * D + f0);
      float* ar = As + r * kHLD + f0;
      ar[0] *= k.x;
      ar[1] *= k.y;
      ar[2] *= k.z;
      ar[3] *= k.w;
    }
  }
  lds_barrier();
  // ---- logits [16][16]: waves 0-3 = K quarters, summed in wave order
  if (wave < 4) {
    const int kq = Dp / 4;   // Dp % 16 == 0 -> multiple of 4
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < kq / 4; ++s) {
      const int k = wave * kq + 4 * s + fq;
      acc = mfma4(As[fr * kHLD + k], whs[k * 17 + fr], acc);
    }
    *reinterpret_cast<f32x4*>(&lgp[wave][lane * 4]) = acc;
  }
  lds_barrier();
  if (wave == 0) {
    f32x4 lg = *reinterpret_cast<const f32x4*>(&lgp[0][lane * 4]);
#pragma unroll
    for (int w = 1; w < 4; ++w) lg += *reinterpret_cast<const f32x4*>(&lgp[w][lane * 4]);
    float la = 0.f, ca = 0.f, na = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = fq * 4 + i, r = r0 + rl;
      const bool valid = r < B, cv = fr < NC;
      const float z = cv ? lg[i] + bias : -3.0e38f;
      const float m = row16_max(z);
      const float ex = cv ? __expf(z - m) : 0.f;
      const float sum = row16_sum(ex);
      const float pr = ex / sum;
      const int label = (valid && a.labels) ? lab[i] : 0;
      const int amx = row16_min(cv && z == m ? fr : 64);
      const float zl = __shfl(z, (lane & ~15) | (label & 15), 64);
      if (valid && fr == 0) {
        la += __logf(sum) + m - zl;
        ca += (amx == label) ? 1.f : 0.f;
        na += 1.f;
      }
      if (a.mode == 2 && valid && cv) a.out[(size_t)r * NC + fr] = a.out_softmax ? pr : z;
      dls[rl * 17 + fr] = (train && valid && cv) ? (pr - (fr == label ? 1.f : 0.f)) * a.scale : 0.f;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      la += __shfl_xor(la, o, 64);
      ca += __shfl_xor(ca, o, 64);
      na += __shfl_xor(na, o, 64);
    }
    if (a.metrics && lane == 0 && na > 0.f) {
      atomicAdd(a.metrics + 0, la);
      atomicAdd(a.metrics + 1, ca);
      atomicAdd(a.metrics + 2, na);
    }
  }
  stamp(a.stamps, 2);
  if (!train) return;
  lds_barrier();
  // ---- training: the tile's dbh / dWh partials, g and the dense BN's backward partial sums
  if (tid < 16) {
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += dls[r * 17 + tid];
    if (tid < NC) a.dbh_part[(size_t)rt * NC + tid] = s;
  }
  const int ntf = Dp / 16;
  float* dwp = a.dwh_part + (size_t)rt * D * NC;
  for (int ft = wave; ft < ntf; ft += NTHH / 64) {
    // dWh^T tile [feature][class] = act^T . dl over the 16 rows
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r = 4 * s + fq;
      acc = mfma4(As[r * kHLD + ft * 16 + fr], dls[r * 17 + fr], acc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int fi = ft * 16 + fq * 4 + i;
      if (fi < D && fr < NC) dwp[(size_t)fi * NC + fr] = acc[i];
    }
    // g [row][feature] = dl . Wh^T through the dropout / ReLU masks
    f32x4 gg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 4 * s + fq;
      gg = mfma4(dls[fr * 17 + c], whs[(ft * 16 + fr) * 17 + c], gg);
    }
    const int fg = ft * 16 + fr;
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = fq * 4 + i, r = r0 + rl;
      float gv = 0.f;
      if (r < B && fg < D) {
        const float act = As[rl * kHLD + fg];
        // act > 0 <=> ReLU passed AND dropout kept; the kept scale is 1/keep
        gv = act > 0.f ? (a.drop_on ? gg[i] * (1.f / (1.f - a.rate)) : gg[i]) : 0.f;
        s1 += gv;
        s2 += (double)(gv * Xh[rl * kHLD + fg]);
      }
      if (r < B) a.g[(size_t)r * Dp + fg] = gv;
    }
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (fq == 0) {
      a.gstat[((size_t)rt * 2 + 0) * Dp + fg] = s1;
      a.gstat[((size_t)rt * 2 + 1) * Dp + fg] = s2;
    }
  }
  stamp(a.stamps, 3);
}

// ------------------------------------------------------------------------------------------------
// Dense backward: grid (ceil(K/32), ceil(B/64)): one 32-feature K tile x one 64-row block per
// workgroup, every load in one batch.  dh = dL/dh is finished while staging: the head's g, h and the
// dense BN's backward sums (fixed-order sum of the head's row-tile partials) give
// dh = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)).
//   waves 0-7   dA[64 rows][32] = dh . W^T (row tile w & 3, K half w >> 2) -> g = dA * ReLU mask of
//               the input BN, and that BN's backward sums
//   waves 8-15  the row block's dW partial [32][Dp] = A^T . dh (K half x 16-column tiles); the reduce
//               launch sums the row blocks in order
constexpr int kUDh = 16, kUWk = 8;   // dh block 64 x Dp <= 16384, W rows 32 x D <= 8192
struct DenseBwdArgs {
  int B, K, D, Dp, ldh, nrt;
  Dv dD, dDp, dC;
  const float* in; Bn bn;           // the input layer's raw output and its BN (kBnSaved)
  const float* w;                   // [K][D]
  const float* gh;                  // [B][Dp] the head's g (dL/d dense-BN output)
  const float* h;                   // [B][Dp] the dense pre-activation
  const double* gstat;              // [nrt][2][Dp] the head's backward partial sums
  Bn bnd;                           // the dense BN (kBnSaved)
  float *dbeta_d, *dgamma_d;        // its gradients (nullable)
  float* dwpart;                    // [ceil(B/64)][K][D]
  float* g;                         // [B][K]
  double* acc;                      // [gridDim.x * gridDim.y][2][C] BN backward partial sums of the input layer
  long long* stamps;
};

// The head folded into the dense backward (training; dense_bwd_kernel<true>): every workgroup recomputes the
// head of ALL rows — the dense BN's backward sums need g of every row — from h (in registers, MFMA tile layout),
// dense_fwd's statistics partials and dropout keep flags, Wh, the labels.  Only the activation tile passes through
// LDS (the logits MFMA's A operand); g comes out of the MFMA already in the tile layout, next to the xhat it is
// multiplied by.  Workgroup (0, 0) stores what the head launch stored once (saved / moving statistics, metrics),
// the column-0 workgroups the dWh / dbh partials of their 64 rows.  Opt-in (TDE_BNCNN_HEAD_FOLD=1): it deletes the
// head launch and one boundary, but the 8x head work per workgroup costs more (phase clocks: 7.3 us activations +
// logits + softmax, 11.2 us g + sums + dh, vs the head launch's 7.7 us; Model B 1.019 M -> 0.920 M img/s).
struct HeadFold {
  const double* hstat;           // [nrt][2][Dp] dense_fwd's statistics partials
  const unsigned* keep;          // dense_fwd's keep flags (null: no dropout)
  float inv_keep;                // 1 / (1 - rate)
  int NC;
  const float* wh; const float* bh; const int* labels; float scale;
  float* metrics; float* dwh_part; float* dbh_part;
};
constexpr int kHT = 7;   // head tiles per wave: nrt * Dp / 16 <= 16 * kHT
// phase-A LDS bytes: act [nrt*16][Dp+4] | Wh [Dp][17] | dl [nrt*16][17] | max(BN coefficients, logit halves,
// per-tile backward sums f64)
__host__ __device__ inline int head_fold_lds(int nrt, int Dp) {
  const int u = 4 * 256 * 4 > 16 * 256 * 4 ? 4 * 256 * 4 : 16 * 256 * 4;
  const int gp = nrt * 2 * Dp * 8;
  return (nrt * 16 * (Dp + 4) + Dp * 17 + nrt * 16 * 17) * 4 + (gp > u ? gp : u);
}

template <bool HEAD>
__global__ __launch_bounds__(NTB) void dense_bwd_kernel(DenseBwdArgs a, HeadFold hf) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int C = a.bn.C, K = a.K, D = a.D, Dp = a.Dp, ldh = a.ldh;
  double* cs = reinterpret_cast<double*>(sm);             // [8][2][32]
  float* st = reinterpret_cast<float*>(sm + 16 * 2 * 32 * 8);
  float* dk = st + 4 * 32;                                 // [4][256]: gamma*rstd, mean(g), mean, rstd*mean(g*xhat)
  float* Wk = dk + 4 * 256;                                // [32][ldh]
  float* dhs = Wk + 32 * ldh;                              // [64][ldh]
  float* Ab = dhs + 64 * ldh;                              // [64][33] relu(BN(in))
  float* Xb = Ab + 64 * 33;                                // [64][33] raw in
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int kt0 = blockIdx.x * 32, b0 = blockIdx.y * 64, nb = min(64, a.B - b0);
  stamp(a.stamps, 0);
  Pf<kUWk> pw;
  Pf<2> px;
  // rows are contiguous: the tile is one clamped linear range (no index division in the address math)
  const int wlast = (K - kt0) * D - 1;
  const float* wt = a.w + (size_t)kt0 * D;
  pf_load(pw, 32 * D, [&](int e) { return wt[min(e, wlast)]; });
  pf_load(px, 64 * 32, [&](int e) { return a.in[(size_t)min(b0 + (e >> 5), a.B - 1) * K + min(kt0 + (e & 31), K - 1)]; });
  Pf<HEAD ? 1 : kUDh> pd, ph;
  if constexpr (HEAD) {
    const int B = a.B, nrt = a.nrt, NC = hf.NC, ntf = Dp >> 4, nt = nrt * ntf, ldA = Dp + 4;
    const bool lead = blockIdx.x == 0 && blockIdx.y == 0;
    float* As = reinterpret_cast<float*>(sm);
    float* whs = As + nrt * 16 * ldA;
    float* dls = whs + Dp * 17;
    float* U = dls + nrt * 16 * 17;
    float *mu = U, *rsd = U + 256, *scd = U + 512, *shd = U + 768;
    float* lgp = U;
    double* gp = reinterpret_cast<double*>(U);
    // ---- one batch of loads: h of this lane's head tiles (tile t = wave + 16 j: row tile t / ntf, feature tile
    // t % ntf; rows 4 fq + i, feature fr), their keep flags, Wh, bias / labels, the statistics partials of feature tid
    float hv[kHT][4];
    unsigned kw[kHT];
#pragma unroll
    for (int j = 0; j < kHT; ++j) {
      const int t = wave + 16 * j;
      kw[j] = 0x01010101u;
      if (t < nt) {
        const int rt = t / ntf, fe = (t - rt * ntf) * 16 + fr;
#pragma unroll
        for (int i = 0; i < 4; ++i) hv[j][i] = a.h[(size_t)min(rt * 16 + fq * 4 + i, B - 1) * Dp + fe];
        if (hf.keep) kw[j] = hf.keep[(size_t)t * 64 + lane];
      }
    }
    float wv[4];   // Dp * 16 <= 4 * NTB
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * NTB, fw = e >> 4, c = e & 15;
      wv[u] = (fw < D && c < NC) ? hf.wh[(size_t)fw * NC + c] : 0.f;
    }
    float bias = 0.f;
    int lab[4] = {0, 0, 0, 0};
    if (wave < nrt) {
      if (fr < NC) bias = hf.bh[fr];
#pragma unroll
      for (int i = 0; i < 4; ++i) lab[i] = hf.labels[min(wave * 16 + fq * 4 + i, B - 1)];
    }
    const Bn& bnd = a.bnd;
    const int f = tid;
    const float gm = (f < D && bnd.gamma) ? bnd.gamma[f] : 1.f;
    const float bt = (f < D && bnd.beta) ? bnd.beta[f] : 0.f;
    const bool upd = lead && f < D && bnd.mmean;
    const float om = upd ? bnd.mmean[f] : 0.f, ov = upd ? bnd.mvar[f] : 1.f;
    double S = 0.0, S2 = 0.0;
    if (f < D) {
      for (int p0 = 0; p0 < nrt; p0 += 8) {
        double v1[8], v2[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int p = min(p0 + u, nrt - 1);
          v1[u] = hf.hstat[((size_t)p * 2 + 0) * Dp + f];
          v2[u] = hf.hstat[((size_t)p * 2 + 1) * Dp + f];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (p0 + u < nrt) {
            S += v1[u];
            S2 += v2[u];
          }
      }
    }
    // ---- the dense BN's batch statistics (as the head launch: E[x^2] - E[x]^2 over the f64 partial sums)
    float coef = 0.f;   // gamma * rstd of feature tid
    if (f < Dp) {
      float mean = 0.f, rstd = 1.f;
      if (f < D) {
        const double m = S / B, v = fmax(S2 / B - m * m, 0.0);
        mean = (float)m;
        rstd = (float)(1.0 / sqrt(v + (double)bnd.eps));
        if (lead) {
          bnd.saved[f] = mean;
          bnd.saved[D + f] = rstd;
          if (bnd.mmean) {
            bnd.mmean[f] = om * bnd.momentum + mean * (1.f - bnd.momentum);
            bnd.mvar[f] = ov * bnd.momentum + (float)v * bnd.bessel * (1.f - bnd.momentum);
          }
        }
        coef = gm * rstd;
      }
      mu[f] = mean;
      rsd[f] = rstd;
      scd[f] = coef;
      shd[f] = f < D ? bt - mean * gm * rstd : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + u * NTB;
      if (e < Dp * 16) whs[(e >> 4) * 17 + (e & 15)] = wv[u];
    }
    lds_barrier();
    stamp(a.stamps, 1);
    // ---- activations (ReLU, dropout) -> LDS; hv becomes xhat
#pragma unroll
    for (int j = 0; j < kHT; ++j) {
      const int t = wave + 16 * j;
      if (t < nt) {
        const int rt = t / ntf, fe = (t - rt * ntf) * 16 + fr;
        const float m_ = mu[fe], r_ = rsd[fe], s_ = scd[fe], h_ = shd[fe];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl = rt * 16 + fq * 4 + i;
          float act = 0.f, x = 0.f;
          if (rl < B && fe < D) {
            x = (hv[j][i] - m_) * r_;
            act = fmaxf(fmaf(hv[j][i], s_, h_), 0.f);
            if (hf.keep) act = ((kw[j] >> (8 * i)) & 1u) ? act * hf.inv_keep : 0.f;
          }
          As[rl * ldA + fe] = act;
          hv[j][i] = x;
        }
      }
    }
    lds_barrier();
    // ---- logits [nrt*16][16]: wave = row tile (w & 7) x feature half (w >> 3), the halves summed in order
    {
      const int rt = wave & 7, kh = wave >> 3, kq = Dp >> 1;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (rt < nrt)
        for (int s4 = 0; s4 < kq / 4; ++s4) {
          const int k = kh * kq + 4 * s4 + fq;
          acc = mfma4(As[(rt * 16 + fr) * ldA + k], whs[k * 17 + fr], acc);
        }
      *reinterpret_cast<f32x4*>(&lgp[wave * 256 + lane * 4]) = acc;
    }
    lds_barrier();
    if (wave < nrt) {
      const f32x4 lg = *reinterpret_cast<const f32x4*>(&lgp[wave * 256 + lane * 4]) +
                       *reinterpret_cast<const f32x4*>(&lgp[(wave + 8) * 256 + lane * 4]);
      float la = 0.f, ca = 0.f, na = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = wave * 16 + fq * 4 + i;
        const bool valid = rl < B, cv = fr < NC;
        const float z = cv ? lg[i] + bias : -3.0e38f;
        const float m = row16_max(z);
        const float ex = cv ? __expf(z - m) : 0.f;
        const float sum = row16_sum(ex);
        const float pr = ex / sum;
        const int label = valid ? lab[i] : 0;
        const int amx = row16_min(cv && z == m ? fr : 64);
        const float zl = __shfl(z, (lane & ~15) | (label & 15), 64);
        if (valid && fr == 0) {
          la += __logf(sum) + m - zl;
          ca += (amx == label) ? 1.f : 0.f;
          na += 1.f;
        }
        dls[rl * 17 + fr] = (valid && cv) ? (pr - (fr == label ? 1.f : 0.f)) * hf.scale : 0.f;
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        la += __shfl_xor(la, o, 64);
        ca += __shfl_xor(ca, o, 64);
        na += __shfl_xor(na, o, 64);
      }
      if (lead && hf.metrics && lane == 0 && na > 0.f) {
        atomicAdd(hf.metrics + 0, la);
        atomicAdd(hf.metrics + 1, ca);
        atomicAdd(hf.metrics + 2, na);
      }
    }
    lds_barrier();
    stamp(a.stamps, 2);
    // ---- the column-0 workgroups: dbh / dWh partials of their 64 rows (row tiles rt_lo .. rt_hi-1)
    if (blockIdx.x == 0) {
      const int rt_lo = blockIdx.y * 4, rt_hi = min(nrt, rt_lo + 4);
      if (tid < 64) {
        const int rt = rt_lo + (tid >> 4), c = tid & 15;
        if (rt < rt_hi && c < NC) {
          float sb = 0.f;
          for (int r = 0; r < 16; ++r) sb += dls[(rt * 16 + r) * 17 + c];
          hf.dbh_part[(size_t)rt * NC + c] = sb;
        }
      }
      for (int item = wave; item < (rt_hi - rt_lo) * ntf; item += 16) {
        const int rt = rt_lo + item / ntf, ft = item % ntf;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int r = rt * 16 + 4 * s4 + fq;
          acc = mfma4(As[r * ldA + ft * 16 + fr], dls[r * 17 + fr], acc);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int fi = ft * 16 + fq * 4 + i;
          if (fi < D && fr < NC) hf.dwh_part[((size_t)rt * D + fi) * NC + fr] = acc[i];
        }
      }
    }
    // ---- g = dl . Wh^T through the dropout / ReLU masks (tile layout), per-tile backward partial sums
    float gq[kHT][4];
#pragma unroll
    for (int j = 0; j < kHT; ++j) {
      const int t = wave + 16 * j;
#pragma unroll
      for (int i = 0; i < 4; ++i) gq[j][i] = 0.f;
      if (t < nt) {
        const int rt = t / ntf, ft = t - rt * ntf, fe = ft * 16 + fr;
        f32x4 gg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int c = 4 * s4 + fq;
          gg = mfma4(dls[(rt * 16 + fr) * 17 + c], whs[(ft * 16 + fr) * 17 + c], gg);
        }
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl = rt * 16 + fq * 4 + i;
          float gv = 0.f;
          if (rl < B && fe < D) {
            // act > 0 <=> ReLU passed AND dropout kept; the kept scale is 1/keep
            gv = As[rl * ldA + fe] > 0.f ? (hf.keep ? gg[i] * hf.inv_keep : gg[i]) : 0.f;
            s1 += gv;
            s2 += (double)(gv * hv[j][i]);
          }
          gq[j][i] = gv;
        }
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (fq == 0) {
          // gp aliases the logit halves (read before the last barrier) and not As / whs / dls
          gp[((size_t)rt * 2 + 0) * Dp + fe] = s1;
          gp[((size_t)rt * 2 + 1) * Dp + fe] = s2;
        }
      }
    }
    lds_barrier();
    // ---- the dense BN's backward sums of feature tid over all rows, in row-tile order
    double T1 = 0.0, T2 = 0.0;
    if (tid < Dp)
      for (int rt = 0; rt < nrt; ++rt) {
        T1 += gp[((size_t)rt * 2 + 0) * Dp + tid];
        T2 += gp[((size_t)rt * 2 + 1) * Dp + tid];
      }
    lds_barrier();   // phase A's LDS is free: the dense backward's layout from here on
    if (tid < Dp) {
      dk[tid] = coef;
      dk[256 + tid] = (float)(T1 / B);
      dk[768 + tid] = (float)(T2 / B);
      if (lead && tid < D) {
        if (a.dbeta_d) a.dbeta_d[tid] = (float)T1;
        if (a.dgamma_d) a.dgamma_d[tid] = (float)T2;
      }
    }
    lds_barrier();
    // dh = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) of this workgroup's rows from the tiles in registers
#pragma unroll
    for (int j = 0; j < kHT; ++j) {
      const int t = wave + 16 * j;
      if (t < nt) {
        const int rt = t / ntf, fe = (t - rt * ntf) * 16 + fr;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = rt * 16 + fq * 4 + i - b0;
          if (r >= 0 && r < 64) dhs[r * ldh + fe] = r < nb ? dk[fe] * (gq[j][i] - dk[256 + fe] - hv[j][i] * dk[768 + fe]) : 0.f;
        }
      }
    }
    // rows of the 64-row block past the last head tile
    for (int e = tid; e < 64 * Dp; e += NTB) {
      const int r = e / Dp;
      if (b0 + r >= nrt * 16) dhs[r * ldh + (e - r * Dp)] = 0.f;
    }
    stamp(a.stamps, 3);
  } else {
    const int hlast = nb * Dp - 1;
    const float* ght = a.gh + (size_t)b0 * Dp;
    const float* ht = a.h + (size_t)b0 * Dp;
    pf_load(pd, 64 * Dp, [&](int e) { return ght[min(e, hlast)]; });
    pf_load(ph, 64 * Dp, [&](int e) { return ht[min(e, hlast)]; });
    // the dense BN's backward sums for feature tid (fixed order over the head's row tiles)
    if (tid < Dp) {
      // the saved statistics and gamma join the load batch (not a second round trip after the sums)
      const bool ok = tid < D;
      const float m = ok ? a.bnd.saved[tid] : 0.f, r = ok ? a.bnd.saved[D + tid] : 0.f;
      const float gm = (ok && a.bnd.gamma) ? a.bnd.gamma[tid] : 1.f;
      double S1 = 0.0, S2 = 0.0;
      for (int p0 = 0; p0 < a.nrt; p0 += 8) {
        double v1[8], v2[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int p = min(p0 + u, a.nrt - 1);
          v1[u] = a.gstat[((size_t)p * 2 + 0) * Dp + tid];
          v2[u] = a.gstat[((size_t)p * 2 + 1) * Dp + tid];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (p0 + u < a.nrt) {
            S1 += v1[u];
            S2 += v2[u];
          }
      }
      dk[tid] = ok ? gm * r : 0.f;
      dk[256 + tid] = (float)(S1 / a.B);
      dk[512 + tid] = m;
      dk[768 + tid] = r * (float)(S2 / a.B);
      if (ok && blockIdx.x == 0 && blockIdx.y == 0) {
        if (a.dbeta_d) a.dbeta_d[tid] = (float)S1;
        if (a.dgamma_d) a.dgamma_d[tid] = (float)S2;
      }
    }
  }
  bn_prepare(a.bn, st, false, nullptr);
  if (!HEAD) stamp(a.stamps, 1);
  const float* sc = st;
  const float* sh = st + C;
  const float* mu = st + 2 * C;
  const float* rs = st + 3 * C;
  pf_store(pw, 32 * D, [&](int e, float v) {
    const int kk = dq(e, a.dD), n = e - kk * D;
    Wk[kk * ldh + n] = kt0 + kk < K ? v : 0.f;
  });
  if (Dp > D)
    for (int e = tid; e < 32 * (Dp - D); e += NTB) Wk[(e / (Dp - D)) * ldh + D + e % (Dp - D)] = 0.f;
  if constexpr (!HEAD) {
#pragma unroll
    for (int u = 0; u < kUDh; ++u) {
      const int e = tid + u * NTB;
      if (e < 64 * Dp) {
        const int r = dq(e, a.dDp), n = e - r * Dp;
        // dh = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)), xhat*rstd folded: (h - mean)*rstd*mean(g*xhat)
        const float dh = dk[n] * (pd.v[u] - dk[256 + n] - (ph.v[u] - dk[512 + n]) * dk[768 + n]);
        dhs[r * ldh + n] = r < nb ? dh : 0.f;
      }
    }
  }
  pf_store(px, 64 * 32, [&](int e, float v) {
    const int r = e >> 5, kk = e & 31, kg = kt0 + kk, c = kg - dq(kg, a.dC) * C;
    const bool ok = r < nb && kt0 + kk < K;
    Xb[r * 33 + kk] = ok ? v : 0.f;
    Ab[r * 33 + kk] = ok ? fmaxf(fmaf(v, sc[c], sh[c]), 0.f) : 0.f;
  });
  lds_barrier();
  stamp(a.stamps, HEAD ? 4 : 2);
  if (wave < 8) {
    const int rt = wave & 3, kh = wave >> 2;
    const int k_me = kt0 + kh * 16 + fr, c_me = k_me - dq(k_me, a.dC) * C;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < Dp / 4; s0 += 4) {   // Dp % 16 == 0
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int n = 4 * (s0 + u) + fq;
        acc = mfma4(dhs[(rt * 16 + fr) * ldh + n], Wk[(kh * 16 + fr) * ldh + n], acc);
      }
    }
    // lane: dA[row rt*16 + 4fq + i][feature k_me]
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rt * 16 + fq * 4 + i;
      if (r < nb && k_me < K) {
        const float x = Xb[r * 33 + kh * 16 + fr];
        const float gv = fmaf(x, sc[c_me], sh[c_me]) > 0.f ? acc[i] : 0.f;
        a.g[(size_t)(b0 + r) * K + k_me] = gv;
        s1 += gv;
        s2 += gv * (x - mu[c_me]) * rs[c_me];
      }
    }
    s1 += __shfl_xor(s1, 16, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (fq == 0) {
      cs[(wave * 2 + 0) * 32 + fr] = s1;
      cs[(wave * 2 + 1) * 32 + fr] = s2;
    }
  } else {
    const int ntd = Dp / 16;
    float* dst = a.dwpart + (size_t)blockIdx.y * K * D;
    for (int item = wave - 8; item < 2 * ntd; item += 8) {
      const int kh = item & 1, dt = item >> 1;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int st4 = 0; st4 < 16; ++st4) {
        const int r = 4 * st4 + fq;
        acc = mfma4(Ab[r * 33 + kh * 16 + fr], dhs[r * ldh + dt * 16 + fr], acc);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = kt0 + kh * 16 + fq * 4 + i, n = dt * 16 + fr;
        if (k < K && n < D) dst[(size_t)k * D + n] = acc[i];
      }
    }
  }
  // BN backward sums: feature f of wave w -> channel (kt0 + (w >> 2) * 16 + f) % C
  stamp(a.stamps, HEAD ? 5 : 3);
  lds_barrier();
  if (tid < 2 * C) {
    // the tile's features of channel c: kk = kk0, kk0 + C, ... (< 32), each over the 4 row tiles, in order
    const int j = tid / C, c = tid - j * C;
    const int r0c = kt0 - dq(kt0, a.dC) * C;           // channel of the tile's first feature
    double S = 0.0;
    for (int kk = c >= r0c ? c - r0c : c - r0c + C; kk < 32 && kt0 + kk < K; kk += C)
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) S += cs[((rt + 4 * (kk >> 4)) * 2 + j) * 32 + (kk & 15)];
    a.acc[(size_t)wg_id() * 2 * C + j * C + c] = S;
  }
  stamp(a.stamps, HEAD ? 6 : 4);
}

// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// Conv backward: grid (B, 1 + dgrad); blockIdx.y 0 = the weight gradient of image b, 1 = its input
// gradient (two workgroups per image: all 256 CUs busy at B = 128).
//   both roles: dZ = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) of the image in a zero-bordered LDS
//     grid (this BN's backward sums from the fixed-order partials)
//   weight gradient: items (16-row K tile, pixel split) -> K = the image's output pixels; the split
//     partials summed through LDS in order -> the image's partial dW
//   input gradient, the stride-s conv as a stride-1 "depth-to-space" product: every output-base block
//     (ob_h, ob_w) gathers the same dZ window (taps jh < ceil(kh/sh), jw < ceil(kw/sw)) for all
//     sh*sw sub-pixel classes, so A = that window [blocks x (jh, jw, co)] and B = the class-stacked
//     weights [(jh, jw, co) x (class, ci)] -> dA of the whole sh x sw input block per output row;
//     ReLU mask of the input BN -> g of the previous layer + that BN's backward partial sums
struct ConvBwdArgs {
  ConvBwdP p;
  int B;
  const float* z; Bn bn; BnBwd bb; const float* gout; float count;   // this layer (count = B*Ho*Wo)
  const float* w;
  const float* in; Bn bn_in; float* gin; double* acc_in;             // the input side
  float* dwpart;                     // [B][K][Co]
  long long* stamps;
  const float* wstack;               // input gradient: the class-stacked [Kdp][NP] weights (nullable)
};

__global__ __launch_bounds__(NTB) void conv_bwd_kernel(ConvBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const ConvBwdP& P = a.p;
  const Geo& g = P.g;
  double* cs = reinterpret_cast<double*>(sm + P.o_cs);     // [16][2][64]
  double* red = reinterpret_cast<double*>(sm + P.o_red);
  float* st = reinterpret_cast<float*>(sm + P.o_st);       // this BN: mean, rstd, gamma*rstd
  float* stin = reinterpret_cast<float*>(sm + P.o_stin);   // input BN: sc, sh, mean, rstd
  float* kks = reinterpret_cast<float*>(sm + P.o_kk);      // sum g, sum g*xhat
  float* dz = reinterpret_cast<float*>(sm + P.o_dz);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int b = blockIdx.x;
  const bool dg = blockIdx.y == 1;
  const int C = g.C, Co = g.Co, Mo = P.Mo, K = P.K, Wd = P.Wd, Wp = P.Wp;
  stamp(a.stamps, 0);
  // ---- one batch of global loads
  const int nact = Mo * Co, nimg = g.H * g.W * C, nw = K * Co;
  Pf<kUAct> pg, pz;
  Pf<kUW> pw;
  Pf<kUImg> px;
  {
    const float* gz = a.gout + (size_t)b * nact;
    const float* zz = a.z + (size_t)b * nact;
    const float* im = a.in + (size_t)b * nimg;
    pf_load(pg, nact, [&](int i) { return gz[i]; });
    pf_load(pz, nact, [&](int i) { return zz[i]; });
    pf_load(px, nimg, [&](int i) { return im[i]; });
    if (dg && a.wstack) {
      // the class-stacked weights this step's forward of the layer staged (conv_fwd wstack): contiguous
      pf_load(pw, P.Kdp * P.NP, [&](int i) { return a.wstack[i]; });
    } else if (dg) {
      pf_load(pw, nw, [&](int i) { return a.w[i]; });
    }
  }
  // the per-channel constants: partials of this layer's backward sums (fixed-order sum), saved
  // statistics
  // (issued before the partial sums' adds: their loads and these share one round trip)
  float cmu = 0.f, crs = 0.f, cg = 1.f;
  if (tid < Co) {
    cmu = a.bn.saved[tid];
    crs = a.bn.saved[Co + tid];
    cg = a.bn.gamma ? a.bn.gamma[tid] : 1.f;
  }
  float imu = 0.f, irs = 1.f, ig = 1.f, ib = 0.f;
  const int ti = tid - 64;
  if (ti >= 0 && ti < C && a.bn_in.mode == kBnSaved) {
    imu = a.bn_in.saved[ti];
    irs = a.bn_in.saved[C + ti];
    ig = a.bn_in.gamma ? a.bn_in.gamma[ti] : 1.f;
    ib = a.bn_in.beta ? a.bn_in.beta[ti] : 0.f;
  }
  const int Q = 2 * Co, np = NTB / Q, qq = tid % Q, qpart = tid / Q;
  double tsum = 0.0;
  if (qpart < np) {
    for (int j0 = qpart; j0 < a.bb.npart; j0 += 8 * np) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + u * np;
        v[u] = j < a.bb.npart ? a.bb.acc[j * Q + qq] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) tsum += v[u];
    }
  }
  // LDS the registers do not cover
  for (int i = tid; i < P.Hd * Wd; i += NTB) {
    const int y = dq(i, P.dWd), x = i - y * Wd;
    if (y < P.Ph || y >= P.Ph + g.Ho || x < P.Pw || x >= P.Pw + g.Wo)
      for (int c = 0; c < Co; ++c) dz[i * Co + c] = 0.f;
  }
  if (tid < 32) dz[P.zslot + tid] = 0.f;
  if (!dg) {
    float* Xs = reinterpret_cast<float*>(sm + P.o_xs);
    int* kow = reinterpret_cast<int*>(sm + P.o_kow);
    int2* ptab = reinterpret_cast<int2*>(sm + P.o_ptab);
    for (int i = tid; i < P.Hp * Wp; i += NTB) {
      const int y = dq(i, P.dWp), x = i - y * Wp, iy = y - g.pt, ix = x - g.pl;
      if (iy < 0 || iy >= g.H || ix < 0 || ix >= g.W)
        for (int c = 0; c < C; ++c) Xs[i * C + c] = 0.f;
    }
    for (int k = tid; k < P.Kw16; k += NTB) {
      int off = 0;
      if (k < K) {
        const int t = dq(k, P.dC), ci = k - t * C, ky = dq(t, P.dkw), kx = t - ky * g.kw;
        off = (ky * Wp + kx) * C + ci;
      }
      kow[k] = off;
    }
    for (int p = tid; p < P.wg_split * P.wg_spp * 4; p += NTB) {
      int2 e{0, P.zslot};
      if (p < Mo) {
        const int oh = dq(p, P.dWo), ow = p - oh * g.Wo;
        e = int2{(oh * g.sh * Wp + ow * g.sw) * C, ((oh + P.Ph) * Wd + ow + P.Pw) * Co};
      }
      ptab[p] = e;
    }
  } else {
    float* Wb = reinterpret_cast<float*>(sm + P.o_wb);
    int* kod = reinterpret_cast<int*>(sm + P.o_kod);
    // class-stacked weights: zero where no weight lands (padding rows / columns, taps past the kernel)
    for (int i = a.wstack ? P.Kdp * P.NP : tid; i < P.Kdp * P.NP; i += NTB) {
      const int kk = dq(i, P.dNP), n = i - kk * P.NP;
      bool hole = kk >= P.Kd || n >= P.NC;
      if (!hole) {
        const int t = dq(kk, P.dCo), jh = dq(t, P.dntw), jw = t - jh * P.ntw;
        const int cl = dq(n, P.dC), ry = dq(cl, P.dsw), rx = cl - ry * g.sw;
        hole = ry + g.sh * jh >= g.kh || rx + g.sw * jw >= g.kw;
      }
      if (hole) Wb[i] = 0.f;
    }
    for (int kk = tid; kk < P.Kdp; kk += NTB) {
      int off = 0;
      if (kk < P.Kd) {
        const int t = dq(kk, P.dCo), co = kk - t * Co, jh = dq(t, P.dntw), jw = t - jh * P.ntw;
        off = (-jh * Wd - jw) * Co + co;
      }
      kod[kk] = off;
    }
  }
  if (qpart < np) red[tid] = tsum;
  if (tid < Co) {
    st[tid] = cmu;
    st[Co + tid] = crs;
    st[2 * Co + tid] = cg * crs;
  }
  if (ti >= 0 && ti < C) {
    const bool none = a.bn_in.mode == kBnNone;
    const float sc = ig * irs;
    stin[ti] = none ? 1.f : sc;
    stin[C + ti] = none ? 0.f : ib - imu * sc;
    stin[2 * C + ti] = imu;
    stin[3 * C + ti] = irs;
  }
  lds_barrier();
  parts_to_slots(red, np, Q);
  if (tid < Q) {
    const double S = red[tid];
    kks[tid] = (float)S;
    if (b == 0 && !dg) {
      if (tid < Co && a.bb.dbeta) a.bb.dbeta[tid] = (float)S;
      if (tid >= Co && a.bb.dgamma) a.bb.dgamma[tid - Co] = (float)S;
    }
  }
  lds_barrier();
  stamp(a.stamps, 1);
  // ---- registers -> LDS: dZ, the input (BN + ReLU'd for the weight gradient, raw for the input
  // gradient's mask), the class-stacked weights
  {
    const float inv = 1.f / a.count;
#pragma unroll
    for (int u = 0; u < kUAct; ++u) {
      const int i = tid + u * NTB;
      if (i < nact) {
        const int p = dq(i, P.dCo), co = i - p * Co, oh = dq(p, P.dWo), ow = p - oh * g.Wo;
        const float xh = (pz.v[u] - st[co]) * st[Co + co];
        dz[((oh + P.Ph) * Wd + ow + P.Pw) * Co + co] =
            st[2 * Co + co] * (pg.v[u] - kks[co] * inv - xh * kks[Co + co] * inv);
      }
    }
    if (!dg) {
      float* Xs = reinterpret_cast<float*>(sm + P.o_xs);
      const bool raw = a.bn_in.mode == kBnNone;
      pf_store(px, nimg, [&](int i, float v) {
        const int pix = dq(i, P.dC), c = i - pix * C, y = dq(pix, P.dW), x = pix - y * g.W;
        Xs[((y + g.pt) * Wp + x + g.pl) * C + c] = raw ? v : fmaxf(fmaf(v, stin[c], stin[C + c]), 0.f);
      });
    } else {
      float* Xr = reinterpret_cast<float*>(sm + P.o_xr);
      float* Wb = reinterpret_cast<float*>(sm + P.o_wb);
      pf_store(px, nimg, [&](int i, float v) { Xr[i] = v; });
      if (a.wstack)
        pf_store(pw, P.Kdp * P.NP, [&](int i, float v) { Wb[i] = v; });
      else
        pf_store(pw, nw, [&](int i, float v) {
        const int t = dq(i, P.dCo), co = i - t * Co, t2 = dq(t, P.dC), ci = t - t2 * C;
        const int ky = dq(t2, P.dkw), kx = t2 - ky * g.kw;
        const int jh = dq(ky, P.dsh), jw = dq(kx, P.dsw), cl = (ky - jh * g.sh) * g.sw + kx - jw * g.sw;
        Wb[((jh * P.ntw + jw) * Co + co) * P.NP + cl * C + ci] = v;
      });
    }
  }
  lds_barrier();
  stamp(a.stamps, 2);
  if (!dg) {
    // ---------------- weight gradient
    const float* Xs = reinterpret_cast<const float*>(sm + P.o_xs);
    const int* kow = reinterpret_cast<const int*>(sm + P.o_kow);
    const int2* ptab = reinterpret_cast<const int2*>(sm + P.o_ptab);
    float* part = reinterpret_cast<float*>(sm + P.o_part);
    float* dst = a.dwpart + (size_t)b * K * Co;
    for (int item = wave; item < P.n_wg_items; item += 16) {
      const int kt = item % P.wg_tiles, sp = item / P.wg_tiles;
      const int off = kow[kt * 16 + fr];
      f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      for (int s0 = 0; s0 < P.wg_spp; s0 += 4) {
        int2 t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = ptab[4 * (sp * P.wg_spp + s0 + u) + fq];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float av = Xs[t[u].x + off];
          acc[0] = mfma4(av, dz[t[u].y + fr], acc[0]);
          if (P.nco > 1) acc[1] = mfma4(av, dz[t[u].y + 16 + fr], acc[1]);
        }
      }
      if (P.wg_split == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = kt * 16 + fq * 4 + i;
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const int co = n * 16 + fr;
            if (k < K && n < P.nco && co < Co) dst[(size_t)k * Co + co] = acc[n][i];
          }
        }
      } else {
#pragma unroll
        for (int n = 0; n < 2; ++n)
          if (n < P.nco)
            *reinterpret_cast<f32x4*>(part + ((size_t)((sp * P.wg_tiles + kt) * P.nco + n) * 64 + lane) * 4) = acc[n];
      }
    }
    if (P.wg_split > 1) {
      lds_barrier();
      for (int t = wave; t < P.wg_tiles * P.nco; t += 16) {
        const int kt = t / P.nco, n = t - kt * P.nco;
        f32x4 v = *reinterpret_cast<const f32x4*>(part + ((size_t)(kt * P.nco + n) * 64 + lane) * 4);
        for (int sp = 1; sp < P.wg_split; ++sp)
          v += *reinterpret_cast<const f32x4*>(part + ((size_t)((sp * P.wg_tiles + kt) * P.nco + n) * 64 + lane) * 4);
        const int co = n * 16 + fr;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = kt * 16 + fq * 4 + i;
          if (k < K && co < Co) dst[(size_t)k * Co + co] = v[i];
        }
      }
    }
    stamp(a.stamps, 3);
    return;
  }
  // ---------------- input gradient (depth-to-space)
  const float* Xr = reinterpret_cast<const float*>(sm + P.o_xr);
  const float* Wb = reinterpret_cast<const float*>(sm + P.o_wb);
  const int* kod = reinterpret_cast<const int*>(sm + P.o_kod);
  float* partd = reinterpret_cast<float*>(sm + P.o_partd);
  const int ntile = P.mtd * P.nnt;
  for (int item = wave; item < P.n_dg_items; item += 16) {
    const int kp = item % P.ksd, t = item / P.ksd, nt = t % P.nnt, mtile = t / P.nnt;
    const int m = min(mtile * 16 + fr, P.Md - 1);
    const int obh = dq(m, P.dNbw), obw = m - obh * P.Nbw;
    const int base = ((P.obh0 + obh + P.Ph) * Wd + P.obw0 + obw + P.Pw) * Co;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i0 = 0; i0 < P.spd; i0 += 4) {
      int o[4];
      float bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = 4 * (kp + (i0 + u) * P.ksd) + fq;
        o[u] = kod[k];
        bv[u] = Wb[k * P.NP + nt * 16 + fr];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = mfma4(dz[base + o[u]], bv[u], acc);
    }
    *reinterpret_cast<f32x4*>(partd + ((size_t)(kp * ntile + t) * 64 + lane) * 4) = acc;
  }
  lds_barrier();
  stamp(a.stamps, 3);
  double s1[kMaxDgNT], s2[kMaxDgNT];
#pragma unroll
  for (int n = 0; n < kMaxDgNT; ++n) s1[n] = s2[n] = 0.0;
  float* gin = a.gin + (size_t)b * nimg;
  for (int t = wave; t < ntile; t += 16) {
    const int nt = t % P.nnt, mtile = t / P.nnt;
    f32x4 v = *reinterpret_cast<const f32x4*>(partd + ((size_t)t * 64 + lane) * 4);
    for (int kp = 1; kp < P.ksd; ++kp) v += *reinterpret_cast<const f32x4*>(partd + ((size_t)(kp * ntile + t) * 64 + lane) * 4);
    const int n = nt * 16 + fr;
    if (n >= P.NC) continue;
    const int cl = dq(n, P.dC), ci = n - cl * C, ry = dq(cl, P.dsw), rx = cl - ry * g.sw;
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mtile * 16 + fq * 4 + i;
      if (m >= P.Md) continue;
      const int obh = dq(m, P.dNbw), obw = m - obh * P.Nbw;
      const int ih = (P.obh0 + obh) * g.sh + ry - g.pt, iw = (P.obw0 + obw) * g.sw + rx - g.pl;
      if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) continue;
      const int e = (ih * g.W + iw) * C + ci;
      const float x = Xr[e];
      const float gv = fmaf(x, stin[ci], stin[C + ci]) > 0.f ? v[i] : 0.f;
      gin[e] = gv;
      t1 += gv;
      t2 += (double)(gv * (x - stin[2 * C + ci]) * stin[3 * C + ci]);
    }
#pragma unroll
    for (int q = 0; q < kMaxDgNT; ++q)
      if (q == nt) {
        s1[q] += t1;
        s2[q] += t2;
      }
  }
  // the input BN's backward partial sums: per-wave column sums -> cs[wave][stat][64 columns] -> per
  // channel (columns n with n % C == ci), waves and columns in a fixed order
#pragma unroll
  for (int q = 0; q < kMaxDgNT; ++q) {
    double x1 = s1[q], x2 = s2[q];
    x1 += __shfl_xor(x1, 16, 64);
    x1 += __shfl_xor(x1, 32, 64);
    x2 += __shfl_xor(x2, 16, 64);
    x2 += __shfl_xor(x2, 32, 64);
    if (fq == 0) {
      cs[(wave * 2 + 0) * 64 + q * 16 + fr] = x1;
      cs[(wave * 2 + 1) * 64 + q * 16 + fr] = x2;
    }
  }
  lds_barrier();
  if (tid < 2 * C) {
    // same order as walking w, then the class columns n = c + r*C; the loads of 4 waves are issued as
    // one batch (a runtime-bound loop here was a 64-long chain of dependent LDS round trips, ~3 us)
    const int j = tid / C, c = tid - j * C;
    double S = 0.0;
#pragma unroll 1
    for (int w0 = 0; w0 < 16; w0 += 4) {
      double v[4][kMaxCls];
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int r = 0; r < kMaxCls; ++r) {
          const int n = c + r * C;
          v[w][r] = n < P.NC ? cs[((w0 + w) * 2 + j) * 64 + n] : 0.0;
        }
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int r = 0; r < kMaxCls; ++r) S += v[w][r];
    }
    a.acc_in[(size_t)b * 2 * C + j * C + c] = S;
  }
  stamp(a.stamps, 4);
}

// ------------------------------------------------------------------------------------------------
// Weight-gradient partials (per image for the convs, per row block for the dense layer) -> the flat
// gradient bucket, summed in partial order.  Each workgroup owns 64 elements of one segment; its 4
// waves take every 4th partial with up to 32 loads in flight per thread; fixed combine order.
// Fused step (apply = 1, one replica): the summed gradient is not stored; the optimizer step is applied
// to the weight (and slots) at the element's flat offset right there (Adam's t = the step counter the
// step's first launch advanced), so the separate multi-tensor optimizer launch disappears.  Segments
// whose partial IS the bucket (BN beta / gamma, written by the backward launches) are zeroed after use.
constexpr int kMaxRed = 16;
struct ReduceArgs {
  int n;
  const float* part[kMaxRed];
  float* out[kMaxRed];
  long long len[kMaxRed];
  int cnt[kMaxRed];            // partials of the segment
  int blk0[kMaxRed + 1];       // first workgroup of the segment
  int wide[kMaxRed];           // few partials (<= kWideCnt), len % 4 == 0: 1024 elements per workgroup,
                               // a float4 per thread summed over all partials (16x fewer workgroups)
  int apply;
  float* g;                    // the flat bucket (segment offsets = out[j] - g)
  float *w, *m, *v;
  const long long* iterations;
  OptHyper h;
  long long* stamps;
  // fused DP exchange (step mode "xgmi"): segment push_seg (the Dense kernel's gradient, 94 % of the bytes)
  // goes straight into the xGMI owners' contribution areas of the all-reduce call that follows
  int push_seg;
  XgPush push;
};
__device__ __forceinline__ void reduce_commit(const ReduceArgs& a, int j, long long e, float gs, long long t, bool inplace) {
  if (j == a.push_seg) {
    xg_push_store(a.push, (int)((*a.push.epoch + 1u) & 1u), a.push.off + e, gs);
    return;
  }
  if (!a.apply) {
    a.out[j][e] = gs;
    return;
  }
  const long long f = (a.out[j] - a.g) + e;
  float m = a.h.kind != kOptSGD ? a.m[f] : 0.f, vv = a.h.kind == kOptAdam ? a.v[f] : 0.f;
  a.w[f] = opt_step(a.h, opt_lr_t(a.h, t), a.w[f], gs, m, vv);
  if (a.h.kind != kOptSGD) a.m[f] = m;
  if (a.h.kind == kOptAdam) a.v[f] = vv;
  if (inplace) a.out[j][e] = 0.f;
}

constexpr int kWideCnt = 8;

__global__ __launch_bounds__(NTH) void reduce_kernel(ReduceArgs a) {
  __shared__ float red[4][64];
  const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
  int j = 0;
  while (j + 1 < a.n && (int)blockIdx.x >= a.blk0[j + 1]) ++j;
  if (a.wide[j]) {
    // a float4 of 4 consecutive elements per thread, every partial summed in order by that thread
    const long long len = a.len[j], e0 = ((long long)(blockIdx.x - a.blk0[j]) * NTH + threadIdx.x) * 4;
    if (e0 >= len) return;
    const int cnt = a.cnt[j];
    const float* p = a.part[j];
    const long long t = a.apply && a.h.kind == kOptAdam ? *a.iterations : 0;
    float4 v[kWideCnt];
#pragma unroll
    for (int u = 0; u < kWideCnt; ++u)
      if (u < cnt) v[u] = *reinterpret_cast<const float4*>(p + (size_t)u * len + e0);
    float4 s = v[0];
#pragma unroll
    for (int u = 1; u < kWideCnt; ++u)
      if (u < cnt) {
        s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
      }
    const bool inplace = p == a.out[j];
    if (j == a.push_seg && ((a.push.off | a.push.L) & 3) == 0) {   // one 16-byte store into the owner
      xg_push_store4(a.push, (int)((*a.push.epoch + 1u) & 1u), a.push.off + e0, s);
      xg_push_drain();
      return;
    }
    reduce_commit(a, j, e0 + 0, s.x, t, inplace);
    reduce_commit(a, j, e0 + 1, s.y, t, inplace);
    reduce_commit(a, j, e0 + 2, s.z, t, inplace);
    reduce_commit(a, j, e0 + 3, s.w, t, inplace);
    if (j == a.push_seg) xg_push_drain();
    return;
  }
  const long long len = a.len[j];
  const long long e = (long long)(blockIdx.x - a.blk0[j]) * 64 + l;
  const int cnt = a.cnt[j];
  const float* p = a.part[j];
  const long long ec = e < len ? e : len - 1;
  const long long t = a.apply && a.h.kind == kOptAdam ? *a.iterations : 0;
  float s = 0.f;
  for (int b0 = q; b0 < cnt; b0 += 128) {
    float v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (b0 + 4 * u < cnt) v[u] = p[(size_t)(b0 + 4 * u) * len + ec];
#pragma unroll
    for (int u = 0; u < 32; ++u)
      if (b0 + 4 * u < cnt) s += v[u];
  }
  red[q][l] = s;
  __syncthreads();
  if (q == 0 && e < len) reduce_commit(a, j, e, (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]), t, p == a.out[j]);
  if (j == a.push_seg) xg_push_drain();
}

}  // namespace bncnn
}  // namespace tde

using namespace tde;
using namespace tde::bncnn;

// ---- host entry points (ctypes).  Geometry / BN descriptors are passed as flat C structs.
struct TdeBnGeo { int H, W, C, Ho, Wo, Co, kh, kw, sh, sw, pt, pl; };
struct TdeBn {
  int mode, C;
  const double* acc; int npart; double count;
  const float *gamma, *beta;
  float eps, momentum, bessel;
  float *mmean, *mvar, *saved;
};
struct TdeBnBwd {
  const double* acc; int npart;
  float *dbeta, *dgamma;
};
static Geo geo_of(const TdeBnGeo* g) { return Geo{g->H, g->W, g->C, g->Ho, g->Wo, g->Co, g->kh, g->kw, g->sh, g->sw, g->pt, g->pl}; }
static Bn bn_of(const TdeBn* b) {
  return Bn{b->mode, b->C, b->acc, b->npart, b->count, b->gamma, b->beta, b->eps, b->momentum, b->bessel, b->mmean, b->mvar,
            b->saved};
}
static bool bn_ok(const TdeBn* b) {
  if (!b || b->C < 1 || b->C > 32) return false;
  if ((b->mode == kBnTrain || b->mode == kBnBatch) && (!b->acc || b->npart < 1 || !(b->count > 0))) return false;
  if (b->mode == kBnTrain && !b->saved) return false;
  if (b->mode == kBnMoving && (!b->mmean || !b->mvar)) return false;
  if (b->mode == kBnSaved && !b->saved) return false;
  return b->mode >= kBnNone && b->mode <= kBnSaved;
}

// Diagnostic phase clocks: after tde_bncnn_stamps(base, n), the next n launches record
// stamps[launch][workgroup][slot] (s_memrealtime, 100 MHz) into base (kStampStride per launch).
constexpr int kStampStride = 8192 * kMaxStamps;
static long long* g_stamp_base = nullptr;
static int g_stamp_next = 0, g_stamp_cap = 0;
TDE_API void tde_bncnn_stamps(long long* base, int n) {
  g_stamp_base = base;
  g_stamp_next = 0;
  g_stamp_cap = base ? n : 0;
}
static long long* next_stamps() {
  if (!g_stamp_base || g_stamp_next >= g_stamp_cap) return nullptr;
  return g_stamp_base + (size_t)(g_stamp_next++) * kStampStride;
}

template <typename F>
static void set_lds(F* f, int bytes) {
  (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
static int up(int x, int m) { return (x + m - 1) / m * m; }
constexpr int kMaxLds = 160 * 1024;


static Dv dv(int d) { return Dv{d, 1.0f / (float)d}; }

// Forward conv launch geometry; 0 if it fits (LDS, prefetch registers), <0 otherwise.
static int conv_bwd_plan(const Geo& g, int dgrad, ConvBwdP& P);

static int conv_fwd_plan(const Geo& g, ConvFwdP& P) {
  P = ConvFwdP{};
  P.g = g;
  P.K = g.kh * g.kw * g.C;
  P.M = g.Ho * g.Wo;
  P.Hp = std::max((g.Ho - 1) * g.sh + g.kh, g.pt + g.H);
  P.Wp = std::max((g.Wo - 1) * g.sw + g.kw, g.pl + g.W);
  if (g.C < 1 || g.C > 32 || g.Co < 1 || g.Co > 32) return -1;
  if (g.H * g.W * g.C > kUImg * NTB || P.K * g.Co > kUW * NTB) return -2;
  P.nct = (g.Co + 15) / 16;
  const int steps = (P.K + 3) / 4;
  P.mt = (P.M + 15) / 16;
  P.msplit = P.mt >= 2 ? 2 : 1;
  P.mtw = (P.mt + P.msplit - 1) / P.msplit;
  P.msplit = (P.mt + P.mtw - 1) / P.mtw;
  const int base = P.mtw * P.nct;
  P.ks = 1;
  while (base * P.ks < 16 && P.ks < 8 && (steps + 2 * P.ks - 1) / (2 * P.ks) >= 8) P.ks *= 2;
  P.spp = up((steps + P.ks - 1) / P.ks, 4);
  P.Kpad = 4 * P.ks * P.spp;
  P.dC = dv(g.C);
  P.dCo = dv(g.Co);
  P.dW = dv(g.W);
  P.dWo = dv(g.Wo);
  P.dWp = dv(P.Wp);
  P.dkw = dv(g.kw);
  P.dNTP = dv(P.nct * 16);
  int o = 0;
  P.o_red = o; o += NTB * 8;
  P.o_cs = o; o += 16 * 2 * 32 * 8;
  P.o_st = o; o += 4 * 32 * 4;
  P.o_xs = o; o += up(P.Hp * P.Wp * g.C, 4) * 4;
  P.o_ws = o; o += P.Kpad * P.nct * 16 * 4;
  P.o_koff = o; o += P.Kpad * 4;
  P.o_part = o; o += P.ks * base * 256 * 4;
  P.lds = o;
  return o > kMaxLds ? -3 : 0;
}

// out = {lds, ks, msplit (workgroups per image = statistics partials per image)}
TDE_API int tde_bncnn_conv_fwd_cfg(const TdeBnGeo* gg, int* out) {
  ConvFwdP P;
  const int rc = conv_fwd_plan(geo_of(gg), P);
  out[0] = P.lds;
  out[1] = P.ks;
  out[2] = P.msplit;
  return rc;
}

// z = conv(relu(BN_in(in))); this layer's BN partial sums into acc [B][2][Co] (nullable).
// inc_iter (nullable): the step counter a training step's first launch advances.
TDE_API int tde_bncnn_conv_fwd(const TdeBnGeo* gg, int B, const float* in, const TdeBn* bn_in, const float* w, float* z,
                               double* acc, long long* inc_iter, float* wstack, hipStream_t stream) {
  ConvFwdP P;
  if (conv_fwd_plan(geo_of(gg), P) != 0) return -1;
  if (!bn_ok(bn_in) || bn_in->C != P.g.C || B < 1 || bn_in->mode == kBnSaved) return -2;
  ConvFwdArgs a{P, B, in, bn_of(bn_in), w, z, acc, next_stamps(), inc_iter, wstack, ConvBwdP{}};
  if (wstack) {
    // the whole stack must be covered by the grid's threads, and fit the backward's registers
    if (conv_bwd_plan(P.g, 1, a.sp) != 0 || !a.sp.wgather || a.sp.Kdp * a.sp.NP > B * P.msplit * NTB) return -3;
  }
  set_lds(conv_fwd_kernel, P.lds);
  conv_fwd_kernel<<<dim3(B, P.msplit), NTB, P.lds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// h = relu(BN(in)) . W (final, deterministic) and the dense BN's statistics partials per 16-row tile.
// keep (nullable): the dropout keep flags of the folded head (HeadFold), drawn at step *iter
TDE_API int tde_bncnn_dense_fwd(int B, int K, int D, int Dp, const float* in, const TdeBn* bn, const float* w, float* h,
                                double* hstat, unsigned* keep, float rate, unsigned long long seed, const long long* iter,
                                int layer_id, hipStream_t stream) {
  if (!bn_ok(bn) || bn->mode == kBnSaved || bn->mode == kBnNone || (Dp & 15) || Dp < D || !h || !hstat) return -1;
  if (keep && (!iter || !(rate > 0.f && rate < 1.f))) return -3;
  const bool v4 = (K & 3) == 0 && ((uintptr_t)in & 15) == 0 && up((K + 15) / 16, 16) <= 4 * kDS;
  const int kw = v4 ? up((K + 15) / 16, 16) : up((K + 15) / 16, 4);
  if (kw > 4 * kDS) return -2;
  DenseFwdArgs a{B, K, D, Dp, kw, dv(bn->C), in, bn_of(bn), w, h, hstat, next_stamps(), keep, rate, seed, iter, layer_id};
  if (v4) dense_fwd_kernel<true><<<dim3(Dp / 16, (B + 15) / 16), NTB, 0, stream>>>(a);
  else dense_fwd_kernel<false><<<dim3(Dp / 16, (B + 15) / 16), NTB, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// The head (see HeadArgs): grid ceil(B/16).
TDE_API int tde_bncnn_head(int B, int D, int Dp, int NC, int mode, const float* h, const double* hstat, const TdeBn* bn,
                           float rate, unsigned long long seed, const long long* iter, int layer_id, int drop_on,
                           const float* wh, const float* bh, const int* labels, float scale, float* metrics, float* out,
                           int out_softmax, float* dwh_part, float* dbh_part, float* g, double* gstat,
                           hipStream_t stream) {
  if (!bn || bn->C != D || (Dp & 15) || Dp < D || Dp > kHeadMaxDp || NC < 1 || NC > 16 || B < 1 || !h || !hstat)
    return -1;
  if (!(bn->mode == kBnTrain || bn->mode == kBnMoving || bn->mode == kBnBatch)) return -2;
  if ((bn->mode == kBnTrain && !bn->saved) || ((bn->mode == kBnTrain || bn->mode == kBnMoving) && (!bn->mmean || !bn->mvar)))
    return -2;
  if (mode == 0 && (!dwh_part || !dbh_part || !g || !gstat || !labels || bn->mode != kBnTrain)) return -3;
  if (mode == 2 && !out) return -4;
  if (drop_on && !(rate > 0.f && rate < 1.f)) return -5;
  const int nrt = (B + 15) / 16;
  HeadArgs a{B, D, Dp, NC, mode, nrt, dv(Dp), h, hstat, bn_of(bn), rate, seed, iter, layer_id, drop_on, wh, bh, labels, scale,
             metrics, out, out_softmax, dwh_part, dbh_part, g, gstat, next_stamps()};
  head_kernel<<<nrt, NTHH, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Debug export of the dropout keep scales the head applies at step *iter: out[r * D + f] = 1/(1-rate) or 0
// (keep_scale per element; the head's 4-at-a-time form draws the same values).  Tests pin the fused
// plan's dropout against a float64 oracle with this mask.
__global__ void dropout_mask_kernel(int n, float rate, unsigned long long seed, const long long* iter, int layer,
                                    float* out) {
  const long long it = iter ? *iter : 0;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x)
    out[e] = keep_scale(rate, seed, it, layer, e);
}

TDE_API int tde_bncnn_dropout_mask(int B, int D, float rate, unsigned long long seed, const long long* iter,
                                   int layer_id, float* out, hipStream_t stream) {
  if (B < 1 || D < 1 || !out || !(rate > 0.f && rate < 1.f)) return -1;
  const int n = B * D;
  dropout_mask_kernel<<<(n + 255) / 256, 256, 0, stream>>>(n, rate, seed, iter, layer_id, out);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_bncnn_dense_bwd(int B, int K, int D, int Dp, const float* in, const TdeBn* bn, const float* w,
                                const float* gh, const float* h, const double* gstat, int nrt, const TdeBn* bnd,
                                float* dbeta_d, float* dgamma_d, float* dwpart, float* g, double* acc,
                                hipStream_t stream) {
  if (!bn_ok(bn) || bn->mode != kBnSaved || (Dp & 15) || Dp < D || Dp > 256 || !acc || !gh || !h || !gstat || nrt < 1)
    return -1;
  if (!bnd || !bnd->saved || bnd->C != D) return -1;
  if (32 * D > kUWk * NTB || 64 * Dp > kUDh * NTB || 2 * (Dp / 16) > 32) return -2;
  const int ldh = Dp + 4;
  const int lds = 16 * 2 * 32 * 8 + 4 * 32 * 4 + 4 * 256 * 4 + 32 * ldh * 4 + 64 * ldh * 4 + 2 * 64 * 33 * 4;
  if (lds > kMaxLds) return -3;
  DenseBwdArgs a{};
  a.B = B;
  a.K = K;
  a.D = D;
  a.Dp = Dp;
  a.ldh = ldh;
  a.nrt = nrt;
  a.dD = dv(D);
  a.dDp = dv(Dp);
  a.dC = dv(bn->C);
  a.in = in;
  a.bn = bn_of(bn);
  a.w = w;
  a.gh = gh;
  a.h = h;
  a.gstat = gstat;
  a.bnd = bn_of(bnd);
  a.dbeta_d = dbeta_d;
  a.dgamma_d = dgamma_d;
  a.dwpart = dwpart;
  a.g = g;
  a.acc = acc;
  a.stamps = next_stamps();
  set_lds(dense_bwd_kernel<false>, lds);
  dense_bwd_kernel<false><<<dim3((K + 31) / 32, (B + 63) / 64), NTB, lds, stream>>>(a, HeadFold{});
  TDE_LAUNCH_CHECK();
  return 0;
}

// The training head folded into the dense backward (dense_bwd_kernel<true>; replaces tde_bncnn_head mode 0 +
// tde_bncnn_dense_bwd): bnd in mode kBnTrain (statistics from hstat; saved / moving updated by workgroup (0, 0));
// keep = dense_fwd's keep flags (null: no dropout).  B <= 128, Dp <= 224, NC <= 16.
TDE_API int tde_bncnn_dense_bwd_head(int B, int K, int D, int Dp, int NC, const float* in, const TdeBn* bn, const float* w,
                                     const float* h, const double* hstat, const TdeBn* bnd, const unsigned* keep,
                                     float rate, const float* wh, const float* bh, const int* labels, float scale,
                                     float* metrics, float* dwh_part, float* dbh_part, float* dbeta_d, float* dgamma_d,
                                     float* dwpart, float* g, double* acc, hipStream_t stream) {
  const int nrt = (B + 15) / 16;
  if (!bn_ok(bn) || bn->mode != kBnSaved || (Dp & 15) || Dp < D || !acc || !h || !hstat || B < 1 || B > 128) return -1;
  if (!bnd || bnd->C != D || bnd->mode != kBnTrain || !bnd->saved || !wh || !bh || !labels || !dwh_part || !dbh_part ||
      NC < 1 || NC > 16)
    return -1;
  if (32 * D > kUWk * NTB || Dp * 16 > 4 * NTB || nrt * (Dp / 16) > 16 * kHT || 2 * (Dp / 16) > 32) return -2;
  if (keep && !(rate > 0.f && rate < 1.f)) return -4;
  const int ldh = Dp + 4;
  const int lds_b = 16 * 2 * 32 * 8 + 4 * 32 * 4 + 4 * 256 * 4 + 32 * ldh * 4 + 64 * ldh * 4 + 2 * 64 * 33 * 4;
  const int lds_a = head_fold_lds(nrt, Dp);
  const int lds = lds_a > lds_b ? lds_a : lds_b;
  if (lds > kMaxLds) return -3;
  DenseBwdArgs a{};
  a.B = B;
  a.K = K;
  a.D = D;
  a.Dp = Dp;
  a.ldh = ldh;
  a.nrt = nrt;
  a.dD = dv(D);
  a.dDp = dv(Dp);
  a.dC = dv(bn->C);
  a.in = in;
  a.bn = bn_of(bn);
  a.w = w;
  a.h = h;
  a.bnd = bn_of(bnd);
  a.dbeta_d = dbeta_d;
  a.dgamma_d = dgamma_d;
  a.dwpart = dwpart;
  a.g = g;
  a.acc = acc;
  a.stamps = next_stamps();
  HeadFold hf{hstat, keep, keep ? 1.f / (1.f - rate) : 1.f, NC, wh, bh, labels, scale, metrics, dwh_part, dbh_part};
  set_lds(dense_bwd_kernel<true>, lds);
  dense_bwd_kernel<true><<<dim3((K + 31) / 32, (B + 63) / 64), NTB, lds, stream>>>(a, hf);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Backward conv launch geometry; 0 if it fits, <0 otherwise.
static int conv_bwd_plan(const Geo& g, int dgrad, ConvBwdP& P) {
  P = ConvBwdP{};
  P.g = g;
  P.dgrad = dgrad;
  P.K = g.kh * g.kw * g.C;
  P.Mo = g.Ho * g.Wo;
  if (g.C < 1 || g.C > 32 || g.Co < 1 || g.Co > 32 || g.sh < 1 || g.sw < 1 || g.sh * g.sw > kMaxCls) return -1;
  if (P.Mo * g.Co > kUAct * NTB || g.H * g.W * g.C > kUImg * NTB || (dgrad && P.K * g.Co > kUW * NTB)) return -2;
  P.nco = (g.Co + 15) / 16;
  P.nth = (g.kh + g.sh - 1) / g.sh;
  P.ntw = (g.kw + g.sw - 1) / g.sw;
  P.Ph = dgrad ? P.nth + 1 : 0;
  P.Pw = dgrad ? P.ntw + 1 : 0;
  // bottom / right margin: the largest output-base row (H-1+pt)/sh must stay inside the bordered grid
  P.Hd = g.Ho + 2 * P.Ph + (dgrad ? std::max((g.H - 1 + g.pt) / g.sh - (g.Ho - 1), 0) : 0);
  P.Wd = g.Wo + 2 * P.Pw + (dgrad ? std::max((g.W - 1 + g.pl) / g.sw - (g.Wo - 1), 0) : 0);
  P.Hp = std::max((g.Ho - 1) * g.sh + g.kh, g.pt + g.H);
  P.Wp = std::max((g.Wo - 1) * g.sw + g.kw, g.pl + g.W);
  P.zslot = P.Hd * P.Wd * g.Co;
  // input gradient (depth-to-space): blocks = output-base positions with at least one input pixel
  P.ncls = g.sh * g.sw;
  P.NC = P.ncls * g.C;
  P.NP = (P.NC + 15) / 16 * 16;
  P.nnt = P.NP / 16;
  if (dgrad && P.nnt > kMaxDgNT) return -1;
  P.Kd = P.nth * P.ntw * g.Co;
  P.obh0 = g.pt / g.sh;
  P.obw0 = g.pl / g.sw;
  const int Nbh = (g.H - 1 + g.pt) / g.sh - P.obh0 + 1;
  P.Nbw = (g.W - 1 + g.pl) / g.sw - P.obw0 + 1;
  P.Md = Nbh * P.Nbw;
  P.mtd = (P.Md + 15) / 16;
  const int dsteps = (P.Kd + 3) / 4;
  P.ksd = 1;
  while (P.mtd * P.nnt * P.ksd < 16 && P.ksd < 4 && (dsteps + 2 * P.ksd - 1) / (2 * P.ksd) >= 8) P.ksd *= 2;
  P.spd = up((dsteps + P.ksd - 1) / P.ksd, 4);
  P.Kdp = 4 * P.ksd * P.spd;
  P.n_dg_items = dgrad ? P.mtd * P.nnt * P.ksd : 0;
  // weight gradient: K tiles x pixel splits (~32 items; >= 4 steps per split)
  P.wg_tiles = (P.K + 15) / 16;
  P.Kw16 = P.wg_tiles * 16;
  const int wsteps = (P.Mo + 3) / 4;
  P.wg_split = std::max(1, std::min(std::min(16, 32 / P.wg_tiles), wsteps / 4));
  P.wg_spp = up((wsteps + P.wg_split - 1) / P.wg_split, 4);
  P.n_wg_items = P.wg_tiles * P.wg_split;
  P.dC = dv(g.C);
  P.dCo = dv(g.Co);
  P.dW = dv(g.W);
  P.dWo = dv(g.Wo);
  P.dWd = dv(P.Wd);
  P.dWp = dv(P.Wp);
  P.dkw = dv(g.kw);
  P.dntw = dv(P.ntw);
  P.dNbw = dv(P.Nbw);
  P.dNP = dv(P.NP);
  P.dsh = dv(g.sh);
  P.dsw = dv(g.sw);
  P.wgather = dgrad && P.Kdp * P.NP <= kUW * NTB;
  int o = 0;
  P.o_red = o; o += NTB * 8;
  P.o_cs = o; o += 16 * 2 * 64 * 8;
  P.o_st = o; o += 4 * 32 * 4;
  P.o_stin = o; o += 4 * 32 * 4;
  P.o_kk = o; o += 2 * 32 * 4;
  P.o_dz = o; o += up(P.zslot + 32, 4) * 4;
  P.o_role = o;
  int ow = o;   // weight-gradient role
  P.o_xs = ow; ow += up(P.Hp * P.Wp * g.C, 4) * 4;
  P.o_kow = ow; ow += P.Kw16 * 4;
  P.o_ptab = ow; ow += P.wg_split * P.wg_spp * 4 * 8;
  P.o_part = ow; ow += (P.wg_split > 1 ? P.wg_split * P.wg_tiles * P.nco * 256 : 0) * 4;
  int od = o;   // input-gradient role
  if (dgrad) {
    P.o_xr = od; od += up(g.H * g.W * g.C, 4) * 4;
    P.o_wb = od; od += P.Kdp * P.NP * 4;
    P.o_kod = od; od += P.Kdp * 4;
    P.o_partd = od; od += P.ksd * P.mtd * P.nnt * 256 * 4;
  }
  P.lds = std::max(ow, od);
  // the fast divisions: every dividend stays below 2^21
  return P.lds > kMaxLds ? -3 : 0;
}

// out = {lds, wgrad items, dgrad items, wgrad split, dgrad K split, staged weight floats}
TDE_API int tde_bncnn_conv_bwd_plan(const TdeBnGeo* gg, int dgrad, int* out) {
  ConvBwdP P;
  const int rc = conv_bwd_plan(geo_of(gg), dgrad, P);
  out[0] = P.lds;
  out[1] = P.n_wg_items;
  out[2] = P.n_dg_items;
  out[3] = P.wg_split;
  out[4] = P.ksd;
  out[5] = P.wgather ? P.Kdp * P.NP : 0;   // floats of the forward-staged input-gradient weights
  return rc;
}

TDE_API int tde_bncnn_conv_bwd(const TdeBnGeo* gg, int B, const float* z, const TdeBn* bn, const TdeBnBwd* bb,
                               const float* gout, const float* w, const float* in, const TdeBn* bn_in, float* gin,
                               double* acc_in, float* dwpart, int dgrad, const float* wstack, hipStream_t stream) {
  ConvBwdP P;
  if (conv_bwd_plan(geo_of(gg), dgrad, P) != 0) return -1;
  const Geo& g = P.g;
  if (!bn_ok(bn) || bn->mode != kBnSaved || bn->C != g.Co || !bb || !bb->acc || bb->npart < 1) return -2;
  if (!bn_ok(bn_in) || bn_in->C != g.C || !(bn_in->mode == kBnSaved || bn_in->mode == kBnNone)) return -3;
  if (dgrad && (!gin || !acc_in || bn_in->mode != kBnSaved || !w)) return -4;
  ConvBwdArgs a{};
  a.p = P;
  a.B = B;
  a.z = z;
  a.bn = bn_of(bn);
  a.bb = BnBwd{bb->acc, bb->npart, bb->dbeta, bb->dgamma};
  a.gout = gout;
  a.count = (float)((double)B * g.Ho * g.Wo);
  a.w = w;
  a.in = in;
  a.bn_in = bn_of(bn_in);
  a.gin = gin;
  a.acc_in = acc_in;
  a.dwpart = dwpart;
  a.stamps = next_stamps();
  a.wstack = dgrad ? wstack : nullptr;
  if (a.wstack && !P.wgather) return -5;
  set_lds(conv_bwd_kernel, P.lds);
  conv_bwd_kernel<<<dim3(B, dgrad ? 2 : 1), NTB, P.lds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// n segments: part[j] holds cnt[j] partials of len[j] floats, summed in order into out[j] (views of the
// flat bucket g).  opt (nullable): apply the optimizer step instead of storing (see reduce_kernel).
struct TdeBnOpt {
  int kind;
  float lr, mom, b1, b2, eps;
  float *g, *w, *m, *v;
  const long long* iterations;
};
TDE_API int tde_bncnn_reduce(int n, const int* cnt, const float* const* part, float* const* out, const long long* len,
                             const TdeBnOpt* opt, int push_seg, const XgPush* push, hipStream_t stream) {
  if (n < 1 || n > kMaxRed) return -1;
  ReduceArgs a{};
  a.n = n;
  a.push_seg = -1;
  if (push && push->nranks > 0) {   // push_seg's element e is bucket element push->off + e
    if (opt || push_seg < 0 || push_seg >= n || push->nranks > kXgMaxRanks || push->L <= 0 || !push->epoch) return -4;
    a.push_seg = push_seg;
    a.push = *push;
  }
  a.stamps = next_stamps();
  if (opt) {
    if (!opt->g || !opt->w || !opt->iterations || (opt->kind != kOptSGD && !opt->m) ||
        (opt->kind == kOptAdam && !opt->v))
      return -2;
    a.iterations = opt->iterations;
    a.apply = 1;
    a.g = opt->g;
    a.w = opt->w;
    a.m = opt->m;
    a.v = opt->v;
    a.h = OptHyper{opt->kind, opt->lr, opt->mom, opt->b1, opt->b2, opt->eps};
  }
  int blocks = 0;
  for (int j = 0; j < n; ++j) {
    if (cnt[j] < 1 || len[j] < 1) return -1;
    if (opt && (out[j] < opt->g)) return -3;
    a.part[j] = part[j];
    a.out[j] = out[j];
    a.len[j] = len[j];
    a.cnt[j] = cnt[j];
    a.blk0[j] = blocks;
    a.wide[j] = cnt[j] <= kWideCnt && (len[j] & 3) == 0 && (((uintptr_t)part[j] | (uintptr_t)out[j]) & 15) == 0;
    blocks += a.wide[j] ? (int)((len[j] + 4 * NTH - 1) / (4 * NTH)) : (int)((len[j] + 63) / 64);
  }
  a.blk0[n] = blocks;
  reduce_kernel<<<blocks, NTH, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}
