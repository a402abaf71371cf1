// Float32 forms of the layer-wise kernel library (layers.hip computes in bf16): under the float32
// policy — the reference's precision (distributed_with_keras.py:21; every Keras default of
// mnist_keras_distributed.py:79-115) — any Sequential / functional model that has no hand-fused plan
// runs its whole step on these kernels with f32 activations, f32 activation gradients and the f32 master
// weights read in place (no bf16 shadow anywhere).
//
// * igemm32: ONE implicit-GEMM kernel family on the exact-f32 MFMA v_mfma_f32_16x16x4_f32 for Conv2D
//   fwd / bwd-data / bwd-filter and Dense fwd / bwd-data / bwd-weight, the operand kinds of layers.hip
//   (A gathered NHWC / row-major, B read straight from the HWIO / [in, out] master kernels):
//       kind            A(m,k)                          B(k,n)
//       dense fwd       X[m*lda+k]          (A_ROWK)    W[k*ldb+n]          (B_KN)
//       dense dgrad     dY[m*lda+k]         (A_ROWK)    W[n*ldb+k]          (B_NK)
//       conv fwd        X[b,oh*s-p+kh,..,c] (A_CONV)    W[(kh,kw,c)*Co+n]   (B_KN)
//       conv dgrad      dY[b,(ih+p-kh)/s,.] (A_DGRAD)   W[kh,kw,n,co]       (B_DGRADW)
//       dense wgrad     X[k*lda+m]          (A_COLM)    dY[k*ldb+n]         (B_KN)
//       conv wgrad      X[b,oh*s-p+kh,..,m] (A_WGRAD)   dY[k*Co+n]          (B_KN)
//   64x64 output tiles, 4 waves of 32x32 (2x2 MFMA tiles), 16-k chunks double-buffered through LDS
//   (global loads of chunk c+1 in flight while chunk c feeds the matrix cores, one barrier per chunk).
//   Lane group q of a wave supplies k = 4q..4q+3 of the chunk as ONE float4 LDS read per operand tile
//   (the k order inside a chunk is free: both operands use the same one).  Epilogue: bias, ReLU,
//   store or += (tensors with several consumers), the per-column f64 sum / sum of squares the next
//   BatchNormalization needs, or split-K partials summed in a fixed order by a second launch.
// * bn_fwd32 / bn_bwd32 (reduce + apply) / act_bwd32 / colstats32 with the semantics of their bf16
//   twins (affine + residual + ReLU + Philox dropout, Keras moving statistics), maxpool32 (argmax
//   bytes, gather backward), gap32, pad32, xent32 (f32 dlogits).
#include "tde_common.h"
#include "tde_philox.h"

#include <cstdlib>
#include <cstring>
#include <initializer_list>

namespace tde {
namespace l32 {

struct Geo {  // NHWC input [B,H,W,C], HWIO kernel [KH,KW,C,Co], NHWC output [B,Ho,Wo,Co]
  int B, H, W, C, Ho, Wo, Co, KH, KW, sh, sw, pt, pl;
};

enum AKind { A_ROWK = 0, A_CONV = 1, A_DGRAD = 2, A_COLM = 3, A_WGRAD = 4 };
enum BKind { B_NK = 0, B_DGRADW = 1, B_KN = 2 };

constexpr int KC = 16, LD = KC + 4;   // LDS rows of 16 k + 4 pad floats
constexpr int kSlots = 8;                               // BN statistics slots ([slot][2][C] f64)

struct G32 {
  const float* a;
  long long lda;
  const float* b;
  long long ldb;
  int M, N, K;
  int cps;          // 16-k chunks per split (grid z = split)
  Geo g;
  float* c;
  long long ldc;
  int accum;        // c += result
  float* part;      // split-K partials [split][M][N] (then c is written by g32_reduce)
  const float* bias;
  int relu;
  double* colstats; // [kSlots][2][N]
  // strided conv dgrad, every stride phase (ih % sh, iw % sw) in one launch (grid z = phase; no split):
  // per phase {ph_h, ph_w, Hp, Wp, kh0, kw0, KHp, KWp} — the phase's pixels and the only taps reaching them
  int nph;
  int phs[4][8];
};

// The stride phase of a block (A_DGRAD with nph > 0), else off
struct Ph {
  int on, ph_h, ph_w, Hp, Wp, kh0, kw0, KHp, KWp;
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- A(m, k) element index (or -1 = zero) for the K-contiguous kinds; row state precomputed
struct RowA {
  bool ok;
  long long base;
  int y0, x0;
};

template <int AK>
__device__ __forceinline__ RowA row_a(const G32& p, const Ph& ph, int m) {
  RowA r{m < p.M, 0, 0, 0};
  const int mm = r.ok ? m : 0;
  if (AK == A_ROWK) {
    r.base = (long long)mm * p.lda;
  } else if (AK == A_CONV) {
    const int hw = p.g.Ho * p.g.Wo, b = mm / hw, rem = mm - b * hw, oh = rem / p.g.Wo, ow = rem - oh * p.g.Wo;
    r.y0 = oh * p.g.sh - p.g.pt;
    r.x0 = ow * p.g.sw - p.g.pl;
    r.base = (long long)b * p.g.H * p.g.W;
  } else if (!ph.on) {  // A_DGRAD: m over input pixels
    const int hw = p.g.H * p.g.W, b = mm / hw, rem = mm - b * hw, ih = rem / p.g.W, iw = rem - ih * p.g.W;
    r.y0 = ih + p.g.pt;
    r.x0 = iw + p.g.pl;
    r.base = (long long)b * p.g.Ho * p.g.Wo;
  } else {  // A_DGRAD, one stride phase: y0 / x0 = the output row / col the phase's first tap reaches
    const int hw = ph.Hp * ph.Wp, b = mm / hw, rem = mm - b * hw, ihp = rem / ph.Wp, iwp = rem - ihp * ph.Wp;
    r.y0 = (ihp * p.g.sh + ph.ph_h + p.g.pt - ph.kh0) / p.g.sh;
    r.x0 = (iwp * p.g.sw + ph.ph_w + p.g.pl - ph.kw0) / p.g.sw;
    r.base = (long long)b * p.g.Ho * p.g.Wo;
  }
  return r;
}

template <int AK>
__device__ __forceinline__ long long a_idx(const G32& p, const Ph& ph, const RowA& r, int k) {
  if (!r.ok || k >= p.K) return -1;
  if (AK == A_ROWK) return r.base + k;
  const int Cd = AK == A_CONV ? p.g.C : p.g.Co;
  const int KWd = (AK == A_DGRAD && ph.on) ? ph.KWp : p.g.KW;
  const int kc = k / Cd, c = k - kc * Cd, kh = kc / KWd, kw = kc - kh * KWd;
  if (AK == A_DGRAD && ph.on) {   // phased: tap (kh0 + kh*sh) reaches output row y0 - kh exactly
    const int oh = r.y0 - kh, ow = r.x0 - kw;
    if ((unsigned)oh >= (unsigned)p.g.Ho || (unsigned)ow >= (unsigned)p.g.Wo) return -1;
    return (r.base + (long long)oh * p.g.Wo + ow) * p.g.Co + c;
  }
  if (AK == A_CONV) {
    const int ih = r.y0 + kh, iw = r.x0 + kw;
    if ((unsigned)ih >= (unsigned)p.g.H || (unsigned)iw >= (unsigned)p.g.W) return -1;
    return (r.base + (long long)ih * p.g.W + iw) * p.g.C + c;
  }
  int oh = r.y0 - kh, ow = r.x0 - kw;   // A_DGRAD: (ih + pt - kh) / sh must be exact and in range
  if (oh < 0 || ow < 0) return -1;
  if (p.g.sh != 1) {
    const int q = oh / p.g.sh;
    if (q * p.g.sh != oh) return -1;
    oh = q;
  }
  if (p.g.sw != 1) {
    const int q = ow / p.g.sw;
    if (q * p.g.sw != ow) return -1;
    ow = q;
  }
  if (oh >= p.g.Ho || ow >= p.g.Wo) return -1;
  return (r.base + (long long)oh * p.g.Wo + ow) * p.g.Co + c;
}

// 4 consecutive k of one row: one float4 when they share (kh, kw) and are aligned, else 4 gathers
template <int AK>
__device__ __forceinline__ float4 load_a_k4(const G32& p, const Ph& ph, const RowA& r, int k, bool vec) {
  if (vec) {   // K % 4 == 0 on this path: a quad is wholly in range or wholly out
    const long long i = a_idx<AK>(p, ph, r, k);
    if (i < 0) return float4{0.f, 0.f, 0.f, 0.f};
    return *reinterpret_cast<const float4*>(p.a + i);
  }
  float4 v;
  const long long i0 = a_idx<AK>(p, ph, r, k), i1 = a_idx<AK>(p, ph, r, k + 1), i2 = a_idx<AK>(p, ph, r, k + 2),
                  i3 = a_idx<AK>(p, ph, r, k + 3);
  v.x = i0 < 0 ? 0.f : p.a[i0];
  v.y = i1 < 0 ? 0.f : p.a[i1];
  v.z = i2 < 0 ? 0.f : p.a[i2];
  v.w = i3 < 0 ? 0.f : p.a[i3];
  return v;
}

// ---- B(k, n) for the K-contiguous kinds (image row = n)
template <int BK>
__device__ __forceinline__ long long b_idx_k(const G32& p, const Ph& ph, int n, int k) {
  if (n >= p.N || k >= p.K) return -1;
  if (BK == B_NK) return (long long)n * p.ldb + k;
  // B_DGRADW: k = (kh, kw, co), n = ci -> W[kh][kw][ci][co] (phased: kh = kh0 + kh'*sh, kw = kw0 + kw'*sw)
  const int kc = k / p.g.Co, co = k - kc * p.g.Co;
  if (ph.on) {
    const int khp = kc / ph.KWp, kwp = kc - khp * ph.KWp;
    const int kh = ph.kh0 + khp * p.g.sh, kw = ph.kw0 + kwp * p.g.sw;
    return ((long long)(kh * p.g.KW + kw) * p.g.C + n) * p.g.Co + co;
  }
  return ((long long)kc * p.g.C + n) * p.g.Co + co;
}

template <int BK>
__device__ __forceinline__ float4 load_b_k4(const G32& p, const Ph& ph, int n, int k, bool vec) {
  if (vec) {
    const long long i = b_idx_k<BK>(p, ph, n, k);
    if (i < 0) return float4{0.f, 0.f, 0.f, 0.f};
    return *reinterpret_cast<const float4*>(p.b + i);
  }
  float4 v;
  const long long i0 = b_idx_k<BK>(p, ph, n, k), i1 = b_idx_k<BK>(p, ph, n, k + 1), i2 = b_idx_k<BK>(p, ph, n, k + 2),
                  i3 = b_idx_k<BK>(p, ph, n, k + 3);
  v.x = i0 < 0 ? 0.f : p.b[i0];
  v.y = i1 < 0 ? 0.f : p.b[i1];
  v.z = i2 < 0 ? 0.f : p.b[i2];
  v.w = i3 < 0 ? 0.f : p.b[i3];
  return v;
}

// ---- M-contiguous A kinds (4 consecutive rows at one k)
struct ColA {   // A_WGRAD: the decomposition of the quad's first row m = (kh, kw, ci)
  int kh, kw, ci;
};

__device__ __forceinline__ long long wgrad_idx(const G32& p, int kh, int kw, int ci, int b, int oh, int ow) {
  const int ih = oh * p.g.sh - p.g.pt + kh, iw = ow * p.g.sw - p.g.pl + kw;
  if ((unsigned)ih >= (unsigned)p.g.H || (unsigned)iw >= (unsigned)p.g.W) return -1;
  return (((long long)b * p.g.H + ih) * p.g.W + iw) * p.g.C + ci;
}

template <int AK>
__device__ __forceinline__ float4 load_a_m4(const G32& p, int m, const ColA& w, int k, bool vec) {
  float4 v{0.f, 0.f, 0.f, 0.f};
  if (k >= p.K || m >= p.M) return v;
  if (AK == A_COLM) {
    const long long i = (long long)k * p.lda + m;
    if (vec) return *reinterpret_cast<const float4*>(p.a + i);
    v.x = p.a[i];
    v.y = m + 1 < p.M ? p.a[i + 1] : 0.f;
    v.z = m + 2 < p.M ? p.a[i + 2] : 0.f;
    v.w = m + 3 < p.M ? p.a[i + 3] : 0.f;
    return v;
  }
  // A_WGRAD: k = pixel (b, oh, ow)
  const int hw = p.g.Ho * p.g.Wo, b = k / hw, rem = k - b * hw, oh = rem / p.g.Wo, ow = rem - oh * p.g.Wo;
  if (vec) {   // C % 4 == 0: the 4 rows are ci..ci+3 of one (kh, kw)
    const long long i = wgrad_idx(p, w.kh, w.kw, w.ci, b, oh, ow);
    return i < 0 ? v : *reinterpret_cast<const float4*>(p.a + i);
  }
  float t[4];
  int kh = w.kh, kw = w.kw, ci = w.ci;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    long long i = -1;
    if (m + j < p.M) i = wgrad_idx(p, kh, kw, ci, b, oh, ow);
    t[j] = i < 0 ? 0.f : p.a[i];
    if (++ci == p.g.C) {
      ci = 0;
      if (++kw == p.g.KW) {
        kw = 0;
        ++kh;
      }
    }
  }
  return float4{t[0], t[1], t[2], t[3]};
}

__device__ __forceinline__ float4 load_b_n4(const G32& p, int n, int k, bool vec) {  // B_KN
  float4 v{0.f, 0.f, 0.f, 0.f};
  if (k >= p.K || n >= p.N) return v;
  const long long i = (long long)k * p.ldb + n;
  if (vec) return *reinterpret_cast<const float4*>(p.b + i);
  v.x = p.b[i];
  v.y = n + 1 < p.N ? p.b[i + 1] : 0.f;
  v.z = n + 2 < p.N ? p.b[i + 2] : 0.f;
  v.w = n + 3 < p.N ? p.b[i + 3] : 0.f;
  return v;
}

constexpr bool a_kcontig(int AK) { return AK == A_ROWK || AK == A_CONV || AK == A_DGRAD; }
constexpr bool b_kcontig(int BK) { return BK == B_NK || BK == B_DGRADW; }

// Output tile TBM x TBN with TBM * TBN = 4096 (64x64, 128x32, 256x16): narrow outputs (Model B's 6 / 12 /
// 24 channels, a wider variant's 48) take a narrow tile instead of leaving most of a 64-wide one empty.
// Waves: 2 x 2 of 32x32 (TBN 64), 4 x 1 of 32x32 (TBN 32), 4 x 1 of 64x16 (TBN 16).
template <int AK, int BK, int TBN>
__global__ __launch_bounds__(256) void igemm32_kernel(G32 p_) {
  constexpr int TBM = 4096 / TBN;
  constexpr int NA = TBM / 64;                    // A float4 loads per thread per chunk
  constexpr int NBT = TBN * 4;                    // threads loading one B float4 each per chunk
  constexpr int WAVES_M = TBN == 64 ? 2 : 4, WAVES_N = 4 / WAVES_M;
  constexpr int WR = TBM / WAVES_M, WC = TBN / WAVES_N, MI = WR / 16, NJ = WC / 16;
  __shared__ __attribute__((aligned(16))) float As[2][TBM * LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][TBN * LD];
  G32 p = p_;
  Ph ph{0, 0, 0, 0, 0, 0, 0, 0, 0};
  int split = blockIdx.z;
  if (AK == A_DGRAD && p_.nph > 0) {   // this block's stride phase (grid z = phase, one split)
    const int* t = p_.phs[blockIdx.z];
    ph = Ph{1, t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7]};
    p.M = p.g.B * ph.Hp * ph.Wp;
    p.K = ph.KHp * ph.KWp * p.g.Co;
    p.cps = (p.K + KC - 1) / KC;
    split = 0;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int m0 = blockIdx.x * TBM, n0 = blockIdx.y * TBN;
  if (m0 >= p.M) return;   // a phase smaller than the grid's largest
  const int nch = (p.K + KC - 1) / KC;
  const int c_lo = split * p.cps, c_hi = min(nch, c_lo + p.cps);

  // load slots: K-contiguous operand -> float4 i = (row i/4, k quad i%4); M/N-contiguous operand ->
  // (k = i / (rows/4), row quad 4 * (i % (rows/4)))
  int ra[NA], ka[NA];
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    const int i = tid + s * 256;
    ra[s] = a_kcontig(AK) ? i >> 2 : 4 * (i % (TBM / 4));
    ka[s] = a_kcontig(AK) ? 4 * (i & 3) : i / (TBM / 4);
  }
  const bool bload = tid < NBT;
  const int rb = b_kcontig(BK) ? tid >> 2 : 4 * (tid % (TBN / 4));
  const int kb = b_kcontig(BK) ? 4 * (tid & 3) : tid / (TBN / 4);
  RowA rowa[NA];
  ColA cola[NA];
#pragma unroll
  for (int s = 0; s < NA; ++s) {
    rowa[s] = RowA{};
    cola[s] = ColA{};
    if (a_kcontig(AK)) {
      rowa[s] = row_a<AK>(p, ph, m0 + ra[s]);
    } else if (AK == A_WGRAD) {
      const int m = min(m0 + ra[s], p.M - 1), kc = m / p.g.C;
      cola[s] = ColA{kc / p.g.KW, kc - (kc / p.g.KW) * p.g.KW, m - kc * p.g.C};
    }
  }
  // vector legality (whole quads inside one (kh, kw) group, 16-byte aligned)
  bool avec, bvec;
  if (AK == A_ROWK) avec = (p.lda & 3) == 0 && (p.K & 3) == 0 && ((uintptr_t)p.a & 15) == 0;
  else if (AK == A_CONV) avec = (p.g.C & 3) == 0 && ((uintptr_t)p.a & 15) == 0;
  else if (AK == A_DGRAD) avec = (p.g.Co & 3) == 0 && ((uintptr_t)p.a & 15) == 0;
  else if (AK == A_COLM) avec = (p.lda & 3) == 0 && (p.M & 3) == 0 && ((uintptr_t)p.a & 15) == 0;
  else avec = (p.g.C & 3) == 0 && ((uintptr_t)p.a & 15) == 0;
  if (BK == B_NK) bvec = (p.ldb & 3) == 0 && (p.K & 3) == 0 && ((uintptr_t)p.b & 15) == 0;
  else if (BK == B_DGRADW) bvec = (p.g.Co & 3) == 0 && ((uintptr_t)p.b & 15) == 0;
  else bvec = (p.ldb & 3) == 0 && (p.N & 3) == 0 && ((uintptr_t)p.b & 15) == 0;

  auto load = [&](int ch, float4* av, float4& bv) {
    const int k0 = ch * KC;
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      if (a_kcontig(AK)) av[s] = load_a_k4<AK>(p, ph, rowa[s], k0 + ka[s], avec);
      else av[s] = load_a_m4<AK>(p, m0 + ra[s], cola[s], k0 + ka[s], avec);
    }
    bv = float4{0.f, 0.f, 0.f, 0.f};
    if (bload) {
      if (b_kcontig(BK)) bv = load_b_k4<BK>(p, ph, n0 + rb, k0 + kb, bvec);
      else bv = load_b_n4(p, n0 + rb, k0 + kb, bvec);
    }
  };
  auto store = [&](int buf, const float4* av, const float4& bv) {
#pragma unroll
    for (int s = 0; s < NA; ++s) {
      if (a_kcontig(AK)) {
        *reinterpret_cast<float4*>(&As[buf][ra[s] * LD + ka[s]]) = av[s];
      } else {
        As[buf][(ra[s] + 0) * LD + ka[s]] = av[s].x;
        As[buf][(ra[s] + 1) * LD + ka[s]] = av[s].y;
        As[buf][(ra[s] + 2) * LD + ka[s]] = av[s].z;
        As[buf][(ra[s] + 3) * LD + ka[s]] = av[s].w;
      }
    }
    if (bload) {
      if (b_kcontig(BK)) {
        *reinterpret_cast<float4*>(&Bs[buf][rb * LD + kb]) = bv;
      } else {
        Bs[buf][(rb + 0) * LD + kb] = bv.x;
        Bs[buf][(rb + 1) * LD + kb] = bv.y;
        Bs[buf][(rb + 2) * LD + kb] = bv.z;
        Bs[buf][(rb + 3) * LD + kb] = bv.w;
      }
    }
  };

  const int wm = (wave / WAVES_N) * WR, wn = (wave % WAVES_N) * WC;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (c_lo < c_hi) {
    float4 av[NA], bv;
    load(c_lo, av, bv);
    store(0, av, bv);
    __syncthreads();
    for (int ch = c_lo; ch < c_hi; ++ch) {
      const int buf = (ch - c_lo) & 1;
      const bool more = ch + 1 < c_hi;
      if (more) load(ch + 1, av, bv);
      float4 a4[MI], b4[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) a4[i] = *reinterpret_cast<const float4*>(&As[buf][(wm + i * 16 + fr) * LD + 4 * fq]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) b4[j] = *reinterpret_cast<const float4*>(&Bs[buf][(wn + j * 16 + fr) * LD + 4 * fq]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          acc[i][j] = mfma4(a4[i].x, b4[j].x, acc[i][j]);
          acc[i][j] = mfma4(a4[i].y, b4[j].y, acc[i][j]);
          acc[i][j] = mfma4(a4[i].z, b4[j].z, acc[i][j]);
          acc[i][j] = mfma4(a4[i].w, b4[j].w, acc[i][j]);
        }
      if (more) store(buf ^ 1, av, bv);
      __syncthreads();
    }
  }

  // ---- epilogue: acc[i][j][r] = C[m0 + wm + 16i + 4fq + r][n0 + wn + 16j + fr]
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wn + j * 16 + fr;
    const bool nok = n < p.N;
    double s1 = 0.0, s2 = 0.0;
    const float bias = (p.bias && nok) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + 4 * fq + r;
        if (!nok || m >= p.M) continue;
        float v = acc[i][j][r];
        if (p.part) {
          p.part[((size_t)split * p.M + m) * p.N + n] = v;
          continue;
        }
        v += bias;
        if (p.relu) v = fmaxf(v, 0.f);
        long long row = m;
        if (AK == A_DGRAD && ph.on) {   // phase row -> input pixel
          const int hw = ph.Hp * ph.Wp, b = m / hw, rem = m - b * hw, ihp = rem / ph.Wp, iwp = rem - ihp * ph.Wp;
          row = ((long long)b * p.g.H + ihp * p.g.sh + ph.ph_h) * p.g.W + iwp * p.g.sw + ph.ph_w;
        }
        float* dst = p.c + (size_t)row * p.ldc + n;
        if (p.accum) v += *dst;
        *dst = v;
        s1 += v;
        s2 += (double)v * v;
      }
    if (p.colstats && !p.part) {
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (fq == 0 && nok) {
        double* cs = p.colstats + (size_t)((blockIdx.x + blockIdx.y * gridDim.x) % kSlots) * 2 * p.N;
        atomicAdd(cs + n, s1);
        atomicAdd(cs + p.N + n, s2);
      }
    }
  }
}

// split-K: c (= or +=) sum of the partials (+ bias, ReLU, column statistics).  Deterministic: each of the
// 8 thread groups of a block sums splits g, g+8, ... of its 32 elements in order, the groups combine in
// order through LDS (the 4 loads of a group thread in flight together: no per-split round trip).
__global__ __launch_bounds__(256) void g32_reduce_kernel(const float* __restrict__ part, int splits, int M, int N,
                                                         float* c, long long ldc, int accum, const float* bias,
                                                         int relu, double* colstats) {
  __shared__ float red[8][33];
  const long long n = (long long)M * N;
  const int el = threadIdx.x & 31, g = threadIdx.x >> 5;
  const long long e = (long long)blockIdx.x * 32 + el;
  float s = 0.f;
  if (e < n) {
    int z = g;
    for (; z + 24 < splits; z += 32) {
      const float a0 = part[(size_t)z * n + e], a1 = part[(size_t)(z + 8) * n + e];
      const float a2 = part[(size_t)(z + 16) * n + e], a3 = part[(size_t)(z + 24) * n + e];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; z < splits; z += 8) s += part[(size_t)z * n + e];
  }
  red[g][el] = s;
  __syncthreads();
  if (g == 0 && e < n) {
    float t = red[0][el];
#pragma unroll
    for (int q = 1; q < 8; ++q) t += red[q][el];
    const long long m = e / N, col = e - m * N;
    if (bias) t += bias[col];
    if (relu) t = fmaxf(t, 0.f);
    float* d = c + m * ldc + col;
    if (accum) t += *d;
    *d = t;
    if (colstats) {
      double* cs = colstats + (size_t)(blockIdx.x % kSlots) * 2 * N;
      atomicAdd(cs + col, (double)t);
      atomicAdd(cs + N + col, (double)t * t);
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// Elementwise / reduction kernels.  Channel-reduction kernels use a [64 channels] x [4 row groups]
// block walking a range of rows (coalesced for C >= 64; correct for any C).
struct Drop {
  float rate;  // 0 = off
  unsigned long long seed;
  const long long* iter;
  int iter_offset;
  int layer_id;
};
__device__ __forceinline__ float keep(const Drop& d, long long e) {
  return philox_keep(d.rate, d.seed, (d.iter ? *d.iter : 0) + d.iter_offset, d.layer_id, e);
}

constexpr int kRowsPerBlock = 64;

// per-channel f64 sum / sum of squares of x [R][C] into stats [kSlots][2][C]
// Channel-reduction launch layout.  A wave's 64 lanes cover Cw = min(C, 64) channels x rpw = 64 / Cw rows
// (narrow layers — Model B's 6 / 12 / 24 channels — keep every lane busy instead of C of 64), 4 waves per
// block, each thread 16 rows: a block covers 64 * rpw rows of a 64-channel group.  Sums combine in a fixed
// order (lane rows, then waves) before one atomic per channel per block.
struct ChanLayout {
  int Cw, rpw, c, lr, rg, rows;   // channel group width, rows per wave slice, this lane's channel / row
  bool on;
  __device__ ChanLayout(int C) {
    const int lane = threadIdx.x & 63;
    Cw = C < 64 ? C : 64;
    rpw = 64 / Cw;
    lr = lane / Cw;
    c = blockIdx.x * 64 + (lane - lr * Cw);
    rg = threadIdx.x >> 6;
    rows = 64 * rpw;
    on = lr < rpw && c < C;
  }
  __device__ long long row0() const { return (long long)blockIdx.y * rows + rg * rpw + lr; }
  __device__ int step() const { return 4 * rpw; }
};
__host__ inline dim3 chan_grid(long long R, int C) {
  const int Cw = C < 64 ? C : 64, rows = 64 * (64 / Cw);
  return dim3((C + 63) / 64, (unsigned)((R + rows - 1) / rows));
}
// red: [256] per sum; returns the block's sum for this thread's channel on lanes lr == 0 of wave 0
__device__ __forceinline__ double chan_block_sum(const double* red, const ChanLayout& L) {
  double t = 0.0;
  for (int q = 0; q < 4; ++q)
    for (int l = 0; l < L.rpw; ++l) t += red[q * 64 + l * L.Cw + (threadIdx.x & 63)];
  return t;
}

__global__ __launch_bounds__(256) void colstats32_kernel(const float* __restrict__ x, long long R, int C,
                                                         double* stats) {
  __shared__ double red[2][256];
  const ChanLayout L(C);
  double s1 = 0.0, s2 = 0.0;
  if (L.on) {
    const long long r1 = min((long long)(blockIdx.y + 1) * L.rows, R);
    const int st = L.step();
    for (long long row = L.row0(); row < r1; row += 8 * st) {   // 8 rows' loads in flight per round trip
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = row + u * st < r1 ? x[(row + u * st) * C + L.c] : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        s1 += v[u];
        s2 += (double)v[u] * v[u];
      }
    }
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (L.rg == 0 && L.lr == 0 && L.on) {
    double* st = stats + (size_t)(blockIdx.y % kSlots) * 2 * C;
    atomicAdd(st + L.c, chan_block_sum(red[0], L));
    atomicAdd(st + C + L.c, chan_block_sum(red[1], L));
  }
}

struct BnF {
  const float* y;
  float* out;
  const float* res;
  long long R;
  int C, mode;          // 0 identity (ReLU / dropout / add only), 1 batch statistics, 2 moving statistics
  const double* stats;  // [kSlots][2][C]
  float* saved;         // [2][C] mean, rstd (mode 1)
  const float *gamma, *beta;
  float eps;
  float *mmean, *mvar;
  float momentum, bessel;
  double* zero_buf;     // [kSlots][2][C] backward accumulators of this layer (zeroed here)
  int relu;
  Drop drop;
};

constexpr int kMaxC32 = 2048;

__global__ __launch_bounds__(256) void bn_fwd32_kernel(BnF a) {
  __shared__ float sc[kMaxC32], sf[kMaxC32];
  const int C = a.C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float scale = 1.f, shift = 0.f;
    if (a.mode != 0) {
      float mean, var;
      if (a.mode == 1) {
        double s1 = 0.0, s2 = 0.0;
        for (int sl = 0; sl < kSlots; ++sl) {
          s1 += a.stats[(size_t)sl * 2 * C + c];
          s2 += a.stats[(size_t)sl * 2 * C + C + c];
        }
        const double md = s1 / (double)a.R, vd = fmax(s2 / (double)a.R - md * md, 0.0);
        mean = (float)md;
        var = (float)vd;
        const float rstd = (float)(1.0 / sqrt(vd + (double)a.eps));
        if (blockIdx.x == 0) {
          a.saved[c] = mean;
          a.saved[C + c] = rstd;
          if (a.mmean) {
            a.mmean[c] = a.mmean[c] * a.momentum + mean * (1.f - a.momentum);
            a.mvar[c] = a.mvar[c] * a.momentum + var * a.bessel * (1.f - a.momentum);
          }
        }
        const float g = a.gamma ? a.gamma[c] : 1.f;
        scale = g * rstd;
        shift = (a.beta ? a.beta[c] : 0.f) - mean * scale;
      } else {
        mean = a.mmean[c];
        var = a.mvar[c];
        const float rstd = rsqrtf(var + a.eps);
        const float g = a.gamma ? a.gamma[c] : 1.f;
        scale = g * rstd;
        shift = (a.beta ? a.beta[c] : 0.f) - mean * scale;
      }
    }
    if (blockIdx.x == 0 && a.zero_buf)
      for (int sl = 0; sl < kSlots; ++sl) {
        a.zero_buf[(size_t)sl * 2 * C + c] = 0.0;
        a.zero_buf[(size_t)sl * 2 * C + C + c] = 0.0;
      }
    sc[c] = scale;
    sf[c] = shift;
  }
  __syncthreads();
  const long long n = a.R * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    float z = a.y[e] * sc[c] + sf[c];
    if (a.res) z += a.res[e];
    if (a.relu) z = fmaxf(z, 0.f);
    if (a.drop.rate > 0.f) z *= keep(a.drop, e);
    a.out[e] = z;
  }
}

struct BnB {
  const float* dout;
  const float* y;
  const float* res;
  long long R;
  int C, mode;          // 0 identity, 1 batch statistics
  const float* saved;   // [2][C] mean, rstd
  const float *gamma, *beta;
  int relu;
  Drop drop;
  double* dstats;       // [kSlots][2][C] sum dz, sum dz*xhat
  float* dx;
  int dx_accum;
  float* dres;
  int dres_accum;
  float *dgamma, *dbeta;
  double* zero_fwd;     // [kSlots][2][C] forward statistics of this layer (zeroed by the apply pass)
};

// dz = dout * keep * (z > 0), z = bn(y) + res recomputed; xhat = (y - mean) * rstd
__device__ __forceinline__ void bn_dz(const BnB& a, long long e, int c, float& dz, float& xh) {
  float sc = 1.f, sf = 0.f, mu = 0.f, rs = 1.f;
  if (a.mode == 1) {
    mu = a.saved[c];
    rs = a.saved[a.C + c];
    const float g = a.gamma ? a.gamma[c] : 1.f;
    sc = g * rs;
    sf = (a.beta ? a.beta[c] : 0.f) - mu * sc;
  }
  const float v = a.y[e];
  const float z = v * sc + sf + (a.res ? a.res[e] : 0.f);
  float g = a.dout[e];
  if (a.drop.rate > 0.f) g *= keep(a.drop, e);
  if (a.relu && !(z > 0.f)) g = 0.f;
  dz = g;
  xh = (v - mu) * rs;
}

__global__ __launch_bounds__(256) void bn_bwd32_reduce_kernel(BnB a) {
  __shared__ double red[2][256];
  const int C = a.C;
  const ChanLayout L(C);
  double s1 = 0.0, s2 = 0.0;
  if (L.on) {
    const int c = L.c;
    float sc = 1.f, sf = 0.f, mu = 0.f, rs = 1.f;
    if (a.mode == 1) {
      mu = a.saved[c];
      rs = a.saved[C + c];
      sc = (a.gamma ? a.gamma[c] : 1.f) * rs;
      sf = (a.beta ? a.beta[c] : 0.f) - mu * sc;
    }
    const long long r1 = min((long long)(blockIdx.y + 1) * L.rows, a.R);
    const int st = L.step();
    for (long long row = L.row0(); row < r1; row += 8 * st) {   // 8 rows' loads in flight per round trip
      float yv[8], gv[8], rv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long long r = row + u * st;
        const bool ok = r < r1;
        const long long e = r * C + c;
        yv[u] = ok ? a.y[e] : 0.f;
        gv[u] = ok ? a.dout[e] : 0.f;
        rv[u] = (ok && a.res) ? a.res[e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long long r = row + u * st;
        if (r >= r1) continue;
        const float z = yv[u] * sc + sf + rv[u];
        float g = gv[u];
        if (a.drop.rate > 0.f) g *= keep(a.drop, r * C + c);
        if (a.relu && !(z > 0.f)) g = 0.f;
        s1 += g;
        s2 += (double)g * ((yv[u] - mu) * rs);
      }
    }
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (L.rg == 0 && L.lr == 0 && L.on) {
    double* ds = a.dstats + (size_t)(blockIdx.y % kSlots) * 2 * C;
    atomicAdd(ds + L.c, chan_block_sum(red[0], L));
    atomicAdd(ds + C + L.c, chan_block_sum(red[1], L));
  }
}

__global__ __launch_bounds__(256) void bn_bwd32_apply_kernel(BnB a) {
  __shared__ float k1[kMaxC32], k2[kMaxC32];
  const int C = a.C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    if (a.mode == 1) {
      double sdz = 0.0, sdx = 0.0;
      for (int sl = 0; sl < kSlots; ++sl) {
        sdz += a.dstats[(size_t)sl * 2 * C + c];
        sdx += a.dstats[(size_t)sl * 2 * C + C + c];
      }
      k1[c] = (float)(sdz / (double)a.R);
      k2[c] = (float)(sdx / (double)a.R);
      if (blockIdx.x == 0) {
        if (a.dbeta) a.dbeta[c] += (float)sdz;
        if (a.dgamma) a.dgamma[c] += (float)sdx;
      }
    } else {
      k1[c] = k2[c] = 0.f;
    }
    if (blockIdx.x == 0 && a.zero_fwd)
      for (int sl = 0; sl < kSlots; ++sl) {
        a.zero_fwd[(size_t)sl * 2 * C + c] = 0.0;
        a.zero_fwd[(size_t)sl * 2 * C + C + c] = 0.0;
      }
  }
  __syncthreads();
  const long long n = a.R * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    float dz, xh;
    bn_dz(a, e, c, dz, xh);
    float dxv = dz;
    if (a.mode == 1) {   // gamma * rstd * (dz - mean(dz) - xhat * mean(dz * xhat))
      const float g = a.gamma ? a.gamma[c] : 1.f;
      dxv = g * a.saved[C + c] * (dz - k1[c] - xh * k2[c]);
    }
    if (a.dx) a.dx[e] = a.dx_accum ? a.dx[e] + dxv : dxv;
    if (a.dres) a.dres[e] = a.dres_accum ? a.dres[e] + dz : dz;
  }
}

// bias / ReLU backward: dz = dout * (out > 0); dbias[c] += sum_rows dz
__global__ __launch_bounds__(256) void act_bwd32_kernel(const float* __restrict__ dout, const float* __restrict__ out,
                                                        long long R, int C, int relu, float* dz, float* dbias) {
  __shared__ double red[256];
  const ChanLayout L(C);
  double s = 0.0;
  if (L.on) {
    const long long r1 = min((long long)(blockIdx.y + 1) * L.rows, R);
    const int st = L.step();
    for (long long row = L.row0(); row < r1; row += 8 * st) {   // 8 rows' loads in flight per round trip
      float gv[8], ov[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long long r = row + u * st;
        gv[u] = r < r1 ? dout[r * C + L.c] : 0.f;
        ov[u] = (r < r1 && relu) ? out[r * C + L.c] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long long r = row + u * st;
        if (r >= r1) continue;
        const float g = (relu && !(ov[u] > 0.f)) ? 0.f : gv[u];
        if (dz) dz[r * C + L.c] = g;
        s += g;
      }
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (L.rg == 0 && L.lr == 0 && L.on && dbias) atomicAdd(dbias + L.c, (float)chan_block_sum(red, L));
}

// max pooling over KHxKW windows (stride sh/sw, top/left pads pt/pl; padded cells never win);
// idx = argmax window position kh*KW + kw
__global__ __launch_bounds__(256) void maxpool32_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                            unsigned char* idx, Geo g) {
  const int n = g.B * g.Ho * g.Wo * g.C;   // < 2^31 (host check): 32-bit index math
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    int q = e / g.C;
    const int c = e - q * g.C;
    int q2 = q / g.Wo;
    const int ow = q - q2 * g.Wo;
    const int b = q2 / g.Ho, oh = q2 - b * g.Ho;
    float best = -INFINITY;
    int bi = 0;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.sh - g.pt + kh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.sw - g.pl + kw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        const float v = x[(((long long)b * g.H + ih) * g.W + iw) * g.C + c];
        if (v > best) {
          best = v;
          bi = kh * g.KW + kw;
        }
      }
    }
    y[e] = best;
    if (idx) idx[e] = (unsigned char)bi;
  }
}

// gather backward: dx[b, ih, iw, c] (+)= sum of dy over the windows whose argmax is (ih, iw)
__global__ __launch_bounds__(256) void maxpool32_bwd_kernel(const float* __restrict__ dy,
                                                            const unsigned char* __restrict__ idx, float* dx, Geo g,
                                                            int accum) {
  const int n = g.B * g.H * g.W * g.C;   // < 2^31 (host check): 32-bit index math
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    int q = e / g.C;
    const int c = e - q * g.C;
    int q2 = q / g.W;
    const int iw = q - q2 * g.W;
    const int b = q2 / g.H, ih = q2 - b * g.H;
    float s = 0.f;
    const int ohl = max(0, (ih + g.pt - g.KH + g.sh) / g.sh), ohh = min(g.Ho - 1, (ih + g.pt) / g.sh);
    const int owl = max(0, (iw + g.pl - g.KW + g.sw) / g.sw), owh = min(g.Wo - 1, (iw + g.pl) / g.sw);
    for (int oh = ohl; oh <= ohh; ++oh) {
      const int kh = ih + g.pt - oh * g.sh;
      if (kh < 0 || kh >= g.KH) continue;
      for (int ow = owl; ow <= owh; ++ow) {
        const int kw = iw + g.pl - ow * g.sw;
        if (kw < 0 || kw >= g.KW) continue;
        const long long o = (((long long)b * g.Ho + oh) * g.Wo + ow) * g.C + c;
        if (idx[o] == (unsigned char)(kh * g.KW + kw)) s += dy[o];
      }
    }
    dx[e] = accum ? dx[e] + s : s;
  }
}

// Max-pool backward fused with the ReLU / bias backward of the layer that produced the pool's input
// (Conv2D / Dense with activation="relu" feeding only this pool, non-overlapping windows): the window's
// winner gets dy * (y > 0) (y = the pooled value = the winner's ReLU output), every other input cell 0,
// and dbias[c] += that over the pooled cells — the separate act_bwd pass over the 4x larger input tensor
// (read dz, read the activation, write dz) disappears.
// Thread = (one input row (b, ih), one channel quad): it walks the row's windows left to right, so the
// index arithmetic is per row, each pooled (dy, y, argmax) quad is loaded once for the KW cells it covers,
// and the 16-byte stores of consecutive cells of one channel quad stream.  Block: 16 quads x 16 rows.
constexpr int kPoolRowsPerBlock = 16;   // input rows per block (one per row group): ~104 blocks per 64
                                        // channels for Model A wide (and as many same-address bias adds)
__global__ __launch_bounds__(256) void maxpool32_bwd_relu_kernel(const float* __restrict__ dy,
                                                                 const float* __restrict__ y,
                                                                 const unsigned char* __restrict__ idx,
                                                                 float* __restrict__ dx, float* dbias, Geo g, int accum) {
  __shared__ float red[16][65];
  const int cq = threadIdx.x & 15, rg = threadIdx.x >> 4, c = blockIdx.x * 64 + 4 * cq;
  const int nrows = g.B * g.H;   // input rows (b, ih); B*H*W*C < 2^31 (host check)
  float4 s{0.f, 0.f, 0.f, 0.f};
  if (c < g.C) {
    const int r1 = min((int)(blockIdx.y + 1) * kPoolRowsPerBlock, nrows);
    for (int row = blockIdx.y * kPoolRowsPerBlock + rg; row < r1; row += 16) {
      const int b = row / g.H, ih = row - b * g.H;
      const int oh = (ih + g.pt) / g.sh, kh = ih + g.pt - oh * g.sh;
      const bool rok = oh < g.Ho && kh < g.KH;   // the row lies inside a window row
      float* drow = dx + ((long long)row * g.W) * g.C + c;
      const long long prow = (((long long)b * g.Ho + oh) * g.Wo) * g.C + c;
      // windows in groups of 4: their pooled loads in flight together
      for (int ow0 = 0; ow0 * g.sw - g.pl < g.W; ow0 += 4) {
        float4 gv[4], yv[4];
        uchar4 iv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ow = ow0 + u;
          gv[u] = yv[u] = float4{0.f, 0.f, 0.f, 0.f};
          iv[u] = uchar4{255, 255, 255, 255};
          if (rok && ow < g.Wo) {
            const long long o = prow + (long long)ow * g.C;
            iv[u] = *reinterpret_cast<const uchar4*>(idx + o);
            gv[u] = *reinterpret_cast<const float4*>(dy + o);
            yv[u] = *reinterpret_cast<const float4*>(y + o);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int ow = ow0 + u;
          // the cells iw = ow*sw - pl + kw, kw < sw (kw >= KW: between windows, 0)
          for (int kw = 0; kw < g.sw; ++kw) {
            const int iw = ow * g.sw - g.pl + kw;
            if (iw < 0 || iw >= g.W) continue;
            float4 v{0.f, 0.f, 0.f, 0.f};
            if (rok && ow < g.Wo && kw < g.KW) {
              const unsigned char want = (unsigned char)(kh * g.KW + kw);
              v.x = (iv[u].x == want && yv[u].x > 0.f) ? gv[u].x : 0.f;
              v.y = (iv[u].y == want && yv[u].y > 0.f) ? gv[u].y : 0.f;
              v.z = (iv[u].z == want && yv[u].z > 0.f) ? gv[u].z : 0.f;
              v.w = (iv[u].w == want && yv[u].w > 0.f) ? gv[u].w : 0.f;
            }
            float4* d = reinterpret_cast<float4*>(drow + (long long)iw * g.C);
            if (accum) {
              const float4 o = *d;
              *d = float4{o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w};
            } else {
              *d = v;
            }
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
          }
        }
      }
    }
  }
  if (!dbias) return;
  red[rg][4 * cq + 0] = s.x;
  red[rg][4 * cq + 1] = s.y;
  red[rg][4 * cq + 2] = s.z;
  red[rg][4 * cq + 3] = s.w;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int cc = blockIdx.x * 64 + threadIdx.x;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][threadIdx.x];
    if (cc < g.C) atomicAdd(dbias + cc, t);
  }
}

__global__ __launch_bounds__(256) void gap32_kernel(const float* __restrict__ src, float* dst, int B, int HW, int C,
                                                    int backward, int accum) {
  if (!backward) {   // y[b, c] = mean over HW
    const long long n = (long long)B * C;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
      const long long b = e / C, c = e - b * C;
      float s = 0.f;
      for (int i = 0; i < HW; ++i) s += src[(b * HW + i) * C + c];
      dst[e] = s / (float)HW;
    }
  } else {           // dx[b, i, c] (+)= dy[b, c] / HW
    const long long n = (long long)B * HW * C;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
      const long long c = e % C, b = e / ((long long)HW * C);
      const float v = src[b * C + c] / (float)HW;
      dst[e] = accum ? dst[e] + v : v;
    }
  }
}

// zero padding: forward y = pad(x); backward dx (+)= crop(dy)
__global__ __launch_bounds__(256) void pad32_kernel(const float* __restrict__ src, float* dst, Geo g, int backward,
                                                    int accum) {
  const long long n = backward ? (long long)g.B * g.H * g.W * g.C : (long long)g.B * g.Ho * g.Wo * g.C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % g.C);
    long long q = e / g.C;
    if (!backward) {
      const int ow = (int)(q % g.Wo);
      q /= g.Wo;
      const int oh = (int)(q % g.Ho);
      const int b = (int)(q / g.Ho);
      const int ih = oh - g.pt, iw = ow - g.pl;
      dst[e] = ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
                   ? src[(((long long)b * g.H + ih) * g.W + iw) * g.C + c]
                   : 0.f;
    } else {
      const int iw = (int)(q % g.W);
      q /= g.W;
      const int ih = (int)(q % g.H);
      const int b = (int)(q / g.H);
      const float v = src[(((long long)b * g.Ho + ih + g.pt) * g.Wo + iw + g.pl) * g.C + c];
      dst[e] = accum ? dst[e] + v : v;
    }
  }
}

// softmax cross-entropy over C classes, one wave per row: loss / accuracy metrics, f32 dlogits
// (scaled), probabilities (or the logits themselves); the first block advances the step counter
__global__ __launch_bounds__(256) void xent32_kernel(const float* __restrict__ logits, const int* __restrict__ labels,
                                                     int B, int C, float scale, float* dlogits, float* metrics,
                                                     float* probs, int probs_are_logits, long long* iterations) {
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  __shared__ float part[4][2];
  float loss = 0.f, corr = 0.f;
  const bool ok = row < B;
  if (ok) {
    const float* l = logits + (long long)row * C;
    float mx = -INFINITY;
    int am = 0x7fffffff;
    for (int c = lane; c < C; c += 64)
      if (l[c] > mx) {
        mx = l[c];
        am = c;
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
    for (int c = lane; c < C; c += 64) se += expf(l[c] - mx);
    se = wave_sum(se);
    const int y = labels[row];
    const float ly = (y >= 0 && y < C) ? l[y] : mx;
    loss = mx + logf(se) - ly;
    corr = (am == y) ? 1.f : 0.f;
    const float inv = 1.f / se;
    for (int c = lane; c < C; c += 64) {
      const float pr = expf(l[c] - mx) * inv;
      if (dlogits) dlogits[(long long)row * C + c] = (pr - (c == y ? 1.f : 0.f)) * scale;
      if (probs) probs[(long long)row * C + c] = probs_are_logits ? l[c] : pr;
    }
  }
  if (lane == 0) {
    part[threadIdx.x >> 6][0] = ok ? loss : 0.f;
    part[threadIdx.x >> 6][1] = ok ? corr : 0.f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (metrics) {
      atomicAdd(&metrics[0], (part[0][0] + part[1][0]) + (part[2][0] + part[3][0]));
      atomicAdd(&metrics[1], (part[0][1] + part[1][1]) + (part[2][1] + part[3][1]));
      atomicAdd(&metrics[2], (float)min(4, B - (int)blockIdx.x * 4));
    }
    if (iterations && blockIdx.x == 0) *iterations += 1;
  }
}

inline int grid1(long long n) {
  const long long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : g > 4096 ? 4096 : g);
}

inline Geo geo_of(const int* g) {
  return Geo{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12]};
}

// Output tile width.  Default 64 (64x64 tiles): measured on the narrow-output models (Model B x2: Co 12 /
// 24 / 48) the 256x16 / 128x32 tiles were SLOWER (0.587 / 0.555 ms per step vs 0.515, profiles/r5_f32/):
// these GEMMs are bound by the A-operand gathers, which a narrow tile does not reduce (one N tile either
// way) while it cuts the number of blocks 2-4x.  TDE_IGEMM32_TBN = 16 / 32 / 64 forces one width; "area"
// picks the TBN in {64, 32, 16} (TBM = 4096 / TBN) of least padded output area (experiments).
static int tile_n(int M, int N) {
  static const int force = [] {
    const char* e = getenv("TDE_IGEMM32_TBN");
    if (!e) return 64;
    if (!strcmp(e, "area")) return 0;
    return atoi(e);
  }();
  if (force == 16 || force == 32 || force == 64) return force;
  int best = 64;
  long long best_area = -1;
  for (int tbn : {64, 32, 16}) {
    const int tbm = 4096 / tbn;
    const long long area = (long long)((M + tbm - 1) / tbm) * tbm * ((N + tbn - 1) / tbn) * tbn;
    if (best_area < 0 || area < best_area) {
      best_area = area;
      best = tbn;
    }
  }
  return best;
}

template <int AK, int BK>
static void go32(const G32& p, int M, int N, int gz, hipStream_t s) {
  const int tbn = tile_n(M, N), tbm = 4096 / tbn;
  const dim3 grid((M + tbm - 1) / tbm, (N + tbn - 1) / tbn, gz);
  if (tbn == 16) igemm32_kernel<AK, BK, 16><<<grid, 256, 0, s>>>(p);
  else if (tbn == 32) igemm32_kernel<AK, BK, 32><<<grid, 256, 0, s>>>(p);
  else igemm32_kernel<AK, BK, 64><<<grid, 256, 0, s>>>(p);
}

}  // namespace l32
}  // namespace tde

using namespace tde;
using namespace tde::l32;

// C[M,N] (= or +=) A.B on the f32 MFMA (+bias, +ReLU, +column statistics).  geo: 13 ints (B,H,W,C,Ho,Wo,
// Co,KH,KW,sh,sw,pt,pl) for the conv kinds.  splits > 1: K split over grid z into `part` ([splits][M][N],
// bias / ReLU / statistics not allowed) and summed in split order into c.
// phase (nullable): strided conv dgrad with every stride phase in one launch — {nph, then 8 ints per phase
// (ph_h, ph_w, Hp, Wp, kh0, kw0, KHp, KWp)}; M / K are then the largest phase's (grid), splits must be 1.
TDE_API int tde_igemm32(const float* a, long long lda, int akind, const float* b, long long ldb, int bkind, int M,
                        int N, int K, const int* geo, float* c, long long ldc, int accum, const float* bias, int relu,
                        double* colstats, int splits, float* part, const int* phase, hipStream_t stream) {
  if (M < 1 || N < 1 || K < 0 || !a || !b || !c || ldc < N) return -1;
  if ((akind == A_CONV || akind == A_DGRAD || akind == A_WGRAD || bkind == B_DGRADW) && !geo) return -2;
  const int nch = (K + KC - 1) / KC;
  if (splits < 1) splits = 1;
  if (splits > nch) splits = nch > 0 ? nch : 1;
  const int cps = nch > 0 ? (nch + splits - 1) / splits : 1;
  splits = nch > 0 ? (nch + cps - 1) / cps : 1;
  if (splits > 1 && !part) return -3;
  const int nph = phase ? phase[0] : 0;
  if (phase && (akind != A_DGRAD || bkind != B_DGRADW || nph < 1 || nph > 4 || splits > 1)) return -5;
  G32 p{};
  p.a = a;
  p.lda = lda;
  p.b = b;
  p.ldb = ldb;
  p.M = M;
  p.N = N;
  p.K = K;
  p.cps = cps;
  if (geo) p.g = geo_of(geo);
  p.c = c;
  p.ldc = ldc;
  p.accum = accum;
  p.part = splits > 1 ? part : nullptr;
  p.bias = bias;
  p.relu = relu;
  p.colstats = colstats;
  p.nph = nph;
  for (int i = 0; i < nph; ++i)
    for (int j = 0; j < 8; ++j) p.phs[i][j] = phase[1 + 8 * i + j];
  const int gz = nph > 0 ? nph : splits;
  const int key = akind * 8 + bkind;
  switch (key) {
    case A_ROWK * 8 + B_KN: go32<A_ROWK, B_KN>(p, M, N, gz, stream); break;
    case A_ROWK * 8 + B_NK: go32<A_ROWK, B_NK>(p, M, N, gz, stream); break;
    case A_CONV * 8 + B_KN: go32<A_CONV, B_KN>(p, M, N, gz, stream); break;
    case A_DGRAD * 8 + B_DGRADW: go32<A_DGRAD, B_DGRADW>(p, M, N, gz, stream); break;
    case A_COLM * 8 + B_KN: go32<A_COLM, B_KN>(p, M, N, gz, stream); break;
    case A_WGRAD * 8 + B_KN: go32<A_WGRAD, B_KN>(p, M, N, gz, stream); break;
    default: return -4;
  }
  TDE_LAUNCH_CHECK();
  if (splits > 1) {
    const long long nb = ((long long)M * N + 31) / 32;
    g32_reduce_kernel<<<(unsigned)nb, 256, 0, stream>>>(part, splits, M, N, c, ldc, accum, bias, relu, colstats);
    TDE_LAUNCH_CHECK();
  }
  return 0;
}

TDE_API int tde_colstats32(const float* x, long long R, int C, double* stats, hipStream_t stream) {
  if (R < 1 || C < 1) return -1;
  colstats32_kernel<<<chan_grid(R, C), 256, 0, stream>>>(x, R, C, stats);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_bn_fwd32(const float* y, float* out, const float* res, long long R, int C, int mode,
                         const double* stats, float* saved, const float* gamma, const float* beta, float eps,
                         float* mmean, float* mvar, float momentum, float bessel, double* zero_buf, int relu,
                         float rate, unsigned long long seed, const long long* iter, int iter_offset, int layer_id,
                         hipStream_t stream) {
  if (R < 1 || C < 1 || C > kMaxC32) return -1;
  if ((mode == 1 && (!stats || !saved)) || (mode == 2 && (!mmean || !mvar))) return -2;
  BnF a{y, out, res, R, C, mode, stats, saved, gamma, beta, eps, mmean, mvar, momentum, bessel, zero_buf, relu,
        Drop{rate, seed, iter, iter_offset, layer_id}};
  bn_fwd32_kernel<<<grid1(R * C), 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_bn_bwd32(const float* dout, const float* y, const float* res, long long R, int C, int mode,
                         const float* saved, const float* gamma, const float* beta, int relu, float rate,
                         unsigned long long seed, const long long* iter, int iter_offset, int layer_id, double* dstats,
                         float* dx, int dx_accum, float* dres, int dres_accum, float* dgamma, float* dbeta,
                         double* zero_fwd, hipStream_t stream) {
  if (R < 1 || C < 1 || C > kMaxC32) return -1;
  if (mode == 1 && (!saved || !dstats)) return -2;
  BnB a{dout, y, res, R, C, mode, saved, gamma, beta, relu, Drop{rate, seed, iter, iter_offset, layer_id}, dstats,
        dx, dx_accum, dres, dres_accum, dgamma, dbeta, zero_fwd};
  if (mode == 1) {
    bn_bwd32_reduce_kernel<<<chan_grid(R, C), 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
  }
  bn_bwd32_apply_kernel<<<grid1(R * C), 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_act_bwd32(const float* dout, const float* out, long long R, int C, int relu, float* dz, float* dbias,
                          hipStream_t stream) {
  if (R < 1 || C < 1 || (relu && !out)) return -1;
  act_bwd32_kernel<<<chan_grid(R, C), 256, 0, stream>>>(dout, out, R, C, relu, dz, dbias);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_maxpool32(const float* x, float* y, unsigned char* idx, const float* dy, float* dx, int dx_accum,
                          const int* geo, int backward, hipStream_t stream) {
  const Geo g = geo_of(geo);
  if (g.KH * g.KW > 255 || (long long)g.B * g.H * g.W * g.C >= (1ll << 31)) return -1;
  if (!backward) {
    maxpool32_fwd_kernel<<<grid1((long long)g.B * g.Ho * g.Wo * g.C), 256, 0, stream>>>(x, y, idx, g);
  } else {
    if (!idx || !dy || !dx) return -2;
    maxpool32_bwd_kernel<<<grid1((long long)g.B * g.H * g.W * g.C), 256, 0, stream>>>(dy, idx, dx, g, dx_accum);
  }
  TDE_LAUNCH_CHECK();
  return 0;
}

// Fused max-pool + ReLU (+ bias) backward (see maxpool32_bwd_relu_kernel): non-overlapping windows
// (stride >= window), C % 4 == 0, 16-byte aligned tensors.
TDE_API int tde_maxpool32_bwd_relu(const float* dy, const float* y, const unsigned char* idx, float* dx, float* dbias,
                                   int dx_accum, const int* geo, hipStream_t stream) {
  const Geo g = geo_of(geo);
  if (!dy || !y || !idx || !dx || (g.C & 3) || g.sh < g.KH || g.sw < g.KW || g.KH * g.KW > 255 ||
      (((uintptr_t)dy | (uintptr_t)y | (uintptr_t)dx) & 15) || ((uintptr_t)idx & 3))
    return -1;
  const long long npix = (long long)g.B * g.H * g.W;
  if (npix >= (1ll << 31)) return -1;
  const int nrows = g.B * g.H;
  maxpool32_bwd_relu_kernel<<<dim3((g.C + 63) / 64, (unsigned)((nrows + kPoolRowsPerBlock - 1) / kPoolRowsPerBlock)),
                              256, 0, stream>>>(dy, y, idx, dx, dbias, g, dx_accum);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_gap32(const float* src, float* dst, int B, int HW, int C, int backward, int accum, hipStream_t stream) {
  gap32_kernel<<<grid1((long long)B * (backward ? HW : 1) * C), 256, 0, stream>>>(src, dst, B, HW, C, backward, accum);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_pad32(const float* src, float* dst, const int* geo, int backward, int accum, hipStream_t stream) {
  const Geo g = geo_of(geo);
  pad32_kernel<<<grid1((long long)g.B * g.Ho * g.Wo * g.C), 256, 0, stream>>>(src, dst, g, backward, accum);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_xent32(const float* logits, const int* labels, int B, int C, float scale, float* dlogits,
                       float* metrics, float* probs, int probs_are_logits, long long* iterations, hipStream_t stream) {
  if (B < 1 || C < 1) return -1;
  xent32_kernel<<<(B + 3) / 4, 256, 0, stream>>>(logits, labels, B, C, scale, dlogits, metrics, probs,
                                                 probs_are_logits, iterations);
  TDE_LAUNCH_CHECK();
  return 0;
}
