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

namespace tde {
namespace l32 {

struct Geo {  // NHWC input [B,H,W,C], HWIO kernel [KH,KW,C,Co], NHWC output [B,Ho,Wo,Co]
  int B, H, W, C, Ho, Wo, Co, KH, KW, sh, sw, pt, pl;
};

enum AKind { A_ROWK = 0, A_CONV = 1, A_DGRAD = 2, A_COLM = 3, A_WGRAD = 4 };
enum BKind { B_NK = 0, B_DGRADW = 1, B_KN = 2 };

constexpr int BM = 64, BN = 64, KC = 16, LD = KC + 4;   // LDS rows of 16 k + 4 pad floats
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
__device__ __forceinline__ RowA row_a(const G32& p, int m) {
  RowA r{m < p.M, 0, 0, 0};
  const int mm = r.ok ? m : 0;
  if (AK == A_ROWK) {
    r.base = (long long)mm * p.lda;
  } else if (AK == A_CONV) {
    const int hw = p.g.Ho * p.g.Wo, b = mm / hw, rem = mm - b * hw, oh = rem / p.g.Wo, ow = rem - oh * p.g.Wo;
    r.y0 = oh * p.g.sh - p.g.pt;
    r.x0 = ow * p.g.sw - p.g.pl;
    r.base = (long long)b * p.g.H * p.g.W;
  } else {  // A_DGRAD: m over input pixels
    const int hw = p.g.H * p.g.W, b = mm / hw, rem = mm - b * hw, ih = rem / p.g.W, iw = rem - ih * p.g.W;
    r.y0 = ih + p.g.pt;
    r.x0 = iw + p.g.pl;
    r.base = (long long)b * p.g.Ho * p.g.Wo;
  }
  return r;
}

template <int AK>
__device__ __forceinline__ long long a_idx(const G32& p, const RowA& r, int k) {
  if (!r.ok || k >= p.K) return -1;
  if (AK == A_ROWK) return r.base + k;
  const int Cd = AK == A_CONV ? p.g.C : p.g.Co;
  const int kc = k / Cd, c = k - kc * Cd, kh = kc / p.g.KW, kw = kc - kh * p.g.KW;
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
__device__ __forceinline__ float4 load_a_k4(const G32& p, const RowA& r, int k, bool vec) {
  if (vec) {   // K % 4 == 0 on this path: a quad is wholly in range or wholly out
    const long long i = a_idx<AK>(p, r, k);
    if (i < 0) return float4{0.f, 0.f, 0.f, 0.f};
    return *reinterpret_cast<const float4*>(p.a + i);
  }
  float4 v;
  const long long i0 = a_idx<AK>(p, r, k), i1 = a_idx<AK>(p, r, k + 1), i2 = a_idx<AK>(p, r, k + 2),
                  i3 = a_idx<AK>(p, r, k + 3);
  v.x = i0 < 0 ? 0.f : p.a[i0];
  v.y = i1 < 0 ? 0.f : p.a[i1];
  v.z = i2 < 0 ? 0.f : p.a[i2];
  v.w = i3 < 0 ? 0.f : p.a[i3];
  return v;
}

// ---- B(k, n) for the K-contiguous kinds (image row = n)
template <int BK>
__device__ __forceinline__ long long b_idx_k(const G32& p, int n, int k) {
  if (n >= p.N || k >= p.K) return -1;
  if (BK == B_NK) return (long long)n * p.ldb + k;
  // B_DGRADW: k = (kh, kw, co), n = ci -> W[kh][kw][ci][co]
  const int kc = k / p.g.Co, co = k - kc * p.g.Co;
  return ((long long)kc * p.g.C + n) * p.g.Co + co;
}

template <int BK>
__device__ __forceinline__ float4 load_b_k4(const G32& p, int n, int k, bool vec) {
  if (vec) {
    const long long i = b_idx_k<BK>(p, n, k);
    if (i < 0) return float4{0.f, 0.f, 0.f, 0.f};
    return *reinterpret_cast<const float4*>(p.b + i);
  }
  float4 v;
  const long long i0 = b_idx_k<BK>(p, n, k), i1 = b_idx_k<BK>(p, n, k + 1), i2 = b_idx_k<BK>(p, n, k + 2),
                  i3 = b_idx_k<BK>(p, n, k + 3);
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

template <int AK, int BK>
__global__ __launch_bounds__(256) void igemm32_kernel(G32 p) {
  __shared__ __attribute__((aligned(16))) float As[2][BM * LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int nch = (p.K + KC - 1) / KC;
  const int c_lo = blockIdx.z * p.cps, c_hi = min(nch, c_lo + p.cps);

  // this thread's load slots: K-contiguous operand -> row tid/4, k quad tid%4;
  // M/N-contiguous operand -> k = tid/16, row quad 4*(tid%16)
  const int ra = a_kcontig(AK) ? tid >> 2 : 4 * (tid & 15);
  const int ka = a_kcontig(AK) ? 4 * (tid & 3) : tid >> 4;
  const int rb = b_kcontig(BK) ? tid >> 2 : 4 * (tid & 15);
  const int kb = b_kcontig(BK) ? 4 * (tid & 3) : tid >> 4;
  RowA rowa{};
  ColA cola{};
  if (a_kcontig(AK)) {
    rowa = row_a<AK>(p, m0 + ra);
  } else if (AK == A_WGRAD) {
    const int m = min(m0 + ra, p.M - 1), kc = m / p.g.C;
    cola = ColA{kc / p.g.KW, kc - (kc / p.g.KW) * p.g.KW, m - kc * p.g.C};
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

  auto load = [&](int ch, float4& av, float4& bv) {
    const int k0 = ch * KC;
    if (a_kcontig(AK)) av = load_a_k4<AK>(p, rowa, k0 + ka, avec);
    else av = load_a_m4<AK>(p, m0 + ra, cola, k0 + ka, avec);
    if (b_kcontig(BK)) bv = load_b_k4<BK>(p, n0 + rb, k0 + kb, bvec);
    else bv = load_b_n4(p, n0 + rb, k0 + kb, bvec);
  };
  auto store = [&](int buf, const float4& av, const float4& bv) {
    if (a_kcontig(AK)) {
      *reinterpret_cast<float4*>(&As[buf][ra * LD + ka]) = av;
    } else {
      As[buf][(ra + 0) * LD + ka] = av.x;
      As[buf][(ra + 1) * LD + ka] = av.y;
      As[buf][(ra + 2) * LD + ka] = av.z;
      As[buf][(ra + 3) * LD + ka] = av.w;
    }
    if (b_kcontig(BK)) {
      *reinterpret_cast<float4*>(&Bs[buf][rb * LD + kb]) = bv;
    } else {
      Bs[buf][(rb + 0) * LD + kb] = bv.x;
      Bs[buf][(rb + 1) * LD + kb] = bv.y;
      Bs[buf][(rb + 2) * LD + kb] = bv.z;
      Bs[buf][(rb + 3) * LD + kb] = bv.w;
    }
  };

  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (c_lo < c_hi) {
    float4 av, bv;
    load(c_lo, av, bv);
    store(0, av, bv);
    __syncthreads();
    for (int ch = c_lo; ch < c_hi; ++ch) {
      const int buf = (ch - c_lo) & 1;
      const bool more = ch + 1 < c_hi;
      if (more) load(ch + 1, av, bv);
      float4 a4[2], b4[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a4[i] = *reinterpret_cast<const float4*>(&As[buf][(wm + i * 16 + fr) * LD + 4 * fq]);
#pragma unroll
      for (int j = 0; j < 2; ++j) b4[j] = *reinterpret_cast<const float4*>(&Bs[buf][(wn + j * 16 + fr) * LD + 4 * fq]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
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
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + j * 16 + fr;
    const bool nok = n < p.N;
    double s1 = 0.0, s2 = 0.0;
    const float bias = (p.bias && nok) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + 4 * fq + r;
        if (!nok || m >= p.M) continue;
        float v = acc[i][j][r];
        if (p.part) {
          p.part[((size_t)blockIdx.z * p.M + m) * p.N + n] = v;
          continue;
        }
        v += bias;
        if (p.relu) v = fmaxf(v, 0.f);
        float* dst = p.c + (size_t)m * p.ldc + n;
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

// split-K: c (= or +=) sum of the partials in split order (deterministic)
__global__ __launch_bounds__(256) void g32_reduce_kernel(const float* __restrict__ part, int splits, int M, int N,
                                                         float* c, long long ldc, int accum) {
  const long long n = (long long)M * N;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += part[(size_t)z * n + e];
    const long long m = e / N, col = e - m * N;
    float* d = c + m * ldc + col;
    *d = accum ? *d + s : s;
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
__global__ __launch_bounds__(256) void colstats32_kernel(const float* __restrict__ x, long long R, int C,
                                                         double* stats) {
  __shared__ double red[2][4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6, c = blockIdx.x * 64 + lane;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const long long r1 = min((long long)(blockIdx.y + 1) * kRowsPerBlock, R);
    for (long long row = (long long)blockIdx.y * kRowsPerBlock + rg; row < r1; row += 4) {
      const double v = x[row * C + c];
      s1 += v;
      s2 += v * v;
    }
  }
  red[0][rg][lane] = s1;
  red[1][rg][lane] = s2;
  __syncthreads();
  if (rg == 0 && c < C) {
    double* st = stats + (size_t)(blockIdx.y % kSlots) * 2 * C;
    atomicAdd(st + c, (red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]));
    atomicAdd(st + C + c, (red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]));
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
  __shared__ double red[2][4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6, c = blockIdx.x * 64 + lane, C = a.C;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const long long r1 = min((long long)(blockIdx.y + 1) * kRowsPerBlock, a.R);
    for (long long row = (long long)blockIdx.y * kRowsPerBlock + rg; row < r1; row += 4) {
      float dz, xh;
      bn_dz(a, row * C + c, c, dz, xh);
      s1 += dz;
      s2 += (double)dz * xh;
    }
  }
  red[0][rg][lane] = s1;
  red[1][rg][lane] = s2;
  __syncthreads();
  if (rg == 0 && c < C) {
    double* ds = a.dstats + (size_t)(blockIdx.y % kSlots) * 2 * C;
    atomicAdd(ds + c, (red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]));
    atomicAdd(ds + C + c, (red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]));
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
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6, c = blockIdx.x * 64 + lane;
  double s = 0.0;
  if (c < C) {
    const long long r1 = min((long long)(blockIdx.y + 1) * kRowsPerBlock, R);
    for (long long row = (long long)blockIdx.y * kRowsPerBlock + rg; row < r1; row += 4) {
      const long long e = row * C + c;
      float g = dout[e];
      if (relu && !(out[e] > 0.f)) g = 0.f;
      if (dz) dz[e] = g;
      s += g;
    }
  }
  red[rg][lane] = s;
  __syncthreads();
  if (rg == 0 && c < C && dbias) atomicAdd(dbias + c, (float)((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])));
}

// max pooling over KHxKW windows (stride sh/sw, top/left pads pt/pl; padded cells never win);
// idx = argmax window position kh*KW + kw
__global__ __launch_bounds__(256) void maxpool32_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                            unsigned char* idx, Geo g) {
  const long long n = (long long)g.B * g.Ho * g.Wo * g.C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % g.C);
    long long q = e / g.C;
    const int ow = (int)(q % g.Wo);
    q /= g.Wo;
    const int oh = (int)(q % g.Ho);
    const int b = (int)(q / g.Ho);
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
  const long long n = (long long)g.B * g.H * g.W * g.C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % g.C);
    long long q = e / g.C;
    const int iw = (int)(q % g.W);
    q /= g.W;
    const int ih = (int)(q % g.H);
    const int b = (int)(q / g.H);
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

template <int AK, int BK>
static void go32(const G32& p, dim3 grid, hipStream_t s) {
  igemm32_kernel<AK, BK><<<grid, 256, 0, s>>>(p);
}

}  // namespace l32
}  // namespace tde

using namespace tde;
using namespace tde::l32;

// C[M,N] (= or +=) A.B on the f32 MFMA (+bias, +ReLU, +column statistics).  geo: 13 ints (B,H,W,C,Ho,Wo,
// Co,KH,KW,sh,sw,pt,pl) for the conv kinds.  splits > 1: K split over grid z into `part` ([splits][M][N],
// bias / ReLU / statistics not allowed) and summed in split order into c.
TDE_API int tde_igemm32(const float* a, long long lda, int akind, const float* b, long long ldb, int bkind, int M,
                        int N, int K, const int* geo, float* c, long long ldc, int accum, const float* bias, int relu,
                        double* colstats, int splits, float* part, hipStream_t stream) {
  if (M < 1 || N < 1 || K < 1 || !a || !b || !c || ldc < N) return -1;
  if ((akind == A_CONV || akind == A_DGRAD || akind == A_WGRAD || bkind == B_DGRADW) && !geo) return -2;
  const int nch = (K + KC - 1) / KC;
  if (splits < 1) splits = 1;
  if (splits > nch) splits = nch;
  const int cps = (nch + splits - 1) / splits;
  splits = (nch + cps - 1) / cps;
  if (splits > 1 && (!part || bias || relu || colstats)) return -3;
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
  const dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
  const int key = akind * 8 + bkind;
  switch (key) {
    case A_ROWK * 8 + B_KN: go32<A_ROWK, B_KN>(p, grid, stream); break;
    case A_ROWK * 8 + B_NK: go32<A_ROWK, B_NK>(p, grid, stream); break;
    case A_CONV * 8 + B_KN: go32<A_CONV, B_KN>(p, grid, stream); break;
    case A_DGRAD * 8 + B_DGRADW: go32<A_DGRAD, B_DGRADW>(p, grid, stream); break;
    case A_COLM * 8 + B_KN: go32<A_COLM, B_KN>(p, grid, stream); break;
    case A_WGRAD * 8 + B_KN: go32<A_WGRAD, B_KN>(p, grid, stream); break;
    default: return -4;
  }
  TDE_LAUNCH_CHECK();
  if (splits > 1) {
    g32_reduce_kernel<<<grid1((long long)M * N), 256, 0, stream>>>(part, splits, M, N, c, ldc, accum);
    TDE_LAUNCH_CHECK();
  }
  return 0;
}

TDE_API int tde_colstats32(const float* x, long long R, int C, double* stats, hipStream_t stream) {
  if (R < 1 || C < 1) return -1;
  colstats32_kernel<<<dim3((C + 63) / 64, (unsigned)((R + kRowsPerBlock - 1) / kRowsPerBlock)), 256, 0, stream>>>(
      x, R, C, stats);
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
    bn_bwd32_reduce_kernel<<<dim3((C + 63) / 64, (unsigned)((R + kRowsPerBlock - 1) / kRowsPerBlock)), 256, 0,
                             stream>>>(a);
    TDE_LAUNCH_CHECK();
  }
  bn_bwd32_apply_kernel<<<grid1(R * C), 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_act_bwd32(const float* dout, const float* out, long long R, int C, int relu, float* dz, float* dbias,
                          hipStream_t stream) {
  if (R < 1 || C < 1 || (relu && !out)) return -1;
  act_bwd32_kernel<<<dim3((C + 63) / 64, (unsigned)((R + kRowsPerBlock - 1) / kRowsPerBlock)), 256, 0, stream>>>(
      dout, out, R, C, relu, dz, dbias);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_maxpool32(const float* x, float* y, unsigned char* idx, const float* dy, float* dx, int dx_accum,
                          const int* geo, int backward, hipStream_t stream) {
  const Geo g = geo_of(geo);
  if (g.KH * g.KW > 255) return -1;
  if (!backward) {
    maxpool32_fwd_kernel<<<grid1((long long)g.B * g.Ho * g.Wo * g.C), 256, 0, stream>>>(x, y, idx, g);
  } else {
    if (!idx || !dy || !dx) return -2;
    maxpool32_bwd_kernel<<<grid1((long long)g.B * g.H * g.W * g.C), 256, 0, stream>>>(dy, idx, dx, g, dx_accum);
  }
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
