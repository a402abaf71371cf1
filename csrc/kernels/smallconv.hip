// Direct (VALU) convolution for narrow layers — Model B's Conv2D(1->6, 3x3), Conv2D(6->12, 6x6/2),
// Conv2D(12->24, 6x6/2) (mnist_keras_distributed.py:83-98).
//
// With C_out <= 32 a 16x16 MFMA tile is mostly padding and the implicit-GEMM gathers of 1-12 channel
// pixels are scalar, so the matrix-core path is latency-bound on index math.  Here one thread owns
// one pixel and ALL its channels in registers (template CO/CI = channel count rounded up to 8):
//  * fwd:   out[p][0..Co) = sum_k x[p,k] * W[k][0..Co)      (bf16 W, broadcast from LDS as f32)
//           + the per-channel BN statistics of the stored bf16 values (wave shuffles -> LDS -> f64 atomics)
//  * dgrad: dx[p][0..C) = sum over the taps that hit p (stride phase computed, no zero taps)
//           of dy[o][co] * W[kh][kw][0..C)[co]
//  * wgrad: filters small enough for registers (K*Co <= 128, Model B's first conv) reduce over all
//           pixels per thread; wider weight gradients stay on the MFMA implicit GEMM (split-K).
#include "tde_common.h"

namespace tde {

struct SGeo {
  int B, H, W, C, Ho, Wo, Co, KH, KW, sh, sw, pt, pl;
};

constexpr int kSmallLds = 15360;  // f32 weight elements staged in LDS (60 KiB: the block's total stays < 64 KiB)

template <int CO>
__global__ __launch_bounds__(256) void smallconv_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                            const float* __restrict__ bias, int relu,
                                                            bf16* __restrict__ y, double* __restrict__ colstats,
                                                            SGeo g) {
  __shared__ float ws[kSmallLds];
  __shared__ float st[2][CO];
  const int K = g.KH * g.KW * g.C;
  for (int i = threadIdx.x; i < K * CO; i += blockDim.x) {
    const int k = i / CO, co = i - k * CO;
    ws[i] = co < g.Co ? bf2f(w[k * g.Co + co]) : 0.f;
  }
  if (threadIdx.x < 2 * CO) (&st[0][0])[threadIdx.x] = 0.f;
  __syncthreads();
  const int npix = g.B * g.Ho * g.Wo;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  float acc[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) acc[c] = 0.f;
  const bool ok = p < npix;
  if (ok) {
    const int hw = g.Ho * g.Wo;
    const int b = p / hw, r = p - b * hw;
    const int oh = r / g.Wo, ow = r - oh * g.Wo;
    const int y0 = oh * g.sh - g.pt, x0 = ow * g.sw - g.pl;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = y0 + kh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = x0 + kw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        const bf16* xp = x + (((long long)b * g.H + ih) * g.W + iw) * g.C;
        const float* wp = ws + ((kh * g.KW + kw) * g.C) * CO;
        for (int ci = 0; ci < g.C; ++ci) {
          const float xv = bf2f(xp[ci]);
#pragma unroll
          for (int c = 0; c < CO; ++c) acc[c] = fmaf(xv, wp[ci * CO + c], acc[c]);
        }
      }
    }
  }
  float s1[CO], s2[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    float v = acc[c] + ((bias && c < g.Co) ? bias[c] : 0.f);
    const float q = bf2f(f2bf(v));
    s1[c] = ok ? q : 0.f;
    s2[c] = ok ? q * q : 0.f;
    if (relu) v = fmaxf(v, 0.f);
    acc[c] = v;
  }
  if (ok) {
    bf16* yp = y + (long long)p * g.Co;
    if (g.Co == CO && (CO % 8) == 0) {
#pragma unroll
      for (int c = 0; c < CO; c += 8) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[c + j]);
        *reinterpret_cast<bf16x8*>(yp + c) = o;
      }
    } else {
#pragma unroll
      for (int c = 0; c < CO; ++c)
        if (c < g.Co) yp[c] = f2bf(acc[c]);
    }
  }
  if (!colstats) return;
#pragma unroll
  for (int c = 0; c < CO; ++c) {
    const float a = wave_sum(s1[c]), b2 = wave_sum(s2[c]);
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&st[0][c], a);
      atomicAdd(&st[1][c], b2);
    }
  }
  __syncthreads();
  if (threadIdx.x < g.Co) {  // slotted statistics (layers.hip kStatSlots = 8)
    double* cs = colstats + (size_t)(blockIdx.x % 8) * 2 * g.Co;
    atomicAdd(&cs[threadIdx.x], (double)st[0][threadIdx.x]);
    atomicAdd(&cs[g.Co + threadIdx.x], (double)st[1][threadIdx.x]);
  }
}

template <int CI>
__global__ __launch_bounds__(256) void smallconv_dgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ w,
                                                              bf16* __restrict__ dx, int accum, SGeo g) {
  __shared__ float ws[kSmallLds];  // [kh][kw][co][ci] so the inner ci loop reads a broadcast row
  const int taps = g.KH * g.KW;
  for (int i = threadIdx.x; i < taps * g.Co * CI; i += blockDim.x) {
    const int ci = i % CI;
    const int t = i / CI;
    const int co = t % g.Co, tap = t / g.Co;
    ws[i] = ci < g.C ? bf2f(w[(tap * g.C + ci) * g.Co + co]) : 0.f;
  }
  __syncthreads();
  const int npix = g.B * g.H * g.W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int hw = g.H * g.W;
  const int b = p / hw, r = p - b * hw;
  const int ih = r / g.W, iw = r - ih * g.W;
  float acc[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) acc[c] = 0.f;
  const int ty = ih + g.pt, tx = iw + g.pl;
  // taps with (ty - kh) % sh == 0: start at the matching phase, step by the stride
  for (int kh = ty % g.sh; kh < g.KH; kh += g.sh) {
    const int oh = (ty - kh) / g.sh;
    if (ty - kh < 0 || oh >= g.Ho) continue;
    for (int kw = tx % g.sw; kw < g.KW; kw += g.sw) {
      const int ow = (tx - kw) / g.sw;
      if (tx - kw < 0 || ow >= g.Wo) continue;
      const bf16* dp = dy + (((long long)b * g.Ho + oh) * g.Wo + ow) * g.Co;
      const float* wp = ws + (kh * g.KW + kw) * g.Co * CI;
      for (int co = 0; co < g.Co; ++co) {
        const float gv = bf2f(dp[co]);
#pragma unroll
        for (int c = 0; c < CI; ++c) acc[c] = fmaf(gv, wp[co * CI + c], acc[c]);
      }
    }
  }
  bf16* xp = dx + (long long)p * g.C;
#pragma unroll
  for (int c = 0; c < CI; ++c) {
    if (c >= g.C) break;
    float v = acc[c];
    if (accum) v += bf2f(xp[c]);
    xp[c] = f2bf(v);
  }
}


// The same input gradient with the filter's output-channel count and the taps per kernel row reaching a
// pixel (KWP = ceil(KW / sw)) known at compile time (Model B's Conv2D(6 -> 12, 6x6, stride 2)): the KWP
// taps of a kernel row load their CO-channel dy vectors (8-byte loads) together before any FMA, so a
// pixel waits ceil(KH / sh) memory latencies instead of one per tap and channel.
template <int CI, int CO, int KWP>
__global__ __launch_bounds__(256) void smallconv_dgrad_c_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ w,
                                                                bf16* __restrict__ dx, int accum, SGeo g) {
  static_assert(CO % 4 == 0, "8-byte dy vectors");
  __shared__ float ws[kSmallLds];  // [kh][kw][co][ci]
  const int taps = g.KH * g.KW;
  for (int i = threadIdx.x; i < taps * CO * CI; i += blockDim.x) {
    const int ci = i % CI;
    const int t = i / CI;
    const int co = t % CO, tap = t / CO;
    ws[i] = ci < g.C ? bf2f(w[(tap * g.C + ci) * CO + co]) : 0.f;
  }
  __syncthreads();
  const int npix = g.B * g.H * g.W;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const int hw = g.H * g.W;
  const int b = p / hw, r = p - b * hw;
  const int ih = r / g.W, iw = r - ih * g.W;
  float acc[CI];
#pragma unroll
  for (int c = 0; c < CI; ++c) acc[c] = 0.f;
  const int ty = ih + g.pt, tx = iw + g.pl;
  const int kw0 = tx % g.sw;
  for (int kh = ty % g.sh; kh < g.KH; kh += g.sh) {
    const int oh = (ty - kh) / g.sh;
    if (ty - kh < 0 || oh >= g.Ho) continue;
    bf16x4 d[KWP][CO / 4];
    bool ok[KWP];
#pragma unroll
    for (int j = 0; j < KWP; ++j) {
      const int kw = kw0 + j * g.sw;
      const int ow = (tx - kw) / g.sw;
      ok[j] = kw < g.KW && tx - kw >= 0 && ow < g.Wo;
      const bf16* dp = dy + (((long long)b * g.Ho + oh) * g.Wo + (ok[j] ? ow : 0)) * CO;
#pragma unroll
      for (int q = 0; q < CO / 4; ++q) {
        if (ok[j]) {
          d[j][q] = *reinterpret_cast<const bf16x4*>(dp + 4 * q);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) d[j][q][e] = (bf16)0.0f;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < KWP; ++j) {
      if (!ok[j]) continue;
      const float* wp = ws + (kh * g.KW + kw0 + j * g.sw) * CO * CI;
#pragma unroll
      for (int co = 0; co < CO; ++co) {
        const float gv = bf2f(d[j][co / 4][co % 4]);
#pragma unroll
        for (int c = 0; c < CI; ++c) acc[c] = fmaf(gv, wp[co * CI + c], acc[c]);
      }
    }
  }
  bf16* xp = dx + (long long)p * g.C;
#pragma unroll
  for (int c = 0; c < CI; ++c) {
    if (c >= g.C) break;
    float v = acc[c];
    if (accum) v += bf2f(xp[c]);
    xp[c] = f2bf(v);
  }
}

// Weight gradient of a layer whose whole filter fits in registers (K = KH*KW*C <= 128/CO, e.g. Model B's
// Conv2D(1->6, 3x3): K = 9): dW[k][co] += sum_p x_patch(p)[k] * dy[p][co].  The implicit GEMM would run
// M = K rows of a 64-row MFMA tile with scalar C = 1 gathers over a 100k-pixel reduction; here each thread
// keeps all K x CO partial sums in registers over a grid-stride run of pixels, the block folds them with
// DPP row reductions + LDS, and one f32 atomic per (k, co) per block lands in the gradient bucket.
// Filters with more than KMAX taps (LeNet-5 conv1: 5x5x1 -> 6, K = 25) split the taps over blockIdx.y.
template <int CO>
__global__ __launch_bounds__(256) void smallconv_wgrad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                              float* __restrict__ dw, SGeo g) {
  constexpr int KMAX = 128 / CO;
  __shared__ float red[4][KMAX * CO];
  const int kbase = blockIdx.y * KMAX;
  const int K = min(KMAX, g.KH * g.KW * g.C - kbase);   // taps [kbase, kbase + K) of this block
  float acc[KMAX][CO];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[k][c] = 0.f;
  const int npix = g.B * g.Ho * g.Wo;
  const int hw = g.Ho * g.Wo;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += gridDim.x * blockDim.x) {
    const int b = p / hw, r = p - b * hw;
    const int oh = r / g.Wo, ow = r - oh * g.Wo;
    const int y0 = oh * g.sh - g.pt, x0 = ow * g.sw - g.pl;
    float d[CO];
    const bf16* dp = dy + (long long)p * g.Co;
#pragma unroll
    for (int c = 0; c < CO; ++c) d[c] = c < g.Co ? bf2f(dp[c]) : 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {
        const int ci = (kbase + k) % g.C, t = (kbase + k) / g.C;
        const int kw = t % g.KW, kh = t / g.KW;
        const int ih = y0 + kh, iw = x0 + kw;
        float xv = 0.f;
        if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
          xv = bf2f(x[(((long long)b * g.H + ih) * g.W + iw) * g.C + ci]);
#pragma unroll
        for (int c = 0; c < CO; ++c) acc[k][c] = fmaf(xv, d[c], acc[k][c]);
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    if (k < K) {
#pragma unroll
      for (int c = 0; c < CO; ++c) {
        const float v = rows4_sum(row16_sum(acc[k][c]));
        if (lane == 0) red[wave][k * CO + c] = v;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * CO; i += blockDim.x) {
    const int k = i / CO, c = i - k * CO;
    if (c < g.Co) atomicAdd(&dw[(kbase + k) * g.Co + c], (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]));
  }
}

}  // namespace tde

using namespace tde;

static SGeo sgeo(const int* geo) {
  return SGeo{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
}

static int round8(int c) { return (c + 7) / 8 * 8; }

// w: bf16 HWIO weight shadow (what the MFMA path reads too), widened to f32 in LDS
TDE_API int tde_smallconv_fwd(const bf16* x, const bf16* w, const float* bias, int relu, bf16* y, double* colstats,
                              const int* geo, hipStream_t stream) {
  const SGeo g = sgeo(geo);
  const int co = round8(g.Co);
  if (co > 32 || g.KH * g.KW * g.C * co > kSmallLds) return -1;
  if ((long long)g.B * g.H * g.W * g.C >= (1LL << 31) || (long long)g.B * g.Ho * g.Wo * g.Co >= (1LL << 31)) return -4;
  const int npix = g.B * g.Ho * g.Wo;
  const int grid = (npix + 255) / 256;
  switch (co) {
    case 8: smallconv_fwd_kernel<8><<<grid, 256, 0, stream>>>(x, w, bias, relu, y, colstats, g); break;
    case 16: smallconv_fwd_kernel<16><<<grid, 256, 0, stream>>>(x, w, bias, relu, y, colstats, g); break;
    case 24: smallconv_fwd_kernel<24><<<grid, 256, 0, stream>>>(x, w, bias, relu, y, colstats, g); break;
    default: smallconv_fwd_kernel<32><<<grid, 256, 0, stream>>>(x, w, bias, relu, y, colstats, g); break;
  }
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_smallconv_dgrad(const bf16* dy, const bf16* w, bf16* dx, int accum, const int* geo,
                                hipStream_t stream) {
  const SGeo g = sgeo(geo);
  const int ci = round8(g.C);
  if (ci > 32 || g.KH * g.KW * g.Co * ci > kSmallLds) return -1;
  if ((long long)g.B * g.H * g.W * g.C >= (1LL << 31) || (long long)g.B * g.Ho * g.Wo * g.Co >= (1LL << 31)) return -4;
  const int npix = g.B * g.H * g.W;
  const int grid = (npix + 255) / 256;
  static const bool generic_only = getenv("TDE_SMALLCONV_DGRAD_GENERIC") != nullptr;
  if (!generic_only && ci == 8 && g.Co == 12 && (g.KW + g.sw - 1) / g.sw == 3 && ((uintptr_t)dy & 7) == 0) {
    smallconv_dgrad_c_kernel<8, 12, 3><<<grid, 256, 0, stream>>>(dy, w, dx, accum, g);  // Model B conv2
    TDE_LAUNCH_CHECK();
    return 0;
  }
  switch (ci) {
    case 8: smallconv_dgrad_kernel<8><<<grid, 256, 0, stream>>>(dy, w, dx, accum, g); break;
    case 16: smallconv_dgrad_kernel<16><<<grid, 256, 0, stream>>>(dy, w, dx, accum, g); break;
    case 24: smallconv_dgrad_kernel<24><<<grid, 256, 0, stream>>>(dy, w, dx, accum, g); break;
    default: smallconv_dgrad_kernel<32><<<grid, 256, 0, stream>>>(dy, w, dx, accum, g); break;
  }
  TDE_LAUNCH_CHECK();
  return 0;
}

// <= g_sw_max / 128 tap chunks of 128 partial sums (TDE_SMALLCONV_WGRAD_MAX, default 1024 = 8 chunks)
static int g_sw_max = [] {
  const char* e = getenv("TDE_SMALLCONV_WGRAD_MAX");
  return e ? atoi(e) : 1024;
}();
// dw: f32 [KH*KW*C][Co] slice of the gradient bucket (accumulated with atomics)
TDE_API int tde_smallconv_wgrad(const bf16* x, const bf16* dy, float* dw, const int* geo, hipStream_t stream) {
  const SGeo g = sgeo(geo);
  const int co = round8(g.Co);
  const int K = g.KH * g.KW * g.C;
  const int cot = co == 24 ? 32 : co;   // the kernel instance the switch below picks
  if (co > 32 || K * co > g_sw_max) return -1;
  if ((long long)g.B * g.H * g.W * g.C >= (1LL << 31) || (long long)g.B * g.Ho * g.Wo * g.Co >= (1LL << 31)) return -4;
  const int npix = g.B * g.Ho * g.Wo;
  // ~2 pixels per thread, at most g_wg_grid_max blocks (every block ends in K x Co same-address atomics)
  static const int gmax = [] {
    const char* e = getenv("TDE_SMALLCONV_WGRAD_GRID");
    return e ? atoi(e) : 256;
  }();
  static const int ppt = [] {
    const char* e = getenv("TDE_SMALLCONV_WGRAD_PPT");
    return e ? atoi(e) : 2;
  }();
  int grid = (npix + 256 * ppt - 1) / (256 * ppt);
  grid = grid < 1 ? 1 : (grid > gmax ? gmax : grid);
  const int kchunks = (K + 128 / cot - 1) / (128 / cot);
  const dim3 gr(grid, kchunks);
  switch (co) {
    case 8: smallconv_wgrad_kernel<8><<<gr, 256, 0, stream>>>(x, dy, dw, g); break;
    case 16: smallconv_wgrad_kernel<16><<<gr, 256, 0, stream>>>(x, dy, dw, g); break;
    default: smallconv_wgrad_kernel<32><<<gr, 256, 0, stream>>>(x, dy, dw, g); break;
  }
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_smallconv_wgrad_ok(int C, int Co, int KH, int KW) {
  return round8(Co) <= 32 && KH * KW * C * round8(Co) <= g_sw_max;
}

TDE_API int tde_smallconv_ok(int C, int Co, int KH, int KW, int dgrad) {
  if (dgrad) return round8(C) <= 32 && KH * KW * Co * round8(C) <= kSmallLds;
  return round8(Co) <= 32 && KH * KW * C * round8(Co) <= kSmallLds;
}
