// Layer-wise gfx950 kernel library: every Conv2D / Dense / BatchNormalization /
// Activation / Dropout / MaxPooling2D / GlobalAveragePooling2D / ZeroPadding2D /
// Add layer of a Keras model (Model B of mnist_keras_distributed.py:79-109 ==
// tf2_mnist_distributed.py:105-135, the ResNet-18 stress config, and any other
// Sequential / functional model built from those layers).
//
// * igemm: ONE implicit-GEMM MFMA kernel family for Conv2D fwd / bwd-data /
//   bwd-filter and Dense fwd / bwd-data / bwd-weight.  C[M,N] = sum_k A(m,k) B(k,n)
//   where A and B are *gathered* (im2col never materialised) straight from the
//   NHWC bf16 activations / HWIO bf16 weight shadows into LDS:
//       kind            A(m,k)                           B(k,n)
//       dense fwd/dgrad X[m*lda+k]            (A_ROWK)   Wt[n*ldb+k]         (B_NK)
//       conv fwd        X[b,oh*s-p+kh,..,ci]  (A_CONV)   Wt[co][kh,kw,ci]    (B_NK)
//       conv dgrad      dY[b,(ih+p-kh)/s,..]  (A_DGRAD)  W[kh,kw,n,co]       (B_DGRADW)
//       dense wgrad     X[k*lda+m]            (A_COLM)   dY[k*ldb+n]         (B_KN)
//       conv wgrad      X[b,oh*s-p+kh,..,ci]  (A_WGRAD)  dY[p*Co+n]          (B_KN)
//   Tiles are 64x64x32 (4 waves of 32x32 = 2x2 MFMA 16x16x32 bf16), operands are
//   double-buffered through LDS (global loads of tile k+1 in flight while tile k
//   feeds the matrix cores, one barrier per k-step).  K-contiguous operands move
//   as 16-byte vectors; M/N-contiguous ones (weight grads) are loaded as 16-byte
//   vectors along M/N and transposed on the LDS write.  The epilogue fuses bias,
//   ReLU, bf16 store (or +=, for tensors with several consumers), f32 store /
//   split-K atomics (weight grads), and the per-channel sum / sum-of-squares that
//   the following BatchNormalization needs (DPP/shuffle column reduction + one
//   atomic per column per wave) — the BN statistics never re-read the activation.
// * bn_fwd: batch-stat (or moving-stat) affine + residual add + ReLU + Philox
//   dropout in one pass; block 0 also updates the moving statistics (Keras
//   momentum semantics, Bessel-corrected variance for 4-D input) and zeroes the
//   backward accumulators of the same layer.  Dropout masks are never stored:
//   the backward regenerates them from the counter-based Philox stream.
// * bn_bwd_reduce / bn_bwd_apply: BN + ReLU + dropout backward (per-channel
//   reductions in LDS, then the dx / residual-grad / dgamma / dbeta pass).
// * maxpool (argmax bytes, gather backward), global average pool, zero-padding,
//   bias/ReLU backward with the bias-grad column sum, and a general softmax
//   cross-entropy (+accuracy, +dlogits, +probabilities) for any class count.
#include "tde_common.h"
#include "tde_philox.h"

#include <initializer_list>

namespace tde {

struct Geo {  // NHWC input [B,H,W,C], HWIO kernel [KH,KW,C,Co], NHWC output [B,Ho,Wo,Co]
  int B, H, W, C, Ho, Wo, Co, KH, KW, sh, sw, pt, pl;
};

enum AKind { A_ROWK = 0, A_CONV = 1, A_DGRAD = 2, A_COLM = 3, A_WGRAD = 4 };
enum BKind { B_NK = 0, B_DGRADW = 1, B_KN = 2 };

// The backward sums of the BatchNormalization whose OUTPUT gradient an input-gradient GEMM produces (it is the
// last writer of that gradient): sum g and sum g * xhat per channel with g = the stored gradient masked by the
// BN's ReLU (z = y * gamma * rstd + beta - mean * gamma * rstd + res > 0), xhat = (y - mean) * rstd — what
// bn_bwd_reduce_*_kernel computes in its own pass, taken in the GEMM's epilogue instead (that pass then vanishes;
// the BN backward runs its apply pass only).  dstats: [kStatSlots][2][C] f32, zeroed by the BN forward.
struct BnSum {
  const bf16* y;       // [rows][C] the BN input (this GEMM's output layout)
  const bf16* res;     // [rows][C] the BN's residual input, or null
  const float* saved;  // [2][C] batch mean, rstd
  const float* gamma;  // nullable
  const float* beta;   // nullable
  int relu;
  float* dstats;       // null: off
};

struct IGemmArgs {
  const bf16* a;
  long long lda;
  const bf16* b;
  long long ldb;
  int M, N, K;
  int ktiles_per_split;
  Geo g;
  int avec, bvec;
  float* cf;
  long long ldc;
  int cf_mode;  // 0 none, 1 store, 2 atomic add
  float alpha;
  bf16* cb;
  long long ldcb;
  int cb_accum;
  const float* bias;
  int relu;
  double* colstats;  // [2][N] sum / sum of squares of the STORED (bf16-rounded) values
  // strided-conv dgrad, one stride phase (ih % sh, iw % sw) per launch: rows are that phase's
  // pixels and K runs over only the taps kh = kh0 + i*sh, kw = kw0 + j*sw that reach them
  int ph_on, ph_h, ph_w, Hp, Wp, kh0, kw0, KHp, KWp;
  int xcd;  // 1: XCD-aware tile order (consecutive tiles share an XCD's L2)
  int a_bytes, b_bytes;  // operand sizes for the buffer-resource range checks of the LDS-DMA path (< 2^31)
  // LDS-DMA weight gradient: pixels in row-padded order k = (oh * B + b) * 2^wp_log + ow (K = Ho*B*2^wp_log;
  // the padding columns ow >= Wo read zeros); a_shift = (pt*W + pl)*C elements below X for the A resource
  int wp_log, a_shift;
  // A_CONV LDS-DMA with whole-kernel-row k-tiles (C * KW == KB, no padding, valid geometry): the packed
  // stem (tde_stem_pack) runs through this
  int rowtile;
  // strided dgrad, all stride phases in ONE launch (grid z = phase; splits must be 1): per phase
  // {ph_h, ph_w, Hp, Wp, kh0, kw0, KHp, KWp}; M and K follow per phase, grid x covers the largest M
  int nph;
  int phs[4][8];
  BnSum bs;   // input gradients only: the consumer BN's backward sums in the epilogue (bs.dstats null = off)
};

constexpr int TK = 32;  // MFMA k-slice
// BN statistics accumulate into kStatSlots interleaved copies ([slot][2][C] f64, slot = block % slots)
// so thousands of producer workgroups do not serialise on the same 2*C addresses; readers sum slots.
constexpr int kStatSlots = 8;

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)0.0f;
  return r;
}

// ---- LDS images.
// K-contiguous operands: [rows][KB + 8] (8-element pad: the 16-byte fragment reads are conflict-free).
// Row-contiguous operands (weight grads: channels are contiguous, the reduction runs over pixels):
// [k = 32][128] image with 256-byte rows and an XOR chunk swizzle, read back transposed with
// ds_read_b64_tr_b16 (CDNA4 hardware transpose): conflict-free for the 16x16x32 operand.
// RW = 128: 256-byte rows, XOR of the 16-byte chunk index with ((row&3)<<2)|((row>>2)&3).
// RW = 64: 128-byte rows (2 rows per 64 banks); the chunk pair is XORed with (row bit 1, row bit 3)
// so the 8 rows one 32-lane half of a transposed read touches land in 8 distinct bank groups.
template <int RW>
__device__ __forceinline__ int swzc(int row) {  // XOR applied to the 16-byte chunk index of image row `row`
  if (RW == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
}
template <int RW>
__device__ __forceinline__ int swz(int row, int ch) {
  return 2 * RW * row + 16 * (ch ^ swzc<RW>(row));
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// 16x16x32 operand fragment (rows mb..mb+15 of the image's 128 columns, k 0..31) via two
// transposed 4x16 reads per 16-lane group.
template <int RW>
__device__ __forceinline__ bf16x8 tr_frag(const bf16* img, int mb, int lane, int k0) {
  const int g = k0 / 8 + (lane >> 4), i = lane & 15, q = i >> 2, pp = i & 3;
  const int ch = (mb >> 3) + (pp >> 1);
  const char* base = reinterpret_cast<const char*>(img);
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + swz<RW>(8 * g + q, ch) + 8 * (pp & 1)));
  const v4i16 hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + swz<RW>(8 * g + 4 + q, ch) + 8 * (pp & 1)));
  // concatenate as 16-bit integers, then reinterpret the whole vector (element-wise bf16 casts of
  // the intrinsic's result mis-assemble the fragment)
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// 32x32x16 operand fragment (rows mb..mb+31, k k0..k0+15; k0 % 16 == 0): every 16-lane group runs the same
// two transposed 4x16 reads as tr_frag, at image rows of k group k0/8 + (lane>>5) and columns
// mb + 16*((lane>>4)&1) .. +15, so lane l receives A[mb + (l&31)][k0 + 8*(l>>5) .. +7].
template <int RW>
__device__ __forceinline__ bf16x8 tr_frag32(const bf16* img, int mb, int lane, int k0) {
  const int g = k0 / 8 + (lane >> 5), i = lane & 15, q = i >> 2, pp = i & 3;
  const int ch = ((mb + 16 * ((lane >> 4) & 1)) >> 3) + (pp >> 1);
  const char* base = reinterpret_cast<const char*>(img);
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + swz<RW>(8 * g + q, ch) + 8 * (pp & 1)));
  const v4i16 hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + swz<RW>(8 * g + 4 + q, ch) + 8 * (pp & 1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

// ---- A(m, k), K-vector kinds: a thread's rows are fixed for the whole K loop; its k offset
// advances by 32 per step, decomposed incrementally into (kh, kw, c) (no divisions in the loop).
struct ARow {
  bool ok;
  long long base;  // ROWK: m*lda ; CONV/DGRAD: pixel index of (b, y0, x0) in the gathered tensor
  int y0, x0;      // CONV: oh*sh-pt, ow*sw-pl ; DGRAD: ih+pt, iw+pl
};

struct KPos {  // decomposition of k = (kh*KW + kw)*Cd + c
  int kh, kw, c;
};

__device__ __forceinline__ void kpos_advance(KPos& s, int d, int Cd, int KW) {
  s.c += d;
  while (s.c >= Cd) {
    s.c -= Cd;
    if (++s.kw == KW) {
      s.kw = 0;
      ++s.kh;
    }
  }
}

__device__ __forceinline__ KPos kpos_of(int k, int Cd, int KW) {
  const int kc = k / Cd;
  const int kh = kc / KW;
  return KPos{kh, kc - kh * KW, k - kc * Cd};
}

template <int AK>
__device__ __forceinline__ ARow a_row(const IGemmArgs& p, int m) {
  ARow r;
  r.ok = m < p.M;
  const int mm = r.ok ? m : 0;
  r.base = 0;
  r.y0 = r.x0 = 0;
  if (AK == A_ROWK) {
    r.base = (long long)mm * p.lda;
  } else if (AK == A_CONV) {
    const int hw = p.g.Ho * p.g.Wo;
    const int b = mm / hw, rem = mm - b * hw;
    const int oh = rem / p.g.Wo, ow = rem - oh * p.g.Wo;
    r.y0 = oh * p.g.sh - p.g.pt;
    r.x0 = ow * p.g.sw - p.g.pl;
    r.base = (long long)b * p.g.H * p.g.W;
  } else if (!p.ph_on) {  // A_DGRAD: m over input pixels, gathers dY
    const int hw = p.g.H * p.g.W;
    const int b = mm / hw, rem = mm - b * hw;
    const int ih = rem / p.g.W, iw = rem - ih * p.g.W;
    r.y0 = ih + p.g.pt;
    r.x0 = iw + p.g.pl;
    r.base = (long long)b * p.g.Ho * p.g.Wo;
  } else {  // A_DGRAD, one stride phase: y0/x0 = the output row/col hit by tap (kh0, kw0)
    const int hw = p.Hp * p.Wp;
    const int b = mm / hw, rem = mm - b * hw;
    const int ihp = rem / p.Wp, iwp = rem - ihp * p.Wp;
    r.y0 = (ihp * p.g.sh + p.ph_h + p.g.pt - p.kh0) / p.g.sh;
    r.x0 = (iwp * p.g.sw + p.ph_w + p.g.pl - p.kw0) / p.g.sw;
    r.base = (long long)b * p.g.Ho * p.g.Wo;
  }
  return r;
}

// element index of A(m, k) at decomposition s (or -1 = zero); k < K checked by the caller
template <int AK>
__device__ __forceinline__ long long a_idx(const IGemmArgs& p, const ARow& r, const KPos& s, int k) {
  if (AK == A_ROWK) return r.base + k;
  if (AK == A_CONV) {
    const int ih = r.y0 + s.kh, iw = r.x0 + s.kw;
    if ((unsigned)ih >= (unsigned)p.g.H || (unsigned)iw >= (unsigned)p.g.W) return -1;
    return (r.base + (long long)ih * p.g.W + iw) * p.g.C + s.c;
  }
  if (p.ph_on) {  // phased: tap (kh0 + kh'*sh) reaches output row y0 - kh' exactly
    const int oh = r.y0 - s.kh, ow = r.x0 - s.kw;
    if ((unsigned)oh >= (unsigned)p.g.Ho || (unsigned)ow >= (unsigned)p.g.Wo) return -1;
    return (r.base + (long long)oh * p.g.Wo + ow) * p.g.Co + s.c;
  }
  // A_DGRAD: oh = (ih + pt - kh) / sh must be exact and in range
  int oh = r.y0 - s.kh, ow = r.x0 - s.kw;
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
  return (r.base + (long long)oh * p.g.Wo + ow) * p.g.Co + s.c;
}

template <int AK, int VEC>
__device__ __forceinline__ bf16x8 load_a_k8(const IGemmArgs& p, const ARow& r, const KPos& s, int k, int Cd) {
  if (!r.ok) return zero8();
  if (VEC || p.avec) {  // 8 consecutive k share (kh, kw): one 16-byte load
    if (k >= p.K) return zero8();
    const long long i = a_idx<AK>(p, r, s, k);
    if (i < 0) return zero8();
    return *reinterpret_cast<const bf16x8*>(p.a + i);
  }
  bf16x8 v;
  KPos t = s;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const long long i = (k + j < p.K) ? a_idx<AK>(p, r, t, k + j) : -1;
    v[j] = i < 0 ? (bf16)0.0f : p.a[i];
    if (AK != A_ROWK) kpos_advance(t, 1, Cd, (AK == A_DGRAD && p.ph_on) ? p.KWp : p.g.KW);
  }
  return v;
}

// ---- B(k, n), K-vector kinds (image row = n)
template <int BK_>
__device__ __forceinline__ long long b_idx_k(const IGemmArgs& p, int n, const KPos& s, int k) {
  if (BK_ == B_NK) return (long long)n * p.ldb + k;
  // B_DGRADW: k = (kh,kw,co), n = ci  ->  W[kh][kw][ci][co]
  if (p.ph_on)
    return ((long long)((p.kh0 + s.kh * p.g.sh) * p.g.KW + p.kw0 + s.kw * p.g.sw) * p.g.C + n) * p.g.Co + s.c;
  return ((long long)(s.kh * p.g.KW + s.kw) * p.g.C + n) * p.g.Co + s.c;
}

template <int BK_, int VEC>
__device__ __forceinline__ bf16x8 load_b_k8(const IGemmArgs& p, int n, const KPos& s, int k) {
  if (n >= p.N) return zero8();
  if (VEC || p.bvec) {
    if (k >= p.K) return zero8();
    return *reinterpret_cast<const bf16x8*>(p.b + b_idx_k<BK_>(p, n, s, k));
  }
  bf16x8 v;
  KPos t = s;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = (k + j < p.K) ? p.b[b_idx_k<BK_>(p, n, t, k + j)] : (bf16)0.0f;
    if (BK_ == B_DGRADW) kpos_advance(t, 1, p.g.Co, p.ph_on ? p.KWp : p.g.KW);
  }
  return v;
}

// ---- row-vector kinds: 8 consecutive rows m..m+7 at one k
struct WRow {  // A_WGRAD: the decomposition of the slot's first row m = (kh, kw, ci)
  int kh, kw, ci;
  bool ok;
};

struct PixPos {  // pixel k = (b, oh, ow), advanced incrementally
  int b, oh, ow;
};

__device__ __forceinline__ void pix_advance(PixPos& q, int d, int Ho, int Wo) {
  q.ow += d;
  while (q.ow >= Wo) {
    q.ow -= Wo;
    if (++q.oh == Ho) {
      q.oh = 0;
      ++q.b;
    }
  }
}

__device__ __forceinline__ long long wgrad_idx(const IGemmArgs& p, int kh, int kw, int ci, const PixPos& q) {
  const int ih = q.oh * p.g.sh - p.g.pt + kh, iw = q.ow * p.g.sw - p.g.pl + kw;
  if ((unsigned)ih >= (unsigned)p.g.H || (unsigned)iw >= (unsigned)p.g.W) return -1;
  return (((long long)q.b * p.g.H + ih) * p.g.W + iw) * p.g.C + ci;
}

template <int AK, int VEC>
__device__ __forceinline__ bf16x8 load_a_m8(const IGemmArgs& p, int m, const WRow& w, const PixPos& q, int k) {
  if (k >= p.K || m >= p.M) return zero8();
  if (AK == A_COLM) {
    const long long i = (long long)k * p.lda + m;
    if (VEC || p.avec) return *reinterpret_cast<const bf16x8*>(p.a + i);
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (m + j < p.M) ? p.a[i + j] : (bf16)0.0f;
    return v;
  }
  if (VEC || p.avec) {  // C % 8 == 0: the 8 rows are ci..ci+7 of one (kh, kw)
    const long long i = wgrad_idx(p, w.kh, w.kw, w.ci, q);
    if (i < 0) return zero8();
    return *reinterpret_cast<const bf16x8*>(p.a + i);
  }
  bf16x8 v;
  int kh = w.kh, kw = w.kw, ci = w.ci;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    long long i = -1;
    if (m + j < p.M) i = wgrad_idx(p, kh, kw, ci, q);
    v[j] = i < 0 ? (bf16)0.0f : p.a[i];
    if (++ci == p.g.C) {
      ci = 0;
      if (++kw == p.g.KW) {
        kw = 0;
        ++kh;
      }
    }
  }
  return v;
}

template <int VEC>
__device__ __forceinline__ bf16x8 load_b_n8(const IGemmArgs& p, int n, int k) {
  // B_KN: B(k, n) = b[k*ldb + n]
  if (k >= p.K || n >= p.N) return zero8();
  const long long i = (long long)k * p.ldb + n;
  if (VEC || p.bvec) return *reinterpret_cast<const bf16x8*>(p.b + i);
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (n + j < p.N) ? p.b[i + j] : (bf16)0.0f;
  return v;
}

// 16 zero bytes: the global_load_lds source of every padding / out-of-range slot.
__device__ __attribute__((aligned(16))) bf16 g_zero16[8];

// Raw buffer resource (base, byte range) and its 16-byte LDS-DMA load (buffer_load_dwordx4 ... lds:
// lane i lands at lds + 16 i; offsets at or beyond the range read zeros).  The resource type exists
// for the device target only, so the host pass of the kernels sees empty stand-ins.
struct BufRes {
#if defined(__HIP_DEVICE_COMPILE__)
  __amdgpu_buffer_rsrc_t r;
#endif
};
__device__ __forceinline__ BufRes buf_res(const void* base, int bytes) {
  BufRes b;
#if defined(__HIP_DEVICE_COMPILE__)
  b.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
#endif
  return b;
}
__device__ __forceinline__ void buf_lds16(const BufRes& b, char* lds, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(b.r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
#endif
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// VEC = 1: both operands are 16-byte gatherable (channel counts % 8 == 0, aligned) — the scalar
// fallbacks are compiled out of the hot loop.
// S > 0 (K-vector A and B, VEC only): the operands go global -> LDS directly (global_load_lds
// dwordx4 into lane-linear images whose 16-byte chunks are XOR-swizzled on the SOURCE address), S
// LDS stages with S-1 k-tiles in flight across the per-step barrier (counted vmcnt, raw s_barrier),
// instead of the register-staged double buffer.
// WGM: waves along M (4 / WGM along N); the register-staged path is 2 x 2.
// MF: MFMA shape of the LDS-DMA paths, 16 (v_mfma_f32_16x16x32_bf16) or 32 (v_mfma_f32_32x32x16_bf16: half the
// instructions per flop; the wave tile must be a multiple of 32 in both directions).  The LDS images are the same
// for both shapes; only the fragment reads and the accumulator -> (row, column) map of the epilogue differ.
template <int AK, int BK_, int BM, int BN, int KB, int VEC, int S = 0, int WGM = 2, int MF = 16>
__global__ __launch_bounds__(256) void igemm_kernel(IGemmArgs p_) {
  IGemmArgs p = p_;
  if (AK == A_DGRAD && p_.nph > 0) {  // multi-phase strided dgrad: this block's phase is blockIdx.z
    const int* ph = p_.phs[blockIdx.z];
    p.ph_on = 1;
    p.ph_h = ph[0];
    p.ph_w = ph[1];
    p.Hp = ph[2];
    p.Wp = ph[3];
    p.kh0 = ph[4];
    p.kw0 = ph[5];
    p.KHp = ph[6];
    p.KWp = ph[7];
    p.M = p.g.B * p.Hp * p.Wp;
    p.K = p.KHp * p.KWp * p.g.Co;
    p.ktiles_per_split = (p.K + KB - 1) / KB;
    if ((int)blockIdx.x * BM >= p.M) return;  // grid x covers the largest phase
  }
  constexpr bool AKV = (AK == A_ROWK || AK == A_CONV || AK == A_DGRAD);  // K-vector A
  constexpr bool BKV = (BK_ == B_NK || BK_ == B_DGRADW);                 // K-vector B
  constexpr bool GLDS = S > 0;
  static_assert(!GLDS || (AKV && BKV && VEC) || (AK == A_WGRAD && BK_ == B_KN && VEC),
                "LDS-DMA staging: 16-byte K-vector operands, or the row-padded weight gradient");
  constexpr int LDKB = GLDS ? KB : KB + 8;         // K-vector image row: KB k (+ 8 pad unless swizzled)
  constexpr int AIMG = AKV ? BM * LDKB : KB * BM;  // elements per buffer
  constexpr int BIMG = BKV ? BN * LDKB : KB * BN;
  constexpr int NBUF = GLDS ? S : 2;
  constexpr int AS = BM * KB / 2048;  // 16-byte slots per thread (either image kind)
  constexpr int BS = BN * KB / 2048;
  constexpr int KV = KB / 8, RSK = 256 / KV;  // K-vector: vectors per row, rows per slot step
  // row-vector images: CH 16-byte chunks per k row, a slot step covers 256/CH k rows
  constexpr int CHA = BM / 8, RSA = 256 / CHA, CHB = BN / 8, RSB = 256 / CHB;
  constexpr int WGN = 4 / WGM;
  static_assert(GLDS || WGM == 2, "wave layouts other than 2 x 2 are built for the glds path only");
  constexpr int WTM = BM / WGM, WTN = BN / WGN, MI = WTM / 16, NI = WTN / 16;
  static_assert(MF == 16 || (MF == 32 && GLDS && WTM % 32 == 0 && WTN % 32 == 0), "32x32 MFMA: LDS-DMA paths, 32-multiple wave tiles");
  // fragment grid of a wave: FI x FJ fragments of FW x FW, RPL accumulator registers per lane each
  constexpr int FW = MF, FI = WTM / FW, FJ = WTN / FW, RPL = MF == 32 ? 16 : 4;
  // glds images: a wave instruction fills 1024 B = RPI rows of KV chunks; rows are read 16 at a time
  // (one per lane of a 16-lane group) at one logical chunk, so the physical chunk is XORed with
  // (row / rows-per-256B-bank-row) to land the 16 reads in 16 distinct bank slots
  constexpr int RPI = 64 / KV, RPB = 128 / KB;
  __shared__ __attribute__((aligned(16))) bf16 smem[NBUF * (AIMG + BIMG)];
  bf16* const As = smem;
  bf16* const Bs = smem + NBUF * AIMG;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  // Workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share an L2): remap the
  // linear id so every XCD owns a contiguous run of tiles — M-major neighbours then share the B
  // tile (and the A rows of the next N column) in one L2.  Bijective for any grid size.
  int bx = blockIdx.x, by = blockIdx.y, bz = (AK == A_DGRAD && p.nph > 0) ? 0 : (int)blockIdx.z;
  if (p.xcd && !(AK == A_DGRAD && p.nph > 0)) {
    const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
    if (nwg > 8) {
      const int bid = bx + gx * (by + gy * bz);
      const int q = nwg >> 3, r = nwg & 7, x8 = bid & 7;
      const int L = (x8 < r ? x8 * (q + 1) : r * (q + 1) + (x8 - r) * q) + (bid >> 3);
      bx = L % gx;
      by = (L / gx) % gy;
      bz = L / (gx * gy);
    }
  }
  const int m0 = bx * BM, n0 = by * BN;  // M-major: neighbours share the B tile in L2
  const int kt0 = bz * p.ktiles_per_split;
  const int kt1 = min((p.K + KB - 1) / KB, kt0 + p.ktiles_per_split);
  if (kt0 >= kt1 && p.cf_mode == 2) return;  // empty split contributes nothing (mode 3 stores its zeros)

  // ---- loader state
  const int lk = (tid % KV) * 8;  // K-vector: k offset of every slot of this thread
  const int lr = tid / KV;        // K-vector: row of slot 0 (slot i: lr + RSK*i)
  const int vka = tid / CHA, vca = tid % CHA;  // row-vector A: k row (+RSA per slot), m chunk
  const int vkb = tid / CHB, vcb = tid % CHB;
  ARow ar[AS];
  WRow wr[AS];
  KPos ka{0, 0, 0}, kb{0, 0, 0};
  PixPos pa{0, 0, 0};
  const int KW = (AK == A_DGRAD && p.ph_on) ? p.KWp : p.g.KW;  // taps per kernel row of this K
  const int Cda = (AK == A_CONV) ? p.g.C : p.g.Co;
  if (AKV) {
#pragma unroll
    for (int i = 0; i < AS; ++i) ar[i] = a_row<AK>(p, m0 + lr + RSK * i);
    if (AK != A_ROWK) ka = kpos_of(kt0 * KB + lk, Cda, KW);
  } else {
#pragma unroll
    for (int i = 0; i < AS; ++i) {
      const int m = m0 + vca * 8;  // every slot shares the chunk (k rows vka + RSA*i)
      if (AK == A_WGRAD) {
        const int mm = m < p.M ? m : 0;
        const KPos t = kpos_of(mm, p.g.C, KW);
        wr[i] = WRow{t.kh, t.kw, t.c, m < p.M};
      }
    }
    if (AK == A_WGRAD) {
      const int k = kt0 * KB + vka;
      const int hw = p.g.Ho * p.g.Wo;
      const int b = k / hw, rem = k - b * hw;
      pa = PixPos{b, rem / p.g.Wo, rem - (rem / p.g.Wo) * p.g.Wo};
    }
  }
  if (BK_ == B_DGRADW) kb = kpos_of(kt0 * KB + lk, p.g.Co, KW);

  // Weight-gradient VEC fast path (the host guarantees 32-bit offsets): every thread's 8 rows are
  // one tap (kh, kw) and 8 channels; each slot walks its pixel forward by KB per k-step with
  // incremental offsets (adds and a rare wrap), no per-step index multiplications.
  constexpr bool WFAST = (AK == A_WGRAD && VEC);
  constexpr bool BFAST = (BK_ == B_KN && VEC);
  struct WSlot {
    int ow, oh, ih, iw, rowoff, coloff, bo;
  };
  WSlot ws[WFAST ? AS : 1];
  int wci = 0, wHWC = 0, wBHWC = 0;
  bool wok = false;
  if constexpr (WFAST) {
    const int m = m0 + vca * 8;
    wok = m < p.M;
    const KPos t = kpos_of(wok ? m : 0, p.g.C, p.g.KW);
    const int WC = p.g.W * p.g.C;
    wHWC = p.g.H * WC;
    wBHWC = p.g.B * wHWC;
    wci = t.c;
    const int hw = p.g.Ho * p.g.Wo;
#pragma unroll
    for (int i = 0; i < AS; ++i) {
      const int k = kt0 * KB + vka + RSA * i;
      const int b = k / hw, rem = k - b * hw, oh = rem / p.g.Wo, ow = rem - oh * p.g.Wo;
      const int ih = oh * p.g.sh - p.g.pt + t.kh, iw = ow * p.g.sw - p.g.pl + t.kw;
      ws[i] = WSlot{ow, oh, ih, iw, ih * WC, iw * p.g.C, b * wHWC};
    }
  }
  int bo_off[BFAST ? BS : 1];
  if constexpr (BFAST) {
#pragma unroll
    for (int i = 0; i < BS; ++i) bo_off[i] = (kt0 * KB + vkb + RSB * i) * (int)p.ldb + n0 + vcb * 8;
  }

  bf16x8 ra[AS], rb[BS];
  auto gload = [&](int kt) {
    const int k0 = kt * KB;
    if (AKV) {
#pragma unroll
      for (int i = 0; i < AS; ++i) ra[i] = load_a_k8<AK, VEC>(p, ar[i], ka, k0 + lk, Cda);
    } else if constexpr (WFAST) {
      // KB pixels = qW output rows + rW columns (block-uniform)
      const int qW = KB / p.g.Wo, rW = KB - qW * p.g.Wo;
      const int WC = p.g.W * p.g.C, drow = p.g.sh * WC, wrapr = p.g.Ho * p.g.sh * WC;
      const int wrapc = p.g.Wo * p.g.sw * p.g.C, dcol = rW * p.g.sw * p.g.C, drowq = qW * drow;
#pragma unroll
      for (int i = 0; i < AS; ++i) {
        WSlot& w = ws[i];
        const bool ok = wok && w.bo < wBHWC && (unsigned)w.ih < (unsigned)p.g.H && (unsigned)w.iw < (unsigned)p.g.W;
        ra[i] = ok ? *reinterpret_cast<const bf16x8*>(p.a + (w.bo + w.rowoff + w.coloff + wci)) : zero8();
        // next k-tile: KB pixels further
        w.ow += rW;
        w.iw += rW * p.g.sw;
        w.coloff += dcol;
        w.oh += qW;
        w.ih += qW * p.g.sh;
        w.rowoff += drowq;
        if (w.ow >= p.g.Wo) {
          w.ow -= p.g.Wo;
          w.iw -= p.g.Wo * p.g.sw;
          w.coloff -= wrapc;
          ++w.oh;
          w.ih += p.g.sh;
          w.rowoff += drow;
        }
        while (w.oh >= p.g.Ho) {
          w.oh -= p.g.Ho;
          w.ih -= p.g.Ho * p.g.sh;
          w.rowoff -= wrapr;
          w.bo += wHWC;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < AS; ++i) {
        PixPos q = pa;
        if (AK == A_WGRAD && i) pix_advance(q, RSA * i, p.g.Ho, p.g.Wo);
        ra[i] = load_a_m8<AK, VEC>(p, m0 + vca * 8, wr[i], q, k0 + vka + RSA * i);
      }
    }
    if (BKV) {
#pragma unroll
      for (int i = 0; i < BS; ++i) rb[i] = load_b_k8<BK_, VEC>(p, n0 + lr + RSK * i, kb, k0 + lk);
    } else if constexpr (BFAST) {
      const bool nok = n0 + vcb * 8 < p.N;
#pragma unroll
      for (int i = 0; i < BS; ++i) {
        rb[i] = (nok && k0 + vkb + RSB * i < p.K) ? *reinterpret_cast<const bf16x8*>(p.b + bo_off[i]) : zero8();
        bo_off[i] += KB * (int)p.ldb;
      }
    } else {
#pragma unroll
      for (int i = 0; i < BS; ++i) rb[i] = load_b_n8<VEC>(p, n0 + vcb * 8, k0 + vkb + RSB * i);
    }
    // advance the incremental decompositions to the next k-tile
    if (AKV && AK != A_ROWK) kpos_advance(ka, KB, Cda, KW);
    if (AK == A_WGRAD && !WFAST) pix_advance(pa, KB, p.g.Ho, p.g.Wo);
    if (BK_ == B_DGRADW) kpos_advance(kb, KB, p.g.Co, KW);
  };
  auto sstore = [&](int buf) {
    bf16* a = As + buf * AIMG;
    bf16* b = Bs + buf * BIMG;
    if (AKV) {
#pragma unroll
      for (int i = 0; i < AS; ++i) *reinterpret_cast<bf16x8*>(a + (lr + RSK * i) * LDKB + lk) = ra[i];
    } else {
#pragma unroll
      for (int i = 0; i < AS; ++i)
        *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(a) + swz<BM>(vka + RSA * i, vca)) = ra[i];
    }
    if (BKV) {
#pragma unroll
      for (int i = 0; i < BS; ++i) *reinterpret_cast<bf16x8*>(b + (lr + RSK * i) * LDKB + lk) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < BS; ++i)
        *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(b) + swz<BN>(vkb + RSB * i, vcb)) = rb[i];
    }
  };

  f32x4 acc[MF == 16 ? MI : 1][MF == 16 ? NI : 1];
  f32x16 acc2[MF == 32 ? FI : 1][MF == 32 ? FJ : 1];
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc2[i][j][r] = 0.f;
  }
  // accumulator register r of fragment (i, j) -> its value, and its row within the fragment
  auto accv = [&](int i, int j, int r) -> float {
    if constexpr (MF == 32) return acc2[i][j][r];
    else return acc[i][j][r];
  };
  auto frow = [&](int r) -> int { return MF == 32 ? 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3) : (lane >> 4) * 4 + r; };
  const int fcl = lane & (FW - 1);   // the lane's column within a fragment

  // BN backward sums (p.bs, input gradients on the LDS-DMA path): the BN input y (and residual) of this thread's
  // epilogue chunks (rows m0 + (tid + 256 i) / (BN / 8), 8 columns at n0 + 8 (tid % (BN / 8))) are loaded here,
  // before the K loop, so the epilogue never waits on them; tiles with more than 4 chunks per thread load them in
  // the epilogue instead
  constexpr int BCH = BM * (BN / 8) / 256;
  constexpr bool BPRE = GLDS && AKV && BCH <= 4;
  bf16x8 pyv[BPRE ? BCH : 1], prv[BPRE ? BCH : 1];
  if constexpr (BPRE) {
    if (p.bs.dstats) {
#pragma unroll
      for (int i = 0; i < BCH; ++i) {
        const int c = tid + 256 * i, lr = c / (BN / 8), ch = c - lr * (BN / 8);
        const int mrow = m0 + lr, col0 = n0 + ch * 8;
        const bool ok = mrow < p.M && col0 < p.N;
        const long long eo = (long long)(ok ? mrow : 0) * p.ldcb + (ok ? col0 : 0);
        pyv[i] = ok ? *reinterpret_cast<const bf16x8*>(p.bs.y + eo) : zero8();
        prv[i] = (ok && p.bs.res) ? *reinterpret_cast<const bf16x8*>(p.bs.res + eo) : zero8();
      }
    }
  }

  const int fr = lane & 15, fk = (lane >> 4) * 8;
  if constexpr (GLDS && !AKV) {
    // Weight gradient dW[(kh,kw,ci), co] = sum over pixels of X(pixel shifted by the tap)[ci] * dY[pixel][co],
    // both operands row-vector images [k][BM|BN] (XOR-swizzled 16-byte chunks, read back transposed), filled
    // by LDS-DMA.  The pixel (K) order is row-padded and batch-inner: k = (oh * B + b) * Wp + ow with Wp a
    // power of two >= Wo dividing KB, so a k-tile covers RT = KB / Wp whole output rows (oh fixed, b0..b0+RT-1;
    // the host guarantees B % RT == 0).  Every slot's byte offset is then fixed for the whole loop except
    // for the kernel-row bounds check of A, redone when oh changes (every B / RT k-tiles); the k-tile's
    // (b0, oh) position is the scalar soffset; padding columns, padding pixels and rows past M / N read zeros.
    constexpr int kOOB = (int)0x80000000u;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const Geo& g = p.g;
    const int Wp = 1 << p.wp_log, RT = KB >> p.wp_log;
    const int HWC = g.H * g.W * g.C, HoWoCo = g.Ho * g.Wo * g.Co;
    const BufRes rsa = buf_res(reinterpret_cast<const char*>(p.a) - 2 * (long long)p.a_shift, p.a_bytes);
    const BufRes rsb = buf_res(p.b, p.b_bytes);
    constexpr int RPA = 1024 / (BM * 2), RPB_ = 1024 / (BN * 2);  // k rows per 1 KiB LDS-DMA instruction
    int afix[AS], akh[AS], avo[AS], bvo[BS];
    bool aok[AS];
#pragma unroll
    for (int i = 0; i < AS; ++i) {
      const int row = (wv * AS + i) * RPA + lane / CHA;
      const int m = m0 + ((lane % CHA) ^ swzc<BM>(row)) * 8;
      const int rr = row >> p.wp_log, ow = row & (Wp - 1);
      const KPos t = kpos_of(m < p.M ? m : 0, g.C, g.KW);
      const int iw = ow * g.sw - g.pl + t.kw;
      aok[i] = m < p.M && ow < g.Wo && (unsigned)iw < (unsigned)g.W;
      afix[i] = rr * HWC + (t.kh * g.W + ow * g.sw + t.kw) * g.C + t.c;  // >= 0 relative to X - a_shift
      akh[i] = t.kh - g.pt;
      avo[i] = kOOB;
    }
#pragma unroll
    for (int j = 0; j < BS; ++j) {
      const int row = (wv * BS + j) * RPB_ + lane / CHB;
      const int n = n0 + ((lane % CHB) ^ swzc<BN>(row)) * 8;
      const int rr = row >> p.wp_log, ow = row & (Wp - 1);
      bvo[j] = (n < p.N && ow < g.Wo) ? (rr * HoWoCo + ow * g.Co + n) * 2 : kOOB;
    }
    const int R0 = kt0 * RT;  // pixel row (oh * B + b) of the next k-tile to issue
    int noh = R0 / g.B, nb0 = R0 - noh * g.B;
    bool newoh = true;
    char* const lds = reinterpret_cast<char*>(smem);
    auto issue = [&](int stage) {
      const int oh = noh, b0 = nb0;
      const bool fresh = newoh;
      nb0 += RT;
      newoh = nb0 >= g.B;
      if (newoh) {
        nb0 -= g.B;
        ++noh;
      }
      if (fresh) {
#pragma unroll
        for (int i = 0; i < AS; ++i)
          avo[i] = (aok[i] && (unsigned)(oh * g.sh + akh[i]) < (unsigned)g.H) ? afix[i] * 2 : kOOB;
      }
      const int soa = (b0 * HWC + oh * g.sh * g.W * g.C) * 2;
      const int sob = (b0 * HoWoCo + oh * g.Wo * g.Co) * 2;
      char* ab = lds + stage * AIMG * 2 + wv * AS * 1024;
      char* bb = lds + NBUF * AIMG * 2 + stage * BIMG * 2 + wv * BS * 1024;
#pragma unroll
      for (int i = 0; i < AS; ++i) buf_lds16(rsa, ab + i * 1024, avo[i], soa);
#pragma unroll
      for (int j = 0; j < BS; ++j) buf_lds16(rsb, bb + j * 1024, bvo[j], sob);
    };
    auto compute = [&](int stage) {
      const bf16* a = As + stage * AIMG;
      const bf16* b = Bs + stage * BIMG;
      if constexpr (MF == 32) {
#pragma unroll
        for (int kk = 0; kk < KB; kk += 16) {
          bf16x8 af[FI], bfr[FJ];
#pragma unroll
          for (int i = 0; i < FI; ++i) af[i] = tr_frag32<BM>(a, wm * WTM + i * 32, lane, kk);
#pragma unroll
          for (int j = 0; j < FJ; ++j) bfr[j] = tr_frag32<BN>(b, wn * WTN + j * 32, lane, kk);
#pragma unroll
          for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int j = 0; j < FJ; ++j) acc2[i][j] = mfma32(af[i], bfr[j], acc2[i][j]);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < KB; kk += 32) {
          bf16x8 af[MI], bfr[NI];
#pragma unroll
          for (int i = 0; i < MI; ++i) af[i] = tr_frag<BM>(a, wm * WTM + i * 16, lane, kk);
#pragma unroll
          for (int j = 0; j < NI; ++j) bfr[j] = tr_frag<BN>(b, wn * WTN + j * 16, lane, kk);
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        }
      }
    };
    const int nk = kt1 - kt0;
    if (nk > 0) {
#pragma unroll
      for (int st = 0; st < S - 1; ++st)
        if (st < nk) issue(st);
      int cst = 0, ist = S - 1;
      for (int rel = 0; rel < nk; ++rel) {
        const int after = min(S - 2, nk - 1 - rel);
        if (after >= 2) vm_wait<2 * (AS + BS)>();
        else if (after == 1) vm_wait<AS + BS>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        if (rel + S - 1 < nk) issue(ist);
        compute(cst);
        cst = cst == S - 1 ? 0 : cst + 1;
        ist = ist == S - 1 ? 0 : ist + 1;
      }
      vm_wait<0>();
    }
  } else if constexpr (GLDS) {
    // LDS-DMA staging (buffer_load_dwordx4 ... lds over raw buffer resources of A and B).
    // Instruction j = wave*AS + i fills rows j*RPI + lane/KV, physical chunk lane%KV, which holds
    // logical chunk (lane%KV) ^ swz(row).  The host only takes this path when every k-tile lies inside
    // ONE filter tap (C, resp. Co, a multiple of KB) and both operands are < 2 GiB.  A slot's 32-bit
    // byte offset (VGPR) is fixed for the whole loop (B, dense A) or recomputed only when the k-tile
    // enters a new filter tap (conv A: two range compares and a select per slot); the k-tile's
    // channel / k / tap offset is the block-uniform soffset (SGPR); padding and out-of-range slots
    // read zeros through the buffer range check (offset 2^31).  The loop is unrolled by the stage
    // count, so stage bases are immediates and no per-k-tile VALU address math remains.
    constexpr int kOOB = (int)0x80000000u;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const BufRes rsa = buf_res(p.a, p.a_bytes), rsb = buf_res(p.b, p.b_bytes);
    int arow[AS], ay0[AS], ax0[AS], avo[AS], bvo[BS], alch[AS], blch[BS];
#pragma unroll
    for (int i = 0; i < AS; ++i) {
      const int row = (wv * AS + i) * RPI + lane / KV;
      const int lch = (lane % KV) ^ ((row / RPB) & (KV - 1));
      const int m = m0 + row;
      const bool ok = m < p.M;
      alch[i] = lch;
      if (AK == A_ROWK) {
        avo[i] = ok ? (int)(((long long)m * p.lda + lch * 8) * 2) : kOOB;
        arow[i] = ay0[i] = ax0[i] = 0;
      } else {
        const ARow r = a_row<AK>(p, m);
        const int Wd = AK == A_CONV ? p.g.W : p.g.Wo, Cd0 = AK == A_CONV ? p.g.C : p.g.Co;
        arow[i] = (int)((r.base + (long long)r.y0 * Wd + r.x0) * Cd0) + lch * 8;   // may be < 0 (padding)
        ay0[i] = r.ok ? r.y0 : -(1 << 28);   // an invalid row never passes the range check
        ax0[i] = r.x0;
        avo[i] = kOOB;
      }
    }
#pragma unroll
    for (int j = 0; j < BS; ++j) {
      const int row = (wv * BS + j) * RPI + lane / KV;
      const int lch = (lane % KV) ^ ((row / RPB) & (KV - 1));
      const int n = n0 + row;
      blch[j] = lch;
      if (BK_ == B_NK) bvo[j] = n < p.N ? (int)(((long long)n * p.ldb + lch * 8) * 2) : kOOB;
      else bvo[j] = n < p.N ? (n * p.g.Co + lch * 8) * 2 : kOOB;   // W[kh][kw][n][co]
    }
    // per-lane LDS fragment offsets (bytes) of row i = 0 / column j = 0 at each 32-wide k slice: the
    // XOR swizzle of a row does not change over the 16-row steps of i / j (16 / RPB is a multiple of KV)
    // (32x32x16: rows lane&31 at chunk kk/8 + lane>>5 per 16-wide k step; the XOR is invariant over 32-row steps too)
    constexpr int KST = MF == 32 ? 16 : 32;
    int offa[KB / KST], offb[KB / KST];
#pragma unroll
    for (int kk = 0; kk < KB; kk += KST) {
      const int c = MF == 32 ? kk / 8 + (lane >> 5) : kk / 8 + (lane >> 4);
      const int fl = MF == 32 ? (lane & 31) : fr;
      const int ra0 = wm * WTM + fl, rb0 = wn * WTN + fl;
      offa[kk / KST] = (ra0 * KB + ((c ^ ((ra0 / RPB) & (KV - 1))) << 3)) * 2;
      offb[kk / KST] = (rb0 * KB + ((c ^ ((rb0 / RPB) & (KV - 1))) << 3)) * 2;
    }
    // row-tile mode (A_CONV): a k-tile is one whole kernel row (its chunks are the row's taps), so the
    // bookkeeping below runs with one "tap" of KB channels per kernel row
    const bool rowtile = AK == A_CONV && p.rowtile;
    const int KWd = rowtile ? 1 : ((AK == A_DGRAD && p.ph_on) ? p.KWp : p.g.KW);  // taps per kernel row of this K
    // block-uniform tap (th, tw) and channel offset c0 of the next k-tile to issue: decomposed once,
    // then advanced by KB per issue (issues run in k order)
    const int Cd = rowtile ? KB : ((AK == A_CONV) ? p.g.C : p.g.Co);
    const int Creal = (AK == A_CONV) ? p.g.C : p.g.Co;
    const int Hl = AK == A_CONV ? p.g.H : p.g.Ho, Wl = AK == A_CONV ? p.g.W : p.g.Wo;
    const int tsgn = AK == A_CONV ? 1 : -1;   // conv reads pixel (y0 + th, x0 + tw), dgrad (y0 - th, x0 - tw)
    int nth = 0, ntw = 0, nc0 = kt0 * KB;
    if (AK != A_ROWK || BK_ == B_DGRADW) {
      const int t = (kt0 * KB) / Cd;
      nc0 = kt0 * KB - t * Cd;
      nth = t / KWd;
      ntw = t - nth * KWd;
    }
    bool newtap = true;   // the first issue of the block computes its tap's slot offsets
    char* const lds = reinterpret_cast<char*>(smem);
    auto issue = [&](int stage, int kt) {
      const int k0 = kt * KB;
      const int th = nth, tw = ntw, c0 = (AK != A_ROWK || BK_ == B_DGRADW) ? nc0 : k0;
      const bool fresh = newtap;
      if (AK != A_ROWK || BK_ == B_DGRADW) {
        nc0 += KB;
        newtap = nc0 >= Cd;
        if (newtap) {
          nc0 -= Cd;
          if (++ntw == KWd) {
            ntw = 0;
            ++nth;
          }
        }
      }
      if (AK != A_ROWK && fresh) {
        const int tapoff = tsgn * (th * Wl + tw) * Creal;
#pragma unroll
        for (int i = 0; i < AS; ++i) {
          const bool v = (unsigned)(ay0[i] + tsgn * th) < (unsigned)Hl && (unsigned)(ax0[i] + tsgn * tw) < (unsigned)Wl;
          avo[i] = v ? (arow[i] + tapoff) * 2 : kOOB;
        }
      }
      const int soa = (AK == A_ROWK ? k0 : c0) * 2;
      int sob = k0 * 2;
      if (BK_ == B_DGRADW) {
        const int kh = p.ph_on ? p.kh0 + th * p.g.sh : th, kw = p.ph_on ? p.kw0 + tw * p.g.sw : tw;
        sob = ((kh * p.g.KW + kw) * p.g.C * p.g.Co + c0) * 2;
      }
      char* ab = lds + stage * AIMG * 2 + wv * AS * 1024;
      char* bb = lds + NBUF * AIMG * 2 + stage * BIMG * 2 + wv * BS * 1024;
      if (k0 + KB > p.K) {   // partial last k-tile (dense K % KB != 0; K % 8 == 0): chunks past K read zeros
#pragma unroll
        for (int i = 0; i < AS; ++i)
          buf_lds16(rsa, ab + i * 1024, k0 + alch[i] * 8 < p.K ? avo[i] : kOOB, soa);
#pragma unroll
        for (int j = 0; j < BS; ++j)
          buf_lds16(rsb, bb + j * 1024, k0 + blch[j] * 8 < p.K ? bvo[j] : kOOB, sob);
      } else {
#pragma unroll
        for (int i = 0; i < AS; ++i)
          buf_lds16(rsa, ab + i * 1024, avo[i], soa);
#pragma unroll
        for (int j = 0; j < BS; ++j)
          buf_lds16(rsb, bb + j * 1024, bvo[j], sob);
      }
    };
    auto compute = [&](int stage) {   // stage: block-uniform; 4 VALU adds form the k-tile's read bases
      const char* a = lds + stage * AIMG * 2;
      const char* b = lds + NBUF * AIMG * 2 + stage * BIMG * 2;
      if constexpr (MF == 32) {
#pragma unroll
        for (int kk = 0; kk < KB; kk += 16) {
          bf16x8 af[FI], bfr[FJ];
          const char* ak = a + offa[kk / 16];
          const char* bk = b + offb[kk / 16];
#pragma unroll
          for (int i = 0; i < FI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ak + i * 32 * KB * 2);
#pragma unroll
          for (int j = 0; j < FJ; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(bk + j * 32 * KB * 2);
#pragma unroll
          for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int j = 0; j < FJ; ++j) acc2[i][j] = mfma32(af[i], bfr[j], acc2[i][j]);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < KB; kk += 32) {
          bf16x8 af[MI], bfr[NI];
          const char* ak = a + offa[kk / 32];
          const char* bk = b + offb[kk / 32];
#pragma unroll
          for (int i = 0; i < MI; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ak + i * 16 * KB * 2);
#pragma unroll
          for (int j = 0; j < NI; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(bk + j * 16 * KB * 2);
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
        }
      }
    };
    const int nk = kt1 - kt0;
    if (nk > 0) {
#pragma unroll
      for (int st = 0; st < S - 1; ++st)
        if (st < nk) issue(st, kt0 + st);
      int cst = 0, ist = S - 1;   // compute / issue stage (scalar rotation, no modulo)
      for (int rel = 0; rel < nk; ++rel) {
        const int after = min(S - 2, nk - 1 - rel);  // k-tiles already issued behind this one
        if (after >= 2) vm_wait<2 * (AS + BS)>();
        else if (after == 1) vm_wait<AS + BS>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();  // stage cst visible to all waves; stage ist free
        if (rel + S - 1 < nk) issue(ist, kt0 + rel + S - 1);
        compute(cst);
        cst = cst == S - 1 ? 0 : cst + 1;
        ist = ist == S - 1 ? 0 : ist + 1;
      }
      vm_wait<0>();
    }
  } else if (kt0 < kt1) {
    gload(kt0);
    sstore(0);
    __syncthreads();
    int buf = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) gload(kt + 1);
      const bf16* a = As + buf * AIMG;
      const bf16* b = Bs + buf * BIMG;
#pragma unroll
      for (int kk = 0; kk < KB; kk += 32) {
        bf16x8 af[MI], bfr[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int r = wm * WTM + i * 16;
          if (AKV) af[i] = *reinterpret_cast<const bf16x8*>(a + (r + fr) * LDKB + kk + fk);
          else af[i] = tr_frag<BM>(a, r, lane, kk);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int c = wn * WTN + j * 16;
          if (BKV) bfr[j] = *reinterpret_cast<const bf16x8*>(b + (c + fr) * LDKB + kk + fk);
          else bfr[j] = tr_frag<BN>(b, c, lane, kk);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
      if (more) {
        sstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
      }
    }
  }

  // ---- epilogue, bf16 activation outputs of the glds kernels: the accumulator tile goes through
  // LDS (f32, MFMA layout in, row-contiguous out) so the global stores are 16-byte row chunks, not
  // 2-byte scattered per-lane stores; per-column BN statistics are still taken in the MFMA layout.
  constexpr int TLD = BN + 16;  // f32 row stride: the 4 row groups of a 16-lane MFMA column hit 4 bank quarters
  constexpr bool LDS_EPI = GLDS && (size_t)BM * TLD * 4 + 4 * 16 * 2 * 4 * 8 <= sizeof(smem);
  if constexpr (LDS_EPI) {
    if (p.cb && p.cf_mode == 0) {
      float* T = reinterpret_cast<float*>(smem);
      float* red = T + BM * TLD;  // [WGM][WGN][NI][2][16] statistics partials
      __syncthreads();            // every wave is done reading the last stage
      float e1[FJ], e2[FJ];
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int lc = wn * WTN + j * FW + fcl, col = n0 + lc;
        const bool cok = col < p.N;
        const float bv = (p.bias && cok) ? p.bias[col] : 0.f;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < FI; ++i) {
#pragma unroll
          for (int r = 0; r < RPL; ++r) {
            const int lr = wm * WTM + i * FW + frow(r);
            float v = p.alpha * accv(i, j, r) + bv;
            if (p.colstats && cok && m0 + lr < p.M) {
              const float q = bf2f(f2bf(v));
              s1 += q;
              s2 += q * q;
            }
            if (p.relu) v = fmaxf(v, 0.f);
            T[lr * TLD + lc] = v;
          }
        }
        if (p.colstats) {
          if (MF == 16) {
            s1 += __shfl_xor(s1, 16, 64);
            s2 += __shfl_xor(s2, 16, 64);
          }
          s1 += __shfl_xor(s1, 32, 64);
          s2 += __shfl_xor(s2, 32, 64);
        }
        e1[j] = s1;
        e2[j] = s2;
      }
      if (p.colstats && lane < FW) {
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          red[(((wm * WGN + wn) * FJ + j) * 2 + 0) * FW + lane] = e1[j];
          red[(((wm * WGN + wn) * FJ + j) * 2 + 1) * FW + lane] = e2[j];
        }
      }
      __syncthreads();
      if (p.colstats && wm == 0 && lane < FW) {
        double* st = p.colstats + (size_t)(bx % kStatSlots) * 2 * p.N;
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
          const int col = n0 + wn * WTN + j * FW + lane;
          if (col >= p.N) continue;
          float a1 = 0.f, a2 = 0.f;
#pragma unroll
          for (int w = 0; w < WGM; ++w) {
            a1 += red[(((w * WGN + wn) * FJ + j) * 2 + 0) * FW + lane];
            a2 += red[(((w * WGN + wn) * FJ + j) * 2 + 1) * FW + lane];
          }
          atomicAdd(&st[col], (double)a1);
          atomicAdd(&st[p.N + col], (double)a2);
        }
      }
      // row-contiguous 8-column chunks: 16-byte bf16 stores (read-add-store for accumulated outputs)
      constexpr int CPRW = BN / 8;
      const bool vst = (p.ldcb % 8) == 0 && ((uintptr_t)p.cb & 15) == 0;
      // BN backward sums (p.bs): this thread's 8 columns are fixed (256 % CPRW == 0); their BN coefficients
      const bool bsum = p.bs.dstats != nullptr;
      float bsc[8], bsf[8], bmu[8], brs[8], q1[8], q2[8];
      if (bsum) {
        const int cc0 = n0 + (tid % CPRW) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cc = min(cc0 + j, p.N - 1);
          const float mu = p.bs.saved[cc], rs = p.bs.saved[p.N + cc];
          const float gm = p.bs.gamma ? p.bs.gamma[cc] : 1.f;
          bsc[j] = gm * rs;
          bsf[j] = (p.bs.beta ? p.bs.beta[cc] : 0.f) - mu * gm * rs;
          bmu[j] = mu;
          brs[j] = rs;
          q1[j] = q2[j] = 0.f;
        }
      }
      for (int c = tid; c < BM * CPRW; c += 256) {
        const int lr = c / CPRW, ch = c - lr * CPRW;
        const int mrow = m0 + lr, col0 = n0 + ch * 8;
        if (mrow >= p.M || col0 >= p.N) continue;
        long long row = mrow;
        if (AK == A_DGRAD && p.ph_on) {  // phase row -> input pixel
          const int hw = p.Hp * p.Wp;
          const int b = mrow / hw, rem = mrow - b * hw;
          const int ihp = rem / p.Wp, iwp = rem - ihp * p.Wp;
          row = ((long long)b * p.g.H + ihp * p.g.sh + p.ph_h) * p.g.W + iwp * p.g.sw + p.ph_w;
        }
        const float4 lo = *reinterpret_cast<const float4*>(T + lr * TLD + ch * 8);
        const float4 hi = *reinterpret_cast<const float4*>(T + lr * TLD + ch * 8 + 4);
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        bf16* q = p.cb + row * p.ldcb + col0;
        if (vst && col0 + 8 <= p.N) {
          if (p.cb_accum) {
            const bf16x8 o = *reinterpret_cast<const bf16x8*>(q);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += bf2f(o[e]);
          }
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e]);
          *reinterpret_cast<bf16x8*>(q) = o;
          if (bsum) {   // (host: vst and N % 8 == 0 whenever p.bs is on)
            bf16x8 yv, rv = zero8();
            if constexpr (BPRE) {
              const int ci = (c - tid) / 256;   // this thread's chunk index (the loop is unrolled by the compiler
#pragma unroll                                  // only as far as BCH; select the prefetched registers)
              for (int i = 0; i < BCH; ++i)
                if (i == ci) {
                  yv = pyv[i];
                  rv = prv[i];
                }
            } else {
              const long long eo = row * p.ldcb + col0;
              yv = *reinterpret_cast<const bf16x8*>(p.bs.y + eo);
              if (p.bs.res) rv = *reinterpret_cast<const bf16x8*>(p.bs.res + eo);
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float yy = bf2f(yv[e]);
              const float z = yy * bsc[e] + bsf[e] + bf2f(rv[e]);
              const float g = (p.bs.relu && !(z > 0.f)) ? 0.f : bf2f(o[e]);   // the stored gradient
              q1[e] += g;
              q2[e] += g * ((yy - bmu[e]) * brs[e]);
            }
          }
        } else {
          for (int e = 0; e < 8 && col0 + e < p.N; ++e) q[e] = f2bf(v[e] + (p.cb_accum ? bf2f(q[e]) : 0.f));
        }
      }
      if (bsum) {
        // threads of one column chunk: lanes l, l ^ CPRW, ... of each wave, then the 4 waves through LDS (T is
        // free after the barrier); one f32 atomic pair per column and workgroup into slot bx % kStatSlots.
        // (LDS ds_add_f32 into one [2][BN] row instead of the permutes: 8-way contended, the input gradients
        // 500 -> 612 us per step; profiles/r6_bnsum/)
#pragma unroll
        for (int o = CPRW; o < 64; o <<= 1)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            q1[e] += __shfl_xor(q1[e], o, 64);
            q2[e] += __shfl_xor(q2[e], o, 64);
          }
        __syncthreads();
        float* bred = reinterpret_cast<float*>(smem);   // [4 waves][2][BN]
        if (lane < CPRW) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            bred[(wave * 2 + 0) * BN + lane * 8 + e] = q1[e];
            bred[(wave * 2 + 1) * BN + lane * 8 + e] = q2[e];
          }
        }
        __syncthreads();
        if (tid < BN && n0 + tid < p.N) {
          float a1 = 0.f, a2 = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            a1 += bred[(w * 2 + 0) * BN + tid];
            a2 += bred[(w * 2 + 1) * BN + tid];
          }
          float* ds = p.bs.dstats + (size_t)(bx % kStatSlots) * 2 * p.N;
          atomicAdd(&ds[n0 + tid], a1);
          atomicAdd(&ds[p.N + n0 + tid], a2);
        }
      }
      return;
    }
  }
  float sp1[FJ], sp2[FJ];  // per-column statistics of this wave (valid in lanes 0..FW-1)
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int col = n0 + wn * WTN + j * FW + fcl;
    const bool cok = col < p.N;
    const float bv = (p.bias && cok) ? p.bias[col] : 0.f;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const int mrow = m0 + wm * WTM + i * FW + frow(r);
        if (!cok || mrow >= p.M) continue;
        int row = mrow;
        if (AK == A_DGRAD && p.ph_on) {  // phase row -> input pixel
          const int hw = p.Hp * p.Wp;
          const int b = mrow / hw, rem = mrow - b * hw;
          const int ihp = rem / p.Wp, iwp = rem - ihp * p.Wp;
          row = (b * p.g.H + ihp * p.g.sh + p.ph_h) * p.g.W + iwp * p.g.sw + p.ph_w;
        }
        float v = p.alpha * accv(i, j, r) + bv;
        if (p.colstats) {
          // statistics of exactly the tensor BN will normalise (the bf16 activation)
          const float q = p.cb ? bf2f(f2bf(v)) : v;
          s1 += q;
          s2 += q * q;
        }
        if (p.relu) v = fmaxf(v, 0.f);
        if (AK == A_WGRAD || AK == A_COLM) {  // weight gradients: M * ldc < 2^31
          const int e = row * (int)p.ldc + col;
          if (p.cf_mode == 2) atomicAdd(&p.cf[e], v);
          else if (p.cf_mode == 3) p.cf[(long long)bz * p.M * p.ldc + e] = v;
          else if (p.cf_mode == 1) p.cf[e] = v;
        } else if (p.cf_mode == 1) {
          p.cf[(long long)row * p.ldc + col] = v;
        } else if (p.cf_mode == 2) {
          atomicAdd(&p.cf[(long long)row * p.ldc + col], v);
        } else if (p.cf_mode == 3) {
          p.cf[(long long)bz * p.M * p.ldc + (long long)row * p.ldc + col] = v;
        }
        if (p.cb) {
          bf16* q = &p.cb[(long long)row * p.ldcb + col];
          if (p.cb_accum) v += bf2f(*q);
          *q = f2bf(v);
        }
      }
    }
    if (p.colstats) {
      if (MF == 16) {
        s1 += __shfl_xor(s1, 16, 64);
        s2 += __shfl_xor(s2, 16, 64);
      }
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
    }
    sp1[j] = s1;
    sp2[j] = s2;
  }
  if (p.colstats) {
    // the WGM waves sharing a column range combine through LDS: one atomic per column per block
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [WGM][WGN][FJ][2][FW]
    if (wm > 0 && lane < FW) {
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        red[(((wm * WGN + wn) * FJ + j) * 2 + 0) * FW + lane] = sp1[j];
        red[(((wm * WGN + wn) * FJ + j) * 2 + 1) * FW + lane] = sp2[j];
      }
    }
    __syncthreads();
    if (wm == 0 && lane < FW) {
      double* st = p.colstats + (size_t)(bx % kStatSlots) * 2 * p.N;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int col = n0 + wn * WTN + j * FW + lane;
        if (col >= p.N) continue;
        float a1 = sp1[j], a2 = sp2[j];
#pragma unroll
        for (int w = 1; w < WGM; ++w) {
          a1 += red[(((w * WGN + wn) * FJ + j) * 2 + 0) * FW + lane];
          a2 += red[(((w * WGN + wn) * FJ + j) * 2 + 1) * FW + lane];
        }
        atomicAdd(&st[col], (double)a1);
        atomicAdd(&st[p.N + col], (double)a2);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Philox4x32-10: tde_philox.h (counter-based: masks are regenerated, never stored)

struct Drop {
  float rate;  // 0 = off
  unsigned long long seed;
  const long long* iter;
  int iter_offset;
  int layer_id;
};

// keep-scale (0 or 1/(1-rate)) of the 8 consecutive elements e0..e0+7 (e0 % 8 == 0)
// the keep-scale of one element (the same Philox stream drop8 draws: counter e / 4, word e % 4)
__device__ __forceinline__ float drop1(const Drop& d, long long e) {
  const long long it = (d.iter ? *d.iter : 0) + d.iter_offset;
  const uint2 key{(unsigned)d.seed, (unsigned)(d.seed >> 32)};
  const float keep = 1.f - d.rate;
  const unsigned long long c = (unsigned long long)(e >> 2);
  const uint4 r = philox(uint4{(unsigned)c, (unsigned)(c >> 32), (unsigned)it, (unsigned)d.layer_id}, key);
  const int q = (int)(e & 3);
  const unsigned w = q == 0 ? r.x : q == 1 ? r.y : q == 2 ? r.z : r.w;
  return ((w >> 8) * (1.f / 16777216.f) < keep) ? 1.f / keep : 0.f;
}

__device__ __forceinline__ void drop8(const Drop& d, long long e0, float* ks) {
  const long long it = (d.iter ? *d.iter : 0) + d.iter_offset;
  const uint2 key{(unsigned)d.seed, (unsigned)(d.seed >> 32)};
  const float keep = 1.f - d.rate, inv = 1.f / keep;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const unsigned long long c = (unsigned long long)(e0 >> 2) + h;
    const uint4 r = philox(uint4{(unsigned)c, (unsigned)(c >> 32), (unsigned)it, (unsigned)d.layer_id}, key);
    const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) ks[h * 4 + q] = ((w[q] >> 8) * (1.f / 16777216.f) < keep) ? inv : 0.f;
  }
}

// ---------------------------------------------------------------------------------------
// BatchNormalization (+ residual + ReLU + dropout) forward
struct BnFwdArgs {
  const bf16* y;
  bf16* out;
  const bf16* res;
  long long R;  // rows (= elements / C)
  int C;
  int mode;  // 0 identity (ReLU/dropout/add only), 1 batch statistics, 2 moving statistics
  const double* stats;  // [2][C] sum, sumsq (mode 1; f64 so E[y^2]-E[y]^2 does not cancel)
  float* saved;        // [2][C] mean, rstd (mode 1, written by block 0)
  const float* gamma;
  const float* beta;
  float eps;
  float* mmean;
  float* mvar;
  float momentum, bessel;
  float* zero_buf;  // [kStatSlots][2][C] backward accumulators of this layer (zeroed by block 0)
  int relu;
  Drop drop;
};

constexpr int kMaxC = 2048;

__global__ __launch_bounds__(256) void bn_fwd_kernel(BnFwdArgs a) {
  __shared__ float sc[kMaxC], sf[kMaxC];
  const int C = a.C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float scale = 1.f, shift = 0.f;
    if (a.mode != 0) {
      float mean, var;
      if (a.mode == 1) {
        double s1 = 0.0, s2 = 0.0;
        for (int sl = 0; sl < kStatSlots; ++sl) {
          s1 += a.stats[sl * 2 * C + c];
          s2 += a.stats[sl * 2 * C + C + c];
        }
        const double md = s1 / (double)a.R;
        mean = (float)md;
        var = (float)fmax(s2 / (double)a.R - md * md, 0.0);
      } else {
        mean = a.mmean[c];
        var = a.mvar[c];
      }
      const float rstd = rsqrtf(var + a.eps);
      const float g = a.gamma ? a.gamma[c] : 1.f;
      scale = g * rstd;
      shift = (a.beta ? a.beta[c] : 0.f) - mean * scale;
      if (blockIdx.x == 0 && a.mode == 1) {
        a.saved[c] = mean;
        a.saved[C + c] = rstd;
        if (a.mmean) {
          a.mmean[c] = a.mmean[c] * a.momentum + mean * (1.f - a.momentum);
          a.mvar[c] = a.mvar[c] * a.momentum + var * a.bessel * (1.f - a.momentum);
        }
      }
    }
    if (blockIdx.x == 0 && a.zero_buf) {
      for (int sl = 0; sl < kStatSlots; ++sl) {
        a.zero_buf[sl * 2 * C + c] = 0.f;
        a.zero_buf[sl * 2 * C + C + c] = 0.f;
      }
    }
    sc[c] = scale;
    sf[c] = shift;
  }
  __syncthreads();
  const long long n = a.R * C;
  const long long nchunk = (n + 7) / 8;
  const bool vec = (n % 8) == 0;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < nchunk;
       q += (long long)gridDim.x * blockDim.x) {
    const long long e0 = q * 8;
    float v[8], r[8], ks[8];
    if (vec) {
      const bf16x8 yv = *reinterpret_cast<const bf16x8*>(a.y + e0);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(yv[j]);
      if (a.res) {
        const bf16x8 rv = *reinterpret_cast<const bf16x8*>(a.res + e0);
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = bf2f(rv[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = e0 + j < n ? bf2f(a.y[e0 + j]) : 0.f;
        r[j] = (a.res && e0 + j < n) ? bf2f(a.res[e0 + j]) : 0.f;
      }
    }
    if (a.drop.rate > 0.f) drop8(a.drop, e0, ks);
    int c = (int)((unsigned)e0 % (unsigned)C);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float z = v[j] * sc[c] + sf[c];
      if (a.res) z += r[j];
      if (a.relu) z = fmaxf(z, 0.f);
      if (a.drop.rate > 0.f) z *= ks[j];
      o[j] = f2bf(z);
      if (++c == C) c = 0;
    }
    if (vec) {
      *reinterpret_cast<bf16x8*>(a.out + e0) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (e0 + j < n) a.out[e0 + j] = o[j];
    }
  }
}

// ---------------------------------------------------------------------------------------
// BN (+ residual + ReLU + dropout) backward.  dz = dout * keep * (z > 0) where z is the
// pre-ReLU value recomputed from y (and the residual); xhat = (y - mean) * rstd.
struct BnBwdArgs {
  const bf16* dout;
  const bf16* y;
  const bf16* res;
  long long R;
  int C;
  int mode;  // 0 identity, 1 batch statistics
  const float* saved;  // [2][C] mean, rstd
  const float* gamma;
  const float* beta;
  int relu;
  Drop drop;
  float* dstats;  // [kStatSlots][2][C] sum dz, sum dz*xhat (slot = block % kStatSlots)
  bf16* dx;
  int dx_accum;
  bf16* dres;
  int dres_accum;
  float* dgamma;
  float* dbeta;
  double* zero_fwd;  // [2][C] forward statistics of this layer (zeroed by block 0 of the apply pass)
};

struct BnPre {
  float sc, sf, mean, rstd;
};

__device__ __forceinline__ void bn_dz8(const BnBwdArgs& a, const float* sc, const float* sf, const float* mu,
                                       const float* rs, long long e0, long long n, bool vec, float* dz,
                                       float* xh) {
  float v[8], r[8], d[8], ks[8];
  if (vec) {
    const bf16x8 yv = *reinterpret_cast<const bf16x8*>(a.y + e0);
    const bf16x8 dv = *reinterpret_cast<const bf16x8*>(a.dout + e0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = bf2f(yv[j]);
      d[j] = bf2f(dv[j]);
      r[j] = 0.f;
    }
    if (a.res) {
      const bf16x8 rv = *reinterpret_cast<const bf16x8*>(a.res + e0);
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = bf2f(rv[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = e0 + j < n;
      v[j] = ok ? bf2f(a.y[e0 + j]) : 0.f;
      d[j] = ok ? bf2f(a.dout[e0 + j]) : 0.f;
      r[j] = (ok && a.res) ? bf2f(a.res[e0 + j]) : 0.f;
    }
  }
  if (a.drop.rate > 0.f) drop8(a.drop, e0, ks);
  int c = (int)((unsigned)e0 % (unsigned)a.C);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float z = v[j] * sc[c] + sf[c] + r[j];
    float g = d[j];
    if (a.drop.rate > 0.f) g *= ks[j];
    if (a.relu && !(z > 0.f)) g = 0.f;
    dz[j] = (e0 + j < n) ? g : 0.f;
    xh[j] = (v[j] - mu[c]) * rs[c];
    if (++c == a.C) c = 0;
  }
}

__device__ __forceinline__ void bn_bwd_prologue(const BnBwdArgs& a, float* sc, float* sf, float* mu, float* rs) {
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    if (a.mode == 1) {
      const float mean = a.saved[c], rstd = a.saved[a.C + c];
      const float g = a.gamma ? a.gamma[c] : 1.f;
      sc[c] = g * rstd;
      sf[c] = (a.beta ? a.beta[c] : 0.f) - mean * g * rstd;
      mu[c] = mean;
      rs[c] = rstd;
    } else {
      sc[c] = 1.f;
      sf[c] = 0.f;
      mu[c] = 0.f;
      rs[c] = 1.f;
    }
  }
}

constexpr int kMaxCB = 1024;

__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(BnBwdArgs a) {
  __shared__ float sc[kMaxCB], sf[kMaxCB], mu[kMaxCB], rs[kMaxCB], s1[kMaxCB], s2[kMaxCB];
  bn_bwd_prologue(a, sc, sf, mu, rs);
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) s1[c] = s2[c] = 0.f;
  __syncthreads();
  const long long n = a.R * a.C;
  const long long nchunk = (n + 7) / 8;
  const bool vec = (n % 8) == 0;
  // When the grid stride is a multiple of C (host picks such grids) every thread always sees the
  // same 8 channels: accumulate in registers and touch LDS once at the end.
  const long long first = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 8;
  const bool fixed = ((long long)gridDim.x * blockDim.x * 8) % a.C == 0;
  float r1[8], r2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r1[j] = r2[j] = 0.f;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < nchunk;
       q += (long long)gridDim.x * blockDim.x) {
    const long long e0 = q * 8;
    float dz[8], xh[8];
    bn_dz8(a, sc, sf, mu, rs, e0, n, vec, dz, xh);
    if (fixed) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        r1[j] += dz[j];
        r2[j] += dz[j] * xh[j];
      }
    } else {
      int c = (int)((unsigned)e0 % (unsigned)a.C);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        atomicAdd(&s1[c], dz[j]);
        atomicAdd(&s2[c], dz[j] * xh[j]);
        if (++c == a.C) c = 0;
      }
    }
  }
  if (fixed && first < n) {
    int c = (int)((unsigned)first % (unsigned)a.C);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(&s1[c], r1[j]);
      atomicAdd(&s2[c], r2[j]);
      if (++c == a.C) c = 0;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float* ds = a.dstats + (size_t)(blockIdx.x % kStatSlots) * 2 * a.C;
    atomicAdd(&ds[c], s1[c]);
    atomicAdd(&ds[a.C + c], s2[c]);
  }
}

// Deterministic mode: dstats[p][0|1][c] = sum dz, sum dz*xhat over rows p (mod kStatSlots), in row order,
// plain stores (every slot written); one channel per thread, 4 row lanes summed in a fixed order.
__global__ __launch_bounds__(256) void bn_bwd_reduce_det_kernel(BnBwdArgs a) {
  __shared__ float sc[kMaxCB], sf[kMaxCB], mu[kMaxCB], rs[kMaxCB];
  __shared__ double red[2][4][64];
  bn_bwd_prologue(a, sc, sf, mu, rs);
  __syncthreads();
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6, c = blockIdx.x * 64 + cl, p = blockIdx.y;
  double s1 = 0.0, s2 = 0.0;
  if (c < a.C)
    for (long long r = p + (long long)kStatSlots * rl; r < a.R; r += 4LL * kStatSlots) {
      const long long e = r * a.C + c;
      const float v = bf2f(a.y[e]);
      const float z = v * sc[c] + sf[c] + (a.res ? bf2f(a.res[e]) : 0.f);
      float g = bf2f(a.dout[e]);
      if (a.drop.rate > 0.f) g *= drop1(a.drop, e);
      if (a.relu && !(z > 0.f)) g = 0.f;
      s1 += g;
      s2 += (double)(g * ((v - mu[c]) * rs[c]));
    }
  red[0][rl][cl] = s1;
  red[1][rl][cl] = s2;
  __syncthreads();
  if (rl == 0 && c < a.C) {
    float* ds = a.dstats + (size_t)p * 2 * a.C;
    ds[c] = (float)((red[0][0][cl] + red[0][1][cl]) + (red[0][2][cl] + red[0][3][cl]));
    ds[a.C + c] = (float)((red[1][0][cl] + red[1][1][cl]) + (red[1][2][cl] + red[1][3][cl]));
  }
}

// Narrow layers (C <= CM, C % 8 != 0: Model B's 6 / 12 channel BNs): one thread per ROW keeps all
// C channels' partial sums in registers (no per-element channel arithmetic, no LDS atomics); the
// block folds them with DPP row reductions and lands 2C global atomics.  Batch-statistics mode
// without dropout only (the general kernel covers the rest).
template <int CM>
__global__ __launch_bounds__(256) void bn_bwd_reduce_rows_kernel(BnBwdArgs a) {
  __shared__ float red[4][2 * CM];
  const int C = a.C;
  float sc[CM], sf[CM], mu[CM], rs[CM], r1[CM], r2[CM];
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    const bool ok = c < C;
    mu[c] = ok ? a.saved[c] : 0.f;
    rs[c] = ok ? a.saved[C + c] : 0.f;
    const float g = (ok && a.gamma) ? a.gamma[c] : 1.f;
    sc[c] = g * rs[c];
    sf[c] = ((ok && a.beta) ? a.beta[c] : 0.f) - mu[c] * sc[c];
    r1[c] = r2[c] = 0.f;
  }
  for (long long row = blockIdx.x * (long long)blockDim.x + threadIdx.x; row < a.R;
       row += (long long)gridDim.x * blockDim.x) {
    const long long e = row * C;
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      if (c < C) {
        const float v = bf2f(a.y[e + c]);
        const float z = v * sc[c] + sf[c] + (a.res ? bf2f(a.res[e + c]) : 0.f);
        float g = bf2f(a.dout[e + c]);
        if (a.relu && !(z > 0.f)) g = 0.f;
        r1[c] += g;
        r2[c] += g * (v - mu[c]) * rs[c];
      }
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < CM; ++c) {
    if (c < C) {
      const float t1 = rows4_sum(row16_sum(r1[c])), t2 = rows4_sum(row16_sum(r2[c]));
      if (lane == 0) {
        red[wave][c] = t1;
        red[wave][CM + c] = t2;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * C) {
    const int c = threadIdx.x % C, w = threadIdx.x / C;
    const float v = (red[0][w * CM + c] + red[1][w * CM + c]) + (red[2][w * CM + c] + red[3][w * CM + c]);
    atomicAdd(a.dstats + (size_t)(blockIdx.x % kStatSlots) * 2 * C + w * C + c, v);
  }
}

// Few rows (a Dense layer's BN: R = batch, e.g. Model B's BatchNormalization after Dense(200) at batch 128):
// one block per 64 channels, a wave per row quarter walking its rows with 128-byte coalesced loads, the four
// partials folded in LDS and ONE atomic pair per channel (the generic kernel runs 25 blocks with per-element
// LDS atomics).  Batch statistics; dropout masks regenerated per element (drop1).
constexpr int kBnColsRows = 16;  // rows per block (grid y): 4 per wave
__global__ __launch_bounds__(256) void bn_bwd_reduce_cols_kernel(BnBwdArgs a) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int C = a.C;
  float r1 = 0.f, r2 = 0.f;
  if (c < C) {
    const float mu = a.saved[c], rs = a.saved[C + c];
    const float sc = (a.gamma ? a.gamma[c] : 1.f) * rs;
    const float sf = (a.beta ? a.beta[c] : 0.f) - mu * sc;
    const long long r1e = min((long long)(blockIdx.y + 1) * kBnColsRows, a.R);
#pragma unroll
    for (long long row = (long long)blockIdx.y * kBnColsRows + rg; row < r1e; row += 4) {
      const long long e = row * C + c;
      const float v = bf2f(a.y[e]);
      const float z = v * sc + sf + (a.res ? bf2f(a.res[e]) : 0.f);
      float g = bf2f(a.dout[e]);
      if (a.drop.rate > 0.f) g *= drop1(a.drop, e);
      if (a.relu && !(z > 0.f)) g = 0.f;
      r1 += g;
      r2 += g * (v - mu) * rs;
    }
  }
  red[0][rg][lane] = r1;
  red[1][rg][lane] = r2;
  __syncthreads();
  if (rg == 0 && c < C) {
    atomicAdd(&a.dstats[c], (red[0][0][lane] + red[0][1][lane]) + (red[0][2][lane] + red[0][3][lane]));
    atomicAdd(&a.dstats[C + c], (red[1][0][lane] + red[1][1][lane]) + (red[1][2][lane] + red[1][3][lane]));
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(BnBwdArgs a) {
  __shared__ float sc[kMaxCB], sf[kMaxCB], mu[kMaxCB], rs[kMaxCB], k1[kMaxCB], k2[kMaxCB];
  bn_bwd_prologue(a, sc, sf, mu, rs);
  const float invR = 1.f / (float)a.R;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    if (a.mode == 1) {
      float sdz = 0.f, sdx = 0.f;
      for (int sl = 0; sl < kStatSlots; ++sl) {
        sdz += a.dstats[sl * 2 * a.C + c];
        sdx += a.dstats[sl * 2 * a.C + a.C + c];
      }
      k1[c] = sdz * invR;
      k2[c] = sdx * invR;
      if (blockIdx.x == 0) {
        if (a.dbeta) a.dbeta[c] += sdz;
        if (a.dgamma) a.dgamma[c] += sdx;
      }
    } else {
      k1[c] = k2[c] = 0.f;
    }
    if (blockIdx.x == 0 && a.zero_fwd) {
      for (int sl = 0; sl < kStatSlots; ++sl) {
        a.zero_fwd[sl * 2 * a.C + c] = 0.0;
        a.zero_fwd[sl * 2 * a.C + a.C + c] = 0.0;
      }
    }
  }
  __syncthreads();
  const long long n = a.R * a.C;
  const long long nchunk = (n + 7) / 8;
  const bool vec = (n % 8) == 0;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < nchunk;
       q += (long long)gridDim.x * blockDim.x) {
    const long long e0 = q * 8;
    float dz[8], xh[8];
    bn_dz8(a, sc, sf, mu, rs, e0, n, vec, dz, xh);
    int c = (int)((unsigned)e0 % (unsigned)a.C);
    float dx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // mode 0: dx = dz (sc = 1); mode 1: dx = gamma*rstd*(dz - mean(dz) - xhat*mean(dz*xhat))
      dx[j] = sc[c] * (dz[j] - k1[c] - xh[j] * k2[c]);
      if (a.mode == 0) dx[j] = dz[j];
      if (++c == a.C) c = 0;
    }
    if (a.dx) {
      bf16x8 o;
      if (a.dx_accum) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(dx[j] + (e0 + j < n ? bf2f(a.dx[e0 + j]) : 0.f));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(dx[j]);
      }
      if (vec) {
        *reinterpret_cast<bf16x8*>(a.dx + e0) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (e0 + j < n) a.dx[e0 + j] = o[j];
      }
    }
    if (a.dres) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (e0 + j >= n) break;
        const float v = dz[j] + (a.dres_accum ? bf2f(a.dres[e0 + j]) : 0.f);
        a.dres[e0 + j] = f2bf(v);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Channel-tiled BN kernels (C % 8 == 0 and C <= 64 or C % 64 == 0; 16-byte aligned tensors).
// A block owns CG = min(C, 64) channels and a strided set of rows: each thread keeps its 8
// channels' coefficients in registers (no per-element LDS lookups), the per-channel prologue
// touches only CG channels (not all C: the 8 f64 statistic slots of a C=512 layer are 64 KB per
// block otherwise), the reduction ends with 2*CG atomics per block, and U=4 rows are loaded
// before any is used so enough bytes are in flight to cover HBM latency with few blocks.
struct BnTile {
  int cg, tpr, rp, g, c0;  // channels per group, threads per row, rows per pass, group, first channel
  long long row, stride;   // first row of this thread, row stride
  bool active;
};

__device__ __forceinline__ BnTile bn_tile(int C) {
  BnTile t;
  t.cg = C < 64 ? C : 64;
  t.tpr = t.cg >> 3;
  t.rp = blockDim.x / t.tpr;
  const int ng = C / t.cg;
  t.g = blockIdx.x % ng;
  const int rb = blockIdx.x / ng, nrb = gridDim.x / ng;
  const int tid = threadIdx.x;
  t.active = tid < t.rp * t.tpr;
  t.c0 = t.g * t.cg + (tid % t.tpr) * 8;
  t.row = (long long)rb * t.rp + tid / t.tpr;
  t.stride = (long long)nrb * t.rp;
  return t;
}

__device__ __forceinline__ void ld8(const bf16* p, float* v) {
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(x[j]);
}

__device__ __forceinline__ void st8(bf16* p, const float* v) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
  *reinterpret_cast<bf16x8*>(p) = o;
}

constexpr int kBnU = 4;

__global__ __launch_bounds__(256) void bn_fwd_tiled_kernel(BnFwdArgs a) {
  __shared__ float lsc[64], lsf[64];
  const int C = a.C;
  const BnTile t = bn_tile(C);
  if (threadIdx.x < t.cg) {
    const int c = t.g * t.cg + threadIdx.x;
    const bool first = blockIdx.x < C / t.cg;  // row-block 0 of this channel group
    float scale = 1.f, shift = 0.f;
    if (a.mode != 0) {
      float mean, var;
      if (a.mode == 1) {
        double s1 = 0.0, s2 = 0.0;
#pragma unroll
        for (int sl = 0; sl < kStatSlots; ++sl) {
          s1 += a.stats[sl * 2 * C + c];
          s2 += a.stats[sl * 2 * C + C + c];
        }
        const double md = s1 / (double)a.R;
        mean = (float)md;
        var = (float)fmax(s2 / (double)a.R - md * md, 0.0);
      } else {
        mean = a.mmean[c];
        var = a.mvar[c];
      }
      const float rstd = rsqrtf(var + a.eps);
      const float g = a.gamma ? a.gamma[c] : 1.f;
      scale = g * rstd;
      shift = (a.beta ? a.beta[c] : 0.f) - mean * scale;
      if (first && a.mode == 1) {
        a.saved[c] = mean;
        a.saved[C + c] = rstd;
        if (a.mmean) {
          a.mmean[c] = a.mmean[c] * a.momentum + mean * (1.f - a.momentum);
          a.mvar[c] = a.mvar[c] * a.momentum + var * a.bessel * (1.f - a.momentum);
        }
      }
    }
    if (first && a.zero_buf) {
#pragma unroll
      for (int sl = 0; sl < kStatSlots; ++sl) {
        a.zero_buf[sl * 2 * C + c] = 0.f;
        a.zero_buf[sl * 2 * C + C + c] = 0.f;
      }
    }
    lsc[threadIdx.x] = scale;
    lsf[threadIdx.x] = shift;
  }
  __syncthreads();
  if (!t.active) return;
  const int lc = t.c0 - t.g * t.cg;
  float sc[8], sf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = lsc[lc + j];
    sf[j] = lsf[lc + j];
  }
  const long long nr = t.row < a.R ? (a.R - t.row + t.stride - 1) / t.stride : 0;
  for (long long i = 0; i < nr; i += kBnU) {
    bf16x8 v[kBnU], r[kBnU];
#pragma unroll
    for (int u = 0; u < kBnU; ++u) {
      if (i + u < nr) {
        const long long e = (t.row + (i + u) * t.stride) * C + t.c0;
        v[u] = *reinterpret_cast<const bf16x8*>(a.y + e);
        if (a.res) r[u] = *reinterpret_cast<const bf16x8*>(a.res + e);
      }
    }
#pragma unroll
    for (int u = 0; u < kBnU; ++u) {
      if (i + u < nr) {
        const long long e = (t.row + (i + u) * t.stride) * C + t.c0;
        float ks[8];
        if (a.drop.rate > 0.f) drop8(a.drop, e, ks);
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float z = bf2f(v[u][j]) * sc[j] + sf[j];
          if (a.res) z += bf2f(r[u][j]);
          if (a.relu) z = fmaxf(z, 0.f);
          if (a.drop.rate > 0.f) z *= ks[j];
          o[j] = z;
        }
        st8(a.out + e, o);
      }
    }
  }
}

// per-thread coefficients of the tiled backward: sc/sf rebuild z, mu/rs give xhat
struct BnBwdRegs {
  float sc[8], sf[8], mu[8], rs[8];
};

__device__ __forceinline__ void bn_dz8_regs(const BnBwdArgs& a, const BnBwdRegs& k, const bf16x8& yv,
                                            const bf16x8& dv, const bf16x8& rv, long long e, float* dz, float* xh) {
  float ks[8];
  if (a.drop.rate > 0.f) drop8(a.drop, e, ks);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = bf2f(yv[j]);
    const float z = v * k.sc[j] + k.sf[j] + bf2f(rv[j]);
    float g = bf2f(dv[j]);
    if (a.drop.rate > 0.f) g *= ks[j];
    if (a.relu && !(z > 0.f)) g = 0.f;
    dz[j] = g;
    xh[j] = (v - k.mu[j]) * k.rs[j];
  }
}

__device__ __forceinline__ void bn_bwd_tiled_prologue(const BnBwdArgs& a, const BnTile& t, float* l) {
  // l: [4][64] sc, sf, mu, rs of the block's channel group
  if (threadIdx.x < t.cg) {
    const int c = t.g * t.cg + threadIdx.x;
    float sc = 1.f, sf = 0.f, mu = 0.f, rs = 1.f;
    if (a.mode == 1) {
      mu = a.saved[c];
      rs = a.saved[a.C + c];
      const float g = a.gamma ? a.gamma[c] : 1.f;
      sc = g * rs;
      sf = (a.beta ? a.beta[c] : 0.f) - mu * sc;
    }
    l[threadIdx.x] = sc;
    l[64 + threadIdx.x] = sf;
    l[128 + threadIdx.x] = mu;
    l[192 + threadIdx.x] = rs;
  }
}

__device__ __forceinline__ void bn_bwd_regs(const BnTile& t, const float* l, BnBwdRegs& k) {
  const int lc = t.c0 - t.g * t.cg;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k.sc[j] = l[lc + j];
    k.sf[j] = l[64 + lc + j];
    k.mu[j] = l[128 + lc + j];
    k.rs[j] = l[192 + lc + j];
  }
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_tiled_kernel(BnBwdArgs a) {
  __shared__ float l[256];
  __shared__ float red[2][2048];  // [rp][cg] partials (rp * cg = 256 / tpr * 8 * tpr = 2048)
  const BnTile t = bn_tile(a.C);
  bn_bwd_tiled_prologue(a, t, l);
  __syncthreads();
  float r1[8], r2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r1[j] = r2[j] = 0.f;
  if (t.active) {
    BnBwdRegs k;
    bn_bwd_regs(t, l, k);
    const long long nr = t.row < a.R ? (a.R - t.row + t.stride - 1) / t.stride : 0;
    for (long long i = 0; i < nr; i += kBnU) {
      bf16x8 v[kBnU], d[kBnU], r[kBnU];
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (i + u < nr) {
          const long long e = (t.row + (i + u) * t.stride) * a.C + t.c0;
          v[u] = *reinterpret_cast<const bf16x8*>(a.y + e);
          d[u] = *reinterpret_cast<const bf16x8*>(a.dout + e);
          if (a.res) {
            r[u] = *reinterpret_cast<const bf16x8*>(a.res + e);
          } else {
            r[u] = zero8();
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kBnU; ++u) {
        if (i + u < nr) {
          const long long e = (t.row + (i + u) * t.stride) * a.C + t.c0;
          float dz[8], xh[8];
          bn_dz8_regs(a, k, v[u], d[u], r[u], e, dz, xh);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            r1[j] += dz[j];
            r2[j] += dz[j] * xh[j];
          }
        }
      }
    }
    const int slot = (int)(threadIdx.x / t.tpr) * t.cg + (t.c0 - t.g * t.cg);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][slot + j] = r1[j];
      red[1][slot + j] = r2[j];
    }
  }
  __syncthreads();
  // 256 threads fold the rp rows: thread -> (channel tid % cg, part tid / cg)
  const int nparts = blockDim.x / t.cg;
  const int c = threadIdx.x % t.cg, part = threadIdx.x / t.cg;
  float s1 = 0.f, s2 = 0.f;
  if (part < nparts)
    for (int row = part; row < t.rp; row += nparts) {
      s1 += red[0][row * t.cg + c];
      s2 += red[1][row * t.cg + c];
    }
  __syncthreads();
  float* fold = &red[0][0];  // reuse: [2][256]
  fold[threadIdx.x] = part < nparts ? s1 : 0.f;
  fold[256 + threadIdx.x] = part < nparts ? s2 : 0.f;
  __syncthreads();
  if (threadIdx.x < t.cg) {
    float a1 = 0.f, a2 = 0.f;
    for (int p = 0; p < nparts; ++p) {
      a1 += fold[p * t.cg + threadIdx.x];
      a2 += fold[256 + p * t.cg + threadIdx.x];
    }
    float* ds = a.dstats + (size_t)(blockIdx.x % kStatSlots) * 2 * a.C;
    const int cc = t.g * t.cg + threadIdx.x;
    atomicAdd(&ds[cc], a1);
    atomicAdd(&ds[a.C + cc], a2);
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_tiled_kernel(BnBwdArgs a) {
  __shared__ float l[384];  // sc, sf, mu, rs, k1, k2
  const BnTile t = bn_tile(a.C);
  bn_bwd_tiled_prologue(a, t, l);
  if (threadIdx.x < t.cg) {
    const int c = t.g * t.cg + threadIdx.x;
    const bool first = blockIdx.x < a.C / t.cg;
    float k1 = 0.f, k2 = 0.f;
    if (a.mode == 1) {
      float sdz = 0.f, sdx = 0.f;
#pragma unroll
      for (int sl = 0; sl < kStatSlots; ++sl) {
        sdz += a.dstats[sl * 2 * a.C + c];
        sdx += a.dstats[sl * 2 * a.C + a.C + c];
      }
      k1 = sdz / (float)a.R;
      k2 = sdx / (float)a.R;
      if (first) {
        if (a.dbeta) a.dbeta[c] += sdz;
        if (a.dgamma) a.dgamma[c] += sdx;
      }
    }
    if (first && a.zero_fwd) {
#pragma unroll
      for (int sl = 0; sl < kStatSlots; ++sl) {
        a.zero_fwd[sl * 2 * a.C + c] = 0.0;
        a.zero_fwd[sl * 2 * a.C + a.C + c] = 0.0;
      }
    }
    l[256 + threadIdx.x] = k1;
    l[320 + threadIdx.x] = k2;
  }
  __syncthreads();
  if (!t.active) return;
  BnBwdRegs k;
  bn_bwd_regs(t, l, k);
  const int lc = t.c0 - t.g * t.cg;
  float k1[8], k2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k1[j] = l[256 + lc + j];
    k2[j] = l[320 + lc + j];
  }
  const long long nr = t.row < a.R ? (a.R - t.row + t.stride - 1) / t.stride : 0;
  constexpr int U = 2;  // 3-5 streams per row: fewer rows in flight keep the VGPR count low
  for (long long i = 0; i < nr; i += U) {
    bf16x8 v[U], d[U], r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i + u < nr) {
        const long long e = (t.row + (i + u) * t.stride) * a.C + t.c0;
        v[u] = *reinterpret_cast<const bf16x8*>(a.y + e);
        d[u] = *reinterpret_cast<const bf16x8*>(a.dout + e);
        if (a.res) {
          r[u] = *reinterpret_cast<const bf16x8*>(a.res + e);
        } else {
          r[u] = zero8();
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (i + u < nr) {
        const long long e = (t.row + (i + u) * t.stride) * a.C + t.c0;
        float dz[8], xh[8], dx[8];
        bn_dz8_regs(a, k, v[u], d[u], r[u], e, dz, xh);
#pragma unroll
        for (int j = 0; j < 8; ++j) dx[j] = a.mode == 1 ? k.sc[j] * (dz[j] - k1[j] - xh[j] * k2[j]) : dz[j];
        if (a.dx) {
          if (a.dx_accum) {
            float o[8];
            ld8(a.dx + e, o);
#pragma unroll
            for (int j = 0; j < 8; ++j) dx[j] += o[j];
          }
          st8(a.dx + e, dx);
        }
        if (a.dres) {
          if (a.dres_accum) {
            float o[8];
            ld8(a.dres + e, o);
#pragma unroll
            for (int j = 0; j < 8; ++j) dz[j] += o[j];
          }
          st8(a.dres + e, dz);
        }
      }
    }
  }
}

// rows per block: target `blocks` blocks in total, at least kBnU rows per thread when there is work
static inline int bn_tiled_grid(long long R, int C, int blocks) {
  const int cg = C < 64 ? C : 64, tpr = cg / 8, rp = 256 / tpr, ng = C / cg;
  long long nrb = (R + rp - 1) / rp;            // one row per thread
  long long want = (blocks + ng - 1) / ng;
  if (nrb > want) nrb = want;
  if (nrb < 1) nrb = 1;
  return (int)(nrb * ng);
}

// ---------------------------------------------------------------------------------------
// bias / ReLU backward of a Conv2D/Dense with a fused activation: dz = dout*(out>0),
// dbias[c] += sum_rows dz.
__global__ __launch_bounds__(256) void act_bwd_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ out,
                                                      long long R, int C, int relu, bf16* __restrict__ dz,
                                                      float* __restrict__ dbias) {
  __shared__ float s1[kMaxCB];
  for (int c = threadIdx.x; c < C; c += blockDim.x) s1[c] = 0.f;
  __syncthreads();
  const long long n = R * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    float g = bf2f(dout[e]);
    if (relu && !(bf2f(out[e]) > 0.f)) g = 0.f;
    if (dz) dz[e] = f2bf(g);
    if (dbias) atomicAdd(&s1[(int)((unsigned)e % (unsigned)C)], g);
  }
  if (!dbias) return;
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) atomicAdd(&dbias[c], s1[c]);
}

// ---------------------------------------------------------------------------------------
// Max pooling (NHWC) with the window argmax stored as one byte per output.
struct PoolArgs {
  const bf16* x;
  bf16* y;
  unsigned char* idx;
  const bf16* dy;
  bf16* dx;
  int dx_accum;
  Geo g;  // C = channels, Co unused, KH/KW window, sh/sw strides, pt/pl pads
};

__global__ __launch_bounds__(256) void maxpool_fwd_kernel(PoolArgs a) {
  const Geo& g = a.g;
  const long long n = (long long)g.B * g.Ho * g.Wo * g.C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const unsigned ue = (unsigned)e;
    const int c = (int)(ue % (unsigned)g.C);
    unsigned t = ue / (unsigned)g.C;
    const int ow = (int)(t % (unsigned)g.Wo);
    t /= (unsigned)g.Wo;
    const int oh = (int)(t % (unsigned)g.Ho);
    const int b = (int)(t / (unsigned)g.Ho);
    float best = -INFINITY;
    int bi = 0;
    for (int i = 0; i < g.KH; ++i) {
      const int ih = oh * g.sh - g.pt + i;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int j = 0; j < g.KW; ++j) {
        const int iw = ow * g.sw - g.pl + j;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        const float v = bf2f(a.x[(((long long)b * g.H + ih) * g.W + iw) * g.C + c]);
        if (v > best) {
          best = v;
          bi = i * g.KW + j;
        }
      }
    }
    a.y[e] = f2bf(best);
    if (a.idx) a.idx[e] = (unsigned char)bi;
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(PoolArgs a) {
  const Geo& g = a.g;
  const long long n = (long long)g.B * g.H * g.W * g.C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const unsigned ue = (unsigned)e;
    const int c = (int)(ue % (unsigned)g.C);
    unsigned t = ue / (unsigned)g.C;
    const int iw = (int)(t % (unsigned)g.W);
    t /= (unsigned)g.W;
    const int ih = (int)(t % (unsigned)g.H);
    const int b = (int)(t / (unsigned)g.H);
    float s = 0.f;
    const int ty = ih + g.pt, tx = iw + g.pl;
    const int oh_lo = ty >= g.KH ? (ty - g.KH) / g.sh + 1 : 0, oh_hi = min(g.Ho - 1, ty / g.sh);
    const int ow_lo = tx >= g.KW ? (tx - g.KW) / g.sw + 1 : 0, ow_hi = min(g.Wo - 1, tx / g.sw);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int i = ty - oh * g.sh;
      if (i < 0 || i >= g.KH) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int j = tx - ow * g.sw;
        if (j < 0 || j >= g.KW) continue;
        const long long o = (((long long)b * g.Ho + oh) * g.Wo + ow) * g.C + c;
        if (a.idx[o] == (unsigned char)(i * g.KW + j)) s += bf2f(a.dy[o]);
      }
    }
    if (a.dx_accum) s += bf2f(a.dx[e]);
    a.dx[e] = f2bf(s);
  }
}

// Channel-vectorised max pooling (C % 8 == 0): one thread per (pixel, 8 channels); index math
// once per thread, 16-byte loads/stores, the 8 argmax bytes as one 8-byte word.
__global__ __launch_bounds__(256) void maxpool_fwd8_kernel(PoolArgs a) {
  const Geo& g = a.g;
  const int C8 = g.C >> 3;
  const int n = g.B * g.Ho * g.Wo * C8;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c8 = e % C8;
    int t = e / C8;
    const int ow = t % g.Wo;
    t /= g.Wo;
    const int oh = t % g.Ho;
    const int b = t / g.Ho;
    float best[8];
    unsigned char bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    for (int i = 0; i < g.KH; ++i) {
      const int ih = oh * g.sh - g.pt + i;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int jj = 0; jj < g.KW; ++jj) {
        const int iw = ow * g.sw - g.pl + jj;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(a.x + ((((long long)b * g.H + ih) * g.W + iw) * g.C + c8 * 8));
        const unsigned char w = (unsigned char)(i * g.KW + jj);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(v[j]);
          if (f > best[j]) {
            best[j] = f;
            bi[j] = w;
          }
        }
      }
    }
    bf16x8 o;
    unsigned long long packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(best[j]);
      packed |= (unsigned long long)bi[j] << (8 * j);
    }
    *reinterpret_cast<bf16x8*>(a.y + (long long)e * 8) = o;
    if (a.idx) *reinterpret_cast<unsigned long long*>(a.idx + (long long)e * 8) = packed;
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd8_kernel(PoolArgs a) {
  const Geo& g = a.g;
  const int C8 = g.C >> 3;
  const int n = g.B * g.H * g.W * C8;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c8 = e % C8;
    int t = e / C8;
    const int iw = t % g.W;
    t /= g.W;
    const int ih = t % g.H;
    const int b = t / g.H;
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
    const int ty = ih + g.pt, tx = iw + g.pl;
    const int oh_lo = ty >= g.KH ? (ty - g.KH) / g.sh + 1 : 0, oh_hi = min(g.Ho - 1, ty / g.sh);
    const int ow_lo = tx >= g.KW ? (tx - g.KW) / g.sw + 1 : 0, ow_hi = min(g.Wo - 1, tx / g.sw);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int i = ty - oh * g.sh;
      if (i < 0 || i >= g.KH) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int jj = tx - ow * g.sw;
        if (jj < 0 || jj >= g.KW) continue;
        const long long o = ((((long long)b * g.Ho + oh) * g.Wo + ow) * g.C + c8 * 8);
        const unsigned long long id = *reinterpret_cast<const unsigned long long*>(a.idx + o);
        const bf16x8 d = *reinterpret_cast<const bf16x8*>(a.dy + o);
        const unsigned w = (unsigned)(i * g.KW + jj);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((id >> (8 * j)) & 0xFF) == w) s[j] += bf2f(d[j]);
      }
    }
    bf16x8* q = reinterpret_cast<bf16x8*>(a.dx + (long long)e * 8);
    bf16x8 o;
    if (a.dx_accum) {
      const bf16x8 prev = *q;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(s[j] + bf2f(prev[j]));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(s[j]);
    }
    *q = o;
  }
}

// MaxPool backward when every input pixel is covered by at most 2 x 2 windows (3x3/2, 2x2/2, ...):
// one grid row per input row (b, ih) so the output-row candidates are block-uniform scalars, and a
// thread issues all (up to 4) argmax-byte + dy loads before using any of them.
__global__ __launch_bounds__(256) void maxpool_bwd8_w2_kernel(PoolArgs a) {
  const Geo& g = a.g;
  const int C8 = g.C >> 3;
  const int row = blockIdx.y;
  const int b = row / g.H, ih = row - b * g.H;
  const int ty = ih + g.pt;
  const int oh_lo = ty >= g.KH ? (ty - g.KH) / g.sh + 1 : 0, oh_hi = min(g.Ho - 1, ty / g.sh);
  const int n = g.W * C8;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int iw = e / C8, c8 = e - iw * C8;
    const int tx = iw + g.pl;
    const int ow_lo = tx >= g.KW ? (tx - g.KW) / g.sw + 1 : 0, ow_hi = min(g.Wo - 1, tx / g.sw);
    unsigned long long id[4];
    bf16x8 d[4];
    unsigned wi[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = oh_lo + (q >> 1), ow = ow_lo + (q & 1);
      id[q] = ~0ull;  // byte 0xFF never equals a window index (host: KH*KW < 255)
      wi[q] = 0;
      if (oh <= oh_hi && ow <= ow_hi) {
        const long long o = (((long long)b * g.Ho + oh) * g.Wo + ow) * g.C + c8 * 8;
        id[q] = *reinterpret_cast<const unsigned long long*>(a.idx + o);
        d[q] = *reinterpret_cast<const bf16x8*>(a.dy + o);
        wi[q] = (unsigned)((ty - oh * g.sh) * g.KW + (tx - ow * g.sw));
      }
    }
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (((id[q] >> (8 * j)) & 0xFF) == wi[q]) s[j] += bf2f(d[q][j]);
    bf16x8* out = reinterpret_cast<bf16x8*>(a.dx + (((long long)row * g.W + iw) * g.C + c8 * 8));
    bf16x8 o;
    if (a.dx_accum) {
      const bf16x8 prev = *out;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(s[j] + bf2f(prev[j]));
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(s[j]);
    }
    *out = o;
  }
}

// Pair variant of the above for windows where two horizontally adjacent input pixels see at most
// 2 output columns together ((KW + sw) / sw <= 2: 3x3/2, 2x2/2): a thread owns input columns
// (2t, 2t+1), so the <= 4 argmax + dy loads serve two outputs (half the load instructions).
__global__ __launch_bounds__(256) void maxpool_bwd8_w2p_kernel(PoolArgs a) {
  const Geo& g = a.g;
  const int C8 = g.C >> 3;
  const int row = blockIdx.y;
  const int b = row / g.H, ih = row - b * g.H;
  const int ty = ih + g.pt;
  const int oh_lo = ty >= g.KH ? (ty - g.KH) / g.sh + 1 : 0, oh_hi = min(g.Ho - 1, ty / g.sh);
  const int W2 = (g.W + 1) >> 1;
  const int n = W2 * C8;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int iw2 = e / C8, c8 = e - iw2 * C8;
    const int iw0 = 2 * iw2;
    const int tx0 = iw0 + g.pl;
    const int ow_lo = tx0 >= g.KW ? (tx0 - g.KW) / g.sw + 1 : 0, ow_hi = min(g.Wo - 1, (tx0 + 1) / g.sw);
    unsigned long long id[4];
    bf16x8 d[4];
    unsigned wi0[4], wi1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int oh = oh_lo + (q >> 1), ow = ow_lo + (q & 1);
      id[q] = ~0ull;  // byte 0xFF never equals a window index (host: KH*KW < 255)
      wi0[q] = wi1[q] = 0x100u;  // matches no argmax byte (0xFF included: id[q] of a missing window)
      d[q] = zero8();
      if (oh <= oh_hi && ow <= ow_hi) {
        const long long o = (((long long)b * g.Ho + oh) * g.Wo + ow) * g.C + c8 * 8;
        id[q] = *reinterpret_cast<const unsigned long long*>(a.idx + o);
        d[q] = *reinterpret_cast<const bf16x8*>(a.dy + o);
        const int i = ty - oh * g.sh, j0 = tx0 - ow * g.sw;
        if (j0 >= 0 && j0 < g.KW) wi0[q] = (unsigned)(i * g.KW + j0);
        if (j0 + 1 >= 0 && j0 + 1 < g.KW) wi1[q] = (unsigned)(i * g.KW + j0 + 1);
      }
    }
    float s0[8], s1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned w = (unsigned)((id[q] >> (8 * j)) & 0xFF);
        const float v = bf2f(d[q][j]);
        if (w == wi0[q]) s0[j] += v;
        if (w == wi1[q]) s1[j] += v;
      }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int iw = iw0 + h;
      if (iw >= g.W) break;
      const float* sv = h ? s1 : s0;
      bf16x8* out = reinterpret_cast<bf16x8*>(a.dx + (((long long)row * g.W + iw) * g.C + c8 * 8));
      bf16x8 o;
      if (a.dx_accum) {
        const bf16x8 prev = *out;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(sv[j] + bf2f(prev[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(sv[j]);
      }
      *out = o;
    }
  }
}

// ---------------------------------------------------------------------------------------
// BatchNorm + ReLU + MaxPool forward in one pass (the ResNet stem: conv1_bn -> conv1_relu -> pool1).
// The BN output (the largest activation of the network, 112x112x64 per image) is never stored: each
// pooled output reads its window of the conv output y, normalises + rectifies every element exactly
// as bn_fwd would store it (bf16-rounded), and keeps the max and its window index for the pool's
// backward.  The BN backward recomputes z from y, so nothing downstream needs the BN output.
__global__ __launch_bounds__(256) void bn_relu_maxpool_fwd_kernel(BnFwdArgs a, PoolArgs pa) {
  __shared__ float sc[kMaxC], sf[kMaxC];
  const int C = a.C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mean, var;
    if (a.mode == 1) {
      double s1 = 0.0, s2 = 0.0;
      for (int sl = 0; sl < kStatSlots; ++sl) {
        s1 += a.stats[sl * 2 * C + c];
        s2 += a.stats[sl * 2 * C + C + c];
      }
      const double md = s1 / (double)a.R;
      mean = (float)md;
      var = (float)fmax(s2 / (double)a.R - md * md, 0.0);
    } else {
      mean = a.mmean[c];
      var = a.mvar[c];
    }
    const float rstd = rsqrtf(var + a.eps);
    const float scale = (a.gamma ? a.gamma[c] : 1.f) * rstd;
    if (blockIdx.x == 0 && a.mode == 1) {
      a.saved[c] = mean;
      a.saved[C + c] = rstd;
      if (a.mmean) {
        a.mmean[c] = a.mmean[c] * a.momentum + mean * (1.f - a.momentum);
        a.mvar[c] = a.mvar[c] * a.momentum + var * a.bessel * (1.f - a.momentum);
      }
    }
    if (blockIdx.x == 0 && a.zero_buf) {
      for (int sl = 0; sl < kStatSlots; ++sl) {
        a.zero_buf[sl * 2 * C + c] = 0.f;
        a.zero_buf[sl * 2 * C + C + c] = 0.f;
      }
    }
    sc[c] = scale;
    sf[c] = (a.beta ? a.beta[c] : 0.f) - mean * scale;
  }
  __syncthreads();
  const Geo& g = pa.g;
  const int C8 = C >> 3;
  const int n = g.B * g.Ho * g.Wo * C8;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c8 = e % C8;
    int t = e / C8;
    const int ow = t % g.Wo;
    t /= g.Wo;
    const int oh = t % g.Ho;
    const int b = t / g.Ho;
    float k[8], s[8], best[8];
    unsigned char bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      k[j] = sc[c8 * 8 + j];
      s[j] = sf[c8 * 8 + j];
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    auto take = [&](const bf16x8& v, unsigned char w) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // the value bn_fwd would store: bf16(relu(y * scale + shift))
        const float f = bf2f(f2bf(fmaxf(fmaf(bf2f(v[j]), k[j], s[j]), 0.f)));
        if (f > best[j]) {
          best[j] = f;
          bi[j] = w;
        }
      }
    };
    if (g.KH == 3 && g.KW == 3) {
      // the ResNet stem's 3x3 window: all 9 loads issued before the first comparison (one memory round trip, not
      // nine), then taken in the same (i, jj) order
      bf16x8 v[9];
      bool ok[9];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
          const int ih = oh * g.sh - g.pt + i, iw = ow * g.sw - g.pl + jj;
          ok[i * 3 + jj] = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          v[i * 3 + jj] = ok[i * 3 + jj]
                              ? *reinterpret_cast<const bf16x8*>(a.y + ((((long long)b * g.H + ih) * g.W + iw) * C + c8 * 8))
                              : zero8();
        }
#pragma unroll
      for (int w = 0; w < 9; ++w)
        if (ok[w]) take(v[w], (unsigned char)w);
    } else {
      for (int i = 0; i < g.KH; ++i) {
        const int ih = oh * g.sh - g.pt + i;
        if ((unsigned)ih >= (unsigned)g.H) continue;
        for (int jj = 0; jj < g.KW; ++jj) {
          const int iw = ow * g.sw - g.pl + jj;
          if ((unsigned)iw >= (unsigned)g.W) continue;
          take(*reinterpret_cast<const bf16x8*>(a.y + ((((long long)b * g.H + ih) * g.W + iw) * C + c8 * 8)),
               (unsigned char)(i * g.KW + jj));
        }
      }
    }
    bf16x8 o;
    unsigned long long packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(best[j]);
      packed |= (unsigned long long)bi[j] << (8 * j);
    }
    *reinterpret_cast<bf16x8*>(pa.y + (long long)e * 8) = o;
    if (pa.idx) *reinterpret_cast<unsigned long long*>(pa.idx + (long long)e * 8) = packed;
  }
}

// Backward of the fused stem: BN backward whose output gradient is the MaxPool's input gradient,
// gathered on the fly from the pooled gradient + argmax bytes (as maxpool_bwd8_w2p_kernel does, <= 2 x 2
// windows per pixel) instead of being stored and re-read.  PASS 0: per-channel sums of dz and dz * xhat
// (dz = gathered gradient, bf16-rounded as the pool backward would store it, masked by the ReLU) into
// dstats; PASS 1: dx = scale * (dz - mean(dz) - xhat * mean(dz * xhat)) (+ dbeta / dgamma, zero the
// forward statistics), as bn_bwd_apply_tiled_kernel.  A thread owns input pixels (2t, 2t+1) of one row
// and 8 channels; 256 % (C / 8) == 0 keeps its channels fixed over the grid stride.
constexpr int kBnPoolRow = 4096;  // elements of one staged pooled row (Wo * C)
// dynamic LDS of bn_pool_bwd_kernel: [6][C] coefficients, then PASS 0's fold [256][16] f32 aliased with the
// two staged pooled rows (dy bf16 + argmax bytes) — sized per launch so small layers keep more blocks per CU
static size_t bn_pool_bwd_lds(int C, int rowlen) {
  const size_t stage = (size_t)2 * rowlen * 3, fold = 256 * 16 * 4;
  return (size_t)6 * C * 4 + ((stage > fold ? stage : fold) + 15) / 16 * 16;
}
template <int PASS>
__global__ __launch_bounds__(256) void bn_pool_bwd_kernel(BnBwdArgs a, PoolArgs pa) {
  extern __shared__ __attribute__((aligned(16))) float bn_pool_dyn[];
  const int C = a.C;
  float* const l0 = bn_pool_dyn;  // [6][C]: sc, sf, mu, rs, k1, k2
  float* const fold = bn_pool_dyn + ((6 * C + 3) & ~3);
  auto l = [&](int q, int c) -> float& { return l0[q * C + c]; };
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float mu = a.saved[c], rs = a.saved[C + c];
    const float sc = (a.gamma ? a.gamma[c] : 1.f) * rs;
    l(0, c) = sc;
    l(1, c) = (a.beta ? a.beta[c] : 0.f) - mu * sc;
    l(2, c) = mu;
    l(3, c) = rs;
    if (PASS == 1) {
      float sdz = 0.f, sdx = 0.f;
#pragma unroll
      for (int sl = 0; sl < kStatSlots; ++sl) {
        sdz += a.dstats[sl * 2 * C + c];
        sdx += a.dstats[sl * 2 * C + C + c];
      }
      l(4, c) = sdz / (float)a.R;
      l(5, c) = sdx / (float)a.R;
      if (blockIdx.x == 0) {
        if (a.dbeta) a.dbeta[c] += sdz;
        if (a.dgamma) a.dgamma[c] += sdx;
        if (a.zero_fwd)
          for (int sl = 0; sl < kStatSlots; ++sl) {
            a.zero_fwd[sl * 2 * C + c] = 0.0;
            a.zero_fwd[sl * 2 * C + C + c] = 0.0;
          }
      }
    }
  }
  const Geo& g = pa.g;
  const int C8 = C >> 3, W2 = (g.W + 1) >> 1;
  const int c8 = threadIdx.x % C8;
  float k[6][8];
  float r1[8], r2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r1[j] = r2[j] = 0.f;
  const int rowlen = g.Wo * C;  // elements of one pooled row (host: <= kBnPoolRow)
  bf16* const sdy = reinterpret_cast<bf16*>(fold);                              // [2][rowlen]
  unsigned char* const sid = reinterpret_cast<unsigned char*>(sdy + 2 * rowlen);  // [2][rowlen]
  for (int row = blockIdx.x; row < g.B * g.H; row += gridDim.x) {
    const int b = row / g.H, ih = row - b * g.H;
    const int ty = ih + g.pt;
    const int oh_lo = ty >= g.KH ? (ty - g.KH) / g.sh + 1 : 0, oh_hi = min(g.Ho - 1, ty / g.sh);
    __syncthreads();  // coefficients written (first row) / the previous row's gathers done
    if (row == (int)blockIdx.x) {
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) k[q][j] = (PASS == 1 || q < 4) ? l(q, c8 * 8 + j) : 0.f;
    }
    // the <= 2 pooled rows this input row reads: 16-byte coalesced loads of dy and the argmax bytes into LDS
    // (all of a thread's loads issued before any LDS write: one memory latency per row, not one per chunk;
    // rowlen <= kBnPoolRow = 4096 gives <= 2 dy chunks and 1 argmax chunk per thread per pooled row)
    {
      const int nr = oh_hi - oh_lo + 1;
      bf16x8 sv[4];
      uint4 si[2];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = t >> 1, i = threadIdx.x + (t & 1) * 256;
        const long long o = ((long long)b * g.Ho + oh_lo + r) * rowlen;
        sv[t] = (r < nr && i < rowlen / 8) ? *reinterpret_cast<const bf16x8*>(pa.dy + o + i * 8) : zero8();
      }
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const long long o = ((long long)b * g.Ho + oh_lo + r) * rowlen;
        si[r] = (r < nr && (int)threadIdx.x < rowlen / 16) ? *reinterpret_cast<const uint4*>(pa.idx + o + threadIdx.x * 16)
                                                           : uint4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = t >> 1, i = threadIdx.x + (t & 1) * 256;
        if (r < nr && i < rowlen / 8) *reinterpret_cast<bf16x8*>(sdy + r * rowlen + i * 8) = sv[t];
      }
#pragma unroll
      for (int r = 0; r < 2; ++r)
        if (r < nr && (int)threadIdx.x < rowlen / 16) *reinterpret_cast<uint4*>(sid + r * rowlen + threadIdx.x * 16) = si[r];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < W2 * C8; e += blockDim.x) {
      const int iw2 = e / C8;
      const int iw0 = 2 * iw2, tx0 = iw0 + g.pl;
      const int ow_lo = tx0 >= g.KW ? (tx0 - g.KW) / g.sw + 1 : 0, ow_hi = min(g.Wo - 1, (tx0 + 1) / g.sw);
      const long long px0 = (long long)row * g.W + iw0;
      bf16x8 yv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h)
        yv[h] = iw0 + h < g.W ? *reinterpret_cast<const bf16x8*>(a.y + (px0 + h) * C + c8 * 8) : zero8();
      float s0[8], s1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s0[j] = s1[j] = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int oh = oh_lo + (q >> 1), ow = ow_lo + (q & 1);
        if (oh > oh_hi || ow > ow_hi) continue;
        const int lo = (q >> 1) * rowlen + ow * C + c8 * 8;
        const unsigned long long id = *reinterpret_cast<const unsigned long long*>(sid + lo);
        const bf16x8 d = *reinterpret_cast<const bf16x8*>(sdy + lo);
        const int i = ty - oh * g.sh, j0 = tx0 - ow * g.sw;
        const unsigned w0 = (j0 >= 0 && j0 < g.KW) ? (unsigned)(i * g.KW + j0) : 0x100u;
        const unsigned w1 = (j0 + 1 >= 0 && j0 + 1 < g.KW) ? (unsigned)(i * g.KW + j0 + 1) : 0x100u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned w = (unsigned)((id >> (8 * j)) & 0xFF);
          const float v = bf2f(d[j]);
          if (w == w0) s0[j] += v;
          if (w == w1) s1[j] += v;
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (iw0 + h >= g.W) break;
        const float* sv = h ? s1 : s0;
        float dx[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bf2f(yv[h][j]);
          const float z = v * k[0][j] + k[1][j];
          const float dz = (a.relu && !(z > 0.f)) ? 0.f : bf2f(f2bf(sv[j]));  // the pool backward's stored value
          const float xh = (v - k[2][j]) * k[3][j];
          if (PASS == 0) {
            r1[j] += dz;
            r2[j] += dz * xh;
          } else {
            dx[j] = k[0][j] * (dz - k[4][j] - xh * k[5][j]);
          }
        }
        if (PASS == 1) {
          bf16x8* out = reinterpret_cast<bf16x8*>(a.dx + (px0 + h) * C + c8 * 8);
          bf16x8 o;
          if (a.dx_accum) {
            const bf16x8 prev = *out;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = f2bf(dx[j] + bf2f(prev[j]));
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = f2bf(dx[j]);
          }
          *out = o;
        }
      }
    }
  }
  if (PASS == 0) {
    // fold the 256 / C8 threads of each channel octet, then one atomic pair per channel per block
    __syncthreads();  // the staged pooled rows share this LDS
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      fold[threadIdx.x * 16 + j] = r1[j];
      fold[threadIdx.x * 16 + 8 + j] = r2[j];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const int o8 = c >> 3, j = c & 7;
      float a1 = 0.f, a2 = 0.f;
      for (int t = o8; t < 256; t += C8) {
        a1 += fold[t * 16 + j];
        a2 += fold[t * 16 + 8 + j];
      }
      float* ds = a.dstats + (size_t)(blockIdx.x % kStatSlots) * 2 * C;
      atomicAdd(&ds[c], a1);
      atomicAdd(&ds[C + c], a2);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Global average pooling [B,HW,C] -> [B,C] and its backward; zero padding / its crop.
__global__ __launch_bounds__(256) void gap_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B, int HW,
                                                      int C) {
  const long long n = (long long)B * C;
  const float inv = 1.f / (float)HW;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)((unsigned)e % (unsigned)C);
    const long long b = (unsigned)e / (unsigned)C;
    const bf16* p = x + b * HW * C + c;
    float s = 0.f;
    for (int i = 0; i < HW; ++i) s += bf2f(p[(long long)i * C]);
    y[e] = f2bf(s * inv);
  }
}

// 64-channel groups (C % 64 == 0, 16-byte aligned): block (b, group) = 8 threads per 8-channel chunk x 32 pixel
// slices, one 16-byte load per pixel, then a 32-way LDS reduction — every load of the block in flight together
// (the per-element form walks HW serially per thread: 13.4 us for ResNet-18's 64x7x7x512)
__global__ __launch_bounds__(256) void gap_fwd_vec_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int B,
                                                          int HW, int C) {
  __shared__ float part[32][65];
  const int groups = C / 64;
  const int b = blockIdx.x / groups, c0 = (blockIdx.x - b * groups) * 64;
  const int ch = threadIdx.x & 7, sl = threadIdx.x >> 3;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bf16* p = x + (long long)b * HW * C + c0 + ch * 8;
  for (int i = sl; i < HW; i += 32) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(p + (long long)i * C);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += bf2f(v[e]);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[sl][ch * 8 + e] = s[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = 0.f;
#pragma unroll 8
    for (int q = 0; q < 32; ++q) t += part[q][threadIdx.x];
    y[(long long)b * C + c0 + threadIdx.x] = f2bf(t * (1.f / (float)HW));
  }
}

__global__ __launch_bounds__(256) void gap_bwd_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, int B,
                                                      int HW, int C, int accum) {
  const long long n = (long long)B * HW * C;
  const float inv = 1.f / (float)HW;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)((unsigned)e % (unsigned)C);
    const long long b = (unsigned)e / ((unsigned)HW * (unsigned)C);
    float v = bf2f(dy[b * C + c]) * inv;
    if (accum) v += bf2f(dx[e]);
    dx[e] = f2bf(v);
  }
}

// dir 0: y[B,H+t+b,W+l+r,C] = pad(x);  dir 1: dx = crop(dy) (+= when accum)
__global__ __launch_bounds__(256) void pad_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst, Geo g, int dir,
                                                  int accum) {
  // g: H,W input dims; Ho,Wo padded dims; pt,pl offsets
  const long long n = (long long)g.B * g.Ho * g.Wo * g.C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const unsigned ue = (unsigned)e;
    const int c = (int)(ue % (unsigned)g.C);
    unsigned t = ue / (unsigned)g.C;
    const int ow = (int)(t % (unsigned)g.Wo);
    t /= (unsigned)g.Wo;
    const int oh = (int)(t % (unsigned)g.Ho);
    const int b = (int)(t / (unsigned)g.Ho);
    const int ih = oh - g.pt, iw = ow - g.pl;
    const bool in = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
    const long long ie = (((long long)b * g.H + ih) * g.W + iw) * g.C + c;
    if (dir == 0) {
      dst[e] = in ? src[ie] : (bf16)0.0f;
    } else if (in) {
      float v = bf2f(src[e]);
      if (accum) v += bf2f(dst[ie]);
      dst[ie] = f2bf(v);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Softmax cross-entropy over C classes, one wave per row (any C).
struct XentArgs {
  const float* logits;
  long long ldl;
  const int* labels;
  int B, C;
  float scale;
  bf16* dlogits;  // [B][ldd] (softmax - onehot) * scale, or null
  long long ldd;
  float* metrics;  // [4] loss sum, correct, count, 0
  float* probs;    // [B][C] softmax (or logits copy when probs_are_logits)
  int probs_are_logits;
  long long* iterations;
};

// NV > 0: C <= 64 * NV, the row is loaded into registers once (all NV loads in flight together) and the three
// passes (max, sum of exponentials, outputs) run on registers; NV = 0 re-reads the row per pass (any C).
template <int NV>
__global__ __launch_bounds__(256) void xent_kernel(XentArgs a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  __shared__ float part[4][2];
  float loss = 0.f, corr = 0.f;
  const bool ok = row < a.B;
  if (ok) {
    const float* l = a.logits + (long long)row * a.ldl;
    float rv[NV > 0 ? NV : 1];
    if constexpr (NV > 0) {
#pragma unroll
      for (int j = 0; j < NV; ++j) rv[j] = lane + 64 * j < a.C ? l[lane + 64 * j] : -INFINITY;
    }
    auto lv = [&](int j, int c) -> float {
      if constexpr (NV > 0) return rv[j];
      else return l[c];
    };
    const int nit = NV > 0 ? NV : (a.C + 63) / 64;
    float mx = -INFINITY;
    int am = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < nit; ++j) {
      const int c = lane + 64 * j;
      if (c >= a.C) continue;
      const float v = lv(j, c);
      if (v > mx) {
        mx = v;
        am = c;
      }
    }
    // wave argmax (first index of the max)
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
#pragma unroll
    for (int j = 0; j < nit; ++j) {
      const int c = lane + 64 * j;
      if (c < a.C) se += __expf(lv(j, c) - mx);
    }
    se = wave_sum(se);
    const int y = a.labels[row];
    const float lse = mx + __logf(se);
    const float ly = (y >= 0 && y < a.C) ? l[y] : mx;
    loss = lse - ly;
    corr = (am == y) ? 1.f : 0.f;
    const float inv = 1.f / se;
#pragma unroll
    for (int j = 0; j < nit; ++j) {
      const int c = lane + 64 * j;
      if (c >= a.C) continue;
      const float x = lv(j, c);
      const float p = __expf(x - mx) * inv;
      if (a.dlogits) a.dlogits[(long long)row * a.ldd + c] = f2bf((p - (c == y ? 1.f : 0.f)) * a.scale);
      if (a.probs) a.probs[(long long)row * a.C + c] = a.probs_are_logits ? x : p;
    }
  }
  if (lane == 0) {
    part[threadIdx.x >> 6][0] = ok ? loss : 0.f;
    part[threadIdx.x >> 6][1] = ok ? corr : 0.f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float ls = part[0][0] + part[1][0] + part[2][0] + part[3][0];
    const float cs = part[0][1] + part[1][1] + part[2][1] + part[3][1];
    const int cnt = min(4, a.B - (int)blockIdx.x * 4);
    if (a.metrics) {
      atomicAdd(&a.metrics[0], ls);
      atomicAdd(&a.metrics[1], cs);
      atomicAdd(&a.metrics[2], (float)cnt);
    }
    if (a.iterations && blockIdx.x == 0) *a.iterations += 1;
  }
}

// per-channel sum / sum of squares of a [R][C] bf16 tensor (BN after a non-GEMM producer)
__global__ __launch_bounds__(256) void colstats_kernel(const bf16* __restrict__ x, long long R, int C,
                                                       double* __restrict__ stats) {
  __shared__ float s1[kMaxCB], s2[kMaxCB];
  for (int c = threadIdx.x; c < C; c += blockDim.x) s1[c] = s2[c] = 0.f;
  __syncthreads();
  const long long n = R * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float v = bf2f(x[e]);
    const int c = (int)((unsigned)e % (unsigned)C);
    atomicAdd(&s1[c], v);
    atomicAdd(&s2[c], v * v);
  }
  __syncthreads();
  double* st = stats + (size_t)(blockIdx.x % kStatSlots) * 2 * C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    atomicAdd(&st[c], (double)s1[c]);
    atomicAdd(&st[C + c], (double)s2[c]);
  }
}

__global__ __launch_bounds__(256) void cast_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e * 4 < n; e += (long long)gridDim.x * blockDim.x) {
    const long long i = e * 4;
    if (i + 4 <= n) {
      const float4 v = *reinterpret_cast<const float4*>(x + i);
      y[i] = f2bf(v.x);
      y[i + 1] = f2bf(v.y);
      y[i + 2] = f2bf(v.z);
      y[i + 3] = f2bf(v.w);
    } else {
      for (long long j = i; j < n; ++j) y[j] = f2bf(x[j]);
    }
  }
}

// Explicit im2col for convolutions whose input channel count is not a multiple of 8 (the ResNet
// stem, C = 3): out[m][k] = x[b, oh*s-p+kh, ow*s-p+kw, ci] for k = (kh*KW+kw)*C+ci < K, 0 up to Kp
// (Kp = K rounded up to 8), so the GEMM that follows runs the 16-byte vector path on both operands.
// Blocks past the pixel range copy the [Co][K] weight shadow into a [Co][Kp] zero-padded copy.
__global__ __launch_bounds__(256) void im2col_kernel(const bf16* __restrict__ x, Geo g, int Kp,
                                                     bf16* __restrict__ out, const bf16* __restrict__ w_in,
                                                     bf16* __restrict__ w_out, int pix_blocks) {
  const int K = g.KH * g.KW * g.C;
  if ((int)blockIdx.x >= pix_blocks) {  // weight padding blocks
    const int n = g.Co * Kp;
    for (int e = (blockIdx.x - pix_blocks) * blockDim.x + threadIdx.x; e < n;
         e += (gridDim.x - pix_blocks) * blockDim.x) {
      const int co = e / Kp, k = e - co * Kp;
      w_out[e] = k < K ? w_in[co * K + k] : (bf16)0.0f;
    }
    return;
  }
  // (kh, kw, ci) of the first element of every 8-element chunk, once per block (K8 <= 256 chunks)
  __shared__ int tap[256];
  const int K8 = Kp >> 3;
  for (int c = threadIdx.x; c < K8; c += blockDim.x) {
    const int k = c * 8, kc = k / g.C;
    tap[c] = ((kc / g.KW) << 20) | ((kc % g.KW) << 10) | (k - kc * g.C);
  }
  __syncthreads();
  // consecutive threads fill consecutive 16-byte chunks of a patch row (coalesced stores); 32-bit
  // index math throughout (the host checks the sizes)
  const int n = g.B * g.Ho * g.Wo * K8;
  const int hw = g.Ho * g.Wo;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += pix_blocks * blockDim.x) {
    const int m = e / K8, k8 = e - m * K8;
    const int b = m / hw, rem = m - b * hw;
    const int oh = rem / g.Wo, ow = rem - oh * g.Wo;
    const int y0 = oh * g.sh - g.pt, x0 = ow * g.sw - g.pl;
    const int t = tap[k8];
    int kh = t >> 20, kw = (t >> 10) & 1023, ci = t & 1023;
    const int k = k8 * 8;
    const bf16* xb = x + b * g.H * g.W * g.C;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ih = y0 + kh, iw = x0 + kw;
      v[j] = (k + j < K && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W) ? xb[(ih * g.W + iw) * g.C + ci]
                                                                                      : (bf16)0.0f;
      if (++ci == g.C) {
        ci = 0;
        if (++kw == g.KW) {
          kw = 0;
          ++kh;
        }
      }
    }
    *reinterpret_cast<bf16x8*>(out + (long long)m * Kp + k) = v;
  }
}

// Row-staged im2col (the stem: C = 3, 7x7/2): one block per output row (b, oh).  The KH input
// rows that row reads are staged once into LDS with coalesced loads (zero rows / columns for the
// padding), then every output 16-byte chunk is assembled from LDS: element k = (kh, kw, ci) of
// pixel ow sits at LDS offset k + kh*(LROW - KW*C) + PAD + ow*sw*C, so a thread keeps its chunk's 8
// offsets in registers and walks ow with one add: no global gathers, no per-element bounds tests.
// (The gather kernel above issues 8 bounds-checked 2-byte global loads per chunk: issue-bound.)
constexpr int kI2cLds = 16384;  // bf16 elements (32 KB)
// LDS row kh starts at kh*LROW (LROW % 8 == 0); input column iw of it at PAD + (iw + pl)*C, with PAD
// chosen so that column 0 is 16-byte aligned: whole input rows are then staged with 16-byte copies
// (VROW) into a zeroed image.
__global__ __launch_bounds__(256) void im2col_rows_kernel(const bf16* __restrict__ x, Geo g, int Kp, int LROW, int PAD,
                                                          int VROW, bf16* __restrict__ out,
                                                          const bf16* __restrict__ w_in, bf16* __restrict__ w_out,
                                                          int pix_blocks) {
  const int K = g.KH * g.KW * g.C;
  if ((int)blockIdx.x >= pix_blocks) {  // weight padding blocks
    const int n = g.Co * Kp;
    for (int e = (blockIdx.x - pix_blocks) * blockDim.x + threadIdx.x; e < n;
         e += (gridDim.x - pix_blocks) * blockDim.x) {
      const int co = e / Kp, k = e - co * Kp;
      w_out[e] = k < K ? w_in[co * K + k] : (bf16)0.0f;
    }
    return;
  }
  __shared__ __attribute__((aligned(16))) bf16 rows[kI2cLds];
  const int b = blockIdx.x / g.Ho, oh = blockIdx.x - b * g.Ho;
  const int y0 = oh * g.sh - g.pt;
  const bf16* xb = x + (long long)b * g.H * g.W * g.C;
  const int WC = g.W * g.C, span = LROW - PAD;  // span: elements of columns -pl .. (LROW-PAD)/C - pl - 1
  if (VROW) {
    for (int e = threadIdx.x; e < g.KH * LROW / 8; e += blockDim.x)
      *reinterpret_cast<bf16x8*>(rows + e * 8) = zero8();
    __syncthreads();
    const int c8 = WC / 8, col0 = PAD + g.pl * g.C;
    for (int e = threadIdx.x; e < g.KH * c8; e += blockDim.x) {
      const int kh = e / c8, j = e - kh * c8;
      const int ih = y0 + kh;
      if ((unsigned)ih < (unsigned)g.H)
        *reinterpret_cast<bf16x8*>(rows + kh * LROW + col0 + j * 8) =
            *reinterpret_cast<const bf16x8*>(xb + ih * WC + j * 8);
    }
  } else {
    for (int e = threadIdx.x; e < g.KH * span; e += blockDim.x) {
      const int kh = e / span, j = e - kh * span;
      const int ih = y0 + kh;
      const int col = j / g.C, ci = j - col * g.C;
      const int iw = col - g.pl;
      bf16 v = (bf16)0.0f;
      if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W) v = xb[(ih * g.W + iw) * g.C + ci];
      rows[kh * LROW + PAD + j] = v;
    }
  }
  __syncthreads();
  const int K8 = Kp >> 3, P = blockDim.x / K8;
  const int t = threadIdx.x;
  if (t >= P * K8) return;
  const int k8 = t % K8;
  int off[8];
  bool ok[8];
  const int KWC = g.KW * g.C;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k8 * 8 + j;
    ok[j] = k < K;
    const int kh = k / KWC;
    off[j] = ok[j] ? k + kh * (LROW - KWC) + PAD : 0;
  }
  const int dstep = g.sw * g.C;
  bf16* orow = out + (long long)blockIdx.x * g.Wo * Kp + k8 * 8;
  for (int ow = t / K8; ow < g.Wo; ow += P) {
    const int base = ow * dstep;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ok[j] ? rows[off[j] + base] : (bf16)0.0f;
    *reinterpret_cast<bf16x8*>(orow + (long long)ow * Kp) = v;
  }
}

static int grid_for(long long n, int per_thread = 1) {
  const long long t = (n + per_thread - 1) / per_thread;
  long long b = (t + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace tde

using namespace tde;

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Split-K epilogue: the GEMM accumulated into the f32 scratch with atomics; apply bias / statistics /
// ReLU / bf16 (+=) store / f32 store here, and re-zero the scratch for its next use.
__global__ __launch_bounds__(256) void gemm_finalize_kernel(float* __restrict__ scr, int M, int N, float alpha,
                                                            const float* __restrict__ bias, int relu,
                                                            float* __restrict__ cf, long long ldc,
                                                            bf16* __restrict__ cb, long long ldcb, int cb_accum,
                                                            double* __restrict__ colstats) {
  __shared__ float s1[kMaxCB], s2[kMaxCB];
  if (colstats) {
    for (int c = threadIdx.x; c < N; c += blockDim.x) s1[c] = s2[c] = 0.f;
    __syncthreads();
  }
  const long long n = (long long)M * N;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int col = (int)((unsigned long long)e % (unsigned)N);
    const long long row = e / N;
    float v = alpha * scr[e] + (bias ? bias[col] : 0.f);
    scr[e] = 0.f;
    if (colstats) {
      const float q = cb ? bf2f(f2bf(v)) : v;
      atomicAdd(&s1[col], q);
      atomicAdd(&s2[col], q * q);
    }
    if (relu) v = fmaxf(v, 0.f);
    if (cf) cf[row * ldc + col] = v;
    if (cb) {
      bf16* q = &cb[row * ldcb + col];
      if (cb_accum) v += bf2f(*q);
      *q = f2bf(v);
    }
  }
  if (colstats) {
    __syncthreads();
    double* st = colstats + (size_t)(blockIdx.x % kStatSlots) * 2 * N;
    for (int c = threadIdx.x; c < N; c += blockDim.x) {
      atomicAdd(&st[c], (double)s1[c]);
      atomicAdd(&st[N + c], (double)s2[c]);
    }
  }
}

// Tile-selection knobs (bench/resnet_layers.py sweeps them; the defaults are the measured choice):
// weight-grad split-K targets ~g_wg_target workgroups with >= g_wg_min_kt k-tiles per split, and
// g_kb_force (32/64) overrides the K step.
// g_glds selects the global_load_lds pipeline for the K-vector kinds (fwd / dgrad / dense).
static int g_wg_target = 512, g_wg_min_kt = 16, g_kb_force = 0, g_glds = 1, g_big = 0, g_big_min = 192;
// dgrad on 256-row big tiles (which need the KB = 64 step): TDE_IGEMM_BIG_DGRAD=1 / tde_igemm_big_dgrad()
static int g_big_dgrad = [] {
  const char* e = getenv("TDE_IGEMM_BIG_DGRAD");
  return e && e[0] == '1' ? 1 : 0;
}();
// number of big-tile launches since load (tests assert the path ran)
static unsigned long long g_big_launches = 0;
// XCD-aware tile order (TDE_XCD_SWIZZLE = bit mask by GEMM kind, see tde_igemm).  Round 1 (VALU-bound
// loop) measured it neutral; with the LDS-DMA loop it pays for the weight gradients only.
static int g_xcd = -1;
// split-K weight gradients with at most this many splits store partials + reduce; more splits use atomics
// weight gradients with too few workgroups for 128-wide tiles drop to 64 (TDE_WG_SMALL_TILES=0: off)
static int g_wg_small_tiles = [] {
  const char* e = getenv("TDE_WG_SMALL_TILES");
  return e ? atoi(e) : 1;
}();
// (default 256: with the grouped fixed-order reduction the partials beat the f32 atomics of many-way splits —
// ResNet-18 weight gradients 797 -> 727 us per step in isolation, stage-2 3x3 51.6 -> 41.3 us, end to end
// 22.36k -> 22.86k img/s at 64; profiles/r6_splitk/)
static int g_wg_scratch_max = [] {
  const char* e = getenv("TDE_WG_SCRATCH_MAX");
  return e ? atoi(e) : 256;
}();
// weight gradients through the row-padded LDS-DMA path (TDE_WGRAD_DMA=0: the register-staged loaders)
// 0 = off, 1 = 3 LDS stages, 2 = 2 stages, 3 = per shape (default; bench/resnet_layers.py --sweep-wgrad,
// profiles/r2_sweep_wgrad.txt): Co <= 64 (ResNet stage 1) keeps the register-staged loaders (the row padding
// costs more than it saves), strided / 1x1 convs take 128 x 64 tiles at 3 stages (twice the workgroups of
// their short pixel loops), the other convs 128 x 128 at 2 stages (two workgroups per CU)
static int g_wg_dma = [] {
  const char* e = getenv("TDE_WGRAD_DMA");
  return e ? atoi(e) : 3;
}();
TDE_API void tde_igemm_wgrad_dma(int mode) { g_wg_dma = mode; }
static unsigned long long g_wg_dma_launches = 0;   // tests assert the path ran
TDE_API unsigned long long tde_igemm_wgrad_dma_launches() { return g_wg_dma_launches; }
// weight-gradient tile cap under a forced g_wg_dma mode (sweeps): 1 = 128 x 64 / 64 x 128 at most
static int g_wg_tile_cap = 0;
TDE_API void tde_igemm_wgrad_tile_cap(int v) { g_wg_tile_cap = v; }
// fwd / dgrad / dense tile choice: the largest of 128x128, 128x64, 64x64 with >= g_tile_min workgroups.
// 2048 (~8 per CU) measured best on ResNet-18 at batch 64 (bench/resnet_layers.py --sweep-tile: fwd
// 671 -> 637 us, dgrad 832 -> 825 us per step vs 512); TDE_IGEMM_TILE_MIN overrides.
static int g_tile_min = [] {
  const char* e = getenv("TDE_IGEMM_TILE_MIN");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : 2048;
}();
TDE_API void tde_igemm_tile_min(int v) {
  if (v > 0) g_tile_min = v;
}

TDE_API void tde_igemm_big_dgrad(int on) { g_big_dgrad = on ? 1 : 0; }
// LDS-DMA kernels on v_mfma_f32_32x32x16_bf16 instead of 16x16x32 (bit mask by GEMM kind as TDE_XCD_SWIZZLE:
// 1 = fwd / dense, 2 = dgrad, 4 = weight gradients); TDE_MFMA32 overrides.  Default 3: ResNet-18 per layer
// (bench/resnet_layers.py --ab-mfma32, profiles/r6_mfma32/) fwd 508 -> 485 us and dgrad 543 -> 530 us per step
// (every layer 2-7 % faster), while the transposed-read weight gradients lose (stage-2 128x128 tiles 50 -> 65-75 us)
static int mfma32_default() {
  const char* e = getenv("TDE_MFMA32");
  return e ? atoi(e) : 3;
}
static int g_mfma32 = mfma32_default();
TDE_API void tde_igemm_mfma32(int mask) { g_mfma32 = mask < 0 ? mfma32_default() : mask; }  // < 0: the default
static unsigned long long g_m32_launches = 0;   // tests assert the 32x32 kernels ran
TDE_API unsigned long long tde_igemm_mfma32_launches() { return g_m32_launches; }
TDE_API unsigned long long tde_igemm_big_launches() { return g_big_launches; }

TDE_API void tde_igemm_tune(int wg_target, int wg_min_kt, int kb_force, int glds, int big, int big_min) {
  if (wg_target > 0) g_wg_target = wg_target;
  if (wg_min_kt > 0) g_wg_min_kt = wg_min_kt;
  g_kb_force = (kb_force == 32 || kb_force == 64) ? kb_force : 0;
  if (glds >= 0) g_glds = glds;
  if (big >= 0) g_big = big;
  if (big_min > 0) g_big_min = big_min;
}

// Split-K factor of a weight-gradient GEMM (row-contiguous operands, 128/64 tiles): fill the chip with
// ~g_wg_target workgroups, >= g_wg_min_kt k-tiles per split (every split ends in a BM x BN partial
// sum), but never fewer than ~256 workgroups while K allows 2 k-tiles per split (1x1 projections).
static int wgrad_splits(int M, int N, int K, int KB, int* ktiles_per_split, bool cap = false) {
  const int bm = M > 64 ? 128 : 64, bn = (N > 64 && !(cap && bm == 128)) ? 128 : 64;
  const int ktiles = (K + KB - 1) / KB;
  const long long t = (long long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  long long sp = (g_wg_target + t - 1) / t;
  long long maxs = ktiles / g_wg_min_kt > 0 ? ktiles / g_wg_min_kt : 1;
  if (t * maxs < 256) {
    const long long want = (256 + t - 1) / t, cap = ktiles / 2 > 0 ? ktiles / 2 : 1;
    maxs = want < cap ? want : cap;
  }
  int splits = (int)(sp < maxs ? sp : maxs);
  if (splits < 1) splits = 1;
  const int per = (ktiles + splits - 1) / splits;
  if (ktiles_per_split) *ktiles_per_split = per;
  return ktiles > 0 ? (ktiles + per - 1) / per : 1;
}

// f32 elements of split-K scratch a weight gradient of this shape uses (0: no split)
TDE_API long long tde_igemm_wgrad_scratch_elems(int M, int N, int K) {
  const int KB = g_kb_force ? g_kb_force : (K < 256 ? 32 : 64);
  // the LDS-DMA weight gradient runs over a row-padded pixel count < 2 K: size for that bound (splits grow with K)
  const int sp = wgrad_splits(M, N, K < (1 << 29) ? 2 * K : K, KB, nullptr);
  return (sp > 1 && sp <= g_wg_scratch_max) ? (long long)sp * M * N : 0;
}

// dst[i] += sum_s part[s][i] over contiguous [M*N] (the split-K partials of a weight gradient)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int splits, long long n,
                                                            float* __restrict__ dst) {
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 acc = reinterpret_cast<const float4*>(part)[i];
    for (int s = 1; s < splits; ++s) {
      const float4 v = reinterpret_cast<const float4*>(part + (size_t)s * n)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float4 d = reinterpret_cast<float4*>(dst)[i];
    d.x += acc.x; d.y += acc.y; d.z += acc.z; d.w += acc.w;
    reinterpret_cast<float4*>(dst)[i] = d;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long e = (n4 << 2) + threadIdx.x;
    float acc = 0.f;
    for (int s = 0; s < splits; ++s) acc += part[(size_t)s * n + e];
    dst[e] += acc;
  }
}

// ---- deterministic mode (TDE_DETERMINISTIC=1 / tde_layers_deterministic): every reduction of the layer-wise
// plan runs in a fixed order, so two runs of one configuration are bitwise identical (tests compare bucketed and
// one-bucket data-parallel runs bitwise).  Per-channel sums move out of the GEMM epilogues /
// streaming passes (whose f64 / f32 atomics land in run-dependent order) into the *_det kernels below: grid
// (channel groups of 64, kStatSlots row parts), part p sums rows p, p + 8, ... in row order and STORES slot p
// (readers sum the slots in slot order); split-K weight gradients go through the ordered partial scratch or run
// unsplit; split-K activation GEMMs run unsplit.  Slow (one pass per sum, a few hundred workgroups): a
// reproducibility / test mode, not the benchmarked path.
static int g_det = [] {
  const char* e = getenv("TDE_DETERMINISTIC");
  return (e && e[0] && e[0] != '0') ? 1 : 0;
}();
TDE_API void tde_layers_deterministic(int on) { g_det = on ? 1 : 0; }
TDE_API int tde_layers_is_deterministic() { return g_det; }

// stats[p][0|1][c] = sum / sum of squares of x[r][c] (bf16, row stride ld) over rows r = p (mod kStatSlots)
__global__ __launch_bounds__(256) void colstats_det_kernel(const bf16* __restrict__ x, long long R, int C, long long ld,
                                                           double* __restrict__ stats) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6, c = blockIdx.x * 64 + cl, p = blockIdx.y;
  double s1 = 0.0, s2 = 0.0;
  if (c < C)
    for (long long r = p + (long long)kStatSlots * rl; r < R; r += 4LL * kStatSlots) {
      const double v = (double)bf2f(x[r * ld + c]);
      s1 += v;
      s2 += v * v;
    }
  red[0][rl][cl] = s1;
  red[1][rl][cl] = s2;
  __syncthreads();
  if (rl == 0 && c < C) {
    double* st = stats + (size_t)p * 2 * C;
    st[c] = (red[0][0][cl] + red[0][1][cl]) + (red[0][2][cl] + red[0][3][cl]);
    st[C + c] = (red[1][0][cl] + red[1][1][cl]) + (red[1][2][cl] + red[1][3][cl]);
  }
}

static int colstats_det(const bf16* x, long long R, int C, long long ld, double* stats, hipStream_t stream) {
  colstats_det_kernel<<<dim3((C + 63) / 64, kStatSlots), 256, 0, stream>>>(x, R, C, ld, stats);
  TDE_LAUNCH_CHECK();
  return 0;
}

// dbias[c] += sum over rows of (relu ? (out > 0) * dout : dout), rows in order (one block per 64 channels)
__global__ __launch_bounds__(256) void colsum_det_kernel(const bf16* __restrict__ dout, const bf16* __restrict__ out,
                                                         long long R, int C, int relu, float* __restrict__ dbias) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < C)
    for (long long r = rl; r < R; r += 4) {
      const long long e = r * C + c;
      const float g = bf2f(dout[e]);
      s += (!relu || bf2f(out[e]) > 0.f) ? g : 0.f;
    }
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < C) dbias[c] += (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

// dst[i] += sum over s < splits of part[s][i] (i < n), in split order; also the reduction pass of the halo
// weight gradient (haloconv.hip)
static void splitk_reduce_launch(const float* part, int splits, long long n, float* dst, hipStream_t stream);
TDE_API int tde_splitk_reduce(const float* part, int splits, long long n, float* dst, hipStream_t stream) {
  if (n <= 0 || splits < 1) return 0;
  if (((uintptr_t)part & 15) || ((uintptr_t)dst & 15)) return -3;
  splitk_reduce_launch(part, splits, n, dst, stream);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Many splits (>= 8, n % 4 == 0): block = 64 consecutive elements (16 float4 columns) x 16 split groups, group j
// summing splits j, j + 16, ... in order and the groups summed in a fixed order through LDS — every thread's loads in
// flight together (the one-thread-per-element form walks all splits serially)
__global__ __launch_bounds__(256) void splitk_reduce_grouped_kernel(const float* __restrict__ part, int splits,
                                                                    long long n, float* __restrict__ dst) {
  __shared__ float4 red[16][16];
  const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const long long n4 = n >> 2, i4 = (long long)blockIdx.x * 16 + col;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) {
    const float4* p4 = reinterpret_cast<const float4*>(part);
#pragma unroll 4
    for (int s = grp; s < splits; s += 16) {
      const float4 v = p4[(size_t)s * n4 + i4];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
  }
  red[grp][col] = acc;
  __syncthreads();
  if (grp == 0 && i4 < n4) {
    float4 t = red[0][col];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
      const float4 v = red[j][col];
      t.x += v.x;
      t.y += v.y;
      t.z += v.z;
      t.w += v.w;
    }
    float4* d4 = reinterpret_cast<float4*>(dst);
    float4 d = d4[i4];
    d.x += t.x;
    d.y += t.y;
    d.z += t.z;
    d.w += t.w;
    d4[i4] = d;
  }
}

static void splitk_reduce_launch(const float* part, int splits, long long n, float* dst, hipStream_t stream) {
  if (splits >= 8 && n % 4 == 0 && ((n / 4 + 15) / 16) < (1LL << 31)) {
    splitk_reduce_grouped_kernel<<<(int)((n / 4 + 15) / 16), 256, 0, stream>>>(part, splits, n, dst);
    return;
  }
  long long g = (n / 4 + 255) / 256;
  g = g < 1 ? 1 : (g > 2048 ? 2048 : g);
  splitk_reduce_kernel<<<(int)g, 256, 0, stream>>>(part, splits, n, dst);
}

static int igemm_impl(const bf16* a, long long lda, int akind, const bf16* b, long long ldb, int bkind, int M, int N,
                      int K, const int* geo, int splits, float* cf, long long ldc, int cf_mode, float alpha, bf16* cb,
                      long long ldcb, int cb_accum, const float* bias, int relu, double* colstats, float* scratch,
                      const int* phase, const BnSum* bs, hipStream_t stream);

TDE_API int tde_igemm(const bf16* a, long long lda, int akind, const bf16* b, long long ldb, int bkind, int M, int N,
                      int K, const int* geo, int splits, float* cf, long long ldc, int cf_mode, float alpha, bf16* cb,
                      long long ldcb, int cb_accum, const float* bias, int relu, double* colstats, float* scratch,
                      const int* phase, hipStream_t stream) {
  return igemm_impl(a, lda, akind, b, ldb, bkind, M, N, K, geo, splits, cf, ldc, cf_mode, alpha, cb, ldcb, cb_accum,
                    bias, relu, colstats, scratch, phase, nullptr, stream);
}

// Stride-1 conv input gradient dx (=|+=) conv_transpose(dy, W) whose epilogue also takes the backward sums of the
// BatchNormalization that consumes dx's tensor (BnSum): the LDS-DMA path only (-8 when this shape would run
// another), never under TDE_DETERMINISTIC (-9: the sums are f32 atomics).
TDE_API int tde_igemm_dgrad_bnsum(const bf16* dy, const bf16* w, int M, int N, int K, const int* geo, bf16* dx,
                                  long long ldx, int accum, const BnSum* bs, hipStream_t stream) {
  if (!bs || !bs->dstats || !bs->y || !bs->saved) return -1;
  if (g_det) return -9;
  return igemm_impl(dy, 0, A_DGRAD, w, 0, B_DGRADW, M, N, K, geo, 1, nullptr, 0, 0, 1.f, dx, ldx, accum, nullptr, 0,
                    nullptr, nullptr, nullptr, bs, stream);
}
TDE_API int tde_bnsum_bytes() { return (int)sizeof(BnSum); }

static int igemm_impl(const bf16* a, long long lda, int akind, const bf16* b, long long ldb, int bkind, int M, int N,
                      int K, const int* geo, int splits, float* cf, long long ldc, int cf_mode, float alpha, bf16* cb,
                      long long ldcb, int cb_accum, const float* bias, int relu, double* colstats, float* scratch,
                      const int* phase, const BnSum* bs, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (phase && (akind != A_DGRAD || splits > 1 || colstats)) return -5;
  if (bs && (akind != A_DGRAD || phase || splits > 1 || !cb || colstats || cf || bias || relu || N % 8 ||
             ldcb % 8 || ((uintptr_t)cb & 15) || ((uintptr_t)bs->y & 15) || ((uintptr_t)bs->res & 15)))
    return -8;
  if (g_det && colstats) {
    // statistics of the stored bf16 output in a fixed order, after the GEMM (which runs without them)
    if (!cb || cb_accum || relu) return -7;
    int rc = igemm_impl(a, lda, akind, b, ldb, bkind, M, N, K, geo, splits, cf, ldc, cf_mode, alpha, cb, ldcb,
                        cb_accum, bias, relu, nullptr, scratch, phase, nullptr, stream);
    if (rc) return rc;
    return colstats_det(cb, M, N, ldcb, colstats, stream);
  }
  // deterministic: activation GEMMs unsplit (their split-K partials meet in f32 atomics)
  if (g_det && splits > 1 && (cb || bias || relu || cf_mode == 1)) splits = 1;
  const bool fused_epi = cb || colstats || bias || relu || cf_mode == 1;
  if (splits > 1 && fused_epi) {
    // split-K into the zeroed f32 scratch, then the epilogue pass
    if (!scratch || (colstats && N > kMaxCB)) return -2;
    int rc = igemm_impl(a, lda, akind, b, ldb, bkind, M, N, K, geo, splits, scratch, N, 2, 1.f, nullptr, 0, 0,
                        nullptr, 0, nullptr, nullptr, nullptr, nullptr, stream);
    if (rc) return rc;
    const long long n = (long long)M * N;
    int g = (int)((n + 255) / 256);
    if (g > 1024) g = 1024;
    gemm_finalize_kernel<<<g, 256, 0, stream>>>(scratch, M, N, alpha, bias, relu, cf_mode == 1 ? cf : nullptr, ldc,
                                                 cb, ldcb, cb_accum, colstats);
    TDE_LAUNCH_CHECK();
    return 0;
  }
  IGemmArgs p{};
  if (g_xcd < 0) {
    // bit mask by GEMM kind: 1 = fwd / dense (A_ROWK, A_CONV), 2 = dgrad, 4 = weight gradients
    const char* e = getenv("TDE_XCD_SWIZZLE");
    // default 4: weight gradients only (ResNet-18 wgrad 840 -> 798 us/step; fwd / dgrad 1-3 % slower with it,
    // profiles/r2_xcd_ab.txt)
    g_xcd = e ? atoi(e) : 4;
  }
  const int kind_bit = (akind == A_ROWK || akind == A_CONV) ? 1 : akind == A_DGRAD ? 2 : 4;
  p.xcd = (g_xcd & kind_bit) ? 1 : 0;
  const bool m32 = (g_mfma32 & kind_bit) != 0;
  p.a = a;
  p.lda = lda;
  p.b = b;
  p.ldb = ldb;
  p.M = M;
  p.N = N;
  p.K = K;
  if (geo) {
    Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
    p.g = g;
  }
  int nph = 0;
  if (phase && phase[0] == -1) {
    // multi-phase table {-1, n, n x {ph_h, ph_w, Hp, Wp, kh0, kw0, KHp, KWp}}: one launch, grid z = phase;
    // M / K passed in are the largest over the phases (grid and K-step sizing)
    nph = phase[1];
    if (nph < 1 || nph > 4 || splits > 1) return -5;
    p.nph = nph;
    for (int i = 0; i < nph; ++i)
      for (int j = 0; j < 8; ++j) p.phs[i][j] = phase[2 + 8 * i + j];
    p.ph_on = 1;
    p.Hp = p.phs[0][2];   // host-side checks only; the kernel takes each block's phase from the table
    p.Wp = p.phs[0][3];
    p.KHp = p.phs[0][6];
    p.KWp = p.phs[0][7];
  } else if (phase) {
    p.ph_on = 1;
    p.ph_h = phase[0];
    p.ph_w = phase[1];
    p.Hp = phase[2];
    p.Wp = phase[3];
    p.kh0 = phase[4];
    p.kw0 = phase[5];
    p.KHp = phase[6];
    p.KWp = phase[7];
  }
  // K step: 64 (two MFMA k-slices per barrier) for long reductions; the gathered input gradient
  // measures faster at 32 (ResNet-18 sweep, bench/resnet_layers.py)
  // 256-row big tiles: LDS reads per MFMA flop within the CU's LDS bandwidth; only when they still give
  // >= g_big_min workgroups (tile count independent of the K step)
  const long long big_tiles = (long long)((M + 255) / 256) * ((N + (N <= 64 ? 63 : 127)) / (N <= 64 ? 64 : 128));
  const bool big_shape = splits <= 1 && (N <= 64 || N % 128 == 0) && big_tiles >= g_big_min;
  // dgrad big tiles run at KB = 64 (their only instantiation), so enabling them moves dgrad to KB = 64
  const bool dgrad_big = akind == A_DGRAD && g_big_dgrad && big_shape && p.g.Co % 64 == 0;
  // (the LDS-DMA dgrad runs best at 64 too since its loop lost the per-k-tile address math:
  // profiles/r2_sweep_fd.txt, 18 ResNet-18 dgrads 834 -> ~640 us)
  const int KB = g_kb_force ? g_kb_force
                            : (dgrad_big ? 64 : (akind == A_DGRAD ? (p.g.Co % 64 == 0 ? 64 : 32) : (K < 256 ? 32 : 64)));
  // LDS-DMA weight gradient: pixels in the row-padded order of the kernel's row-vector LDS-DMA path
  // (Wp = pow2 >= Wo dividing KB; B a multiple of the output rows per k-tile; 32-bit operand offsets)
  bool wg_dma = false, wg_cap = false;
  int wg_stages = 3;
  if (akind == A_WGRAD && bkind == B_KN && g_glds && g_wg_dma && KB == 64 && !phase && aligned16(a) && aligned16(b) &&
      (g_wg_dma != 3 || N > 64) &&
      p.g.C % 8 == 0 && p.g.Co % 8 == 0 && ldb == p.g.Co && N == p.g.Co && M == p.g.KH * p.g.KW * p.g.C &&
      K == p.g.B * p.g.Ho * p.g.Wo) {
    int wl = 0;
    while ((1 << wl) < p.g.Wo) ++wl;
    const int RT = wl <= 6 ? 64 >> wl : 0;
    const long long shift = ((long long)p.g.pt * p.g.W + p.g.pl) * p.g.C;
    const long long ae = (long long)p.g.B * p.g.H * p.g.W * p.g.C + shift;
    const long long be = (long long)p.g.B * p.g.Ho * p.g.Wo * p.g.Co;
    const long long kp = (long long)p.g.Ho * p.g.B * (1LL << wl);
    if (RT >= 1 && p.g.B % RT == 0 && ae * 2 < (1LL << 31) - 16 && be * 2 < (1LL << 31) - 16 && kp < (1LL << 30)) {
      wg_dma = true;
      if (g_wg_dma == 3) {
        wg_cap = p.g.sh > 1 || p.g.sw > 1 || (p.g.KH == 1 && p.g.KW == 1);
        wg_stages = wg_cap ? 3 : 2;
      } else {
        wg_cap = g_wg_tile_cap != 0;
        wg_stages = g_wg_dma == 2 ? 2 : 3;
      }
      p.wp_log = wl;
      p.a_shift = (int)shift;
      p.a_bytes = (int)(ae * 2);
      p.b_bytes = (int)(be * 2);
      K = (int)kp;
      p.K = K;
    }
  }
  const int ktiles = (K + KB - 1) / KB;
  const bool auto_splits = splits == 0;
  if (splits < 1) splits = 1;
  if (splits > ktiles) splits = ktiles > 0 ? ktiles : 1;
  if (splits > 1 && (cb || colstats || cf_mode != 2 || bias || relu)) return -2;  // split-K only into f32 atomics
  p.ktiles_per_split = (ktiles + splits - 1) / splits;
  splits = ktiles > 0 ? (ktiles + p.ktiles_per_split - 1) / p.ktiles_per_split : 1;
  const bool al = aligned16(a), bl = aligned16(b);
  switch (akind) {
    case A_ROWK: p.avec = al && lda % 8 == 0 && K % 8 == 0; break;
    case A_CONV: p.avec = al && p.g.C % 8 == 0; break;
    case A_DGRAD: p.avec = al && p.g.Co % 8 == 0; break;
    case A_COLM: p.avec = al && lda % 8 == 0 && (M + 7) / 8 * 8 <= lda; break;  // padded rows read, never stored
    case A_WGRAD: p.avec = al && p.g.C % 8 == 0; break;
    default: return -1;
  }
  switch (bkind) {
    case B_NK: p.bvec = bl && ldb % 8 == 0 && K % 8 == 0; break;
    case B_DGRADW: p.bvec = bl && p.g.Co % 8 == 0; break;
    case B_KN: p.bvec = bl && ldb % 8 == 0 && N % 8 == 0; break;
    default: return -1;
  }
  p.cf = cf;
  p.ldc = ldc;
  p.cf_mode = cf ? cf_mode : 0;
  p.alpha = alpha;
  p.cb = cb;
  p.ldcb = ldcb;
  p.cb_accum = cb_accum;
  p.bias = bias;
  p.relu = relu;
  p.colstats = colstats;
  // tile: weight-grad kinds (row-contiguous operands) use the 128x128 transposed images; the others
  // take the largest tile that still gives >= 2 workgroups per CU
  int bm = 64, bn = 64;
  const bool rowk = (akind == A_COLM || akind == A_WGRAD);
  auto tiles = [&](int tm, int tn) { return (long long)((M + tm - 1) / tm) * ((N + tn - 1) / tn) * splits; };
  if (rowk) {
    bm = M > 64 ? 128 : 64;
    bn = N > 64 ? 128 : 64;
    if (wg_cap && bm == 128 && bn == 128) bn = 64;
    if (auto_splits) {
      splits = wgrad_splits(M, N, K, KB, &p.ktiles_per_split, wg_cap);
    }
    // short reductions (K = a small batch, e.g. a Dense weight gradient at batch 128: 2 splits at most) cannot
    // reach a chip-filling grid by splitting K: take narrower tiles while that still leaves < 256 workgroups
    if (!wg_dma && g_wg_small_tiles) {
      if (bm == 128 && tiles(bm, bn) < 256) bm = 64;
      if (bn == 128 && tiles(bm, bn) < 256) bn = 64;
    }
  } else if (N > 64 && tiles(128, 128) >= g_tile_min) {
    bm = bn = 128;
  } else if (tiles(128, 64) >= g_tile_min || (ktiles >= 16 && tiles(128, 64) >= 256)) {
    // 128x64 also for long K loops that still give >= one workgroup per CU: half the operand re-reads
    // of 64x64 (ResNet-18 14x14x256 convs 34.7 -> 27.1 us; profiles/r2_sweep_fd.txt)
    bm = 128;
  }
  if (g_det && splits > 1) {
    // deterministic: split-K weight gradients only through the ordered partial scratch (the condition below)
    const bool ordered = rowk && auto_splits && splits <= g_wg_scratch_max && scratch && p.cf_mode == 2 &&
                         p.ldc == N && p.cf && ((uintptr_t)p.cf & 15) == 0 && ((uintptr_t)scratch & 15) == 0;
    if (!ordered) {
      splits = 1;
      p.ktiles_per_split = ktiles;
    }
  }
  dim3 grid((M + bm - 1) / bm, (N + bn - 1) / bn, nph > 0 ? nph : splits);
  if (grid.y > 65535 || splits > 65535) return -3;
  // weight-grad split-K with a scratch: every split stores its partial tile (plain stores) and one
  // reduction pass adds them to the gradient, instead of BM x BN memory-side f32 atomics per split
  float* const wg_dst = p.cf;
  const long long wg_ldc = p.ldc;
  const bool wg_scratch = rowk && auto_splits && splits > 1 && splits <= g_wg_scratch_max && scratch &&
                          p.cf_mode == 2 && p.ldc == N && p.cf &&
                          ((uintptr_t)p.cf & 15) == 0 && ((uintptr_t)scratch & 15) == 0;
  if (wg_scratch) {
    p.cf = scratch;
    p.cf_mode = 3;
  }
  const bool vec = p.avec && p.bvec;
  if (rowk && vec && !wg_dma) {  // the weight-gradient fast loaders index with 32-bit offsets
    const long long asz = akind == A_WGRAD ? (long long)p.g.B * p.g.H * p.g.W * p.g.C : (long long)K * lda;
    if (asz >= (1LL << 31) || (long long)K * ldb >= (1LL << 31) || (long long)M * N >= (1LL << 31)) return -6;
  }
  // global_load_lds path: every k-tile inside one filter tap (see igemm_kernel)
  bool ut = true;
  if (akind == A_CONV) {
    ut = p.g.C % KB == 0;
    if (!ut && p.g.C % 8 == 0 && p.g.C * p.g.KW == KB && p.g.pt == 0 && p.g.pl == 0 &&
        (p.g.Ho - 1) * p.g.sh + p.g.KH <= p.g.H && (p.g.Wo - 1) * p.g.sw + p.g.KW <= p.g.W) {
      ut = true;
      p.rowtile = 1;
    }
  }
  if (akind == A_DGRAD) ut = p.g.Co % KB == 0 && (p.ph_on || (p.g.sh == 1 && p.g.sw == 1));
  {
    // LDS-DMA loads address both operands with 32-bit byte offsets under buffer range checks
    long long ae = 0, be = 0;
    if (akind == A_ROWK) ae = (long long)(M - 1) * lda + K;
    else if (akind == A_CONV) ae = (long long)p.g.B * p.g.H * p.g.W * p.g.C;
    else if (akind == A_DGRAD) ae = (long long)p.g.B * p.g.Ho * p.g.Wo * p.g.Co;
    if (bkind == B_NK) be = (long long)(N - 1) * ldb + K;
    else if (bkind == B_DGRADW) be = (long long)p.g.KH * p.g.KW * p.g.C * p.g.Co;
    if (ae * 2 >= (1LL << 31) - 16 || be * 2 >= (1LL << 31) - 16) ut = false;
    if (!wg_dma) {
      p.a_bytes = (int)(ae * 2 < (1LL << 31) ? ae * 2 : 0);
      p.b_bytes = (int)(be * 2 < (1LL << 31) ? be * 2 : 0);
    }
  }
  // big tiles (256 x 64 with 64 x 64 per wave, or 256 x 128 with 128 x 64 per wave): fwd/dense when
  // tuned on (fwd 641 -> 840 us on ResNet-18 with them), dgrad when g_big_dgrad
  const bool big = (g_big || (g_big_dgrad && akind == A_DGRAD)) && KB == 64 && splits == 1 && !rowk && big_shape;
  if (bs) {
    if (!(vec && g_glds && ut && !big)) return -8;   // the BN sums live in the LDS-DMA kernels' LDS epilogue
    p.bs = *bs;
  }
#define TDE_IGEMM(AK_, BK__, BM_, BN_)                                                   \
  do {                                                                                   \
    if (vec) {                                                                           \
      if (KB == 64) igemm_kernel<AK_, BK__, BM_, BN_, 64, 1><<<grid, 256, 0, stream>>>(p); \
      else igemm_kernel<AK_, BK__, BM_, BN_, 32, 1><<<grid, 256, 0, stream>>>(p);          \
    } else {                                                                             \
      if (KB == 64) igemm_kernel<AK_, BK__, BM_, BN_, 64, 0><<<grid, 256, 0, stream>>>(p); \
      else igemm_kernel<AK_, BK__, BM_, BN_, 32, 0><<<grid, 256, 0, stream>>>(p);          \
    }                                                                                    \
  } while (0)
  // K-vector kinds: global_load_lds pipeline, 3 stages at KB = 64 (<= 96 KiB LDS), 4 at KB = 32
#define TDE_IGEMM_KV(AK_, BK__, BM_, BN_)                                                           \
  do {                                                                                              \
    if (vec && g_glds && ut) {                                                                      \
      if (big) ++g_big_launches;                                                                    \
      if (big && N <= 64) {                                                                         \
        grid = dim3((M + 255) / 256, (N + 63) / 64, grid.z);                                        \
        igemm_kernel<AK_, BK__, 256, 64, 64, 1, 3, 4><<<grid, 256, 0, stream>>>(p);                 \
      } else if (big) {                                                                             \
        grid = dim3((M + 255) / 256, (N + 127) / 128, grid.z);                                      \
        igemm_kernel<AK_, BK__, 256, 128, 64, 1, 3, 2><<<grid, 256, 0, stream>>>(p);                \
      } else if (KB == 64) {                                                                        \
        if (m32) ++g_m32_launches;                                                                 \
        if (m32) igemm_kernel<AK_, BK__, BM_, BN_, 64, 1, 3, 2, 32><<<grid, 256, 0, stream>>>(p);   \
        else igemm_kernel<AK_, BK__, BM_, BN_, 64, 1, 3><<<grid, 256, 0, stream>>>(p);              \
      } else {                                                                                      \
        if (m32) ++g_m32_launches;                                                                 \
        if (m32) igemm_kernel<AK_, BK__, BM_, BN_, 32, 1, 4, 2, 32><<<grid, 256, 0, stream>>>(p);   \
        else igemm_kernel<AK_, BK__, BM_, BN_, 32, 1, 4><<<grid, 256, 0, stream>>>(p);              \
      }                                                                                             \
    } else {                                                                                        \
      TDE_IGEMM(AK_, BK__, BM_, BN_);                                                               \
    }                                                                                               \
  } while (0)
  if (akind == A_ROWK && bkind == B_NK) {
    if (bm == 128 && bn == 128) TDE_IGEMM_KV(A_ROWK, B_NK, 128, 128);
    else if (bm == 128) TDE_IGEMM_KV(A_ROWK, B_NK, 128, 64);
    else TDE_IGEMM_KV(A_ROWK, B_NK, 64, 64);
  } else if (akind == A_CONV && bkind == B_NK) {
    if (bm == 128 && bn == 128) TDE_IGEMM_KV(A_CONV, B_NK, 128, 128);
    else if (bm == 128) TDE_IGEMM_KV(A_CONV, B_NK, 128, 64);
    else TDE_IGEMM_KV(A_CONV, B_NK, 64, 64);
  } else if (akind == A_DGRAD && bkind == B_DGRADW) {
    if (bm == 128 && bn == 128) TDE_IGEMM_KV(A_DGRAD, B_DGRADW, 128, 128);
    else if (bm == 128) TDE_IGEMM_KV(A_DGRAD, B_DGRADW, 128, 64);
    else TDE_IGEMM_KV(A_DGRAD, B_DGRADW, 64, 64);
  } else if (akind == A_COLM && bkind == B_KN) {
    if (bm == 128 && bn == 128) TDE_IGEMM(A_COLM, B_KN, 128, 128);
    else if (bm == 128) TDE_IGEMM(A_COLM, B_KN, 128, 64);
    else if (bn == 128) TDE_IGEMM(A_COLM, B_KN, 64, 128);
    else TDE_IGEMM(A_COLM, B_KN, 64, 64);
  } else if (akind == A_WGRAD && bkind == B_KN && wg_dma) {
    ++g_wg_dma_launches;
    if (m32) ++g_m32_launches;
#define TDE_WG_DMA(BM_, BN_, S_)                                                                \
  do {                                                                                          \
    if (m32) igemm_kernel<A_WGRAD, B_KN, BM_, BN_, 64, 1, S_, 2, 32><<<grid, 256, 0, stream>>>(p); \
    else igemm_kernel<A_WGRAD, B_KN, BM_, BN_, 64, 1, S_><<<grid, 256, 0, stream>>>(p);           \
  } while (0)
    if (bm == 128 && bn == 128 && wg_stages == 2) TDE_WG_DMA(128, 128, 2);
    else if (bm == 128 && bn == 128) TDE_WG_DMA(128, 128, 3);
    else if (bm == 128) TDE_WG_DMA(128, 64, 3);
    else if (bn == 128) TDE_WG_DMA(64, 128, 3);
    else TDE_WG_DMA(64, 64, 3);
#undef TDE_WG_DMA
  } else if (akind == A_WGRAD && bkind == B_KN) {
    if (bm == 128 && bn == 128) TDE_IGEMM(A_WGRAD, B_KN, 128, 128);
    else if (bm == 128) TDE_IGEMM(A_WGRAD, B_KN, 128, 64);
    else if (bn == 128) TDE_IGEMM(A_WGRAD, B_KN, 64, 128);
    else TDE_IGEMM(A_WGRAD, B_KN, 64, 64);
  } else {
    return -1;
  }
#undef TDE_IGEMM_KV
#undef TDE_IGEMM
  TDE_LAUNCH_CHECK();
  if (wg_scratch) {
    const long long n = (long long)M * N;
    (void)wg_ldc;
    splitk_reduce_launch(scratch, splits, n, wg_dst, stream);
    TDE_LAUNCH_CHECK();
  }
  return 0;
}

// drop: rate, seed, iter ptr, iter_offset, layer_id
// channel-tiled BN path: 8-channel vectors with whole channel groups of <= 64, 16-byte aligned tensors
static bool bn_tiled_ok(int C, std::initializer_list<const void*> ptrs) {
  if (C % 8 != 0 || (C > 64 && C % 64 != 0)) return false;
  for (const void* p : ptrs)
    if (((uintptr_t)p & 15) != 0) return false;
  return true;
}

// streaming grid: ~16K elements per block (prologue amortised), 512..4096 blocks
// Grid of the streaming BN passes: n / div blocks within [lo, hi] (TDE_BN_STREAM="div,lo,hi"), and of
// the backward reduction (TDE_BN_RED="div,lo,hi"; each of its blocks ends with 2*min(C,64) atomics).
struct BnGrid {
  long long div, lo, hi;
};
static BnGrid bn_grid_env(const char* name, BnGrid d) {
  const char* e = getenv(name);
  if (e) {
    long long a = 0, b = 0, c = 0;
    if (sscanf(e, "%lld,%lld,%lld", &a, &b, &c) == 3 && a > 0 && b > 0 && c >= b) d = BnGrid{a, b, c};
  }
  return d;
}
static int bn_grid_blocks(long long n, const BnGrid& g) {
  const long long b = n / g.div;
  return (int)(b < g.lo ? g.lo : (b > g.hi ? g.hi : b));
}
static int bn_stream_blocks(long long n) {
  static const BnGrid g = bn_grid_env("TDE_BN_STREAM", BnGrid{16384, 512, 4096});
  return bn_grid_blocks(n, g);
}
static int bn_reduce_blocks(long long n) {
  // (round 6 A/B of 16384 / 512 / 2048: +0.3 % end to end within noise, but the kernel statistics show every
  // reduction slower — stage 1 17.5 -> 20 us; profiles/r6_bnsum/: kept 32768 / 256 / 1024)
  static const BnGrid g = bn_grid_env("TDE_BN_RED", BnGrid{32768, 256, 1024});
  return bn_grid_blocks(n, g);
}

TDE_API int tde_bn_fwd(const bf16* y, bf16* out, const bf16* res, long long R, int C, int mode, const double* stats,
                       float* saved, const float* gamma, const float* beta, float eps, float* mmean, float* mvar,
                       float momentum, float bessel, float* zero_buf, int relu, float drop_rate,
                       unsigned long long seed, const long long* iter, int iter_offset, int layer_id,
                       hipStream_t stream) {
  if (C > kMaxC) return -1;
  if (R * C >= (1LL << 31)) return -4;
  BnFwdArgs a{y, out, res, R, C, mode, stats, saved, gamma, beta, eps, mmean, mvar, momentum, bessel, zero_buf, relu,
              Drop{drop_rate, seed, iter, iter_offset, layer_id}};
  if (bn_tiled_ok(C, {y, out, res})) {
    bn_fwd_tiled_kernel<<<bn_tiled_grid(R, C, bn_stream_blocks(R * C)), 256, 0, stream>>>(a);
  } else {
    bn_fwd_kernel<<<grid_for(R * C, 8), 256, 0, stream>>>(a);
  }
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_bn_bwd(const bf16* dout, const bf16* y, const bf16* res, long long R, int C, int mode,
                       const float* saved, const float* gamma, const float* beta, int relu, float drop_rate,
                       unsigned long long seed, const long long* iter, int iter_offset, int layer_id, float* dstats,
                       bf16* dx, int dx_accum, bf16* dres, int dres_accum, float* dgamma, float* dbeta,
                       double* zero_fwd, int sums_ready, hipStream_t stream) {
  if (C > kMaxCB) return -1;
  BnBwdArgs a{dout, y, res, R, C, mode, saved, gamma, beta, relu, Drop{drop_rate, seed, iter, iter_offset, layer_id},
              dstats, dx, dx_accum, dres, dres_accum, dgamma, dbeta, zero_fwd};
  if (R * C >= (1LL << 31)) return -4;
  if (sums_ready && mode == 1) {
    // dstats already hold this BN's backward sums (taken by the epilogue of the input-gradient GEMM that wrote
    // dout last, tde_igemm_dgrad_bnsum): the apply pass only
    if (bn_tiled_ok(C, {dout, y, res, dx, dres}))
      bn_bwd_apply_tiled_kernel<<<bn_tiled_grid(R, C, bn_stream_blocks(R * C)), 256, 0, stream>>>(a);
    else
      bn_bwd_apply_kernel<<<grid_for(R * C, 8), 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
    return 0;
  }
  if (g_det && mode == 1) {
    // fixed-order backward sums into the kStatSlots slots, then the apply pass reads them (it sums slots in order)
    bn_bwd_reduce_det_kernel<<<dim3((C + 63) / 64, kStatSlots), 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
    a.mode = 1;
    if (bn_tiled_ok(C, {dout, y, res, dx, dres}))
      bn_bwd_apply_tiled_kernel<<<bn_tiled_grid(R, C, bn_stream_blocks(R * C)), 256, 0, stream>>>(a);
    else
      bn_bwd_apply_kernel<<<grid_for(R * C, 8), 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
    return 0;
  }
  if (bn_tiled_ok(C, {dout, y, res, dx, dres})) {
    if (mode == 1) {
      // each block ends with 2*min(C,64) global atomics: a moderate grid, deep per-thread ILP
      bn_bwd_reduce_tiled_kernel<<<bn_tiled_grid(R, C, bn_reduce_blocks(R * C)), 256, 0, stream>>>(a);
      TDE_LAUNCH_CHECK();
    }
    bn_bwd_apply_tiled_kernel<<<bn_tiled_grid(R, C, bn_stream_blocks(R * C)), 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
    return 0;
  }
  const int g = grid_for(R * C, 8);
  static const bool cols_off = getenv("TDE_BN_COLS_OFF") != nullptr;
  if (mode == 1 && C > 16 && R <= 1024 && !cols_off) {
    bn_bwd_reduce_cols_kernel<<<dim3((C + 63) / 64, (unsigned)((R + kBnColsRows - 1) / kBnColsRows)), 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
  } else if (mode == 1 && C <= 16 && drop_rate == 0.f) {
    // narrow layers: row-per-thread reduction (~2 rows per thread, <= 256 blocks)
    // rows per block (TDE_BN_ROWS_PER_BLOCK, default 256 = one row per thread; Model B 588k / 593k vs 587k / 590k
    // img/s at 512), at most 1024 blocks
    static const int rpb = [] {
      const char* e = getenv("TDE_BN_ROWS_PER_BLOCK");
      return e && atoi(e) > 0 ? atoi(e) : 256;
    }();
    long long gr = (R + rpb - 1) / rpb;
    gr = gr < 1 ? 1 : (gr > 1024 ? 1024 : gr);
    if (C <= 8) bn_bwd_reduce_rows_kernel<8><<<(int)gr, 256, 0, stream>>>(a);
    else bn_bwd_reduce_rows_kernel<16><<<(int)gr, 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
  } else if (mode == 1) {
    // Reduction grid: <= 2 blocks per CU (each block ends with 2*C global atomics, so more blocks only
    // add contention), rounded to a multiple of C / gcd(2048, C) so the grid stride is a multiple of C
    // and every thread accumulates fixed channels in registers.
    int gr = g < 512 ? g : 512;
    int gc = C, t = 2048;
    while (t) {
      const int r = gc % t;
      gc = t;
      t = r;
    }
    const int mult = C / gc;
    gr = ((gr + mult - 1) / mult) * mult;
    bn_bwd_reduce_kernel<<<gr, 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
  }
  bn_bwd_apply_kernel<<<g, 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_act_bwd(const bf16* dout, const bf16* out, long long R, int C, int relu, bf16* dz, float* dbias,
                        hipStream_t stream) {
  if (R * C >= (1LL << 31)) return -4;
  if (C > kMaxCB) return -1;
  if (g_det && dbias) {
    if (dz) {
      act_bwd_kernel<<<grid_for(R * C, 8), 256, 0, stream>>>(dout, out, R, C, relu, dz, nullptr);
      TDE_LAUNCH_CHECK();
    }
    colsum_det_kernel<<<(C + 63) / 64, 256, 0, stream>>>(dout, out, R, C, relu, dbias);
    TDE_LAUNCH_CHECK();
    return 0;
  }
  act_bwd_kernel<<<grid_for(R * C, 8), 256, 0, stream>>>(dout, out, R, C, relu, dz, dbias);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_maxpool(const bf16* x, bf16* y, unsigned char* idx, const bf16* dy, bf16* dx, int dx_accum,
                        const int* geo, int backward, hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if (g.KH * g.KW > 256) return -1;
  if ((long long)g.B * g.H * g.W * g.C >= (1LL << 31) || (long long)g.B * g.Ho * g.Wo * g.C >= (1LL << 31)) return -4;
  PoolArgs a{x, y, idx, dy, dx, dx_accum, g};
  const bool vec = g.C % 8 == 0 && ((uintptr_t)(backward ? (const void*)dy : (const void*)x) & 15) == 0;
  if (vec) {
    if (!backward) maxpool_fwd8_kernel<<<grid_for((long long)g.B * g.Ho * g.Wo * g.C, 8), 256, 0, stream>>>(a);
    else if ((g.KH + g.sh - 1) / g.sh <= 2 && (g.KW + g.sw - 1) / g.sw <= 2 && g.KH * g.KW < 255 &&
             (long long)g.B * g.H <= 65535) {
      static const bool pair_off = getenv("TDE_MAXPOOL_BWD_SINGLE") != nullptr;
      if (!pair_off && (g.KW + g.sw) / g.sw <= 2) {
        const int per_row = ((g.W + 1) / 2) * (g.C / 8);
        maxpool_bwd8_w2p_kernel<<<dim3((per_row + 255) / 256, g.B * g.H), 256, 0, stream>>>(a);
      } else {
        const int per_row = g.W * (g.C / 8);
        maxpool_bwd8_w2_kernel<<<dim3((per_row + 255) / 256, g.B * g.H), 256, 0, stream>>>(a);
      }
    } else maxpool_bwd8_kernel<<<grid_for((long long)g.B * g.H * g.W * g.C, 8), 256, 0, stream>>>(a);
    TDE_LAUNCH_CHECK();
    return 0;
  }
  if (!backward) maxpool_fwd_kernel<<<grid_for((long long)g.B * g.Ho * g.Wo * g.C), 256, 0, stream>>>(a);
  else maxpool_bwd_kernel<<<grid_for((long long)g.B * g.H * g.W * g.C), 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// BatchNorm (mode 1 batch statistics / 2 moving statistics) + ReLU + MaxPool forward (bn_relu_maxpool_fwd_kernel):
// y [R = B*H*W, C] conv output -> pooled [B, Ho, Wo, C] + argmax bytes; geo = the pool geometry
TDE_API int tde_bn_relu_maxpool_fwd(const bf16* y, long long R, int C, int mode, const double* stats, float* saved,
                                    const float* gamma, const float* beta, float eps, float* mmean, float* mvar,
                                    float momentum, float bessel, float* zero_buf, bf16* pooled, unsigned char* idx,
                                    const int* geo, hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if (C > kMaxC || C % 8 != 0 || g.C != C || (long long)g.B * g.H * g.W != R) return -1;
  if (mode != 1 && mode != 2) return -1;
  if (g.KH * g.KW > 255 || ((uintptr_t)y & 15) != 0 || ((uintptr_t)pooled & 15) != 0) return -1;
  if (R * C >= (1LL << 31)) return -4;
  BnFwdArgs a{y, nullptr, nullptr, R, C, mode, stats, saved, gamma, beta, eps, mmean, mvar, momentum, bessel, zero_buf, 1,
              Drop{0.f, 0, nullptr, 0, 0}};
  PoolArgs pa{y, pooled, idx, nullptr, nullptr, 0, g};
  bn_relu_maxpool_fwd_kernel<<<grid_for((long long)g.B * g.Ho * g.Wo * C, 8), 256, 0, stream>>>(a, pa);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Backward of tde_bn_relu_maxpool_fwd (bn_pool_bwd_kernel): pooled gradient dpool [B, Ho, Wo, C] + argmax bytes
// -> the BN input gradient dx [R, C] (dstats: [slots][2][C] f32, zeroed by the forward)
TDE_API int tde_bn_pool_bwd(const bf16* dpool, const unsigned char* idx, const bf16* y, long long R, int C,
                            const float* saved, const float* gamma, const float* beta, int relu, float* dstats, bf16* dx,
                            int dx_accum, float* dgamma, float* dbeta, double* zero_fwd, const int* geo,
                            hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if (C > 512 || C % 8 != 0 || 256 % (C / 8) != 0 || g.C != C || (long long)g.B * g.H * g.W != R) return -1;
  if ((g.KH + g.sh - 1) / g.sh > 2 || (g.KW + g.sw) / g.sw > 2 || g.KH * g.KW >= 255) return -1;
  if (((uintptr_t)y & 15) != 0 || ((uintptr_t)dx & 15) != 0 || ((uintptr_t)dpool & 15) != 0 || !saved || !dstats)
    return -1;
  if (R * C >= (1LL << 31)) return -4;
  BnBwdArgs a{nullptr, y, nullptr, R, C, 1, saved, gamma, beta, relu, Drop{0.f, 0, nullptr, 0, 0}, dstats, dx,
              dx_accum, nullptr, 0, dgamma, dbeta, zero_fwd};
  PoolArgs pa{nullptr, nullptr, const_cast<unsigned char*>(idx), dpool, dx, dx_accum, g};
  // the staging loads of bn_pool_bwd_kernel cover <= 2 x 256 dy chunks and 256 argmax chunks per pooled row
  if ((long long)g.Wo * C > kBnPoolRow || (g.Wo * C) % 16 != 0 || ((uintptr_t)idx & 15) != 0) return -1;
  if (kBnPoolRow / 8 > 2 * 256 || kBnPoolRow / 16 > 256) return -1;
  // one input row per block iteration (its <= 2 pooled rows staged in LDS); the reduction ends with 2*C
  // atomics per block, so it takes a moderate grid, the apply pass one block per row
  const int rows = g.B * g.H;
  const size_t lds = bn_pool_bwd_lds(C, g.Wo * C);
  bn_pool_bwd_kernel<0><<<rows < 1024 ? rows : 1024, 256, lds, stream>>>(a, pa);
  TDE_LAUNCH_CHECK();
  bn_pool_bwd_kernel<1><<<rows < 16384 ? rows : 16384, 256, lds, stream>>>(a, pa);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_gap(const bf16* x, bf16* y, int B, int HW, int C, int backward, int accum, hipStream_t stream) {
  if ((long long)B * HW * C >= (1LL << 31)) return -4;
  if (!backward && C % 64 == 0 && aligned16(x) && (long long)B * (C / 64) < (1LL << 31))
    gap_fwd_vec_kernel<<<B * (C / 64), 256, 0, stream>>>(x, y, B, HW, C);
  else if (!backward) gap_fwd_kernel<<<grid_for((long long)B * C), 256, 0, stream>>>(x, y, B, HW, C);
  else gap_bwd_kernel<<<grid_for((long long)B * HW * C), 256, 0, stream>>>(x, y, B, HW, C, accum);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_pad(const bf16* src, bf16* dst, const int* geo, int backward, int accum, hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if ((long long)g.B * g.Ho * g.Wo * g.C >= (1LL << 31)) return -4;
  pad_kernel<<<grid_for((long long)g.B * g.Ho * g.Wo * g.C), 256, 0, stream>>>(src, dst, g, backward, accum);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_xent(const float* logits, long long ldl, const int* labels, int B, int C, float scale, bf16* dlogits,
                     long long ldd, float* metrics, float* probs, int probs_are_logits, long long* iterations,
                     hipStream_t stream) {
  if (B <= 0) return 0;
  XentArgs a{logits, ldl, labels, B, C, scale, dlogits, ldd, metrics, probs, probs_are_logits, iterations};
  if (C <= 64 * 16) xent_kernel<16><<<(B + 3) / 4, 256, 0, stream>>>(a);
  else xent_kernel<0><<<(B + 3) / 4, 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_colstats(const bf16* x, long long R, int C, double* stats, hipStream_t stream) {
  if (R * C >= (1LL << 31)) return -4;
  if (C > kMaxCB) return -1;
  if (g_det) return colstats_det(x, R, C, C, stats, stream);
  colstats_kernel<<<grid_for(R * C, 8), 256, 0, stream>>>(x, R, C, stats);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Strided-conv input gradient: zero the input pixels of the stride phases no filter tap reaches (bit
// (ph_h * sw + ph_w) of `untapped`), e.g. 3 of the 4 phases of a 1x1 stride-2 projection; the tapped phases'
// GEMMs then store (not accumulate) their pixels.  16-byte stores over C % 8 == 0 channels.
__global__ __launch_bounds__(256) void dgrad_phase_zero_kernel(bf16* __restrict__ dx, Geo g, unsigned untapped) {
  // 32-bit index math (the host bounds the chunk count below 2^31)
  const int cv = g.C >> 3;
  const int n = g.B * g.H * g.W * cv;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int pix = i / cv, row = pix / g.W, iw = pix - row * g.W, ih = row % g.H;
    if ((untapped >> ((ih % g.sh) * g.sw + iw % g.sw)) & 1u) reinterpret_cast<bf16x8*>(dx)[i] = zero8();
  }
}

TDE_API int tde_dgrad_phase_zero(bf16* dx, const int* geo, unsigned untapped, hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if (g.C % 8 || ((uintptr_t)dx & 15) || g.sh * g.sw > 32) return -1;
  if ((long long)g.B * g.H * g.W * (g.C / 8) >= (1LL << 31)) return -4;
  dgrad_phase_zero_kernel<<<grid_for((long long)g.B * g.H * g.W * (g.C / 8)), 256, 0, stream>>>(dx, g, untapped);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_cast_f32_bf16(const float* x, bf16* y, long long n, hipStream_t stream) {
  if (((uintptr_t)x & 15) != 0) return -1;
  cast_kernel<<<grid_for(n, 4), 256, 0, stream>>>(x, y, n);
  TDE_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------------
// Packed stem (C <= 4 input channels, stride 2 along W: the RGB 7x7/2 stem of ResNet): the zero-padded
// input is re-laid as [B][Hp][Wv][8] with element (b, r, v, 4j + c) = x[b][r - pt][2v + j - pl][c], i.e. a
// "virtual pixel" is two real pixels x 4 channels, and the conv becomes a valid, stride-(sh, 1) conv with
// C' = 8 channels and KW' = ceil(KW / 2) taps on it (weights packed likewise, the phantom taps zero):
// every 16-byte chunk of an implicit-GEMM row is contiguous in memory, so the stem runs through the
// LDS-DMA implicit GEMM (whole-kernel-row k-tiles, C' * KW' = 32) instead of an explicit im2col
// (244 MB per ResNet-18 step at batch 64).  g = the real geometry; Hp / Wv from Ho / Wo.
__global__ __launch_bounds__(256) void stem_pack_kernel(const bf16* __restrict__ x, Geo g, int Hp, int Wv,
                                                        int KWv, bf16* __restrict__ xp,
                                                        const bf16* __restrict__ wt, bf16* __restrict__ wv,
                                                        long long nx_blocks) {
  const int K = g.KH * g.KW * g.C, Kv = g.KH * KWv * 8;
  if ((long long)blockIdx.x >= nx_blocks) {  // weights: wt [Co][K] -> wv [Co][Kv]
    const long long n = (long long)g.Co * Kv;
    for (long long i = ((long long)blockIdx.x - nx_blocks) * 256 + threadIdx.x; i < n; i += 256LL * 8) {
      const int co = (int)(i / Kv), k = (int)(i - (long long)co * Kv);
      const int kh = k / (KWv * 8), r = k - kh * KWv * 8, kv = r >> 3, j = (r >> 2) & 1, c = r & 3;
      const int kw = 2 * kv + j;
      wv[i] = (kw < g.KW && c < g.C) ? wt[(long long)co * K + (kh * g.KW + kw) * g.C + c] : (bf16)0.0f;
    }
    return;
  }
  // input: one thread per virtual pixel (16 bytes out); 32-bit index math (the host bounds nv * 8 < 2^31)
  const int nv = g.B * Hp * Wv;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nv; i += (int)nx_blocks * 256) {
    const int br = i / Wv, v = i - br * Wv;
    const int b = br / Hp, r = br - b * Hp;
    const int ih = r - g.pt;
    bf16x8 o = zero8();
    const int iw0 = 2 * v - g.pl;
    const long long px0 = ((long long)b * g.H + ih) * g.W + iw0;
    if (g.C == 3 && (unsigned)ih < (unsigned)g.H && iw0 >= 0 && iw0 + 1 < g.W && ((px0 * 6) & 3) == 0) {
      // RGB, both real pixels inside: their 6 channels are 12 contiguous, 4-byte aligned bytes
      const unsigned* src = reinterpret_cast<const unsigned*>(x + px0 * 3);
      const unsigned w0 = src[0], w1 = src[1], w2 = src[2];
      unsigned short h[6] = {(unsigned short)w0, (unsigned short)(w0 >> 16), (unsigned short)w1,
                             (unsigned short)(w1 >> 16), (unsigned short)w2, (unsigned short)(w2 >> 16)};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        o[c] = __builtin_bit_cast(bf16, h[c]);
        o[4 + c] = __builtin_bit_cast(bf16, h[3 + c]);
      }
    } else if ((unsigned)ih < (unsigned)g.H) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int iw = 2 * v + j - g.pl;
        if ((unsigned)iw < (unsigned)g.W) {
          const bf16* src = x + (((long long)b * g.H + ih) * g.W + iw) * g.C;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (c < g.C) o[4 * j + c] = src[c];
        }
      }
    }
    *reinterpret_cast<bf16x8*>(xp + (long long)i * 8) = o;
  }
}

// gW[kh][kw][c][co] += gWv[kh][kw/2][4 (kw%2) + c][co]; every gWv element (phantom taps / channels too) is
// zeroed by the thread that read it, re-arming the buffer for the next step's accumulation
__global__ __launch_bounds__(256) void stem_unpack_wgrad_kernel(float* __restrict__ gwv, Geo g, int KWv,
                                                                float* __restrict__ gw) {
  const int nv = g.KH * KWv * 8 * g.Co;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < nv; e += gridDim.x * 256) {
    const int co = e % g.Co, t = e / g.Co, r = t % 8, t2 = t / 8, kv = t2 % KWv, kh = t2 / KWv;
    const int kw = 2 * kv + (r >> 2), c = r & 3;
    const float v = gwv[e];
    gwv[e] = 0.f;
    if (kw < g.KW && c < g.C) gw[((kh * g.KW + kw) * g.C + c) * g.Co + co] += v;
  }
}

// geo: the REAL conv geometry (C <= 4, sw == 2); xp [B][Hp][Wv][8] with Hp = (Ho-1)*sh + KH, Wv = Wo + KWv - 1,
// KWv = ceil(KW / 2); wt/wv optional (weights packed in the same launch)
TDE_API int tde_stem_pack(const bf16* x, const int* geo, bf16* xp, const bf16* wt, bf16* wv, hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if (g.C > 4 || g.sw != 2 || ((uintptr_t)xp & 15)) return -1;
  const int KWv = (g.KW + 1) / 2, Hp = (g.Ho - 1) * g.sh + g.KH, Wv = g.Wo + KWv - 1;
  const long long nv = (long long)g.B * Hp * Wv;
  if (nv * 8 >= (1LL << 31)) return -4;
  long long nxb = (nv + 255) / 256;
  nxb = nxb > 8192 ? 8192 : nxb;
  const int wb = (wt && wv) ? 8 : 0;
  stem_pack_kernel<<<(int)nxb + wb, 256, 0, stream>>>(x, g, Hp, Wv, KWv, xp, wt, wv, nxb);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_stem_unpack_wgrad(float* gwv, const int* geo, float* gw, hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if (g.C > 4 || g.sw != 2) return -1;
  const int nv = g.KH * ((g.KW + 1) / 2) * 8 * g.Co;
  stem_unpack_wgrad_kernel<<<(nv + 255) / 256, 256, 0, stream>>>(gwv, g, (g.KW + 1) / 2, gw);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_im2col(const bf16* x, const int* geo, int Kp, bf16* out, const bf16* w_in, bf16* w_out,
                       hipStream_t stream) {
  Geo g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9], geo[10], geo[11], geo[12]};
  if (Kp % 8 || Kp < g.KH * g.KW * g.C || ((uintptr_t)out & 15)) return -1;
  if (Kp / 8 > 256 || g.C >= 1024 || g.KW >= 1024) return -2;  // per-block tap table / packing
  if ((long long)g.B * g.Ho * g.Wo * (Kp / 8) >= (1LL << 31) || (long long)g.B * g.H * g.W * g.C >= (1LL << 31))
    return -4;
  const int wb = w_in ? 8 : 0;
  // row-staged path: the KH input rows of one output row fit the LDS buffer
  const int SPAN = ((g.Wo - 1) * g.sw + g.KW) * g.C;  // elements of one staged row
  const int PAD = (8 - (g.pl * g.C) % 8) % 8;
  const int LROW = (PAD + SPAN + 7) / 8 * 8;
  const int VROW = (g.W * g.C) % 8 == 0 && ((uintptr_t)x & 15) == 0 && g.pl * g.C + g.W * g.C <= SPAN;
  static const bool rows_off = getenv("TDE_IM2COL_GATHER") != nullptr;
  if (!rows_off && g.KH * LROW <= kI2cLds && Kp / 8 <= 256 && (long long)g.B * g.Ho < (1LL << 30) &&
      (long long)g.B * g.Ho * g.Wo * Kp < (1LL << 40)) {
    const int pix = g.B * g.Ho;
    im2col_rows_kernel<<<pix + wb, 256, 0, stream>>>(x, g, Kp, LROW, PAD, VROW, out, w_in, w_out, pix);
    TDE_LAUNCH_CHECK();
    return 0;
  }
  const int pix = grid_for((long long)g.B * g.Ho * g.Wo * (Kp / 8));
  im2col_kernel<<<pix + wb, 256, 0, stream>>>(x, g, Kp, out, w_in, w_out, pix);
  TDE_LAUNCH_CHECK();
  return 0;
}
