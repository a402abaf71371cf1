// Shared pieces of the fused DWK/TF2M small-CNN step kernels
//   Conv2D(32,3x3,VALID,bias,ReLU) · MaxPooling2D(2) · Flatten · Dense(64) · Dense(C) + SCCE
// (distributed_with_keras.py:33-43, tf2_mnist_distributed.py:66-72).
//
// Two precisions are built from these pieces:
//   convnet.hip      bf16 MFMA (16x16x32) Dense GEMMs over bf16 pooled tiles / weight shadows
//                    (Keras mixed_bfloat16 policy)
//   convnet_f32.hip  exact-f32 MFMA (16x16x4 f32) over f32 tiles and the f32 master weights
//                    (Keras float32 policy: the reference's precision, distributed_with_keras.py:21)
// The conv (VALU, f32), the classifier head (f32 MFMA), the softmax-CE, the fused optimizer
// and the deferred conv update are the same code in both.
#pragma once
#include "tde_optim.h"
#include "tde_xgmi.h"

namespace tde {
namespace cnet {

constexpr int CC = 32;   // conv filters
constexpr int HD = 64;   // Dense units
constexpr int NW = 16;   // waves of a backward workgroup

struct FwdArgs {
  const float* x; const float* wc; const float* bc;
  const void* W1; int ldw1;          // bf16 shadow ([K][HD] rows or [HD][K]) | f32 master [K][HD]
  float* hpre;                       // [B][HD] f32, += (pre-zeroed by the previous backward / head launch)
  void* Pt; int ldPt;                // [K][ldPt] pooled activations, transposed (nullable; bf16 | f32)
  uint64_t* amax; int lda;           // [P][CC/8][lda] pool argmax bytes (nullable)
  int B, H, W;
  long long* stamps;
  int w1_rows;                       // bf16: 1 = W1 is the row-major [K][HD] shadow (ldw1 = HD)
  // deferred conv update (fused step): while *pend the conv weights used are the optimizer
  // step of (wc, bc) with the previous backward's gradients (nullable: use wc, bc as stored)
  const int* pend;
  const float *gwc, *gbc, *mwc, *mbc, *vwc, *vbc;
  const long long* iterations;
  OptHyper h;
  unsigned long long* inc_iter;      // training: block 0 advances the step counter (nullable)
  int hrep; long long hrep_stride;   // hpre replicas: workgroup x adds into replica x % hrep
  int grep; long long grep_stride;   // deferred conv gradient = sum of grep replicas (<= 1: one)
  unsigned long long* fly_count;     // diagnostics (nullable): += 1 per forward that applied a pending update
  // fused step: the head variables this step's backward reads, snapshotted here (nullable hsnap: none).
  // The backward's head workgroup updates W2 / b2 / b1 in place while the trunk workgroups of the same
  // launch read them: they read the snapshot instead, so no workgroup can see a half-updated head.
  const float *hsrc_w2, *hsrc_b2, *hsrc_b1;
  float* hsnap;                      // [64 b1 | 64*hC W2 | hC b2]
  int hC;
};

// Fused step: one forward workgroup copies the head variables into the snapshot the backward reads.
__device__ __forceinline__ void fwd_snap_head(const FwdArgs& a, int nthreads) {
  if (!a.hsnap || blockIdx.x != 0 || blockIdx.y != 0) return;
  const int C = a.hC, n = HD + HD * C + C;
  for (int i = threadIdx.x; i < n; i += nthreads) {
    float v;
    if (i < HD) v = a.hsrc_b1 ? a.hsrc_b1[i] : 0.f;
    else if (i < HD + HD * C) v = a.hsrc_w2[i - HD];
    else v = a.hsrc_b2[i - HD - HD * C];
    a.hsnap[i] = v;
  }
}

// The input rows a workgroup's pooled positions touch (<= XR rows of <= XW floats per image)
// are staged into LDS with coalesced float4 loads: gathering 4x4 patches straight from HBM
// puts 64 distinct cache lines behind every load instruction.
constexpr int XR = 6, XW = 32;
// per-image stride of the staged rows padded to 2 (mod 64) floats: the per-lane (= per-image)
// float2 patch reads then hit distinct bank pairs (168 = 40 mod 64 for MNIST made them 8-way)
__host__ __device__ constexpr int fwd_istride(int W) { return XR * W + ((2 - (XR * W) % 64) + 64) % 64; }
constexpr int kConvW = CC * 10;     // conv taps [9][CC] + bias [CC] (floats), staged in LDS
constexpr int kXrBytes = 64 * (XR * XW + 64) * 4;

// Forward prologue, part 1: the <= XR input rows of the 64 images of this workgroup -> xr.
__device__ __forceinline__ void fwd_stage_x(const FwdArgs& a, float* xr, int b0, int py0, int nrows, int nthreads) {
  const int W = a.W, H = a.H;
  const int istride = fwd_istride(W);
  const int n4 = nrows * W / 4;  // float4 per image
  // all of this thread's row loads are issued before the first LDS store (one round trip)
  constexpr int kU = 8;
  for (int i0 = threadIdx.x; i0 < 64 * n4; i0 += kU * nthreads) {
    float4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * nthreads, bl = i / n4, q = i - bl * n4;
      v[u] = float4{0.f, 0.f, 0.f, 0.f};
      if (i < 64 * n4 && b0 + bl < a.B)
        v[u] = *reinterpret_cast<const float4*>(a.x + (size_t)(b0 + bl) * H * W + (size_t)(2 * py0) * W + q * 4);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = i0 + u * nthreads, bl = i / n4, q = i - bl * n4;
      if (i < 64 * n4) {
        // istride is only 8-byte aligned (bank padding): two 8-byte LDS writes
        float2* d2 = reinterpret_cast<float2*>(xr + bl * istride + q * 4);
        d2[0] = float2{v[u].x, v[u].y};
        d2[1] = float2{v[u].z, v[u].w};
      }
    }
  }
}

// Forward prologue, part 2: the conv weights in effect for this step -> wcs (with the
// deferred update applied while *pend).
__device__ __forceinline__ void fwd_stage_conv(const FwdArgs& a, float* wcs, int nthreads) {
  for (int i = threadIdx.x; i < kConvW; i += nthreads) {
    const bool isb = i >= 9 * CC;
    const int j = isb ? i - 9 * CC : i;
    float w = isb ? a.bc[j] : a.wc[j];
    if (a.pend) {
      const float* gp = isb ? a.gbc + j : a.gwc + j;
      float gv[kMaxGrep];
#pragma unroll
      for (int r = 0; r < kMaxGrep; ++r) gv[r] = (r == 0 || r < a.grep) ? gp[r * a.grep_stride] : 0.f;
      float g = gv[0];
#pragma unroll
      for (int r = 1; r < kMaxGrep; ++r) g += gv[r];
      float m = 0.f, v = 0.f;
      if (a.h.kind != kOptSGD) m = isb ? a.mbc[j] : a.mwc[j];
      if (a.h.kind == kOptAdam) v = isb ? a.vbc[j] : a.vwc[j];
      const long long t = a.h.kind == kOptAdam ? *a.iterations : 0;
      if (*a.pend) w = opt_step(a.h, opt_lr_t(a.h, t), w, g, m, v);
    }
    wcs[i] = w;
  }
}

// The 8 conv channels c0..c0+7 of one wave (wave-uniform LDS broadcast reads).
struct ConvW8 {
  float4 wlo[9], whi[9], blo, bhi;
  __device__ __forceinline__ void load(const float* wcs, int c0) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      wlo[t] = *reinterpret_cast<const float4*>(wcs + t * CC + c0);
      whi[t] = *reinterpret_cast<const float4*>(wcs + t * CC + c0 + 4);
    }
    blo = *reinterpret_cast<const float4*>(wcs + 9 * CC + c0);
    bhi = *reinterpret_cast<const float4*>(wcs + 9 * CC + c0 + 4);
  }
};

__device__ __forceinline__ float f4get(float4 q, int k) { return k == 0 ? q.x : (k == 1 ? q.y : (k == 2 ? q.z : q.w)); }

// Conv 3x3 + bias + ReLU + 2x2 max-pool of one image (lane) at one pooled position for the wave's
// 8 channels: xb points at the top-left of the 4x4 input patch in the staged rows (row stride W).
// out[cc] = pooled activation; packed = 8 argmax bytes (0..3 window slot, 0xFF: ReLU zeroed).
__device__ __forceinline__ void conv_pool8(const float* xb, int W, const ConvW8& cw, float out[8], uint64_t& packed) {
  float patch[16];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float2 u = *reinterpret_cast<const float2*>(xb + r * W);
    const float2 v = *reinterpret_cast<const float2*>(xb + r * W + 2);
    patch[r * 4 + 0] = u.x; patch[r * 4 + 1] = u.y; patch[r * 4 + 2] = v.x; patch[r * 4 + 3] = v.y;
  }
  packed = 0;
#pragma unroll
  for (int cc = 0; cc < 8; ++cc) {
    float wt[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t] = f4get(cc < 4 ? cw.wlo[t] : cw.whi[t], cc & 3);
    const float bcv = f4get(cc < 4 ? cw.blo : cw.bhi, cc & 3);
    float best = -3.0e38f;
    int bi = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int dy = q >> 1, dx = q & 1;
      float z = bcv;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) z = fmaf(patch[(dy + ky) * 4 + dx + kx], wt[ky * 3 + kx], z);
      if (z > best) { best = z; bi = q; }
    }
    out[cc] = fmaxf(best, 0.f);
    packed |= (uint64_t)(best > 0.f ? (unsigned)bi : 0xFFu) << (8 * cc);
  }
}

// Backward of the trunk with the classifier head fused in (the head is
// the same math as head.hip): per 64-image chunk every workgroup recomputes the head from the
// Dense(64) pre-activation (16 KB f32): h = ReLU(hpre + b1) -> logits = h . W2 + b2 (exact f32
// MFMA) -> softmax-CE -> dl = (p - onehot) * scale -> G = dl . W2^T masked by h > 0, straight into
// LDS — the Dense(64) input gradient every workgroup needs anyway.  ONE workgroup (the last) also
// produces the head's side outputs — loss and accuracy, dW2 = h^T . dl, db2, db1 (complete sums,
// no atomics) — and stores them or, in the fused step, applies the update to them.
// hpre is double-buffered by step parity: this launch reads hpre[p] and zeroes hpre[1-p] (read by
// the previous step's backward, accumulated into by the next forward): no in-kernel hand-off.
struct BwdArgs {
  const float* x; const uint64_t* amax; int lda;
  const float* hpre;                 // [B][HD] f32 Dense(64) pre-activation (this step's parity)
  float* hzero;                      // [B][HD] the other parity buffer, zeroed here
  int hrep; long long hrep_stride;   // hpre replicas (summed on load; all zeroed)
  float* cpart;                      // deterministic mode: per-workgroup conv-gradient partials (nullable)
  const float* b1; const float* W2; const float* b2; int C; int pre_relu;
  const int* labels;
  float scale;                       // 1 / global batch (Keras AUTO reduction under a strategy)
  float* metrics;                    // += {loss_sum, correct, count}
  const void* W1; int ldw1;          // bf16 row-major shadow [K][HD] | f32 master [K][HD]
  const void* Pt; int ldPt;          // [K][ldPt] (bf16 | f32)
  float* dW1;                        // [K][HD] f32 (MODE 0: stored)
  float* dwc; float* dbc;            // [9][CC], [CC] (atomic +=)
  int crep; long long crep_stride;   // workgroup x adds into conv-gradient replica x % crep (<= 1: one)
  float *dW2, *db2, *db1;            // MODE 0: head gradients (+= by the head workgroup)
  int B, H, W;
  long long* stamps;
  // fused step (MODE != 0)
  float *w1, *m1, *v1;               // fp32 master [K][HD] (+ slots), updated in place
  bf16* w1r_out;                     // bf16: row-major shadow (== W1), rewritten
  bf16* w1c_out; int ldw1c;          // bf16: transposed shadow [HD][ldw1c] (nullable)
  float *hw, *hm, *hv;               // flat weight / slot buffers (head variables at the offsets below)
  long long off_w2, off_b2, off_b1;  // off_b1 < 0: the Dense(64) has no bias
  const long long* iterations;       // t of this step (advanced by this step's forward)
  long long* iter_prev;              // := t by the head workgroup (read by the next forward)
  OptHyper h;
  FlatApply commit;                  // the previous step's deferred conv update (head workgroup, while *pend)
  int* pend_set;                     // := 1: this step's conv update is deferred
  XgPush push;                       // MODE 0, nranks > 0: dW1 goes to the xGMI owners (fused DP exchange)
};

// Up to NPER elements per thread of a FlatApply's ranges, loaded early into registers and
// updated later (the loads' latency hides behind the caller's work).
template <int NPER>
struct FlatPrefetch {
  int e[NPER];
  float w[NPER], g[NPER], m[NPER], v[NPER];
  __device__ __forceinline__ void load(const FlatApply& f, int tid, int nt) {
#pragma unroll
    for (int k = 0; k < NPER; ++k) {
      int idx = tid + k * nt;
      e[k] = -1;
      for (int r = 0; r < f.nr; ++r) {
        if (idx < f.n[r]) {
          e[k] = f.lo[r] + idx;
          break;
        }
        idx -= f.n[r];
      }
      w[k] = g[k] = m[k] = v[k] = 0.f;
      if (e[k] >= 0) {
        w[k] = f.w[e[k]];
        g[k] = flat_grad(f, e[k]);
        if (f.h.kind != kOptSGD) m[k] = f.m[e[k]];
        if (f.h.kind == kOptAdam) v[k] = f.v[e[k]];
      }
    }
  }
  __device__ __forceinline__ void apply(const FlatApply& f, long long t) {
    const float lr_t = opt_lr_t(f.h, t);
#pragma unroll
    for (int k = 0; k < NPER; ++k) {
      if (e[k] < 0) continue;
      f.w[e[k]] = opt_step(f.h, lr_t, w[k], g[k], m[k], v[k]);
      flat_grad_zero(f, e[k]);
      if (f.h.kind != kOptSGD) f.m[e[k]] = m[k];
      if (f.h.kind == kOptAdam) f.v[e[k]] = v[k];
    }
  }
};

__device__ __forceinline__ f32x4 mfma_f32x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// LDS of the head pieces (16 waves, 64 rows)
constexpr int HS = HD + 4;   // f32 row stride of h
// row strides of dlogits [64][16] and W2 [HD][16]: 17, not 16, so the 16 rows a wave reads at one column
// (dH = dl . W2^T) fall on 16 different LDS banks (stride 16: 8-way conflicts in every workgroup's head)
constexpr int DLS = 17, W2S = 17;
constexpr int kHeadScratch = 64 * HS * 4 + 12 * 64 * 4 * 4 + 64 * DLS * 4;   // hs + part + dls
struct HeadLds {
  float* hs;     // [64][HS]      h = act(hpre + b1)
  float* part;   // [12][64][4]   logits partial sums
  float* dls;    // [64][DLS]     dlogits
  float* w2s;    // [HD][W2S]     W2, classes padded to 16
  float* b2s;    // [16]
  int* labs;     // [64]
  __device__ __forceinline__ static HeadLds carve(unsigned char* scratch, unsigned char* w2, unsigned char* b2,
                                                  unsigned char* lab) {
    HeadLds l;
    l.hs = reinterpret_cast<float*>(scratch);
    l.part = reinterpret_cast<float*>(scratch + 64 * HS * 4);
    l.dls = reinterpret_cast<float*>(scratch + 64 * HS * 4 + 12 * 64 * 4 * 4);
    l.w2s = reinterpret_cast<float*>(w2);
    l.b2s = reinterpret_cast<float*>(b2);
    l.labs = reinterpret_cast<int*>(lab);
    return l;
  }
};
constexpr int kW2Bytes = HD * W2S * 4, kB2Bytes = 16 * 4, kLabBytes = 64 * 4;

// W2 image (classes padded to 16) and b2 into LDS (1024 threads)
__device__ __forceinline__ void head_load_w2(const BwdArgs& a, const HeadLds& l, int tid) {
  const int u = tid >> 4, c = tid & 15;   // 64 x 16
  l.w2s[u * W2S + c] = c < a.C ? a.W2[u * a.C + c] : 0.f;
  if (tid < 16) l.b2s[tid] = tid < a.C ? a.b2[tid] : 0.f;
}

// This workgroup's slice of the other parity buffer of hpre zeroed for the next forward's atomics
__device__ __forceinline__ void zero_other_parity(const BwdArgs& a, int tid) {
  const int n4 = (int)(((a.hrep - 1) * a.hrep_stride + (long long)a.B * HD) / 4);
  const int per = (n4 + gridDim.x - 1) / gridDim.x, beg = blockIdx.x * per;
  const int end = min(n4, beg + per);
  for (int i = beg + tid; i < end; i += 1024) reinterpret_cast<float4*>(a.hzero)[i] = float4{0.f, 0.f, 0.f, 0.f};
}

// hpre[row][c4..c4+3] summed over the replicas (loads issued together).  More than 4 replicas: the
// deterministic mode (TDE_DETERMINISTIC: one replica per forward workgroup, each written by exactly one
// add into zeros), summed in replica order.
__device__ __forceinline__ float4 load_hpre(const BwdArgs& a, int row, int c4) {
  constexpr int kMaxRep = 8;
  if (a.hrep > kMaxRep) {
    float4 s = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.hrep; ++r) {
      const float4 v = *reinterpret_cast<const float4*>(a.hpre + (size_t)r * a.hrep_stride + (size_t)row * HD + c4);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    return s;
  }
  float4 v[kMaxRep];
#pragma unroll
  for (int r = 0; r < kMaxRep; ++r)
    v[r] = r < a.hrep ? *reinterpret_cast<const float4*>(a.hpre + (size_t)r * a.hrep_stride + (size_t)row * HD + c4)
                      : float4{0.f, 0.f, 0.f, 0.f};
  float4 s = v[0];
#pragma unroll
  for (int r = 1; r < kMaxRep; ++r) {
    s.x += v[r].x; s.y += v[r].y; s.z += v[r].z; s.w += v[r].w;
  }
  return s;
}

// h = act(hpre + b1) of this thread's row / 4 units into LDS (rows past nb zeroed)
__device__ __forceinline__ void head_stage(const BwdArgs& a, float4 hv, float4 b1v, int hr, int hc4, int nb,
                                           float* hs) {
  float4 h = float4{hv.x + b1v.x, hv.y + b1v.y, hv.z + b1v.z, hv.w + b1v.w};
  if (a.pre_relu) h = float4{fmaxf(h.x, 0.f), fmaxf(h.y, 0.f), fmaxf(h.z, 0.f), fmaxf(h.w, 0.f)};
  if (hr >= nb) h = float4{0.f, 0.f, 0.f, 0.f};
  *reinterpret_cast<float4*>(hs + hr * HS + hc4) = h;
}

// logits = h . W2 + b2 (exact f32 MFMA; wave = 16-row tile x K quarter), softmax-CE on waves 0..3
// -> dls = dlogits [64][16]; loss / correct / count accumulated into la / ca / na (lanes fr == 0).
// Entered after a barrier that published hs / labs; ends with a barrier that publishes dls.
__device__ __forceinline__ void head_logits_ce(const BwdArgs& a, int nb, const HeadLds& l, int lane, int wave,
                                               float& la, float& ca, float& na) {
  const int fr = lane & 15, fq = lane >> 4, C = a.C;
  f32x4 lg = {0.f, 0.f, 0.f, 0.f};
  {
    const int rt = wave & 3, kq = wave >> 2;
#pragma unroll
    for (int k = kq * 16; k < kq * 16 + 16; k += 4)
      lg = mfma_f32x4(l.hs[(rt * 16 + fr) * HS + k + fq], l.w2s[(k + fq) * W2S + fr], lg);
    if (kq > 0) *reinterpret_cast<f32x4*>(l.part + (((kq - 1) * 4 + rt) * 64 + lane) * 4) = lg;
  }
  lds_barrier();
  if (wave < 4) {
    const int rt = wave;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const f32x4 pv = *reinterpret_cast<const f32x4*>(l.part + ((q * 4 + rt) * 64 + lane) * 4);
      lg[0] += pv[0]; lg[1] += pv[1]; lg[2] += pv[2]; lg[3] += pv[3];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rt * 16 + fq * 4 + i;
      const bool valid = r < nb;
      const bool cv = fr < C;
      const float z = cv ? lg[i] + l.b2s[fr] : -3.0e38f;
      const float m = row16_max(z);
      const float e = cv ? __expf(z - m) : 0.f;
      const float s = row16_sum(e);
      const float pr = e / s;
      const int label = l.labs[r];
      const int amx = row16_min(cv && z == m ? fr : 64);
      const float zl = __shfl(z, (lane & ~15) | (label & 15), 64);
      if (valid && fr == 0) {
        la += __logf(s) + m - zl;
        ca += (amx == label) ? 1.f : 0.f;
        na += 1.f;
      }
      l.dls[r * DLS + fr] = (valid && cv) ? (pr - (fr == label ? 1.f : 0.f)) * a.scale : 0.f;
    }
  }
  lds_barrier();
}

// dH tile of this wave (rows rt*16.., units ut*16.., rt = wave>>2, ut = wave&3) = dl . W2^T, masked
// by h > 0 and rows < nb.  Lane holds dH[rt*16 + 4fq + i][ut*16 + fr].
__device__ __forceinline__ f32x4 head_dh(const BwdArgs& a, int nb, const HeadLds& l, int lane, int wave) {
  const int fr = lane & 15, fq = lane >> 4, rt = wave >> 2, ut = wave & 3;
  f32x4 gh = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 16; k += 4)
    gh = mfma_f32x4(l.dls[(rt * 16 + fr) * DLS + k + fq], l.w2s[(ut * 16 + fr) * W2S + k + fq], gh);
  const int j = ut * 16 + fr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = rt * 16 + fq * 4 + i;
    if ((a.pre_relu && !(l.hs[r * HS + j] > 0.f)) || r >= nb) gh[i] = 0.f;
  }
  return gh;
}

// The head workgroup: loss / accuracy, dW2 = h^T . dl, db2, db1 over all chunks, then stored (MODE 0)
// or updated (fused step; with the previous step's deferred conv update and the flags).
// db1p: 256 floats of LDS scratch outside the head areas.
template <int MODE>
__device__ __forceinline__ void head_workgroup(const BwdArgs& a, const HeadLds& l, float* db1p) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fq = lane >> 4, C = a.C;
  const int hr = tid >> 4, hc4 = (tid & 15) * 4;
  const float4 b1v = a.b1 ? *reinterpret_cast<const float4*>(a.b1 + hc4) : float4{0.f, 0.f, 0.f, 0.f};

  // fused step: the variables this workgroup updates, loaded now.  waves 0..3: W2[wave*16 + 4fq + i][fr]
  // (the dW2 tile layout); wave 4: b2[fr]; wave 5: b1[lane]
  long long e[4] = {-1, -1, -1, -1};
  if (wave < 4 && fr < C) {
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = a.off_w2 + (long long)(wave * 16 + fq * 4 + i) * C + fr;
  } else if (wave == 4 && fq == 0 && fr < C) {
    e[0] = a.off_b2 + fr;
  } else if (wave == 5 && a.off_b1 >= 0) {
    e[0] = a.off_b1 + lane;
  }
  float hwv[4] = {0.f, 0.f, 0.f, 0.f}, hmv[4] = {0.f, 0.f, 0.f, 0.f}, hvv[4] = {0.f, 0.f, 0.f, 0.f};
  long long t_it = 0;
  FlatPrefetch<1> cp;
  int cpend = 0;
  if (MODE != 0) {
    t_it = *a.iterations;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (e[i] < 0) continue;
      hwv[i] = a.hw[e[i]];
      if (MODE == 2 && a.h.kind != kOptSGD) hmv[i] = a.hm[e[i]];
      if (MODE == 2 && a.h.kind == kOptAdam) hvv[i] = a.hv[e[i]];
    }
    if (a.commit.nr > 0) {
      cpend = *a.commit.pend;
      cp.load(a.commit, tid, 1024);
    }
  }

  f32x4 gw = {0.f, 0.f, 0.f, 0.f};
  float db1acc = 0.f, db2acc = 0.f, la = 0.f, ca = 0.f, na = 0.f;
  for (int b0 = 0; b0 < a.B; b0 += 64) {
    const int nb = min(64, a.B - b0);
    float4 hv = {0.f, 0.f, 0.f, 0.f};
    if (hr < nb) hv = load_hpre(a, b0 + hr, hc4);
    const int lab = (tid < nb) ? a.labels[b0 + tid] : 0;
    head_stage(a, hv, b1v, hr, hc4, nb, l.hs);
    if (tid < 64) l.labs[tid] = lab;
    lds_barrier();
    head_logits_ce(a, nb, l, lane, wave, la, ca, na);
    const f32x4 gh = head_dh(a, nb, l, lane, wave);
    db1acc += (gh[0] + gh[1]) + (gh[2] + gh[3]);
    if (wave < 4) {
#pragma unroll
      for (int k = 0; k < 64; k += 4) gw = mfma_f32x4(l.hs[(k + fq) * HS + wave * 16 + fr], l.dls[(k + fq) * DLS + fr], gw);
    } else if (wave == 4) {
#pragma unroll 4
      for (int r = fq * 16; r < fq * 16 + 16; ++r) db2acc += l.dls[r * DLS + fr];
    }
    lds_barrier();
  }
  // db1: over the 4 lane groups, then the 4 row-tile waves of each unit tile; db2: over the lane groups
  db1acc += __shfl_xor(db1acc, 16, 64);
  db1acc += __shfl_xor(db1acc, 32, 64);
  if (fq == 0) db1p[(wave >> 2) * 64 + (wave & 3) * 16 + fr] = db1acc;
  db2acc += __shfl_xor(db2acc, 16, 64);
  db2acc += __shfl_xor(db2acc, 32, 64);
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
  lds_barrier();
  float gv[4] = {0.f, 0.f, 0.f, 0.f};
  float* gdst[4] = {nullptr, nullptr, nullptr, nullptr};
  if (wave < 4 && fr < C) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gv[i] = gw[i];
      gdst[i] = a.dW2 ? a.dW2 + (size_t)(wave * 16 + fq * 4 + i) * C + fr : nullptr;
    }
  } else if (wave == 4 && fq == 0 && fr < C) {
    gv[0] = db2acc;
    gdst[0] = a.db2 ? a.db2 + fr : nullptr;
  } else if (wave == 5 && a.b1) {
    gv[0] = (db1p[lane] + db1p[64 + lane]) + (db1p[128 + lane] + db1p[192 + lane]);
    gdst[0] = a.db1 ? a.db1 + lane : nullptr;
  }
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (gdst[i]) *gdst[i] += gv[i];
    stamp(a.stamps, 7);
    return;
  }
  const float lr_t = opt_lr_t(a.h, t_it);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (e[i] < 0) continue;
    float m = hmv[i], v = hvv[i];
    a.hw[e[i]] = opt_step(a.h, lr_t, hwv[i], gv[i], m, v);
    if (MODE == 2 && a.h.kind != kOptSGD) a.hm[e[i]] = m;
    if (MODE == 2 && a.h.kind == kOptAdam) a.hv[e[i]] = v;
  }
  // the previous step's conv update (its forward used it on the fly; this launch does not read the
  // conv weights): commit it, clear its flag; flag this step's update (the trunk's atomics)
  if (cpend) cp.apply(a.commit, t_it - 1);
  if (tid == 0) {
    if (cpend) *a.commit.pend = 0;
    if (cpend && a.commit.count) atomicAdd(a.commit.count, 1ull);
    if (a.pend_set) *a.pend_set = 1;
    if (a.iter_prev) *a.iter_prev = t_it;
  }
  stamp(a.stamps, 7);   // diagnostics: the head workgroup's end (micro.py)
}

// Reduces the routing accumulators (conv weight / bias gradients: [tap 0..8 | bias 9][CC]) of the
// 16 waves through LDS (red: [NW][16][CC] f32) and adds them into dwc / dbc.
__device__ __forceinline__ void conv_grad_reduce(const BwdArgs& a, const f32x4 accr[2], float* red, int lane, int wave) {
  const int fr = lane & 15, fq = lane >> 4, tid = threadIdx.x;
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[((size_t)wave * 16 + fq * 4 + r) * CC + ct * 16 + fr] = accr[ct][r];
  lds_barrier();
  if (tid < 10 * CC) {
    const int tap = tid / CC, c = tid - tap * CC;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[((size_t)w * 16 + tap) * CC + c];
    if (a.cpart) a.cpart[(size_t)blockIdx.x * 10 * CC + tid] = s;   // deterministic: summed by cgrad_reduce
    else {
      // replicas spread the adds of the ~170 workgroups over crep addresses per value (the contention
      // of 170 same-address float atomics cost ~4 us of the MNIST-CNN backward)
      const long long ro = a.crep > 1 ? (long long)(blockIdx.x % a.crep) * a.crep_stride : 0;
      if (tap < 9) {
        if (a.dwc) atomicAdd(a.dwc + ro + tap * CC + c, s);
      } else if (a.dbc) {
        atomicAdd(a.dbc + ro + c, s);
      }
    }
  }
}

}  // namespace cnet
}  // namespace tde

// ---- host side: the ctypes structs of the entry points and the common argument checks

// Fused-step optimizer description shared by the convnet forward entry points (ctypes struct):
// slots m/v flat like w; iterations = the device step counter.
struct TdeStepOpt {
  int kind;
  float lr, mom, b1, b2, eps;
  float *w, *g, *m, *v;
  const long long* iterations;
  int* pend;
  int grep; long long grep_stride;   // g holds grep replicas (<= 1: one)
  unsigned long long* fly_count;      // diagnostics (nullable): forwards that applied the pending update
  const float *hsrc_w2, *hsrc_b2, *hsrc_b1;   // head snapshot (FwdArgs::hsnap; nullable hsnap: none)
  float* hsnap;
  int hC;
};

// Fused-step description of the backward (ctypes struct).
struct TdeBwdOpt {
  int kind;
  float lr, mom, b1, b2, eps;
  float *w, *m, *v;                   // flat buffers
  long long off_w1, off_w2, off_b2, off_b1;
  void* W1c; int ldw1c;               // bf16: transposed shadow (nullable)
  const long long* iterations;
  long long* iter_prev;
  tde::FlatApply commit;              // previous step's deferred conv update (nr = 0: none)
  int* pend_set;
  int crep; long long crep_stride;    // conv-gradient replicas this step accumulates into (<= 1: one)
};

namespace tde {
namespace cnet {

inline OptHyper hyper_of(const TdeStepOpt* o) { return OptHyper{o->kind, o->lr, o->mom, o->b1, o->b2, o->eps}; }
inline bool opt_ok(const TdeStepOpt* o) {
  return o->w && o->g && o->iterations && (o->kind == kOptSGD || o->m) && (o->kind != kOptAdam || o->v) &&
         (!o->hsnap || (o->hsrc_w2 && o->hsrc_b2 && o->hC >= 1 && o->hC <= 16 && !((uintptr_t)o->hsnap & 15)));
}

// The forward's deferred-update / step-counter / replica fields from the host arguments.
inline void fill_fwd_opt(FwdArgs& a, const TdeStepOpt* opt, long long off_wc, long long off_bc, long long* inc_iter,
                         int hrep, long long hrep_stride) {
  a.inc_iter = (unsigned long long*)inc_iter;
  a.hrep = hrep > 0 ? hrep : 1;
  a.hrep_stride = hrep_stride;
  if (opt) {
    a.pend = opt->pend;
    a.gwc = opt->g + off_wc;
    a.gbc = opt->g + off_bc;
    a.mwc = opt->m ? opt->m + off_wc : nullptr;
    a.mbc = opt->m ? opt->m + off_bc : nullptr;
    a.vwc = opt->v ? opt->v + off_wc : nullptr;
    a.vbc = opt->v ? opt->v + off_bc : nullptr;
    a.iterations = opt->iterations;
    a.h = hyper_of(opt);
    a.grep = opt->grep > 1 ? opt->grep : 1;
    a.grep_stride = opt->grep_stride;
    a.fly_count = opt->fly_count;
    a.hsrc_w2 = opt->hsrc_w2;
    a.hsrc_b2 = opt->hsrc_b2;
    a.hsrc_b1 = opt->hsrc_b1;
    a.hsnap = opt->hsnap;
    a.hC = opt->hC;
  } else {
    a.grep = 1;
    a.grep_stride = 0;
  }
}

// Common validation + fill of the backward arguments (returns 0 or a negative error code).
inline int fill_bwd(BwdArgs& a, const float* x, const void* amax, int lda, const float* hpre, float* hzero, int hrep,
                    long long hrep_stride, const float* b1, const float* W2, const float* b2, int C, int pre_relu,
                    const int* labels, float scale, float* metrics, const void* W1, int ldw1, const void* Pt, int ldPt,
                    float* dW1, float* dwc, float* dbc, float* dW2, float* db2, float* db1, int B, int H, int W,
                    long long* stamps, const TdeBwdOpt* opt) {
  if ((ldw1 & 7) || (ldPt & 7) || ldPt < B || lda < B || C < 1 || C > 16 || !hpre || !hzero || !labels) return -1;
  if ((((uintptr_t)hpre | (uintptr_t)hzero | (uintptr_t)b1) & 15)) return -2;
  if (opt && (!opt->w || !opt->iterations || (opt->kind != kOptSGD && !opt->m) || (opt->kind == kOptAdam && !opt->v) ||
              ldw1 != HD || (opt->W1c && (opt->ldw1c & 3)) || (opt->off_w1 & 3) || opt->commit.nr > kFlatRanges ||
              (opt->commit.nr > 0 && !opt->commit.pend) || (b1 != nullptr) != (opt->off_b1 >= 0)))
    return -4;
  if (opt && opt->commit.nr > 0) {
    int total = 0;
    for (int i = 0; i < opt->commit.nr; ++i) total += opt->commit.n[i];
    if (total > 1024) return -5;
  }
  if (hrep < 1 || hrep > 1024 || (hrep > 1 && (hrep_stride < (long long)B * HD || (hrep_stride & 3)))) return -6;
  a = BwdArgs{};
  a.x = x;
  a.amax = (const uint64_t*)amax;
  a.lda = lda;
  a.hpre = hpre;
  a.hzero = hzero;
  a.hrep = hrep;
  a.hrep_stride = hrep_stride;
  a.b1 = b1;
  a.W2 = W2;
  a.b2 = b2;
  a.C = C;
  a.pre_relu = pre_relu;
  a.labels = labels;
  a.scale = scale;
  a.metrics = metrics;
  a.W1 = W1;
  a.ldw1 = ldw1;
  a.Pt = Pt;
  a.ldPt = ldPt;
  a.dW1 = dW1;
  a.dwc = dwc;
  a.dbc = dbc;
  a.dW2 = dW2;
  a.db2 = db2;
  a.db1 = db1;
  a.B = B;
  a.H = H;
  a.W = W;
  a.stamps = stamps;
  a.off_b1 = -1;
  if (opt) {
    a.w1 = opt->w + opt->off_w1;
    a.m1 = opt->m ? opt->m + opt->off_w1 : nullptr;
    a.v1 = opt->v ? opt->v + opt->off_w1 : nullptr;
    a.w1r_out = (bf16*)W1;
    a.w1c_out = (bf16*)opt->W1c;
    a.ldw1c = opt->ldw1c;
    a.hw = opt->w;
    a.hm = opt->m;
    a.hv = opt->v;
    a.off_w2 = opt->off_w2;
    a.off_b2 = opt->off_b2;
    a.off_b1 = opt->off_b1;
    a.iterations = opt->iterations;
    a.iter_prev = opt->iter_prev;
    a.h = OptHyper{opt->kind, opt->lr, opt->mom, opt->b1, opt->b2, opt->eps};
    a.commit = opt->commit;
    a.pend_set = opt->pend_set;
    a.crep = opt->crep > 1 ? opt->crep : 1;
    a.crep_stride = opt->crep_stride;
  }
  return 0;
}

}  // namespace cnet
}  // namespace tde
