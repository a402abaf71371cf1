// Fused forward and backward of the DWK/TF2M small CNN trunk in float32 — the reference's
// precision (distributed_with_keras.py:21 casts the images to float32; every Keras layer of
// distributed_with_keras.py:33-43 / tf2_mnist_distributed.py:66-72 runs in the float32 policy).
//
// Same dataflow as the bf16 form (convnet.hip; shared pieces in tde_convnet.h), with every
// GEMM on the exact-f32 MFMA v_mfma_f32_16x16x4_f32 (bit-for-bit a k-ordered fmaf chain, no
// reduced-precision operand anywhere) over f32 LDS tiles and the f32 master weights — no bf16
// shadow exists in this form, so the optimizer writes nothing but the master weights.
//
// The f32 MFMA issues at 1/16 of the bf16 rate (MI355X_MICROARCH.md § Matrix cores), so the work
// per workgroup is cut to keep each CU's matrix pipe time small and spread over more CUs:
//   forward   FPW=1 pooled position x 64 images per workgroup (169 workgroups for MNIST);
//             wave w owns the output column tile w of all 4 row tiles (4 independent
//             accumulators, 32 MFMAs), split-K atomics into hpre as in the bf16 form;
//   backward  ONE pooled position per workgroup (169 + the head workgroup); per 64-image chunk
//             waves 0-7 compute dP = G . W1^T (8 tiles x 16 MFMAs) while waves 8-15 compute
//             the position's dW1 rows = P^T . G (8 tiles x 16 MFMAs), then all 16 waves run the
//             routing MFMA dWc[tap][c] = sum_{b,q} X[tap][(b,q)] D[(b,q)][c] (lane group = pool
//             window slot q, 8 MFMAs per wave).
//
// Fragment map of the 16x16x4 f32 MFMA: lane l holds A[l&15][k] and B[k][l&15] with k set by
// (l>>4, step); a lane's k for step s of a 16-k group is fq*16 + 4*((s/4 + fq) & 3) + s%4
// (fq = l>>4), so each lane reads its operands as float4 rows and, with 72-float LDS rows
// (40 for the 32-wide forward tile, 8-k groups), the ds_read_b128 lane groups hit disjoint
// banks (searched exhaustively over strides and per-group rotations).
#include "tde_convnet.h"

namespace tde {
using namespace cnet;

constexpr int PS32 = 40;   // f32 LDS row stride of the forward's pooled tile [64][32]
constexpr int GS32 = 72;   // f32 LDS row stride of the backward's 64-wide operand rows
constexpr int DPS32 = 40;  // f32 LDS row stride of dP [64][32]

constexpr int fwd32_lds(int fpw) { return fpw * 64 * PS32 * 4 + kXrBytes + kConvW * 4; }

// column of the float4 a lane reads for group i of a 32-wide (8 k per lane group) row
__device__ __forceinline__ int k8_col(int fq, int i) { return fq * 8 + 4 * ((i + fq) & 1); }
// ... and of a 64-wide (16 k per lane group) row
__device__ __forceinline__ int k16_col(int fq, int i) { return fq * 16 + 4 * ((i + fq) & 3); }

template <int FPW>
__global__ __launch_bounds__(FPW * 256) void convnet32_fwd_kernel(FwdArgs a) {
  constexpr int NT = FPW * 256;
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  float* Ps = reinterpret_cast<float*>(fsm);                                        // [FPW][64][PS32]
  float* xr = reinterpret_cast<float*>(fsm + FPW * 64 * PS32 * 4);                  // [64][XR][W]
  float* wcs = reinterpret_cast<float*>(fsm + FPW * 64 * PS32 * 4 + kXrBytes);      // [10][CC]
  stamp(a.stamps, 0);
  if (a.inc_iter && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(a.inc_iter, 1ull);
  if (a.fly_count && a.pend && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && *a.pend)
    atomicAdd(a.fly_count, 1ull);
  fwd_snap_head(a, NT);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int W = a.W, H = a.H;
  const int Wp = (W - 2) / 2, Hp = (H - 2) / 2, P = Hp * Wp;
  const int p0 = blockIdx.x * FPW;
  const int b0 = blockIdx.y * 64;
  const int b = b0 + lane;
  const bool bok = b < a.B;
  const int pp = __builtin_amdgcn_readfirstlane(wave >> 2), cg = __builtin_amdgcn_readfirstlane(wave & 3),
            c0 = cg * 8;
  const int p = p0 + pp;
  const bool pok = p < P;
  const int py0 = p0 / Wp;
  const int nrows = min(XR, H - 2 * py0);
  const float* W1 = reinterpret_cast<const float*>(a.W1);
  float* Pt = reinterpret_cast<float*>(a.Pt);

  // B fragments first (independent of the staging below, so their round trip overlaps it):
  // W1[kp*32 + k][nt*16 + fr] for this lane's 8 k of each position (f32 master, [K][HD])
  const int nt = wave & 3;
  float wfr[FPW][8];
#pragma unroll
  for (int ks = 0; ks < FPW; ++ks) {
    const int kp = p0 + ks;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wfr[ks][4 * i + j] = kp < P ? W1[(size_t)(kp * CC + k8_col(fq, i) + j) * a.ldw1 + nt * 16 + fr] : 0.f;
  }
  fwd_stage_x(a, xr, b0, py0, nrows, NT);
  fwd_stage_conv(a, wcs, NT);
  stamp(a.stamps, 1);
  lds_barrier();
  ConvW8 cw;
  cw.load(wcs, c0);

  // ---- phase 1: conv + bias + ReLU + 2x2 max-pool for 8 channels (f32 tile, f32 P^T)
  float out[8];
  if (bok && pok) {
    const int py = p / Wp, px = p - py * Wp;
    uint64_t packed;
    conv_pool8(xr + lane * fwd_istride(W) + (2 * (py - py0)) * W + 2 * px, W, cw, out, packed);
    if (a.amax) a.amax[((size_t)p * (CC / 8) + cg) * a.lda + b] = packed;
  } else {
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) out[cc] = 0.f;
  }
  if (pok && Pt && (bok || b < a.ldPt)) {
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) Pt[(size_t)(p * CC + c0 + cc) * a.ldPt + b] = out[cc];
  }
  {
    float* dst = Ps + ((size_t)pp * 64 + lane) * PS32 + c0;
    *reinterpret_cast<float4*>(dst) = float4{out[0], out[1], out[2], out[3]};
    *reinterpret_cast<float4*>(dst + 4) = float4{out[4], out[5], out[6], out[7]};
  }
  stamp(a.stamps, 2);
  lds_barrier();
  stamp(a.stamps, 3);

  // ---- phase 2: hpre[64 x 64] += Ps(64 x FPW*32) . W1(FPW*32 x 64) on the f32 MFMA; wave = column
  // tile nt of row tiles mt = (wave>>2) + FPW*j (independent accumulators keep the pipe issuing)
  constexpr int NMT = 4 / FPW;
  float* const hrow = a.hpre + (size_t)(blockIdx.x % a.hrep) * a.hrep_stride;
  f32x4 acc[NMT];
#pragma unroll
  for (int j = 0; j < NMT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < FPW; ++ks) {
    if (p0 + ks >= P) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float4 av[NMT];
#pragma unroll
      for (int j = 0; j < NMT; ++j) {
        const int mt = (wave >> 2) + FPW * j;
        av[j] = *reinterpret_cast<const float4*>(Ps + ((size_t)ks * 64 + mt * 16 + fr) * PS32 + k8_col(fq, i));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < NMT; ++j) acc[j] = mfma_f32x4(f4get(av[j], e), wfr[ks][4 * i + e], acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < NMT; ++j) {
    const int mt = (wave >> 2) + FPW * j;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = b0 + mt * 16 + fq * 4 + r;
      if (row < a.B) atomicAdd(hrow + (size_t)row * HD + nt * 16 + fr, acc[j][r]);
    }
  }
  stamp(a.stamps, 4);
}

// LDS carve of the backward (bytes)
constexpr int kG32 = 0;                              // f32 [64 b][GS32]   G = dH (A of dP)
constexpr int kGt32 = kG32 + 64 * GS32 * 4;          // f32 [64 u][GS32]   G^T (B of dW1)
constexpr int kW1s32 = kGt32 + 64 * GS32 * 4;        // f32 [32 c][GS32]   W1 rows (B of dP; the update's w)
constexpr int kPts32 = kW1s32 + 32 * GS32 * 4;       // f32 [32 c][GS32]   P^T rows (A of dW1)
constexpr int kXs32 = kPts32 + 32 * GS32 * 4;        // f32 [64 b][16]     4x4 input patches
constexpr int kAm32 = kXs32 + 64 * 16 * 4;           // u8  [64 b][CC]     pool argmax
constexpr int kR32 = kAm32 + 64 * CC;                // head scratch | dP [64][DPS32] | red [NW][16][CC]
constexpr int kRBytes = kHeadScratch > NW * 16 * CC * 4 ? kHeadScratch : NW * 16 * CC * 4;
static_assert(64 * DPS32 * 4 <= kRBytes, "dP exceeds the shared scratch");
constexpr int kW2s32 = kR32 + kRBytes;
constexpr int kB2s32 = kW2s32 + kW2Bytes;
constexpr int kLab32 = kB2s32 + kB2Bytes;
constexpr int kBwd32Lds = kLab32 + kLabBytes;
static_assert(kBwd32Lds <= 160 * 1024, "backward LDS exceeds a CU");

template <int MODE>
__global__ __launch_bounds__(1024) void convnet32_bwd_kernel(BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* Gs = reinterpret_cast<float*>(smem + kG32);
  float* Gts = reinterpret_cast<float*>(smem + kGt32);
  float* W1s = reinterpret_cast<float*>(smem + kW1s32);
  float* Pts = reinterpret_cast<float*>(smem + kPts32);
  float* xs = reinterpret_cast<float*>(smem + kXs32);
  uint8_t* am = smem + kAm32;
  float* dps = reinterpret_cast<float*>(smem + kR32);
  const HeadLds hl = HeadLds::carve(smem + kR32, smem + kW2s32, smem + kB2s32, smem + kLab32);
  stamp(a.stamps, 0);
  const int W = a.W, H = a.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fq = lane >> 4;
  const float* W1 = reinterpret_cast<const float*>(a.W1);
  const float* Pt = reinterpret_cast<const float*>(a.Pt);

  // the head weights into registers now, stored to LDS with the chunk operands below: every global load
  // of the prologue is in flight before the first LDS store (one round trip, not three)
  const int u2 = tid >> 4, c2 = tid & 15;   // 64 x 16
  const float w2v = c2 < a.C ? a.W2[u2 * a.C + c2] : 0.f;
  const float b2v = (tid < 16 && tid < a.C) ? a.b2[tid] : 0.f;
  zero_other_parity(a, tid);
  if (blockIdx.x == gridDim.x - 1) {
    hl.w2s[u2 * W2S + c2] = w2v;
    if (tid < 16) hl.b2s[tid] = b2v;
    head_workgroup<MODE>(a, hl, Gs);   // the G area is unused there
    return;
  }

  const int Wp = (W - 2) / 2;
  const int p = blockIdx.x;            // one pooled position per workgroup (grid = P + 1)
  const int py = p / Wp, px = p - py * Wp;
  const int hr = tid >> 4, hc4 = (tid & 15) * 4;
  const float4 b1v = a.b1 ? *reinterpret_cast<const float4*>(a.b1 + hc4) : float4{0.f, 0.f, 0.f, 0.f};
  // roles: waves 0-7 dP tile (mt = wave>>1 images, ct = wave&1 channels);
  //        waves 8-15 dW1 tile (rt = v>>2 channels, nt = v&3 units), v = wave-8
  const bool dw_wave = wave >= 8;
  const int v8 = wave & 7;

  f32x4 accw = {0.f, 0.f, 0.f, 0.f};
  f32x4 accr[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};

  // fused step with slots: the dW1-wave's slot values, loaded now (the weights come from W1s)
  f32x4 mp = {0.f, 0.f, 0.f, 0.f}, vp = {0.f, 0.f, 0.f, 0.f};
  long long t_it = 0;
  if (MODE != 0) {
    t_it = *a.iterations;
    if (MODE == 2 && dw_wave) {
      const int rt = v8 >> 2, nt = v8 & 3;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t e = (size_t)(p * CC + rt * 16 + fq * 4 + r) * HD + nt * 16 + fr;
        if (a.h.kind != kOptSGD) mp[r] = a.m1[e];
        if (a.h.kind == kOptAdam) vp[r] = a.v1[e];
      }
    }
  }

  // W1 rows of the position [32][64] f32: loaded once (independent of the image chunk), stored to LDS
  // after the first chunk's loads are issued
  const float2 w1v = *reinterpret_cast<const float2*>(W1 + (size_t)(p * CC + (tid >> 5)) * a.ldw1 + (tid & 31) * 2);

  for (int b0 = 0; b0 < a.B; b0 += 64) {
    const int nb = min(64, a.B - b0);
    // ---- prologue: coalesced loads of this chunk's operands
    float4 hv = {0.f, 0.f, 0.f, 0.f};
    if (hr < nb) hv = load_hpre(a, b0 + hr, hc4);
    const int lab = (tid < nb) ? a.labels[b0 + tid] : 0;
    float2 ptv;
    {
      const int r = tid >> 5, c = (tid & 31) * 2;
      const float* src = Pt + (size_t)(p * CC + r) * a.ldPt + b0 + c;
      ptv.x = c < nb ? src[0] : 0.f;
      ptv.y = c + 1 < nb ? src[1] : 0.f;
    }
    float4 xv = {0.f, 0.f, 0.f, 0.f};
    uint64_t amv = ~0ull;
    if (tid < 256) {
      const int bl = tid >> 2, r = tid & 3;
      if (bl < nb) {
        const float2* row = reinterpret_cast<const float2*>(a.x + (size_t)(b0 + bl) * H * W + (2 * py + r) * W + 2 * px);
        const float2 u = row[0], t = row[1];
        xv = float4{u.x, u.y, t.x, t.y};
      }
      const int cg = tid >> 6, bb = tid & 63;
      if (bb < nb) amv = a.amax[((size_t)p * (CC / 8) + cg) * a.lda + b0 + bb];
    }
    stamp(a.stamps, 1);
    if (b0 == 0) {
      hl.w2s[u2 * W2S + c2] = w2v;
      if (tid < 16) hl.b2s[tid] = b2v;
      *reinterpret_cast<float2*>(W1s + (tid >> 5) * GS32 + (tid & 31) * 2) = w1v;
    }
    head_stage(a, hv, b1v, hr, hc4, nb, hl.hs);
    if (tid < 64) hl.labs[tid] = lab;
    {
      const int r = tid >> 5, c = (tid & 31) * 2;
      *reinterpret_cast<float2*>(Pts + r * GS32 + c) = ptv;
    }
    if (tid < 256) {
      const int bl = tid >> 2, r = tid & 3;
      *reinterpret_cast<float4*>(xs + bl * 16 + r * 4) = xv;
      const int cg = tid >> 6, bb = tid & 63;
      *reinterpret_cast<uint64_t*>(am + bb * CC + cg * 8) = amv;
    }
    lds_barrier();
    // ---- the head recomputed: G = dH (f32) into LDS, row-major and transposed
    {
      float la = 0.f, ca = 0.f, na = 0.f;   // the head workgroup keeps these
      head_logits_ce(a, nb, hl, lane, wave, la, ca, na);
      const f32x4 gh = head_dh(a, nb, hl, lane, wave);
      const int rt = wave >> 2, j = (wave & 3) * 16 + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) Gs[(rt * 16 + fq * 4 + i) * GS32 + j] = gh[i];
      *reinterpret_cast<float4*>(Gts + j * GS32 + rt * 16 + fq * 4) = float4{gh[0], gh[1], gh[2], gh[3]};
    }
    lds_barrier();
    stamp(a.stamps, 2);

    // ---- waves 0-7: dP[b][c] = sum_u G[b][u] W1[c][u];  waves 8-15: dW1[c][u] += sum_b P[b][c] G[b][u]
    {
      const float* Ab = dw_wave ? Pts + ((v8 >> 2) * 16 + fr) * GS32 : Gs + ((v8 >> 1) * 16 + fr) * GS32;
      const float* Bb = dw_wave ? Gts + ((v8 & 3) * 16 + fr) * GS32 : W1s + ((v8 & 1) * 16 + fr) * GS32;
      f32x4 acc = dw_wave ? accw : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 av = *reinterpret_cast<const float4*>(Ab + k16_col(fq, i));
        const float4 bv = *reinterpret_cast<const float4*>(Bb + k16_col(fq, i));
        acc = mfma_f32x4(av.x, bv.x, acc);
        acc = mfma_f32x4(av.y, bv.y, acc);
        acc = mfma_f32x4(av.z, bv.z, acc);
        acc = mfma_f32x4(av.w, bv.w, acc);
      }
      if (dw_wave) {
        accw = acc;
      } else {
        const int mt = v8 >> 1, ct = v8 & 1;
#pragma unroll
        for (int r = 0; r < 4; ++r) dps[(mt * 16 + fq * 4 + r) * DPS32 + ct * 16 + fr] = acc[r];
      }
    }
    lds_barrier();
    stamp(a.stamps, 3);

    // ---- routing MFMA: k = (b, q), lane group fq = window slot q; wave takes images 4w..4w+3
    {
      const int tap = fr, ky = tap / 3, kx = tap - ky * 3, qy = fq >> 1, qx = fq & 1;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int bl = wave * 4 + s;
        const float xa = tap < 9 ? xs[bl * 16 + (qy + ky) * 4 + qx + kx] : (tap == 9 ? 1.f : 0.f);
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const int c = ct * 16 + fr;
          const float d = am[bl * CC + c] == (unsigned)fq ? dps[bl * DPS32 + c] : 0.f;
          accr[ct] = mfma_f32x4(xa, d, accr[ct]);
        }
      }
    }
    lds_barrier();
  }
  stamp(a.stamps, 4);

  if (dw_wave) {
    const int rt = v8 >> 2, nt = v8 & 3;
    const int col = nt * 16 + fr;
    if (MODE != 0) {
      // ---- update this position's Dense(64) rows (complete dW1: the rows belong to this workgroup);
      // the weights were staged into W1s before the chunk loop
      const float lr_t = opt_lr_t(a.h, t_it);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rt * 16 + fq * 4 + r;
        const size_t e = (size_t)(p * CC + row) * HD + col;
        float m = mp[r], v = vp[r];
        a.w1[e] = opt_step(a.h, lr_t, W1s[row * GS32 + col], accw[r], m, v);
        if (MODE == 2 && a.h.kind != kOptSGD) a.m1[e] = m;
        if (MODE == 2 && a.h.kind == kOptAdam) a.v1[e] = v;
      }
    } else if (a.push.nranks > 0) {
      // fused DP exchange: this position's complete dW1 rows [32][64] are staged in W1s (free after the
      // chunk loop) and pushed below as one contiguous 8 KB run of float4 stores
#pragma unroll
      for (int r = 0; r < 4; ++r) W1s[(rt * 16 + fq * 4 + r) * GS32 + col] = accw[r];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) a.dW1[(size_t)(p * CC + rt * 16 + fq * 4 + r) * HD + col] = accw[r];
    }
  }
  conv_grad_reduce(a, accr, dps, lane, wave);   // its barrier also publishes the W1s staging
  if (MODE == 0 && a.push.nranks > 0 && tid < CC * HD / 4) {
    // the rows go straight into the owners' contribution areas of the all-reduce call that follows this
    // launch (its parity from the completed-calls count); the bucket offset is a multiple of 4 (host check)
    const int parity = (int)((*a.push.epoch + 1u) & 1u);
    const int row = tid >> 4, c4 = (tid & 15) * 4;
    xg_push_store4(a.push, parity, a.push.off + (long long)(p * CC + row) * HD + c4,
                   *reinterpret_cast<const float4*>(W1s + row * GS32 + c4));
    xg_push_drain();   // acknowledged before the wave ends
  }
  stamp(a.stamps, 5);
}

}  // namespace tde

using namespace tde;
using namespace tde::cnet;

// Float32 forward: W1 is the f32 master Dense(64) kernel [K][64] (ldw1 = 64), Pt f32 [K][ldPt].
// opt / off_wc / off_bc / inc_iter / hrep as tde_convnet_fwd.
TDE_API int tde_convnet_fwd_f32(const float* x, const float* wc, const float* bc, const float* W1, int ldw1,
                                float* hpre, float* Pt, int ldPt, void* amax, int lda, int B, int H, int W,
                                long long* stamps, const TdeStepOpt* opt, long long off_wc, long long off_bc,
                                long long* inc_iter, int hrep, long long hrep_stride, hipStream_t stream) {
  if ((W & 3) || W > XW || ((W - 2) / 2) < 4 || ldw1 != HD || (Pt && (ldPt & 7)) || (amax && lda < B)) return -1;
  if (((uintptr_t)wc | (uintptr_t)bc | (uintptr_t)W1) & 15) return -2;
  if (opt && (!opt_ok(opt) || !opt->pend)) return -4;
  const int P = ((H - 2) / 2) * ((W - 2) / 2);
  int by = (B + 63) / 64;
  if (Pt) {
    const int byp = (ldPt + 63) / 64;
    if (byp > by) by = byp;
  }
  FwdArgs a{x, wc, bc, W1, ldw1, hpre, Pt, ldPt, (uint64_t*)amax, lda, B, H, W, stamps};
  fill_fwd_opt(a, opt, off_wc, off_bc, inc_iter, hrep, hrep_stride);
  // positions per workgroup (TDE_CONVNET32_FPW = 1|2, default 1)
  static const int fpw = [] {
    const char* e = getenv("TDE_CONVNET32_FPW");
    return (e && atoi(e) == 2) ? 2 : 1;
  }();
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)convnet32_fwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, fwd32_lds(1));
    hipFuncSetAttribute((const void*)convnet32_fwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, fwd32_lds(2));
    attr_set = true;
  }
  const dim3 grid((P + fpw - 1) / fpw, by);
  if (fpw == 1) convnet32_fwd_kernel<1><<<grid, 256, fwd32_lds(1), stream>>>(a);
  else convnet32_fwd_kernel<2><<<grid, 512, fwd32_lds(2), stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Float32 backward: W1 = the f32 master [K][64] (ldw1 = 64; in the fused step the same memory as
// opt->w + opt->off_w1), Pt f32.  Other arguments as tde_convnet_bwd (opt->W1c is ignored).
TDE_API int tde_convnet_bwd_f32(const float* x, const void* amax, int lda, const float* hpre, float* hzero,
                                int hrep, long long hrep_stride, const float* b1, const float* W2, const float* b2,
                                int C, int pre_relu, const int* labels, float scale, float* metrics, const float* W1,
                                int ldw1, const float* Pt, int ldPt, float* dW1, float* dwc, float* dbc, float* dW2,
                                float* db2, float* db1, int B, int H, int W, long long* stamps, const TdeBwdOpt* opt,
                                float* cpart, const XgPush* push, int crep, long long crep_stride,
                                hipStream_t stream) {
  if (ldw1 != HD || ((uintptr_t)W1 & 15) || ((uintptr_t)Pt & 7)) return -1;
  if (push && push->nranks > 0 &&
      (opt || push->nranks > kXgMaxRanks || push->L <= 0 || (push->L & 3) || (push->off & 3) || !push->epoch))
    return -7;
  if (opt && opt->w + opt->off_w1 != W1) return -3;   // the update is applied to the rows it reads
  BwdArgs a;
  const int rc = fill_bwd(a, x, amax, lda, hpre, hzero, hrep, hrep_stride, b1, W2, b2, C, pre_relu, labels, scale,
                          metrics, W1, ldw1, Pt, ldPt, dW1, dwc, dbc, dW2, db2, db1, B, H, W, stamps, opt);
  if (rc) return rc;
  a.cpart = cpart;
  a.w1r_out = nullptr;
  a.w1c_out = nullptr;
  if (push) a.push = *push;
  if (!opt && crep > 1) {   // data-parallel step: conv-gradient replicas summed by the all-reduce
    a.crep = crep;
    a.crep_stride = crep_stride;
  }
  const int P = ((H - 2) / 2) * ((W - 2) / 2);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)convnet32_bwd_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, kBwd32Lds);
    (void)hipFuncSetAttribute((const void*)convnet32_bwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, kBwd32Lds);
    (void)hipFuncSetAttribute((const void*)convnet32_bwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, kBwd32Lds);
    attr_set = true;
  }
  const dim3 grid(P + 1);   // one workgroup per pooled position + the head workgroup
  if (!opt) convnet32_bwd_kernel<0><<<grid, 1024, kBwd32Lds, stream>>>(a);
  else if (opt->kind == kOptSGD) convnet32_bwd_kernel<1><<<grid, 1024, kBwd32Lds, stream>>>(a);
  else convnet32_bwd_kernel<2><<<grid, 1024, kBwd32Lds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Sizes of the ctypes-mirrored fused-step structs (tests/test_abi.py checks the Python mirrors in
// ops/kernels.py against them): out = {TdeStepOpt, TdeBwdOpt, FlatApply, OptHyper}.
TDE_API int tde_cnet_abi_sizes(long long* out, int n) {
  const long long s[] = {(long long)sizeof(TdeStepOpt), (long long)sizeof(TdeBwdOpt), (long long)sizeof(FlatApply),
                         (long long)sizeof(OptHyper)};
  for (int i = 0; i < n && i < 4; ++i) out[i] = s[i];
  return 4;
}
