// Fused forward and backward of the DWK/TF2M small CNN trunk
//   Conv2D(32,3x3,VALID,bias,ReLU) · MaxPooling2D(2) · Flatten · Dense(64)  (matmul part)
// (distributed_with_keras.py:34-37, tf2_mnist_distributed.py:67-70;
//  SURVEY.md §2.5 A1-A4 forward, A10-A13 backward).
//
// Design (latency-bound regime; measured with in-kernel s_memrealtime stamps):
//  * 1024-thread workgroups (16 waves): enough waves per CU to hide load latency;
//  * every global operand is loaded ONCE per workgroup with coalesced 16-byte
//    loads issued in the prologue and staged in LDS (rows padded so the
//    16x16x32 MFMA fragment reads are bank-conflict free);
//  * LDS-only barriers (lds_barrier): the scattered global stores of a phase
//    drain in the background instead of stalling the barrier;
//  * the pool-argmax side output is stored lane-contiguous ([P][C/8][ldA] u64).
//
// Forward: a workgroup owns PPW=4 pooled positions x 64 images.
//   phase 1 (VALU; wave = (position, 8-channel group), lane = image): 3x3 conv of
//           the 2x2 pool window from a 4x4 register patch, bias, ReLU, max ->
//           bf16 pooled tile in LDS, argmax bytes, P^T (for the weight grad);
//   phase 2 (MFMA; wave = 16x16 output tile): tile . W1^T rows of the 4 positions
//           -> split-K partial of the Dense pre-activation, f32 atomics into hpre.
// Backward, per workgroup of 4 positions, looping 64-image chunks:
//   dP   = G . W1[p*32:(p+1)*32]^T      (MFMA; Dense input-gradient, in-kernel)
//   dW1[p*32:(p+1)*32] = P^T . G        (MFMA; Dense weight-gradient rows, stored)
//   route dP through the pool argmax and ReLU mask and reduce over (image, window
//   slot) with MFMA: dWc[tap][c] = sum_k X[tap][k] D[k][c], k=(pos,b,q) — the
//   bias gradient is the extra all-ones tap row.
//
// Fused single-replica step (no gradient all-reduce between backward and update):
// the optimizer runs where each gradient is finished, with no extra launch and no
// cross-workgroup hand-off inside a kernel (on gfx950 an in-kernel release/acquire
// costs about as much as a kernel boundary):
//   * Dense(64) kernel rows: each backward workgroup owns its rows' dW1 completely,
//     so it updates the fp32 rows and rewrites their bf16 shadow in place;
//   * Dense(64) bias, Dense(10) kernel + bias (finished by the head launch): the
//     last backward workgroup updates them;
//   * Conv2D kernel + bias (finished by the backward's atomics): deferred — the next
//     forward computes the updated values on the fly from (w, g, slots) while *pend,
//     and the next head launch (which does not read them) commits them and clears
//     *pend; a flush launch commits them at the end of each execution.
#include "tde_optim.h"

namespace tde {

constexpr int PPW = 4;   // pooled positions per workgroup
constexpr int NW = 16;   // waves per workgroup
constexpr int CC = 32;   // conv filters
constexpr int HD = 64;   // Dense units
constexpr int PSTR = 40; // padded LDS row stride (bf16) of the pooled tile
constexpr int RSTR = 72; // padded LDS row stride (bf16) of 64-wide operand rows

struct ConvNetFwdArgs {
  const float* x; const float* wc; const float* bc;
  const bf16* W1c; int ldw1c;       // [HD][K] bf16 (W1^T shadow)
  float* hpre;                      // [B][HD] f32, += (pre-zeroed by the previous head launch)
  bf16* Pt; int ldPt;               // [K][ldPt] (nullable)
  uint64_t* amax; int lda;          // [P][CC/8][lda] (nullable)
  int B, H, W;
  long long* stamps;
  int w1_rows;                      // 1: W1c is the row-major [K][HD] shadow (ldw1c = HD)
  // deferred conv update (fused step): while *pend the conv weights used are the optimizer
  // step of (wc, bc) with the previous backward's gradients (nullable: use wc, bc as stored)
  const int* pend;
  const float *gwc, *gbc, *mwc, *mbc, *vwc, *vbc;
  const long long* iterations;
  OptHyper h;
};

// The input rows a workgroup's PPW positions touch (<= XR rows of <= XW floats per
// image) are staged into LDS with coalesced float4 loads: gathering 4x4 patches
// straight from HBM puts 64 distinct cache lines behind every load instruction.
constexpr int XR = 6, XW = 32;
// per-image stride of the staged rows padded to 2 (mod 64) floats: the per-lane (= per-image) float2
// patch reads then hit distinct bank pairs (168 = 40 mod 64 for MNIST made them 8-way conflicts)
__host__ __device__ constexpr int fwd_istride(int W) { return XR * W + ((2 - (XR * W) % 64) + 64) % 64; }
constexpr int kConvW = CC * 10;   // conv taps [9][CC] + bias [CC] (floats), staged in LDS
constexpr int fwd_lds(int fpw) { return fpw * 64 * PSTR * 2 + 64 * (XR * XW + 64) * 4 + kConvW * 4; }

// FPW pooled positions x 64 images per workgroup, 4*FPW waves (wave = position x 8-channel
// group).  Phase 1 is VALU-bound: fewer positions per workgroup spread the conv over more CUs
// (FPW=4: 43 workgroups x 16 waves for MNIST; FPW=2: 85 x 8) at the price of more split-K
// atomics in phase 2.
template <int FPW>
__global__ __launch_bounds__(FPW * 256) void convnet_fwd_kernel(ConvNetFwdArgs a) {
  constexpr int NT = FPW * 256;
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  bf16* Ps = reinterpret_cast<bf16*>(fsm);
  float* xr = reinterpret_cast<float*>(fsm + FPW * 64 * PSTR * 2);  // [64][XR][W]
  float* wcs = reinterpret_cast<float*>(fsm + FPW * 64 * PSTR * 2 + 64 * (XR * XW + 64) * 4);  // [10][CC]
  stamp(a.stamps, 0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  const int W = a.W, H = a.H;
  const int Wp = (W - 2) / 2, Hp = (H - 2) / 2, P = Hp * Wp;
  const int p0 = blockIdx.x * FPW;
  const int b0 = blockIdx.y * 64;
  const int b = b0 + lane;
  const bool bok = b < a.B;
  // wave-uniform: the conv weights of this wave's 8 channels are scalar loads (SGPRs), not 72 VGPRs
  const int pp = __builtin_amdgcn_readfirstlane(wave >> 2), cg = __builtin_amdgcn_readfirstlane(wave & 3),
            c0 = cg * 8;
  const int p = p0 + pp;
  const bool pok = p < P;
  const int py0 = p0 / Wp;
  const int nrows = min(XR, H - 2 * py0);
  const int istride = fwd_istride(W);  // floats per staged image (bank-padded)

  // ---- prologue: all global loads, independent, issued back to back
  {
    const int n4 = nrows * W / 4;  // float4 per image
    for (int i = threadIdx.x; i < 64 * n4; i += NT) {
      const int bl = i / n4, q = i - bl * n4;
      float4 v = {0.f, 0.f, 0.f, 0.f};
      if (b0 + bl < a.B)
        v = *reinterpret_cast<const float4*>(a.x + (size_t)(b0 + bl) * H * W + (size_t)(2 * py0) * W + q * 4);
      // istride is only 8-byte aligned (bank padding): two 8-byte LDS writes
      float2* d2 = reinterpret_cast<float2*>(xr + bl * istride + q * 4);
      d2[0] = float2{v.x, v.y};
      d2[1] = float2{v.z, v.w};
    }
  }
  // conv weights in effect for this step -> LDS (with the deferred update applied while *pend)
  for (int i = threadIdx.x; i < kConvW; i += NT) {
    const bool isb = i >= 9 * CC;
    const int j = isb ? i - 9 * CC : i;
    float w = isb ? a.bc[j] : a.wc[j];
    if (a.pend) {
      const float g = isb ? a.gbc[j] : a.gwc[j];
      float m = 0.f, v = 0.f;
      if (a.h.kind != kOptSGD) m = isb ? a.mbc[j] : a.mwc[j];
      if (a.h.kind == kOptAdam) v = isb ? a.vbc[j] : a.vwc[j];
      const long long t = a.h.kind == kOptAdam ? *a.iterations : 0;
      if (*a.pend) w = opt_step(a.h, opt_lr_t(a.h, t), w, g, m, v);
    }
    wcs[i] = w;
  }
  // W1^T fragments of this wave's output tiles: tile t = wave + 4*FPW*j (j < 4/FPW),
  // mt = t>>2 (image rows), nt = t&3 = wave&3 (units) for every j
  const int nt = wave & 3;
  bf16x8 wfr[FPW];
#pragma unroll
  for (int ks = 0; ks < FPW; ++ks) {
    const int kp = p0 + ks;
    if (kp >= P) {
      wfr[ks] = bf16x8{};
    } else if (a.w1_rows) {
      // row-major shadow [K][HD]: 8 K-consecutive elements of column nt*16+fr (16 lanes read
      // 32 contiguous bytes per element row)
      const bf16* src = a.W1c + (size_t)(kp * CC + fk) * a.ldw1c + nt * 16 + fr;
#pragma unroll
      for (int j = 0; j < 8; ++j) wfr[ks][j] = src[(size_t)j * a.ldw1c];
    } else {
      wfr[ks] = *reinterpret_cast<const bf16x8*>(a.W1c + (size_t)(nt * 16 + fr) * a.ldw1c + (size_t)kp * CC + fk);
    }
  }
  stamp(a.stamps, 1);
  lds_barrier();
  // this wave's 8 channels (wave-uniform LDS broadcast reads)
  float4 wlo[9], whi[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const float4 lo = *reinterpret_cast<const float4*>(wcs + t * CC + c0);
    const float4 hi = *reinterpret_cast<const float4*>(wcs + t * CC + c0 + 4);
    wlo[t] = lo;
    whi[t] = hi;
  }
  float4 blo, bhi;
  {
    const float4 lo = *reinterpret_cast<const float4*>(wcs + 9 * CC + c0);
    const float4 hi = *reinterpret_cast<const float4*>(wcs + 9 * CC + c0 + 4);
    blo = lo;
    bhi = hi;
  }

  // ---- phase 1: conv + bias + ReLU + 2x2 max-pool for 8 channels
  bf16x8 outv;
  if (bok && pok) {
    float patch[16];
    {
      const int py = p / Wp, px = p - py * Wp;
      const float* xb = xr + lane * istride + (2 * (py - py0)) * W + 2 * px;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float2 u = *reinterpret_cast<const float2*>(xb + r * W);
        const float2 v = *reinterpret_cast<const float2*>(xb + r * W + 2);
        patch[r * 4 + 0] = u.x; patch[r * 4 + 1] = u.y; patch[r * 4 + 2] = v.x; patch[r * 4 + 3] = v.y;
      }
    }
    uint64_t packed = 0;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      float wt[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float4 q = cc < 4 ? wlo[t] : whi[t];
        const int k = cc & 3;
        wt[t] = k == 0 ? q.x : (k == 1 ? q.y : (k == 2 ? q.z : q.w));
      }
      const float4 bq = cc < 4 ? blo : bhi;
      const int kb = cc & 3;
      const float bcv = kb == 0 ? bq.x : (kb == 1 ? bq.y : (kb == 2 ? bq.z : bq.w));
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
      outv[cc] = f2bf(fmaxf(best, 0.f));
      packed |= (uint64_t)(best > 0.f ? (unsigned)bi : 0xFFu) << (8 * cc);
    }
    if (a.amax) a.amax[((size_t)p * (CC / 8) + cg) * a.lda + b] = packed;
    if (a.Pt) {
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) a.Pt[(size_t)(p * CC + c0 + cc) * a.ldPt + b] = outv[cc];
    }
  } else {
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) outv[cc] = f2bf(0.f);
    if (pok && a.Pt && b < a.ldPt) {
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) a.Pt[(size_t)(p * CC + c0 + cc) * a.ldPt + b] = outv[cc];
    }
  }
  *reinterpret_cast<bf16x8*>(Ps + ((size_t)pp * 64 + lane) * PSTR + c0) = outv;
  stamp(a.stamps, 2);
  lds_barrier();
  stamp(a.stamps, 3);

  // ---- phase 2: hpre[64 x 64] += Ps(64 x FPW*32) . W1^T(FPW*32 x 64); 16x16 tiles over the waves
#pragma unroll
  for (int j = 0; j < 4 / FPW; ++j) {
    const int mt = (wave >> 2) + FPW * j;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < FPW; ++ks) {
      if (p0 + ks < P) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(Ps + ((size_t)ks * 64 + mt * 16 + fr) * PSTR + fk);
        acc = mfma16(av, wfr[ks], acc);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = b0 + mt * 16 + (lane >> 4) * 4 + r;
      if (row < a.B) atomicAdd(a.hpre + (size_t)row * HD + nt * 16 + fr, acc[r]);
    }
  }
  stamp(a.stamps, 4);
}

struct ConvNetBwdArgs {
  const float* x; const uint64_t* amax; int lda;
  const bf16* G; int ldg;            // [B][HD] bf16 (dHpre)
  const bf16* Gt; int ldgt;          // [HD][ldgt] bf16
  const bf16* W1r; int ldw1r;        // [K][HD] bf16 (row-major shadow)
  const bf16* Pt; int ldPt;          // [K][ldPt] bf16
  float* dW1;                        // [K][HD] f32 (stored; unused when apply)
  float* dwc; float* dbc;            // [9][CC], [CC] (atomic +=)
  int B, H, W;
  long long* stamps;
  // fused step: update the Dense(64) kernel rows here instead of storing dW1
  int apply;
  float *w1, *m1, *v1;               // fp32 master [K][HD] (+ slots), updated in place
  bf16* w1r_out;                     // row-major bf16 shadow (== W1r), rewritten
  bf16* w1c_out; int ldw1c;          // transposed bf16 shadow [HD][ldw1c] (nullable)
  const long long* iterations;
  OptHyper h;
  FlatApply head;                    // applied by the last workgroup (head variables), nr = 0: none
  int* pend;                         // set to 1: the conv update is pending (nullable)
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
        g[k] = f.g[e[k]];
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
      f.g[e[k]] = 0.f;
      if (f.h.kind != kOptSGD) f.m[e[k]] = m[k];
      if (f.h.kind == kOptAdam) f.v[e[k]] = v[k];
    }
  }
};

// Elements [start, total) of a FlatApply's ranges, threads tid, tid + nt, ... (no prefetch).
__device__ __forceinline__ void flat_apply_from(const FlatApply& f, long long t, int start, int tid, int nt) {
  int total = 0;
  for (int r = 0; r < f.nr; ++r) total += f.n[r];
  const float lr_t = opt_lr_t(f.h, t);
  for (int idx0 = start + tid; idx0 < total; idx0 += nt) {
    int idx = idx0, e = -1;
    for (int r = 0; r < f.nr; ++r) {
      if (idx < f.n[r]) {
        e = f.lo[r] + idx;
        break;
      }
      idx -= f.n[r];
    }
    float m = f.h.kind != kOptSGD ? f.m[e] : 0.f, v = f.h.kind == kOptAdam ? f.v[e] : 0.f;
    f.w[e] = opt_step(f.h, lr_t, f.w[e], f.g[e], m, v);
    f.g[e] = 0.f;
    if (f.h.kind != kOptSGD) f.m[e] = m;
    if (f.h.kind == kOptAdam) f.v[e] = v;
  }
}

// LDS carve (bytes)
constexpr int kG = 0;                                   // bf16 [64][RSTR]
constexpr int kW1 = kG + 64 * RSTR * 2;                 // bf16 [128][RSTR]
constexpr int kPt = kW1 + 128 * RSTR * 2;               // bf16 [128][RSTR]
constexpr int kGt = kPt + 128 * RSTR * 2;               // bf16 [64][RSTR]
constexpr int kXs = kGt + 64 * RSTR * 2;                // f32  [PPW][64][16]
constexpr int kAm = kXs + PPW * 64 * 16 * 4;            // u8   [PPW][64][CC]
constexpr int kDp = kAm + PPW * 64 * CC;                // f32  [PPW][64][DPS] (reused as red [NW][16][CC])
// dP row stride: 40 floats puts the 4 lane groups of the routing reads (rows 2 apart) on disjoint
// bank quarters (stride 32 made them 4-way LDS bank conflicts)
constexpr int DPS = 40;
constexpr int kBwdLds = kDp + PPW * 64 * DPS * 4;

// MODE 0: store dW1; 1: fused step, SGD; 2: fused step, optimizer with slots (momentum / Adam)
template <int MODE>
__global__ __launch_bounds__(1024) void convnet_bwd_kernel(ConvNetBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* Gs = reinterpret_cast<bf16*>(smem + kG);
  bf16* W1s = reinterpret_cast<bf16*>(smem + kW1);
  bf16* Pts = reinterpret_cast<bf16*>(smem + kPt);
  bf16* Gts = reinterpret_cast<bf16*>(smem + kGt);
  float* xs = reinterpret_cast<float*>(smem + kXs);
  uint8_t* am = smem + kAm;
  float* dps = reinterpret_cast<float*>(smem + kDp);
  float* red = dps;
  stamp(a.stamps, 0);
  const int W = a.W, H = a.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, tid = threadIdx.x;
  const int fr = lane & 15, fq = lane >> 4, fk = fq * 8;
  const int Wp = (W - 2) / 2, Hp = (H - 2) / 2, P = Hp * Wp;
  const int p0 = blockIdx.x * PPW;
  const int nrow = min(PPW, P - p0) * CC;  // valid W1/Pt rows of this workgroup

  f32x4 accw[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  f32x4 accr[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};

  // fused step: this workgroup's fp32 master rows (and slots) and the head variables, loaded
  // now, updated after the chunk loop
  constexpr int NS = MODE == 2 ? 2 : 1;   // slot registers (dummies unless MODE 2)
  f32x4 wp[2], mp[NS], vp[NS];
  long long t_it = 0;
  const bool head_wg = a.head.nr > 0 && blockIdx.x == gridDim.x - 1;
  FlatPrefetch<1> hp;
  if (MODE != 0) {
    if (a.h.kind == kOptAdam || a.head.h.kind == kOptAdam) t_it = *a.iterations;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = wave + 16 * i;
      const int nt = t & 3, rt = t >> 2;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rt * 16 + fq * 4 + r;
        const size_t e = (size_t)(p0 * CC + row) * HD + nt * 16 + fr;
        wp[i][r] = row < nrow ? a.w1[e] : 0.f;
        if (MODE == 2) {
          mp[i % NS][r] = (row < nrow && a.h.kind != kOptSGD) ? a.m1[e] : 0.f;
          vp[i % NS][r] = (row < nrow && a.h.kind == kOptAdam) ? a.v1[e] : 0.f;
        }
      }
    }
    if (head_wg) hp.load(a.head, tid, 1024);
  }

  // W1 rows of the 4 positions: loaded once (independent of the image chunk)
  {
    const int r = tid >> 3, c = (tid & 7) * 8;  // 128 rows x 8 chunks of 16 B
    bf16x8 v = r < nrow ? *reinterpret_cast<const bf16x8*>(a.W1r + (size_t)(p0 * CC + r) * a.ldw1r + c) : bf16x8{};
    *reinterpret_cast<bf16x8*>(W1s + r * RSTR + c) = v;
  }

  for (int b0 = 0; b0 < a.B; b0 += 64) {
    const int nb = min(64, a.B - b0);
    // ---- prologue: coalesced loads of this chunk's operands
    bf16x8 gv = {}, gtv = {}, ptv;
    if (tid < 512) {
      const int r = tid >> 3, c = (tid & 7) * 8;
      if (r < nb) gv = *reinterpret_cast<const bf16x8*>(a.G + (size_t)(b0 + r) * a.ldg + c);
      // Gt rows: unit r, images b0+c .. +8 (zero past B)
      gtv = load_frag(a.Gt + (size_t)r * a.ldgt + b0 + c, b0 + c, a.B, true);
    }
    {
      const int r = tid >> 3, c = (tid & 7) * 8;
      ptv = r < nrow ? load_frag(a.Pt + (size_t)(p0 * CC + r) * a.ldPt + b0 + c, b0 + c, a.B, true) : bf16x8{};
    }
    float4 xv = {0.f, 0.f, 0.f, 0.f};
    {
      const int pp = tid >> 8, bl = (tid >> 2) & 63, r = tid & 3;
      const int p = p0 + pp, b = b0 + bl;
      if (p < P && b < a.B) {
        const int py = p / Wp, px = p - py * Wp;
        const float2* row = reinterpret_cast<const float2*>(a.x + (size_t)b * H * W + (2 * py + r) * W + 2 * px);
        const float2 u = row[0], t = row[1];
        xv = float4{u.x, u.y, t.x, t.y};
      }
    }
    uint64_t amv = ~0ull;
    {
      const int pp = tid >> 8, cg = (tid >> 6) & 3, bl = tid & 63;
      const int p = p0 + pp, b = b0 + bl;
      if (p < P && b < a.B) amv = a.amax[((size_t)p * (CC / 8) + cg) * a.lda + b];
    }
    stamp(a.stamps, 1);
    if (tid < 512) {
      const int r = tid >> 3, c = (tid & 7) * 8;
      *reinterpret_cast<bf16x8*>(Gs + r * RSTR + c) = gv;
      *reinterpret_cast<bf16x8*>(Gts + r * RSTR + c) = gtv;
    }
    {
      const int r = tid >> 3, c = (tid & 7) * 8;
      *reinterpret_cast<bf16x8*>(Pts + r * RSTR + c) = ptv;
    }
    {
      const int pp = tid >> 8, bl = (tid >> 2) & 63, r = tid & 3;
      *reinterpret_cast<float4*>(xs + ((size_t)pp * 64 + bl) * 16 + r * 4) = xv;
    }
    {
      const int pp = tid >> 8, cg = (tid >> 6) & 3, bl = tid & 63;
      *reinterpret_cast<uint64_t*>(am + ((size_t)pp * 64 + bl) * CC + cg * 8) = amv;
    }
    lds_barrier();
    stamp(a.stamps, 2);

    // ---- dP[pp][b][c] = G[b] . W1[pp*32 + c]  (wave = position x 16 images)
    {
      const int pp = wave >> 2, mt = wave & 3;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 av = *reinterpret_cast<const bf16x8*>(Gs + (mt * 16 + fr) * RSTR + ks * 32 + fk);
          const bf16x8 bv = *reinterpret_cast<const bf16x8*>(W1s + (pp * CC + ct * 16 + fr) * RSTR + ks * 32 + fk);
          acc = mfma16(av, bv, acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) dps[((size_t)pp * 64 + mt * 16 + fq * 4 + r) * DPS + ct * 16 + fr] = acc[r];
      }
    }
    // ---- dW1 rows += P^T . G   (32 tiles of 16x16: t = wave, wave+16)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = wave + 16 * i;
      const int nt = t & 3, rt = t >> 2;  // rt: 16-row block (of 8) within the 128 rows
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(Pts + (rt * 16 + fr) * RSTR + ks * 32 + fk);
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(Gts + (nt * 16 + fr) * RSTR + ks * 32 + fk);
        accw[i] = mfma16(av, bv, accw[i]);
      }
    }
    lds_barrier();
    stamp(a.stamps, 3);

    // ---- routing MFMA: k = ((pp*64 + b)*4 + q); 32 k-steps, wave takes ks = wave, wave+16
    {
      const int tap = fr, ky = tap / 3, kx = tap - ky * 3;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int ks = wave + 16 * h2;
        const int kb = ks * 32 + fk;
        const int pp = kb >> 8, bl = (kb >> 2) & 63;
        bf16x8 av;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int bb = bl + (j >> 2), q = j & 3, qy = q >> 1, qx = q & 1;
          float v;
          if (tap < 9) v = xs[((size_t)pp * 64 + bb) * 16 + (qy + ky) * 4 + qx + kx];
          else v = (tap == 9) ? 1.f : 0.f;
          av[j] = f2bf(v);
        }
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const int c = ct * 16 + fr;
          bf16x8 bv;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const size_t idx = ((size_t)pp * 64 + bl + h) * CC + c;
            const unsigned id = am[idx];
            const float dv = dps[((size_t)pp * 64 + bl + h) * DPS + c];
#pragma unroll
            for (int q = 0; q < 4; ++q) bv[h * 4 + q] = f2bf(id == (unsigned)q ? dv : 0.f);
          }
          accr[ct] = mfma16(av, bv, accr[ct]);
        }
      }
    }
    lds_barrier();
  }
  stamp(a.stamps, 4);

  if (MODE != 0) {
    // ---- update this workgroup's Dense(64) rows (complete dW1: rows belong to one workgroup) and
    // rewrite their bf16 shadows; its W1 rows were read into LDS before the chunk loop
    const float lr_t = opt_lr_t(a.h, t_it);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = wave + 16 * i;
      const int nt = t & 3, rt = t >> 2;
      const int col = nt * 16 + fr, row0 = rt * 16 + fq * 4;
      if (row0 >= nrow) continue;   // nrow is a multiple of 32: all 4 rows valid or none
      bf16x4 hv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const size_t e = (size_t)(p0 * CC + row0 + r) * HD + col;
        float m = MODE == 2 ? mp[i % NS][r] : 0.f, v = MODE == 2 ? vp[i % NS][r] : 0.f;
        const float w = opt_step(a.h, lr_t, wp[i][r], accw[i][r], m, v);
        a.w1[e] = w;
        if (MODE == 2 && a.h.kind != kOptSGD) a.m1[e] = m;
        if (MODE == 2 && a.h.kind == kOptAdam) a.v1[e] = v;
        hv[r] = f2bf(w);
        a.w1r_out[e] = hv[r];
      }
      if (a.w1c_out) *reinterpret_cast<bf16x4*>(a.w1c_out + (size_t)col * a.ldw1c + p0 * CC + row0) = hv;
    }
    if (head_wg) {
      hp.apply(a.head, t_it);
      flat_apply_from(a.head, t_it, 1024, tid, 1024);   // elements beyond one per thread (none for MNIST)
    }
    if (a.pend && blockIdx.x == 0 && tid == 0) *a.pend = 1;
  } else {
    // ---- store dW1 tiles (each row of dW1 belongs to exactly one workgroup)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = wave + 16 * i;
      const int nt = t & 3, rt = t >> 2;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rt * 16 + fq * 4 + r;
        if (row < nrow) a.dW1[(size_t)(p0 * CC + row) * HD + nt * 16 + fr] = accw[i][r];
      }
    }
  }
  // ---- reduce routing accumulators over the 16 waves, then 10*CC atomics
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
    if (tap < 9) atomicAdd(a.dwc + tap * CC + c, s);
    else if (a.dbc) atomicAdd(a.dbc + c, s);
  }
  stamp(a.stamps, 5);
}

}  // namespace tde

using namespace tde;

// Specialised for Conv2D(32, 3x3, valid) on 1-channel input + MaxPool(2) + Dense(64).
// Fused-step optimizer description shared by the convnet entry points (ctypes struct):
// slots m/v flat like w; iterations = the device step counter.
struct TdeStepOpt {
  int kind;
  float lr, mom, b1, b2, eps;
  float *w, *g, *m, *v;
  const long long* iterations;
  int* pend;
};

static OptHyper hyper_of(const TdeStepOpt* o) { return OptHyper{o->kind, o->lr, o->mom, o->b1, o->b2, o->eps}; }
static bool opt_ok(const TdeStepOpt* o) {
  return o->w && o->g && o->iterations && (o->kind == kOptSGD || o->m) && (o->kind != kOptAdam || o->v);
}

// w1_rows: W1c is the row-major [K][HD] shadow (ldw1c == HD) instead of [HD][K].
// opt (nullable): deferred conv update {w, g, m, v, pend} with wc/bc at offsets off_wc/off_bc.
TDE_API int tde_convnet_fwd(const float* x, const float* wc, const float* bc, const void* W1c, int ldw1c,
                            float* hpre, void* Pt, int ldPt, void* amax, int lda, int B, int H, int W,
                            long long* stamps, int w1_rows, const TdeStepOpt* opt, long long off_wc,
                            long long off_bc, hipStream_t stream) {
  if ((W & 3) || W > XW || ((W - 2) / 2) < 4 || (ldw1c & 7) || (Pt && (ldPt & 7)) || (amax && lda < B)) return -1;
  if (((uintptr_t)wc | (uintptr_t)bc) & 15) return -2;
  if (w1_rows && ldw1c != HD) return -3;
  if (opt && (!opt_ok(opt) || !opt->pend)) return -4;
  const int P = ((H - 2) / 2) * ((W - 2) / 2);
  int by = (B + 63) / 64;
  if (Pt) {
    const int byp = (ldPt + 63) / 64;
    if (byp > by) by = byp;
  }
  ConvNetFwdArgs a{x, wc, bc, (const bf16*)W1c, ldw1c, hpre, (bf16*)Pt, ldPt, (uint64_t*)amax, lda, B, H, W, stamps};
  a.w1_rows = w1_rows;
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
  }
  // positions per workgroup (TDE_CONVNET_FPW = 1|2|4, default 2)
  static const int fpw = [] {
    const char* e = getenv("TDE_CONVNET_FPW");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 4) ? v : 2;
  }();
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)convnet_fwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, fwd_lds(1));
    hipFuncSetAttribute((const void*)convnet_fwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, fwd_lds(2));
    hipFuncSetAttribute((const void*)convnet_fwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, fwd_lds(4));
    attr_set = true;
  }
  const dim3 grid((P + fpw - 1) / fpw, by);
  if (fpw == 1) convnet_fwd_kernel<1><<<grid, 256, fwd_lds(1), stream>>>(a);
  else if (fpw == 2) convnet_fwd_kernel<2><<<grid, 512, fwd_lds(2), stream>>>(a);
  else convnet_fwd_kernel<4><<<grid, 1024, fwd_lds(4), stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// opt (nullable): fused step — Dense(64) rows at off_w1 updated in place (W1r rewritten; W1c [HD][ldw1c]
// too when non-null), the head variables (ranges = {lo, n} x nr, nr <= kFlatRanges) updated by
// the last workgroup, and *opt->pend set (deferred conv update).
TDE_API int tde_convnet_bwd(const float* x, const void* amax, int lda, const void* G, int ldg, const void* Gt,
                            int ldgt, const void* W1r, int ldw1r, const void* Pt, int ldPt, float* dW1, float* dwc,
                            float* dbc, int B, int H, int W, long long* stamps, const TdeStepOpt* opt,
                            long long off_w1, void* W1c, int ldw1c, const int* ranges, int nr,
                            hipStream_t stream) {
  if ((ldg & 7) || (ldgt & 7) || (ldw1r & 7) || (ldPt & 7) || ldgt < B || ldPt < B || lda < B) return -1;
  if (opt && (!opt_ok(opt) || ldw1r != HD || (W1c && (ldw1c & 3)) || (off_w1 & 3) || nr < 0 || nr > kFlatRanges))
    return -4;
  const int P = ((H - 2) / 2) * ((W - 2) / 2);
  ConvNetBwdArgs a{x, (const uint64_t*)amax, lda, (const bf16*)G, ldg, (const bf16*)Gt, ldgt, (const bf16*)W1r,
                   ldw1r, (const bf16*)Pt, ldPt, dW1, dwc, dbc, B, H, W, stamps};
  if (opt) {
    int total = 0;
    for (int i = 0; i < nr; ++i) total += ranges[2 * i + 1];
    a.apply = 1;
    a.w1 = opt->w + off_w1;
    a.m1 = opt->m ? opt->m + off_w1 : nullptr;
    a.v1 = opt->v ? opt->v + off_w1 : nullptr;
    a.w1r_out = (bf16*)W1r;
    a.w1c_out = (bf16*)W1c;
    a.ldw1c = ldw1c;
    a.iterations = opt->iterations;
    a.h = hyper_of(opt);
    a.head = FlatApply{opt->w, opt->g, opt->m, opt->v, opt->iterations, nullptr, a.h, nr, {0}, {0}};
    for (int i = 0; i < nr; ++i) {
      a.head.lo[i] = ranges[2 * i];
      a.head.n[i] = ranges[2 * i + 1];
    }
    a.pend = opt->pend;
  }
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)convnet_bwd_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, kBwdLds);
    hipFuncSetAttribute((const void*)convnet_bwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, kBwdLds);
    hipFuncSetAttribute((const void*)convnet_bwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, kBwdLds);
    attr_set = true;
  }
  const dim3 grid((P + PPW - 1) / PPW);
  if (!a.apply) convnet_bwd_kernel<0><<<grid, 1024, kBwdLds, stream>>>(a);
  else if (a.h.kind == kOptSGD) convnet_bwd_kernel<1><<<grid, 1024, kBwdLds, stream>>>(a);
  else convnet_bwd_kernel<2><<<grid, 1024, kBwdLds, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Empty kernel: measures the launch/boundary floor of the device (microbenchmarks).
__global__ void noop_kernel() {}
TDE_API int tde_noop(int blocks, int threads, hipStream_t stream) {
  noop_kernel<<<blocks, threads, 0, stream>>>();
  TDE_LAUNCH_CHECK();
  return 0;
}
