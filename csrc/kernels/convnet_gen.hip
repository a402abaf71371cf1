// Fused forward and backward of the DWK/TF2M small CNN at ANY of the common widths, float32
// (distributed_with_keras.py:33-43, tf2_mnist_distributed.py:66-72 with the user's own Conv2D filters /
// Dense units):
//   Conv2D(CC, 3x3, VALID, bias, ReLU) · MaxPooling2D(2) · Flatten · Dense(HD[, ReLU]) · Dense(C <= 16) + SCCE
// for CC in {16, 32, 48, 64} and HD in {32, 64, ..., 256} (templates): the 27 (CC, HD) pairs whose 8-wave backward
// fits a CU's LDS (Conv2D 16 / 32 up to Dense(256), 48 up to 192, 64 up to 160; `fits()` below, mirrored by the
// Python plan's LDS-fit rule), exact-f32 MFMA (v_mfma_f32_16x16x4_f32) over f32 LDS tiles and the f32 master
// weights.  The reference's own Conv2D(32) / Dense(64) keeps its hand-tuned kernels (convnet_f32.hip).  Two step
// forms: "plain" (gradients to the flat bucket, the multi-tensor optimizer after it) and the fused step (the
// optimizer applied inside the backward: Dense rows by their trunk workgroups, the head in place, the conv
// update deferred and committed by the next step's forward; see `opt` / `hopt` / `fcommit` below).
//
//   forward   one pooled position x 64 images per workgroup (4 waves): conv + bias + ReLU + 2x2 max-pool
//             for all CC channels (argmax bytes, the transposed pooled tile Pt), then the position's
//             slice of the Dense(HD) matmul on the MFMA, split-K atomics into hpre replicas
//   backward  one pooled position per workgroup (16 waves) + one head workgroup: every workgroup
//             recomputes the head from hpre (softmax-CE, dH = dl . W2^T masked by ReLU) into LDS, then
//             dP = G . W1p^T and dW1p = P^T . G (complete rows: the position's own), the routing MFMA
//             through the pool argmax / ReLU mask into the conv gradients; the head workgroup makes
//             loss / accuracy, dW2, db2, db1.  hpre is double-buffered by step parity as in the
//             specialised plan (this launch zeroes the other parity).
#include "tde_optim.h"
#include "tde_xgmi.h"

namespace tde {
namespace cgen {

constexpr int XRW = 4;             // input rows per pooled position
constexpr int kMaxBwdThreads = 1024;   // backward workgroup: NW waves (16, or 8 for the register-heavy widths)
constexpr int W2S = 17;            // row stride of W2 / dlogits tiles in LDS

template <int CC>
struct ConvW {   // one channel group of 8: the 9 taps and the bias of channels c0..c0+7 (LDS broadcast)
  float w[9][8], b[8];
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__host__ __device__ constexpr int xr_stride(int W) { return XRW * W + ((2 - (XRW * W) % 64) + 64) % 64; }

}  // namespace cgen
}  // namespace tde

// Fused step, forward side (ops/kernels.py CgenFly): the previous step's conv update applied on the fly
// while *pend (its gradient: grep replicas gwc / gbc + r * grep_stride; the slots at the conv elements;
// Adam's t = *iter_prev), and the head variables copied into the snapshot the backward's trunk reads.
struct TdeCgenFly {
  int kind;
  float lr, mom, b1, b2, eps;
  const int* pend;
  const float* gwc; const float* gbc; int grep; long long grep_stride;
  const float* mwc; const float* mbc; const float* vwc; const float* vbc;
  const long long* iter_prev;
  const float* sb1; const float* sw2; const float* sb2;   // head sources (b1 nullable)
  float* hsnap; int hC;                                     // [b1 HD | W2 HD*hC | b2 hC]
};

namespace tde {
namespace cgen {

struct GFwdArgs {
  const float* x; const float* wc; const float* bc; const float* W1;
  float* hpre; int hrep; long long hrep_stride;
  float* Pt; int ldPt;
  uint64_t* amax; int lda;
  long long* inc_iter;   // step counter advanced by block (0, 0) (nullable; the fused step's, read by the backward)
  TdeCgenFly fly;
  int fly_on;
  long long* stamps;     // diagnostics (nullable): phase clocks per workgroup (bench/cgen_micro.py --phases)
  int B, H, W;
};

template <int CC, int HD>
struct FwdCfg {
  static constexpr int PSS = CC + 4;              // LDS row stride of the pooled tile [64 images][CC]
  static constexpr int NT = HD / 16;              // column tiles of the Dense slice
  static constexpr int NTW = (NT + 3) / 4;        // column tiles per wave
  static constexpr int KQ = CC / 4;               // k per lane group
  static constexpr int kXr = 64 * 130 * 4;        // staged input rows (W <= 32)
  static constexpr int kPs = 64 * PSS * 4;
  static constexpr int kLds = kXr + kPs + 10 * CC * 4;
};

template <int CC, int HD>
__global__ __launch_bounds__(256) void cgen_fwd_kernel(GFwdArgs a) {
  using F = FwdCfg<CC, HD>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* xr = reinterpret_cast<float*>(smem);
  float* Ps = reinterpret_cast<float*>(smem + F::kXr);
  float* wcs = reinterpret_cast<float*>(smem + F::kXr + F::kPs);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int W = a.W, Wp = (W - 2) / 2;
  const int p = blockIdx.x, py = p / Wp, px = p - py * Wp;
  const int b0 = blockIdx.y * 64, b = b0 + lane;
  const bool bok = b < a.B;
  stamp(a.stamps, 0);

  // B fragments of this wave's column tiles first (their round trip overlaps the staging below):
  // W1[p*CC + fq*KQ + s][nt*16 + fr]
  float wfr[F::NTW][F::KQ];
#pragma unroll
  for (int j = 0; j < F::NTW; ++j) {
    const int nt = wave + 4 * j;
#pragma unroll
    for (int s = 0; s < F::KQ; ++s)
      wfr[j][s] = nt < F::NT ? a.W1[(size_t)(p * CC + fq * F::KQ + s) * HD + nt * 16 + fr] : 0.f;
  }
  // the 4 input rows of the position for 64 images (float4 loads, float2 LDS stores: the padded stride is
  // only 8-byte aligned), the conv weights
  const int ist = xr_stride(W), n4 = XRW * W / 4;
  for (int i = tid; i < 64 * n4; i += 256) {
    const int bl = i / n4, q = i - bl * n4;
    float4 v{0.f, 0.f, 0.f, 0.f};
    if (b0 + bl < a.B) v = *reinterpret_cast<const float4*>(a.x + (size_t)(b0 + bl) * a.H * W + (size_t)(2 * py) * W + 4 * q);
    float2* d = reinterpret_cast<float2*>(xr + bl * ist + 4 * q);
    d[0] = float2{v.x, v.y};
    d[1] = float2{v.z, v.w};
  }
  {
    // the conv weights in effect: with the previous step's update (pending) applied on the fly
    const TdeCgenFly& f = a.fly;
    const bool fly = a.fly_on && *f.pend;
    const OptHyper hy{f.kind, f.lr, f.mom, f.b1, f.b2, f.eps};
    const float lr_t = fly ? opt_lr_t(hy, f.kind == kOptAdam ? *f.iter_prev : 0) : 0.f;
    for (int i = tid; i < 10 * CC; i += 256) {
      const bool isb = i >= 9 * CC;
      const int j = isb ? i - 9 * CC : i;
      float w = isb ? a.bc[j] : a.wc[j];
      if (fly) {
        const float* gp = isb ? f.gbc + j : f.gwc + j;
        float gv[kMaxGrep];
#pragma unroll
        for (int r = 0; r < kMaxGrep; ++r) gv[r] = (r == 0 || r < f.grep) ? gp[r * f.grep_stride] : 0.f;
        float g = gv[0];
#pragma unroll
        for (int r = 1; r < kMaxGrep; ++r) g += gv[r];
        float m = 0.f, v = 0.f;
        if (f.kind != kOptSGD) m = isb ? f.mbc[j] : f.mwc[j];
        if (f.kind == kOptAdam) v = isb ? f.vbc[j] : f.vwc[j];
        w = opt_step(hy, lr_t, w, g, m, v);
      }
      wcs[i] = w;
    }
    if (a.fly_on && blockIdx.x == 0 && blockIdx.y == 0) {   // the head as of this step, for the backward's trunk
      const int nh = HD + HD * f.hC + f.hC;
      for (int i = tid; i < nh; i += 256) {
        float v;
        if (i < HD) v = f.sb1 ? f.sb1[i] : 0.f;
        else if (i < HD + HD * f.hC) v = f.sw2[i - HD];
        else v = f.sb2[i - HD - HD * f.hC];
        f.hsnap[i] = v;
      }
    }
  }
  lds_barrier();
  stamp(a.stamps, 1);

  // conv + bias + ReLU + 2x2 max-pool: lane = image, wave = channel groups of 8
  float patch[16];
  {
    const float* xb = xr + lane * ist + 2 * px;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float2 u = *reinterpret_cast<const float2*>(xb + r * W);
      const float2 v = *reinterpret_cast<const float2*>(xb + r * W + 2);
      patch[4 * r] = u.x; patch[4 * r + 1] = u.y; patch[4 * r + 2] = v.x; patch[4 * r + 3] = v.y;
    }
  }
  for (int cg = wave; cg < CC / 8; cg += 4) {
    uint64_t packed = 0;
    float out[8];
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      const int c = cg * 8 + cc;
      float best = -3.0e38f;
      int bi = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int dy = q >> 1, dx = q & 1;
        float z = wcs[9 * CC + c];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) z = fmaf(patch[(dy + ky) * 4 + dx + kx], wcs[(ky * 3 + kx) * CC + c], z);
        if (z > best) { best = z; bi = q; }
      }
      out[cc] = bok ? fmaxf(best, 0.f) : 0.f;
      packed |= (uint64_t)(best > 0.f ? (unsigned)bi : 0xFFu) << (8 * cc);
    }
    if (bok) a.amax[((size_t)p * (CC / 8) + cg) * a.lda + b] = packed;
    if (bok || b < a.ldPt) {
#pragma unroll
      for (int cc = 0; cc < 8; ++cc) a.Pt[(size_t)(p * CC + cg * 8 + cc) * a.ldPt + b] = out[cc];
    }
    float* dst = Ps + lane * F::PSS + cg * 8;
    *reinterpret_cast<float4*>(dst) = float4{out[0], out[1], out[2], out[3]};
    *reinterpret_cast<float4*>(dst + 4) = float4{out[4], out[5], out[6], out[7]};
  }
  lds_barrier();
  stamp(a.stamps, 2);

  // hpre[64 x HD] += Ps(64 x CC) . W1p(CC x HD): wave = column tiles nt = wave + 4j, all 4 row tiles;
  // lane group fq supplies k = fq*KQ .. fq*KQ + KQ-1 (the same k order in A and B)
  if (a.inc_iter && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) a.inc_iter[0] += 1;
  float* const hrow = a.hpre + (size_t)(blockIdx.x % a.hrep) * a.hrep_stride;
#pragma unroll
  for (int j = 0; j < F::NTW; ++j) {
    const int nt = wave + 4 * j;
    if (nt >= F::NT) break;
    f32x4 acc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s4 = 0; s4 < F::KQ; s4 += 4) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const float4 av = *reinterpret_cast<const float4*>(Ps + (mt * 16 + fr) * F::PSS + fq * F::KQ + s4);
        acc[mt] = mfma4(av.x, wfr[j][s4], acc[mt]);
        acc[mt] = mfma4(av.y, wfr[j][s4 + 1], acc[mt]);
        acc[mt] = mfma4(av.z, wfr[j][s4 + 2], acc[mt]);
        acc[mt] = mfma4(av.w, wfr[j][s4 + 3], acc[mt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = b0 + mt * 16 + fq * 4 + r;
        if (row < a.B) atomicAdd(hrow + (size_t)row * HD + nt * 16 + fr, acc[mt][r]);
      }
  }
  stamp(a.stamps, 3);
}

}  // namespace cgen
}  // namespace tde

// The optimizer of the fused generic step (ops/kernels.py CgenOpt): w / m / v point at the Dense kernel's
// elements of the flat buffers.
struct TdeCgenOpt {
  int kind;
  float lr, mom, b1, b2, eps;
  float* w; float* m; float* v;
  const long long* iterations;
};

// Fused step, the backward's head workgroup (ops/kernels.py CgenHead): flat buffers w / m / v, the head's
// element offsets (off_b1 < 0: no bias), t = *iterations; *pend_set = 1 and *iter_prev = t at the end.
struct TdeCgenHead {
  int kind;
  float lr, mom, b1, b2, eps;
  float* w; float* m; float* v;
  long long off_w2, off_b2, off_b1;
  const long long* iterations;
  int* pend_set;
  long long* iter_prev;
};

namespace tde {
namespace cgen {

struct GBwdArgs {
  const float* x; const uint64_t* amax; int lda;
  const float* hpre; float* hzero; int hrep; long long hrep_stride;
  const float* b1; const float* W2; const float* b2; int C; int pre_relu;
  const int* labels; float scale; float* metrics;
  const float* W1; const float* Pt; int ldPt;
  float* dW1; float* dwc; float* dbc; float* dW2; float* db2; float* db1;
  long long* iterations;   // the step counter, advanced by the head workgroup (nullable)
  // fused step (nullable): each trunk workgroup applies the optimizer to its own Dense rows in place instead
  // of storing dW1 (no other workgroup of the launch reads them; t = *oit, advanced by the forward)
  TdeCgenOpt opt;
  int opt_on;
  long long* stamps;   // diagnostics (nullable): per-workgroup phase clocks, bench/cgen_micro.py --phases
  // conv gradients: workgroup x adds into replica x % crep (dwc / dbc + replica * crep_stride): ~170 same-address
  // float atomics per value serialise at the memory side; the consumer sums the replicas
  int crep;
  long long crep_stride;
  // fused step, head workgroup: the head updated in place (the trunk reads the forward's snapshot), the
  // previous step's conv update committed (fcommit, while *fcommit.pend; its forward applied it on the fly),
  // this step's flagged pending
  TdeCgenHead hopt;
  int hopt_on;
  FlatApply fcommit;
  // plain step under the xGMI communicator (nranks > 0): dW1 rows stored straight into the owners'
  // contribution areas of the all-reduce call that follows (the fused data-parallel exchange)
  XgPush push;
  int B, H, W;
};

template <int CC, int HD, int NW>
struct BwdCfg {
  static constexpr int NTH = NW * 64;
  static constexpr int RG = HD + 4;    // row stride of G / h / W1s (floats)
  static constexpr int RP = 64 + 4;    // row stride of P^T rows
  static constexpr int DPS = CC + 4;   // row stride of dP
  static constexpr int T1 = 4 * (CC / 16);              // dP tiles (image tile x channel tile)
  static constexpr int T2 = (CC / 16) * (HD / 16);      // dW1 tiles (channel tile x unit tile)
  static constexpr int TW = (T1 + T2 + NW - 1) / NW;    // tiles per wave
  static constexpr int KG = NW / 4;                     // K groups of the logits MFMA (4 row tiles each)
  static constexpr int UTW = (HD / 16 + NW - 1) / NW;   // head workgroup: dW2 unit tiles per wave
  static constexpr int IPW = 64 / NW;                   // routing: images per wave
  static constexpr int HQ = HD / 4;                     // k per lane group in the dP MFMA
  // LDS carve (bytes).  h and G share one [64][RG] tile: G overwrites h element by element (the lane that
  // masks by h[r][j] writes G[r][j]); the head workgroup takes dW2 = h^T . dl before that.
  static constexpr int kH = 0;
  static constexpr int kW1 = kH + 64 * RG * 4;          // head workgroup: its db1 partials [4][HD] instead
  static constexpr int kPt = kW1 + CC * RG * 4;
  static constexpr int kXs = kPt + CC * RP * 4;
  static constexpr int kAm = kXs + 64 * 16 * 4;
  static constexpr int kDp = kAm + 64 * CC;
  static constexpr int kS = kDp + 64 * DPS * 4;          // logits partials | dlogits; after the chunks the
  static constexpr int kPart = (KG > 1 ? KG - 1 : 1) * 4 * 64 * 4 * 4, kDl = 64 * W2S * 4;   // conv-gradient
  static constexpr int kRed = NW * 10 * CC * 4;                                                // reduction
  static constexpr int kSBytes = kPart + kDl > kRed ? kPart + kDl : kRed;
  static constexpr int kW2 = kS + kSBytes;
  static constexpr int kB2 = kW2 + HD * W2S * 4;
  static constexpr int kLab = kB2 + 16 * 4;
  static constexpr int kLds = kLab + 64 * 4;
  static constexpr bool kFits = kLds <= 160 * 1024 && 4 * HD <= CC * RG;
};

template <int CC, int HD, int NW>
__global__ __launch_bounds__(NW * 64) void cgen_bwd_kernel(GBwdArgs a) {
  using F = BwdCfg<CC, HD, NW>;
  static_assert(F::kFits, "backward LDS exceeds a CU");
  constexpr int kGThreads = F::NTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* hs = reinterpret_cast<float*>(smem + F::kH);
  float* Gs = hs;                                                // G overwrites h in place
  float* W1s = reinterpret_cast<float*>(smem + F::kW1);
  float* db1p = W1s;                                             // head workgroup (it stages no W1 rows)
  float* Pts = reinterpret_cast<float*>(smem + F::kPt);
  float* xs = reinterpret_cast<float*>(smem + F::kXs);
  uint8_t* am = smem + F::kAm;
  float* dps = reinterpret_cast<float*>(smem + F::kDp);
  float* part = reinterpret_cast<float*>(smem + F::kS);
  float* dls = reinterpret_cast<float*>(smem + F::kS + F::kPart);
  float* red = reinterpret_cast<float*>(smem + F::kS);           // after the chunk loop
  float* w2s = reinterpret_cast<float*>(smem + F::kW2);
  float* b2s = reinterpret_cast<float*>(smem + F::kB2);
  int* labs = reinterpret_cast<int*>(smem + F::kLab);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int W = a.W, Wp = (W - 2) / 2, P = ((a.H - 2) / 2) * Wp, C = a.C;
  const bool head_wg = blockIdx.x == gridDim.x - 1;
  stamp(a.stamps, 0);

  // the other parity of hpre zeroed for the next forward's atomics (a slice per workgroup)
  {
    const long long n4 = ((long long)(a.hrep - 1) * a.hrep_stride + (long long)a.B * HD) / 4;
    const long long per = (n4 + gridDim.x - 1) / gridDim.x, beg = blockIdx.x * per, end = min(n4, beg + per);
    for (long long i = beg + tid; i < end; i += kGThreads) reinterpret_cast<float4*>(a.hzero)[i] = float4{0.f, 0.f, 0.f, 0.f};
  }
  // head weights (classes padded to 16)
  for (int i = tid; i < HD * 16; i += kGThreads) {
    const int u = i >> 4, c = i & 15;
    w2s[u * W2S + c] = c < C ? a.W2[u * C + c] : 0.f;
  }
  if (tid < 16) b2s[tid] = tid < C ? a.b2[tid] : 0.f;

  const int p = head_wg ? 0 : blockIdx.x, py = p / Wp, px = p - py * Wp;
  if (!head_wg) {
    for (int i = tid; i < CC * HD / 4; i += kGThreads) {   // W1 rows of the position [CC][HD]
      const int r = i / (HD / 4), c4 = (i - r * (HD / 4)) * 4;
      *reinterpret_cast<float4*>(W1s + r * F::RG + c4) = *reinterpret_cast<const float4*>(a.W1 + (size_t)(p * CC + r) * HD + c4);
    }
  }

  f32x4 accw[F::TW];   // dW1 tile accumulators (persist over the image chunks)
#pragma unroll
  for (int j = 0; j < F::TW; ++j) accw[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accr[CC / 16];
#pragma unroll
  for (int ct = 0; ct < CC / 16; ++ct) accr[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 gw[F::UTW];   // head workgroup: dW2 tiles (unit tiles wave, wave + NW, ...)
#pragma unroll
  for (int j = 0; j < F::UTW; ++j) gw[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float la = 0.f, ca = 0.f, na = 0.f, db2acc = 0.f;
  if (head_wg)
    for (int i = tid; i < 4 * HD; i += kGThreads) db1p[i] = 0.f;

  for (int b0 = 0; b0 < a.B; b0 += 64) {
    const int nb = min(64, a.B - b0);
    // ---- h = act(hpre + b1) for the chunk (replicas summed), labels; trunk: P^T rows, patches, argmax
    for (int i = tid; i < 64 * HD / 4; i += kGThreads) {
      const int r = i / (HD / 4), c4 = (i - r * (HD / 4)) * 4;
      float4 h{0.f, 0.f, 0.f, 0.f};
      if (r < nb) {
        for (int q = 0; q < a.hrep; ++q) {
          const float4 v = *reinterpret_cast<const float4*>(a.hpre + (size_t)q * a.hrep_stride + (size_t)(b0 + r) * HD + c4);
          h.x += v.x; h.y += v.y; h.z += v.z; h.w += v.w;
        }
        if (a.b1) {
          const float4 bb = *reinterpret_cast<const float4*>(a.b1 + c4);
          h.x += bb.x; h.y += bb.y; h.z += bb.z; h.w += bb.w;
        }
        if (a.pre_relu) h = float4{fmaxf(h.x, 0.f), fmaxf(h.y, 0.f), fmaxf(h.z, 0.f), fmaxf(h.w, 0.f)};
      }
      *reinterpret_cast<float4*>(hs + r * F::RG + c4) = h;
    }
    if (tid < 64) labs[tid] = tid < nb ? a.labels[b0 + tid] : 0;
    if (!head_wg) {
      for (int i = tid; i < CC * 16; i += kGThreads) {   // P^T rows of the position: [CC][64 images]
        const int r = i >> 4, c4 = (i & 15) * 4;
        float4 v{0.f, 0.f, 0.f, 0.f};
        const float* src = a.Pt + (size_t)(p * CC + r) * a.ldPt + b0 + c4;
        if (c4 + 3 < nb) v = *reinterpret_cast<const float4*>(src);
        else {
          if (c4 < nb) v.x = src[0];
          if (c4 + 1 < nb) v.y = src[1];
          if (c4 + 2 < nb) v.z = src[2];
        }
        *reinterpret_cast<float4*>(Pts + r * F::RP + c4) = v;
      }
      if (tid < 256) {
        const int bl = tid >> 2, r = tid & 3;
        float4 xv{0.f, 0.f, 0.f, 0.f};
        if (bl < nb) {
          const float2* row = reinterpret_cast<const float2*>(a.x + (size_t)(b0 + bl) * a.H * W + (2 * py + r) * W + 2 * px);
          const float2 u = row[0], t = row[1];
          xv = float4{u.x, u.y, t.x, t.y};
        }
        *reinterpret_cast<float4*>(xs + bl * 16 + r * 4) = xv;
      }
      for (int i = tid; i < 64 * (CC / 8); i += kGThreads) {
        const int cg = i >> 6, bb = i & 63;
        const uint64_t v = bb < nb ? a.amax[((size_t)p * (CC / 8) + cg) * a.lda + b0 + bb] : ~0ull;
        *reinterpret_cast<uint64_t*>(am + bb * CC + cg * 8) = v;
      }
    }
    lds_barrier();
    stamp(a.stamps, 1);

    // ---- logits = h . W2 + b2: wave = (row tile rt, K group kg: K quarters kg, kg + KG, ..); softmax-CE on
    //      waves 0..3 -> dls
    {
      const int rt = wave & 3, kg = wave >> 2;
      f32x4 lg{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kq = kg; kq < 4; kq += F::KG)
#pragma unroll
        for (int k = kq * (HD / 4); k < (kq + 1) * (HD / 4); k += 4)
          lg = mfma4(hs[(rt * 16 + fr) * F::RG + k + fq], w2s[(k + fq) * W2S + fr], lg);
      if (kg > 0) *reinterpret_cast<f32x4*>(part + (((kg - 1) * 4 + rt) * 64 + lane) * 4) = lg;
      lds_barrier();
      if (wave < 4) {
#pragma unroll
        for (int q = 0; q < F::KG - 1; ++q) {
          const f32x4 pv = *reinterpret_cast<const f32x4*>(part + ((q * 4 + rt) * 64 + lane) * 4);
          lg[0] += pv[0]; lg[1] += pv[1]; lg[2] += pv[2]; lg[3] += pv[3];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = rt * 16 + fq * 4 + i;
          const bool valid = r < nb, cv = fr < C;
          const float z = cv ? lg[i] + b2s[fr] : -3.0e38f;
          const float m = row16_max(z);
          const float e = cv ? __expf(z - m) : 0.f;
          const float ssum = row16_sum(e);
          const int label = labs[r];
          const int amx = row16_min(cv && z == m ? fr : 64);
          const float zl = __shfl(z, (lane & ~15) | (label & 15), 64);
          if (valid && fr == 0) {
            la += __logf(ssum) + m - zl;
            ca += (amx == label) ? 1.f : 0.f;
            na += 1.f;
          }
          dls[r * W2S + fr] = (valid && cv) ? (e / ssum - (fr == label ? 1.f : 0.f)) * a.scale : 0.f;
        }
      }
      lds_barrier();
      stamp(a.stamps, 2);
    }
    if (head_wg) {
      // dW2[u][c] += sum_b h[b][u] dl[b][c] (unit tiles ut = wave, wave + NW, ..), db2 — before G overwrites h
#pragma unroll
      for (int j = 0; j < F::UTW; ++j) {
        const int ut = wave + NW * j;
        if (ut < HD / 16) {
#pragma unroll 4
          for (int k = 0; k < 64; k += 4) gw[j] = mfma4(hs[(k + fq) * F::RG + ut * 16 + fr], dls[(k + fq) * W2S + fr], gw[j]);
        }
      }
      if (tid < 16) {
        float s = 0.f;
        for (int r = 0; r < nb; ++r) s += dls[r * W2S + tid];
        db2acc += s;
      }
      lds_barrier();
    }
    // ---- G = dH = dl . W2^T masked by h > 0 (rows < nb), in place of h: tiles (row tile, unit tile) over the
    //      waves
    for (int t = wave; t < 4 * (HD / 16); t += NW) {
      const int rt = t & 3, ut = t >> 2;
      f32x4 gh{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 16; k += 4) gh = mfma4(dls[(rt * 16 + fr) * W2S + k + fq], w2s[(ut * 16 + fr) * W2S + k + fq], gh);
      const int j = ut * 16 + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rt * 16 + fq * 4 + i;
        if ((a.pre_relu && !(hs[r * F::RG + j] > 0.f)) || r >= nb) gh[i] = 0.f;
        Gs[r * F::RG + j] = gh[i];
      }
    }
    if (head_wg) {
      lds_barrier();
      for (int i = tid; i < 4 * HD; i += kGThreads) {   // db1 += sum_b G[b][u]: 4 row groups of 16 images per unit
        const int u = i % HD, rg = i / HD;
        float s = 0.f;
        for (int r = rg * 16; r < rg * 16 + 16; ++r) s += Gs[r * F::RG + u];
        db1p[i] += s;
      }
      lds_barrier();
      continue;
    }
    lds_barrier();
    stamp(a.stamps, 3);

    // ---- tiles over the waves: dP[b][c] = sum_u G[b][u] W1p[c][u] (t < T1), dW1p[c][u] += sum_b P[b][c]
    //      G[b][u] (T1 <= t < T1 + T2; accumulators persist over the chunks)
#pragma unroll
    for (int j = 0; j < F::TW; ++j) {
      const int t = wave + NW * j;
      if (t < F::T1) {
        const int mt = t & 3, ct = t >> 2;
        f32x4 acc{0.f, 0.f, 0.f, 0.f};
        const float* Ab = Gs + (mt * 16 + fr) * F::RG + fq * F::HQ;
        const float* Bb = W1s + (ct * 16 + fr) * F::RG + fq * F::HQ;
#pragma unroll
        for (int s = 0; s < F::HQ; s += 4) {
          const float4 av = *reinterpret_cast<const float4*>(Ab + s);
          const float4 bv = *reinterpret_cast<const float4*>(Bb + s);
          acc = mfma4(av.x, bv.x, acc);
          acc = mfma4(av.y, bv.y, acc);
          acc = mfma4(av.z, bv.z, acc);
          acc = mfma4(av.w, bv.w, acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) dps[(mt * 16 + fq * 4 + r) * F::DPS + ct * 16 + fr] = acc[r];
      } else if (t < F::T1 + F::T2) {
        const int u2 = t - F::T1, rt = u2 % (CC / 16), nt = u2 / (CC / 16);
        // A[row c][k b] = P^T[c][b]; B[k b][col u] = G[b][u]; lane group fq takes images fq*16 .. +15
        const float* Ab = Pts + (rt * 16 + fr) * F::RP + fq * 16;
#pragma unroll
        for (int s = 0; s < 16; s += 4) {
          const float4 av = *reinterpret_cast<const float4*>(Ab + s);
          const float* Bb = Gs + (fq * 16 + s) * F::RG + nt * 16 + fr;
          accw[j] = mfma4(av.x, Bb[0], accw[j]);
          accw[j] = mfma4(av.y, Bb[F::RG], accw[j]);
          accw[j] = mfma4(av.z, Bb[2 * F::RG], accw[j]);
          accw[j] = mfma4(av.w, Bb[3 * F::RG], accw[j]);
        }
      }
    }
    lds_barrier();
    stamp(a.stamps, 4);

    // ---- routing MFMA: dWc[tap][c] += sum over (image, window slot) of X[tap] . dP masked by the argmax;
    //      k = (b, q): lane group fq = window slot q; wave takes images 4w .. 4w+3
    {
      const int tap = fr, ky = tap / 3, kx = tap - ky * 3, qy = fq >> 1, qx = fq & 1;
#pragma unroll
      for (int s = 0; s < F::IPW; ++s) {
        const int bl = wave * F::IPW + s;
        const float xa = tap < 9 ? xs[bl * 16 + (qy + ky) * 4 + qx + kx] : (tap == 9 ? 1.f : 0.f);
#pragma unroll
        for (int ct = 0; ct < CC / 16; ++ct) {
          const int c = ct * 16 + fr;
          const float d = am[bl * CC + c] == (unsigned)fq ? dps[bl * F::DPS + c] : 0.f;
          accr[ct] = mfma4(xa, d, accr[ct]);
        }
      }
    }
    lds_barrier();
    stamp(a.stamps, 5);
  }

  if (head_wg) {
    la = rows4_sum(la);
    ca = rows4_sum(ca);
    na = rows4_sum(na);
    if (wave < 4 && lane == 0 && a.metrics && na > 0.f) {
      atomicAdd(a.metrics + 0, la);
      atomicAdd(a.metrics + 1, ca);
      atomicAdd(a.metrics + 2, na);
    }
    const float db1v = tid < HD ? (db1p[tid] + db1p[HD + tid]) + (db1p[2 * HD + tid] + db1p[3 * HD + tid]) : 0.f;
    if (a.hopt_on) {
      // fused step: the head's update in place, then the previous step's conv update committed
      const TdeCgenHead& o = a.hopt;
      const OptHyper hy{o.kind, o.lr, o.mom, o.b1, o.b2, o.eps};
      const long long t = *o.iterations;
      const float lr_t = opt_lr_t(hy, t);
      auto upd = [&](long long e, float g) {
        float m = o.kind != kOptSGD ? o.m[e] : 0.f;
        float v = o.kind == kOptAdam ? o.v[e] : 0.f;
        o.w[e] = opt_step(hy, lr_t, o.w[e], g, m, v);
        if (o.kind != kOptSGD) o.m[e] = m;
        if (o.kind == kOptAdam) o.v[e] = v;
      };
#pragma unroll
      for (int j = 0; j < F::UTW; ++j) {
        const int ut = wave + NW * j;
        if (ut < HD / 16 && fr < C)
#pragma unroll
          for (int i = 0; i < 4; ++i) upd(o.off_w2 + (long long)(ut * 16 + fq * 4 + i) * C + fr, gw[j][i]);
      }
      if (tid < C) upd(o.off_b2 + tid, db2acc);
      if (tid < HD && o.off_b1 >= 0) upd(o.off_b1 + tid, db1v);
      __shared__ int s_cp;
      if (tid == 0) s_cp = *a.fcommit.pend;
      __syncthreads();
      if (s_cp) flat_apply(a.fcommit, t - 1, tid, kGThreads);
      __syncthreads();
      if (tid == 0) {
        if (s_cp) *a.fcommit.pend = 0;
        *o.pend_set = 1;
        *o.iter_prev = t;
      }
    } else {
#pragma unroll
      for (int j = 0; j < F::UTW; ++j) {
        const int ut = wave + NW * j;
        if (ut < HD / 16 && fr < C && a.dW2)
#pragma unroll
          for (int i = 0; i < 4; ++i) atomicAdd(a.dW2 + (size_t)(ut * 16 + fq * 4 + i) * C + fr, gw[j][i]);
      }
      if (tid < C && a.db2) atomicAdd(a.db2 + tid, db2acc);
      if (tid < HD && a.db1) atomicAdd(a.db1 + tid, db1v);
    }
    if (tid == 0 && a.iterations) a.iterations[0] += 1;
  } else {

  // dW1 rows of the position (complete: this workgroup owns them): stored, or applied in place from the LDS
  // copy of the rows this launch read
  if (a.opt_on) {
    const TdeCgenOpt& o = a.opt;
    const OptHyper hy{o.kind, o.lr, o.mom, o.b1, o.b2, o.eps};
    const float lr_t = opt_lr_t(hy, o.kind == kOptAdam ? *o.iterations : 0);
#pragma unroll
    for (int j = 0; j < F::TW; ++j) {
      const int t = wave + NW * j;
      if (t >= F::T1 && t < F::T1 + F::T2) {
        const int u2 = t - F::T1, rt = u2 % (CC / 16), nt = u2 / (CC / 16);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rt * 16 + fq * 4 + r, col = nt * 16 + fr;
          const size_t e = (size_t)(p * CC + row) * HD + col;
          float m = o.kind != kOptSGD ? o.m[e] : 0.f;
          float v = o.kind == kOptAdam ? o.v[e] : 0.f;
          o.w[e] = opt_step(hy, lr_t, W1s[row * F::RG + col], accw[j][r], m, v);
          if (o.kind != kOptSGD) o.m[e] = m;
          if (o.kind == kOptAdam) o.v[e] = v;
        }
      }
    }
  } else if (a.push.nranks > 0) {
    // the position's complete dW1 rows staged in W1s (its last reader, the dP tiles, finished at the chunk
    // loop's final barrier), then pushed below as contiguous float4 runs
#pragma unroll
    for (int j = 0; j < F::TW; ++j) {
      const int t = wave + NW * j;
      if (t >= F::T1 && t < F::T1 + F::T2) {
        const int u2 = t - F::T1, rt = u2 % (CC / 16), nt = u2 / (CC / 16);
#pragma unroll
        for (int r = 0; r < 4; ++r) W1s[(rt * 16 + fq * 4 + r) * F::RG + nt * 16 + fr] = accw[j][r];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < F::TW; ++j) {
      const int t = wave + NW * j;
      if (t >= F::T1 && t < F::T1 + F::T2) {
        const int u2 = t - F::T1, rt = u2 % (CC / 16), nt = u2 / (CC / 16);
#pragma unroll
        for (int r = 0; r < 4; ++r) a.dW1[(size_t)(p * CC + rt * 16 + fq * 4 + r) * HD + nt * 16 + fr] = accw[j][r];
      }
    }
  }
  // conv gradients: the 16 waves' routing accumulators summed through LDS, one add per value
#pragma unroll
  for (int ct = 0; ct < CC / 16; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int tap = fq * 4 + r;
      if (tap < 10) red[((size_t)wave * 10 + tap) * CC + ct * 16 + fr] = accr[ct][r];
    }
  lds_barrier();
  stamp(a.stamps, 6);
  for (int i = tid; i < 10 * CC; i += kGThreads) {
    const int tap = i / CC, c = i - tap * CC;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[((size_t)w * 10 + tap) * CC + c];
    const long long ro = (long long)(blockIdx.x % a.crep) * a.crep_stride;
    if (tap < 9) atomicAdd(a.dwc + ro + tap * CC + c, s);
    else atomicAdd(a.dbc + ro + c, s);
  }
  if (a.push.nranks > 0) {   // (the barrier above published the W1s staging)
    const int parity = (int)((*a.push.epoch + 1u) & 1u);
    for (int i = tid; i < CC * HD / 4; i += kGThreads) {
      const int row = i / (HD / 4), c4 = (i - row * (HD / 4)) * 4;
      xg_push_store4(a.push, parity, a.push.off + (long long)(p * CC + row) * HD + c4,
                     *reinterpret_cast<const float4*>(W1s + row * F::RG + c4));
    }
    xg_push_drain();   // acknowledged before the wave ends
  }
  stamp(a.stamps, 7);
  }
}

template <int CC, int HD>
static int launch_fwd(const GFwdArgs& a, int P, hipStream_t s) {
  using F = FwdCfg<CC, HD>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)cgen_fwd_kernel<CC, HD>, hipFuncAttributeMaxDynamicSharedMemorySize, F::kLds);
    attr = true;
  }
  int by = (a.B + 63) / 64;
  const int byp = (a.ldPt + 63) / 64;
  if (byp > by) by = byp;
  cgen_fwd_kernel<CC, HD><<<dim3(P, by), 256, F::kLds, s>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

template <int CC, int HD, int NW>
static int launch_bwd_nw(const GBwdArgs& a, int P, hipStream_t s) {
  using F = BwdCfg<CC, HD, NW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)cgen_bwd_kernel<CC, HD, NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              F::kLds);
    attr = true;
  }
  cgen_bwd_kernel<CC, HD, NW><<<P + 1, F::NTH, F::kLds, s>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Waves per backward workgroup: 16 (4 per SIMD, 128 VGPRs each) unless the width's accumulators would spill
// there (TDE_CGEN_WAVES = 8 | 16 forces one).
static int bwd_waves(int CC, int HD) {
  static const int forced = [] {
    const char* e = getenv("TDE_CGEN_WAVES");
    return e ? atoi(e) : 0;
  }();
  if (forced == 8 || forced == 16) return forced;
  return CC * HD >= 6144 ? 8 : 16;
}

// The instantiated family: the backward's LDS at 8 waves fits a CU (Conv2D 16 / 32 up to Dense(256), 48 up to
// 192, 64 up to 160).
template <int CC, int HD>
constexpr bool fits() { return BwdCfg<CC, HD, 8>::kFits; }

template <int CC, int HD>
static int launch_bwd(const GBwdArgs& a, int P, hipStream_t s) {
  if constexpr (!fits<CC, HD>()) {
    return -9;
  } else if constexpr (!BwdCfg<CC, HD, 16>::kFits) {
    return launch_bwd_nw<CC, HD, 8>(a, P, s);
  } else {
    return bwd_waves(CC, HD) == 8 ? launch_bwd_nw<CC, HD, 8>(a, P, s) : launch_bwd_nw<CC, HD, 16>(a, P, s);
  }
}

template <int CC, int HD>
static int launch_fwd_if(const GFwdArgs& a, int P, hipStream_t s) {
  if constexpr (!fits<CC, HD>()) return -9;
  else return launch_fwd<CC, HD>(a, P, s);
}

template <int CC, int HD>
static int supported_if() { return fits<CC, HD>() ? 1 : 0; }

#define TDE_CGEN_CASES_CC(FN, CCV, ...)                                                                   \
  case CCV * 1000 + 32: return FN<CCV, 32>(__VA_ARGS__);   case CCV * 1000 + 64: return FN<CCV, 64>(__VA_ARGS__);   \
  case CCV * 1000 + 96: return FN<CCV, 96>(__VA_ARGS__);   case CCV * 1000 + 128: return FN<CCV, 128>(__VA_ARGS__); \
  case CCV * 1000 + 160: return FN<CCV, 160>(__VA_ARGS__); case CCV * 1000 + 192: return FN<CCV, 192>(__VA_ARGS__); \
  case CCV * 1000 + 224: return FN<CCV, 224>(__VA_ARGS__); case CCV * 1000 + 256: return FN<CCV, 256>(__VA_ARGS__);
#define TDE_CGEN_DISPATCH(FN, CCV, HDV, ...)                                                              \
  switch (CCV * 1000 + HDV) {                                                                              \
    TDE_CGEN_CASES_CC(FN, 16, __VA_ARGS__)                                                                 \
    TDE_CGEN_CASES_CC(FN, 32, __VA_ARGS__)                                                                 \
    TDE_CGEN_CASES_CC(FN, 48, __VA_ARGS__)                                                                 \
    TDE_CGEN_CASES_CC(FN, 64, __VA_ARGS__)                                                                 \
    default: return -9;                                                                                     \
  }

}  // namespace cgen
}  // namespace tde

using namespace tde;
using namespace tde::cgen;

static int supported_code(int CC, int HD) { TDE_CGEN_DISPATCH(supported_if, CC, HD) }

TDE_API int tde_cgen_supported(int CC, int HD) { return supported_code(CC, HD) == 1; }

// Forward (see the header).  x [B][H][W] f32 (C_in = 1), wc [9][CC], bc [CC], W1 [P*CC][HD] f32 master,
// hpre [hrep][>=B][HD] (+=), Pt [P*CC][ldPt], amax [P][CC/8][lda] (8 argmax bytes per u64).  fly (nullable):
// the fused step's deferred conv update and head snapshot (TdeCgenFly).
TDE_API int tde_cgen_fwd(int CC, int HD, const float* x, const float* wc, const float* bc, const float* W1,
                         float* hpre, int hrep, long long hrep_stride, float* Pt, int ldPt, void* amax, int lda,
                         long long* inc_iter, const TdeCgenFly* fly, long long* stamps, int B, int H, int W,
                         hipStream_t stream) {
  if (!tde_cgen_supported(CC, HD) || (W & 3) || W > 32 || H < 4 || W < 4 || ((H - 2) & 1) || ((W - 2) & 1))
    return -1;
  if (fly && (!fly->pend || !fly->gwc || !fly->gbc || fly->grep < 1 || fly->grep > kMaxGrep || !fly->iter_prev ||
              (fly->kind != kOptSGD && (!fly->mwc || !fly->mbc)) || (fly->kind == kOptAdam && (!fly->vwc || !fly->vbc)) ||
              !fly->sw2 || !fly->sb2 || !fly->hsnap || fly->hC < 1 || fly->hC > 16))
    return -3;
  if (!x || !wc || !bc || !W1 || !hpre || !Pt || !amax || (ldPt & 7) || ldPt < B || lda < B || hrep < 1 ||
      (hrep > 1 && hrep_stride < (long long)B * HD) || ((uintptr_t)x & 15) || ((uintptr_t)W1 & 15))
    return -2;
  const int P = ((H - 2) / 2) * ((W - 2) / 2);
  GFwdArgs a{x, wc, bc, W1, hpre, hrep, hrep_stride, Pt, ldPt, (uint64_t*)amax, lda, inc_iter,
             fly ? *fly : TdeCgenFly{}, fly != nullptr, stamps, B, H, W};
  TDE_CGEN_DISPATCH(launch_fwd_if, CC, HD, a, P, stream)
}

// Backward (plain step: gradients out).  hpre / hzero [hrep][>=B][HD] (hzero zeroed here), dW1 [P*CC][HD]
// stored, dwc [9][CC] / dbc [CC] atomically added, dW2 [HD][C] / db2 [C] / db1 [HD] added (nullable);
// iterations (nullable) advanced by one.  opt (nullable): the fused step — dW1 applied to the Dense kernel in
// place by the optimizer instead of stored (dW1 may then be null).  crep / crep_stride: conv-gradient replicas.
// hopt + fcommit (nullable, with opt): the fused step's head update in the head workgroup and the commit of the
// previous step's conv update (b1 / W2 / b2 are then the forward's snapshot).
// push (nullable; plain step): dW1 into the xGMI owners' contribution areas instead of dW1.
TDE_API int tde_cgen_bwd(int CC, int HD, const float* x, const void* amax, int lda, const float* hpre, float* hzero,
                         int hrep, long long hrep_stride, const float* b1, const float* W2, const float* b2, int C,
                         int pre_relu, const int* labels, float scale, float* metrics, const float* W1, const float* Pt,
                         int ldPt, float* dW1, float* dwc, float* dbc, float* dW2, float* db2, float* db1,
                         long long* iterations, const TdeCgenOpt* opt, long long* stamps, int crep,
                         long long crep_stride, const TdeCgenHead* hopt, const FlatApply* fcommit,
                         const XgPush* push, int B, int H, int W, hipStream_t stream) {
  if (!tde_cgen_supported(CC, HD) || C < 1 || C > 16 || W > 32 || (W & 3)) return -1;
  if (opt && (!opt->w || (opt->kind != kOptSGD && !opt->m) || (opt->kind == kOptAdam && (!opt->v || !opt->iterations))))
    return -3;
  if (crep < 1 || crep > 64 || (crep > 1 && crep_stride < 10LL * CC)) return -4;
  if (push && push->nranks > 0 &&
      (opt || push->nranks > kXgMaxRanks || push->L <= 0 || (push->L & 3) || (push->off & 3) || !push->epoch))
    return -6;
  if (hopt && (!opt || !fcommit || !fcommit->pend || fcommit->grep > kMaxGrep || fcommit->nr > kFlatRanges ||
               !hopt->w || (hopt->kind != kOptSGD && !hopt->m) || (hopt->kind == kOptAdam && !hopt->v) ||
               !hopt->iterations || !hopt->pend_set || !hopt->iter_prev))
    return -5;
  if (!x || !amax || !hpre || !hzero || !W2 || !b2 || !labels || !W1 || !Pt || (!dW1 && !opt) || !dwc || !dbc ||
      (ldPt & 7) || ldPt < B || lda < B || hrep < 1 || (hrep > 1 && (hrep_stride < (long long)B * HD || (hrep_stride & 3))) ||
      (((uintptr_t)hpre | (uintptr_t)hzero | (uintptr_t)W1 | (uintptr_t)Pt | (uintptr_t)b1) & 15))
    return -2;
  const int P = ((H - 2) / 2) * ((W - 2) / 2);
  GBwdArgs a{x, (const uint64_t*)amax, lda, hpre, hzero, hrep, hrep_stride, b1, W2, b2, C, pre_relu, labels, scale,
             metrics, W1, Pt, ldPt, dW1, dwc, dbc, dW2, db2, db1, iterations, opt ? *opt : TdeCgenOpt{}, opt != nullptr, stamps,
             crep, crep_stride, hopt ? *hopt : TdeCgenHead{}, hopt != nullptr, fcommit ? *fcommit : FlatApply{},
             push ? *push : XgPush{}, B, H, W};
  TDE_CGEN_DISPATCH(launch_bwd, CC, HD, a, P, stream)
}
