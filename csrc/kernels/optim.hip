// Multi-tensor optimizer apply over the flat parameter buffer: SGD (optionally
// momentum / Nesterov, Keras form) and Adam (Keras/TF form, epsilon added to
// sqrt(v_hat)), in ONE launch for all variables (SURVEY.md §2.5 A14/B17,
// reference: distributed_with_keras.py:42, mnist_keras_distributed.py:111,
// tf2_mnist_distributed.py:137).
//
// The same pass (a) zeroes the gradient buffer for the next step's atomic /
// split-K accumulation and (b) refreshes the bf16 compute copies ("shadows") of
// the weights in the layouts the MFMA kernels read — row-major and, through an
// LDS 16x64 transpose, column-major.  The step counter (`iterations`, Keras
// optimizer.iterations / Estimator global_step) lives on the device and is
// advanced by the step's loss kernel before this launch, so Adam's bias
// correction reads t = iterations with no host round trip and no in-kernel
// cross-workgroup protocol.
//
// Vectorised: float4 loads/stores everywhere (segments are 256-byte aligned).
#include "tde_optim.h"

namespace tde {

struct OptSeg {
  long long off;      // element offset in the flat buffers
  int rows, cols;     // logical 2-D shape (rows*cols elements)
  long long sh_off;   // bf16 row-major shadow offset or -1
  long long sht_off;  // bf16 transposed shadow offset or -1 (tiled blocks)
};

struct OptArgs {
  float* w; float* g; float* m; float* v;
  bf16* shadow;
  const OptSeg* segs;
  const int4* table;        // per block: {seg, kind(0=1d,1=tile), a, b}
  const long long* iterations;
  int kind;                 // 0 sgd, 1 momentum, 2 nesterov, 3 adam
  float lr, mom, b1, b2, eps, grad_scale;
  int zero_grad;
  const float* lr_ptr;      // optional device-resident lr (schedules)
};

constexpr int kChunk = 2048;
constexpr int kTileR = 16;  // rows per transposed-shadow tile (tile = kTileR x 64)

struct Hyper {
  float lr, lr_t;
};

__device__ __forceinline__ float upd1(const OptArgs& a, float w, float g, float& m, float& v, const Hyper& h) {
  const OptHyper oh{a.kind, h.lr, a.mom, a.b1, a.b2, a.eps};
  return opt_step(oh, h.lr_t, w, g * a.grad_scale, m, v);
}

// Update 4 consecutive elements at flat index i (16-byte aligned).
__device__ __forceinline__ float4 upd4(const OptArgs& a, size_t i, const Hyper& h) {
  float4 w = *reinterpret_cast<float4*>(a.w + i);
  const float4 g = *reinterpret_cast<float4*>(a.g + i);
  float4 m = {0.f, 0.f, 0.f, 0.f}, v = {0.f, 0.f, 0.f, 0.f};
  if (a.kind != 0) m = *reinterpret_cast<float4*>(a.m + i);
  if (a.kind == 3) v = *reinterpret_cast<float4*>(a.v + i);
  w.x = upd1(a, w.x, g.x, m.x, v.x, h);
  w.y = upd1(a, w.y, g.y, m.y, v.y, h);
  w.z = upd1(a, w.z, g.z, m.z, v.z, h);
  w.w = upd1(a, w.w, g.w, m.w, v.w, h);
  *reinterpret_cast<float4*>(a.w + i) = w;
  if (a.zero_grad) *reinterpret_cast<float4*>(a.g + i) = float4{0.f, 0.f, 0.f, 0.f};
  if (a.kind != 0) *reinterpret_cast<float4*>(a.m + i) = m;
  if (a.kind == 3) *reinterpret_cast<float4*>(a.v + i) = v;
  return w;
}

__device__ __forceinline__ float upds(const OptArgs& a, size_t i, const Hyper& h) {
  float m = a.kind != 0 ? a.m[i] : 0.f, v = a.kind == 3 ? a.v[i] : 0.f;
  const float w = upd1(a, a.w[i], a.g[i], m, v, h);
  a.w[i] = w;
  if (a.zero_grad) a.g[i] = 0.f;
  if (a.kind != 0) a.m[i] = m;
  if (a.kind == 3) a.v[i] = v;
  return w;
}

__global__ __launch_bounds__(256) void optim_apply_kernel(OptArgs a) {
  __shared__ bf16 tile[kTileR][72];
  const int4 ent = a.table[blockIdx.x];
  const OptSeg s = a.segs[ent.x];
  Hyper h;
  h.lr = a.lr_ptr ? *a.lr_ptr : a.lr;
  h.lr_t = opt_lr_t(OptHyper{a.kind, h.lr, a.mom, a.b1, a.b2, a.eps}, a.kind == kOptAdam ? *a.iterations : 0);
  const int tid = threadIdx.x;

  if (ent.y == 0) {
    const long long n = (long long)s.rows * s.cols;
    const long long beg = (long long)ent.z * kChunk;
    const long long end = beg + kChunk < n ? beg + kChunk : n;
#pragma unroll
    for (int it = 0; it < kChunk / 1024; ++it) {
      const long long e = beg + it * 1024 + tid * 4;
      if (e + 4 <= end) {
        const float4 w = upd4(a, (size_t)(s.off + e), h);
        if (s.sh_off >= 0) {
          bf16x4 hv = {f2bf(w.x), f2bf(w.y), f2bf(w.z), f2bf(w.w)};
          *reinterpret_cast<bf16x4*>(a.shadow + s.sh_off + e) = hv;
        }
      } else {
        for (long long q = e; q < end && q < e + 4; ++q) {
          const float w = upds(a, (size_t)(s.off + q), h);
          if (s.sh_off >= 0) a.shadow[s.sh_off + q] = f2bf(w);
        }
      }
    }
  } else {
    // 16x64 tiles (one float4 per thread): ~4x more workgroups than 64x64 tiles, so
    // a 5408x64 Dense kernel spreads over 338 workgroups instead of 85 CUs.
    const int r0 = ent.z * kTileR, c0 = ent.w * 64;
    const bool vec = (s.cols % 4) == 0;
    {
      const int r = tid >> 4, c = (tid & 15) * 4;
      const int gr = r0 + r, gc = c0 + c;
      if (gr < s.rows) {
        const long long e = (long long)gr * s.cols + gc;
        if (vec && gc + 4 <= s.cols) {
          const float4 w = upd4(a, (size_t)(s.off + e), h);
          bf16x4 hv = {f2bf(w.x), f2bf(w.y), f2bf(w.z), f2bf(w.w)};
          if (s.sh_off >= 0) *reinterpret_cast<bf16x4*>(a.shadow + s.sh_off + e) = hv;
          *reinterpret_cast<bf16x4*>(&tile[r][c]) = hv;
        } else {
          for (int q = 0; q < 4 && gc + q < s.cols; ++q) {
            const float w = upds(a, (size_t)(s.off + e + q), h);
            const bf16 hv = f2bf(w);
            if (s.sh_off >= 0) a.shadow[s.sh_off + e + q] = hv;
            tile[r][c + q] = hv;
          }
        }
      }
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < kTileR * 64 / 256; ++it) {
      const int i = it * 256 + tid;
      const int c = i / kTileR, r = i % kTileR, gr = r0 + r, gc = c0 + c;
      if (gr < s.rows && gc < s.cols) a.shadow[s.sht_off + (long long)gc * s.rows + gr] = tile[r][c];
    }
  }
}

// Writes bf16 shadows from the current weights without updating (init/restore).
__global__ __launch_bounds__(256) void shadow_refresh_kernel(const float* w, bf16* shadow,
                                                             const OptSeg* segs,
                                                             const int4* table) {
  __shared__ bf16 tile[kTileR][66];
  const int4 ent = table[blockIdx.x];
  const OptSeg s = segs[ent.x];
  const int tid = threadIdx.x;
  if (ent.y == 0) {
    const long long n = (long long)s.rows * s.cols;
    const long long beg = (long long)ent.z * kChunk;
    const long long end = beg + kChunk < n ? beg + kChunk : n;
    if (s.sh_off >= 0)
      for (long long e = beg + tid; e < end; e += 256) shadow[s.sh_off + e] = f2bf(w[s.off + e]);
  } else {
    const int r0 = ent.z * kTileR, c0 = ent.w * 64;
    for (int i = tid; i < kTileR * 64; i += 256) {
      const int r = i >> 6, c = i & 63, gr = r0 + r, gc = c0 + c;
      if (gr < s.rows && gc < s.cols) {
        const long long e = (long long)gr * s.cols + gc;
        const bf16 h = f2bf(w[s.off + e]);
        if (s.sh_off >= 0) shadow[s.sh_off + e] = h;
        tile[r][c] = h;
      }
    }
    __syncthreads();
    for (int i = tid; i < kTileR * 64; i += 256) {
      const int c = i / kTileR, r = i % kTileR, gr = r0 + r, gc = c0 + c;
      if (gr < s.rows && gc < s.cols) shadow[s.sht_off + (long long)gc * s.rows + gr] = tile[r][c];
    }
  }
}

// Deferred-update flush (one workgroup): applies the ranges if *pend with t = *iterations, then clears
// *pend.  Without pend (an unconditional update) the ranges are spread over the whole grid.
__global__ __launch_bounds__(256) void flat_apply_kernel(FlatApply f) {
  __shared__ int go;
  if (threadIdx.x == 0) go = f.pend ? *f.pend : 1;
  __syncthreads();
  if (!go) return;
  flat_apply(f, f.h.kind == kOptAdam ? *f.iterations : 0, blockIdx.x * 256 + threadIdx.x, 256 * gridDim.x);
  __syncthreads();
  if (threadIdx.x == 0 && f.pend) *f.pend = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0 && f.count) atomicAdd(f.count, 1ull);
}

}  // namespace tde

using namespace tde;

// ranges: int[2*nr] = {lo0, n0, lo1, n1, ...}
TDE_API int tde_flat_apply(float* w, float* g, float* m, float* v, const long long* iterations, int* pend,
                           int kind, float lr, float mom, float b1, float b2, float eps, const int* ranges,
                           int nr, int grep, long long grep_stride, unsigned long long* count,
                           hipStream_t stream) {
  if (nr < 0 || nr > kFlatRanges || (kind != kOptSGD && !m) || (kind == kOptAdam && (!v || !iterations)))
    return -1;
  FlatApply f{w, g, m, v, iterations, pend, OptHyper{kind, lr, mom, b1, b2, eps}, nr, {0}, {0}, grep, grep_stride, count};
  for (int i = 0; i < nr; ++i) {
    f.lo[i] = ranges[2 * i];
    f.n[i] = ranges[2 * i + 1];
  }
  int maxn = 0;
  for (int i = 0; i < nr; ++i) maxn = f.n[i] > maxn ? f.n[i] : maxn;
  // pend: one workgroup (it reads and clears the flag); otherwise about one element per thread
  const int nb = pend ? 1 : (maxn + 255) / 256 < 1 ? 1 : ((maxn + 255) / 256 > 64 ? 64 : (maxn + 255) / 256);
  flat_apply_kernel<<<nb, 256, 0, stream>>>(f);
  TDE_LAUNCH_CHECK();
  return 0;
}

// Host helper: number of table entries for a segment list (for sizing).
TDE_API int tde_optim_table_size(const void* segs_host, int nseg) {
  const OptSeg* s = (const OptSeg*)segs_host;
  int n = 0;
  for (int i = 0; i < nseg; ++i) {
    if (s[i].sht_off >= 0)
      n += ((s[i].rows + kTileR - 1) / kTileR) * ((s[i].cols + 63) / 64);
    else
      n += (int)(((long long)s[i].rows * s[i].cols + kChunk - 1) / kChunk);
  }
  return n;
}

// Fills `table_host` (int4 per block) for a segment list.
TDE_API int tde_optim_build_table(const void* segs_host, int nseg, void* table_host) {
  const OptSeg* s = (const OptSeg*)segs_host;
  int4* t = (int4*)table_host;
  int n = 0;
  for (int i = 0; i < nseg; ++i) {
    if (s[i].sht_off >= 0) {
      for (int r = 0; r < (s[i].rows + kTileR - 1) / kTileR; ++r)
        for (int c = 0; c < (s[i].cols + 63) / 64; ++c) t[n++] = int4{i, 1, r, c};
    } else {
      int nb = (int)(((long long)s[i].rows * s[i].cols + kChunk - 1) / kChunk);
      for (int b = 0; b < nb; ++b) t[n++] = int4{i, 0, b, 0};
    }
  }
  return n;
}

TDE_API int tde_optim_apply(float* w, float* g, float* m, float* v, void* shadow,
                            const void* segs_dev, const void* table_dev, int nblocks,
                            const long long* iterations, int kind, float lr, float mom, float b1,
                            float b2, float eps, float grad_scale, int zero_grad,
                            const float* lr_ptr, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  if (((uintptr_t)w | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return -1;
  OptArgs a{w, g, m, v, (bf16*)shadow, (const OptSeg*)segs_dev, (const int4*)table_dev,
            iterations, kind, lr, mom, b1, b2, eps, grad_scale, zero_grad, lr_ptr};
  optim_apply_kernel<<<nblocks, 256, 0, stream>>>(a);
  TDE_LAUNCH_CHECK();
  return 0;
}

TDE_API int tde_shadow_refresh(const float* w, void* shadow, const void* segs_dev,
                               const void* table_dev, int nblocks, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  shadow_refresh_kernel<<<nblocks, 256, 0, stream>>>(w, (bf16*)shadow, (const OptSeg*)segs_dev,
                                                     (const int4*)table_dev);
  TDE_LAUNCH_CHECK();
  return 0;
}
