// Multi-tensor optimizer apply over the flat parameter buffer: SGD (optionally
// momentum / Nesterov, Keras form) and Adam (Keras/TF form, epsilon added to
// sqrt(v_hat)), in ONE launch for all variables (SURVEY.md §2.5 A14/B17,
// reference: distributed_with_keras.py:42, mnist_keras_distributed.py:111,
// tf2_mnist_distributed.py:137).
//
// The same pass (a) zeroes the gradient buffer for the next step's atomic /
// split-K accumulation, (b) refreshes the bf16 compute copies ("shadows") of
// the weights in the layouts the MFMA kernels read — row-major and, through an
// LDS 64x64 transpose, column-major — and (c) advances the device-resident
// `iterations` counter (Keras optimizer.iterations / Estimator global_step),
// so a captured hipGraph replays whole training steps with no host work.
#include "tde_common.h"

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
  long long* iterations;
  unsigned* done;
  int kind;                 // 0 sgd, 1 momentum, 2 nesterov, 3 adam
  float lr, mom, b1, b2, eps, grad_scale;
  int zero_grad;
  const float* lr_ptr;      // optional device-resident lr (schedules)
};

constexpr int kChunk = 2048;

__device__ __forceinline__ float opt_update(const OptArgs& a, size_t i, float t_b1, float t_b2,
                                            float lr) {
  float g = a.g[i] * a.grad_scale;
  if (a.zero_grad) a.g[i] = 0.f;
  float w = a.w[i];
  if (a.kind == 0) {
    w -= lr * g;
  } else if (a.kind == 1 || a.kind == 2) {
    float v = a.mom * a.m[i] - lr * g;  // Keras: v = m*v - lr*g ; w += v
    a.m[i] = v;
    w = (a.kind == 2) ? w + a.mom * v - lr * g : w + v;
  } else {
    float m = a.b1 * a.m[i] + (1.f - a.b1) * g;
    float v = a.b2 * a.v[i] + (1.f - a.b2) * g * g;
    a.m[i] = m;
    a.v[i] = v;
    const float lr_t = lr * sqrtf(1.f - t_b2) / (1.f - t_b1);
    w -= lr_t * m / (sqrtf(v) + a.eps);
  }
  a.w[i] = w;
  return w;
}

__global__ __launch_bounds__(256) void optim_apply_kernel(OptArgs a) {
  __shared__ bf16 tile[64][66];
  const int4 ent = a.table[blockIdx.x];
  const OptSeg s = a.segs[ent.x];
  const long long it = __hip_atomic_load(a.iterations, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float t = (float)(it + 1);
  const float t_b1 = a.kind == 3 ? __powf(a.b1, t) : 0.f;
  const float t_b2 = a.kind == 3 ? __powf(a.b2, t) : 0.f;
  const float lr = a.lr_ptr ? *a.lr_ptr : a.lr;
  const int tid = threadIdx.x;

  if (ent.y == 0) {
    const long long n = (long long)s.rows * s.cols;
    const long long beg = (long long)ent.z * kChunk;
    const long long end = beg + kChunk < n ? beg + kChunk : n;
    for (long long e = beg + tid; e < end; e += 256) {
      const float w = opt_update(a, (size_t)(s.off + e), t_b1, t_b2, lr);
      if (s.sh_off >= 0) a.shadow[s.sh_off + e] = f2bf(w);
    }
  } else {
    const int r0 = ent.z * 64, c0 = ent.w * 64;
    for (int i = tid; i < 64 * 64; i += 256) {
      const int r = i >> 6, c = i & 63;
      const int gr = r0 + r, gc = c0 + c;
      if (gr < s.rows && gc < s.cols) {
        const long long e = (long long)gr * s.cols + gc;
        const float w = opt_update(a, (size_t)(s.off + e), t_b1, t_b2, lr);
        const bf16 h = f2bf(w);
        if (s.sh_off >= 0) a.shadow[s.sh_off + e] = h;
        tile[r][c] = h;
      }
    }
    __syncthreads();
    for (int i = tid; i < 64 * 64; i += 256) {
      const int c = i >> 6, r = i & 63;
      const int gr = r0 + r, gc = c0 + c;
      if (gr < s.rows && gc < s.cols) a.shadow[s.sht_off + (long long)gc * s.rows + gr] = tile[r][c];
    }
  }

  // Last block advances the iteration counter.
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    const unsigned ticket = atomicAdd(a.done, 1u);
    if (ticket == gridDim.x - 1) {
      atomicAdd((unsigned long long*)a.iterations, 1ull);
      __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Writes bf16 shadows from the current weights without updating (init/restore).
__global__ __launch_bounds__(256) void shadow_refresh_kernel(const float* w, bf16* shadow,
                                                             const OptSeg* segs,
                                                             const int4* table) {
  __shared__ bf16 tile[64][66];
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
    const int r0 = ent.z * 64, c0 = ent.w * 64;
    for (int i = tid; i < 64 * 64; i += 256) {
      const int r = i >> 6, c = i & 63, gr = r0 + r, gc = c0 + c;
      if (gr < s.rows && gc < s.cols) {
        const long long e = (long long)gr * s.cols + gc;
        const bf16 h = f2bf(w[s.off + e]);
        if (s.sh_off >= 0) shadow[s.sh_off + e] = h;
        tile[r][c] = h;
      }
    }
    __syncthreads();
    for (int i = tid; i < 64 * 64; i += 256) {
      const int c = i >> 6, r = i & 63, gr = r0 + r, gc = c0 + c;
      if (gr < s.rows && gc < s.cols) shadow[s.sht_off + (long long)gc * s.rows + gr] = tile[r][c];
    }
  }
}

}  // namespace tde

using namespace tde;

// Host helper: number of table entries for a segment list (for sizing).
TDE_API int tde_optim_table_size(const void* segs_host, int nseg) {
  const OptSeg* s = (const OptSeg*)segs_host;
  int n = 0;
  for (int i = 0; i < nseg; ++i) {
    if (s[i].sht_off >= 0)
      n += ((s[i].rows + 63) / 64) * ((s[i].cols + 63) / 64);
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
      for (int r = 0; r < (s[i].rows + 63) / 64; ++r)
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
                            long long* iterations, unsigned* done, int kind, float lr,
                            float mom, float b1, float b2, float eps, float grad_scale,
                            int zero_grad, const float* lr_ptr, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  OptArgs a{w, g, m, v, (bf16*)shadow, (const OptSeg*)segs_dev, (const int4*)table_dev,
            iterations, done, kind, lr, mom, b1, b2, eps, grad_scale, zero_grad, lr_ptr};
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
