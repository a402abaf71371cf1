// Device-side optimizer math shared by every kernel that applies an update:
// the multi-tensor optimizer (optim.hip), the fused convnet step (convnet.hip,
// head.hip: updates applied where the gradient is finished) and the xGMI
// all-reduce (xgmi_allreduce.hip: the update applied to the reduced slice).
// Keras forms (distributed_with_keras.py:42,
// mnist_keras_distributed.py:111, tf2_mnist_distributed.py:137):
//   SGD        w -= lr*g
//   momentum   v = mom*v - lr*g ; w += v          (nesterov: w += mom*v - lr*g)
//   Adam       m,v moments ; w -= lr_t*m/(sqrt(v)+eps), lr_t = lr*sqrt(1-b2^t)/(1-b1^t)
#pragma once
#include "tde_common.h"

namespace tde {

enum { kOptSGD = 0, kOptMomentum = 1, kOptNesterov = 2, kOptAdam = 3 };

struct OptHyper {
  int kind;
  float lr, mom, b1, b2, eps;
};

// Adam's bias-corrected step size at step t (t = optimizer.iterations after the
// step's increment; t < 1 is treated as 1); lr for the other kinds.
__device__ __forceinline__ float opt_lr_t(const OptHyper& h, long long t) {
  if (h.kind != kOptAdam) return h.lr;
  const float tf = (float)(t > 0 ? t : 1);
  return h.lr * sqrtf(1.f - __powf(h.b2, tf)) / (1.f - __powf(h.b1, tf));
}

// One element: returns the new weight, updates the slots in place.
__device__ __forceinline__ float opt_step(const OptHyper& h, float lr_t, float w, float g, float& m, float& v) {
  if (h.kind == kOptSGD) return w - h.lr * g;
  if (h.kind == kOptMomentum || h.kind == kOptNesterov) {
    const float nv = h.mom * m - h.lr * g;
    m = nv;
    return h.kind == kOptNesterov ? w + h.mom * nv - h.lr * g : w + nv;
  }
  m = h.b1 * m + (1.f - h.b1) * g;
  v = h.b2 * v + (1.f - h.b2) * g * g;
  return w - lr_t * m / (sqrtf(v) + h.eps);
}

// Update of up to kFlatRanges element ranges of the flat parameter buffers
// (w, g, and the slots the kind uses), gradient zeroed after use.  `pend`
// (nullable) marks a deferred update: applied only while *pend != 0, then cleared.
constexpr int kFlatRanges = 4;
struct FlatApply {
  float* w; float* g; float* m; float* v;
  const long long* iterations;
  int* pend;
  OptHyper h;
  int nr;
  int lo[kFlatRanges], n[kFlatRanges];
  // the gradient is the sum of grep (<= 1: one) replicas g[e + r * grep_stride], all zeroed after use
  int grep;
  long long grep_stride;
  // diagnostics (nullable): += 1 each time the update is applied (deferred-update invariants, program.py)
  unsigned long long* count;
};
constexpr int kMaxGrep = 8;   // gradient replicas: every load issued before the first add (one round trip)
__device__ __forceinline__ float flat_grad(const FlatApply& f, int e) {
  float v[kMaxGrep];
#pragma unroll
  for (int r = 0; r < kMaxGrep; ++r) v[r] = (r == 0 || r < f.grep) ? f.g[e + r * f.grep_stride] : 0.f;
  float g = v[0];
#pragma unroll
  for (int r = 1; r < kMaxGrep; ++r) g += v[r];
  return g;
}
__device__ __forceinline__ void flat_grad_zero(const FlatApply& f, int e) {
#pragma unroll
  for (int r = 0; r < kMaxGrep; ++r)
    if (r == 0 || r < f.grep) f.g[e + r * f.grep_stride] = 0.f;
}

// Threads [tid, tid + nt*k) of the caller apply the ranges with step t.
__device__ __forceinline__ void flat_apply(const FlatApply& f, long long t, int tid, int nt) {
  const float lr_t = opt_lr_t(f.h, t);
  for (int r = 0; r < f.nr; ++r) {
    for (int i = tid; i < f.n[r]; i += nt) {
      const int e = f.lo[r] + i;
      float m = f.h.kind != kOptSGD ? f.m[e] : 0.f;
      float v = f.h.kind == kOptAdam ? f.v[e] : 0.f;
      f.w[e] = opt_step(f.h, lr_t, f.w[e], flat_grad(f, e), m, v);
      flat_grad_zero(f, e);
      if (f.h.kind != kOptSGD) f.m[e] = m;
      if (f.h.kind == kOptAdam) f.v[e] = v;
    }
  }
}

}  // namespace tde
