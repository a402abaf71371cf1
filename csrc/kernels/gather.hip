// Device-resident input pipeline: row gather from an HBM-resident dataset cache.
//
// The reference's input pipelines (distributed_with_keras.py:30 `map(scale).cache().shuffle(10000)`,
// mnist_keras_distributed.py:142-145 `from_tensor_slices(...).shuffle(1000).repeat().batch(bs)`) cache the
// whole (mapped) training set in memory.  On an MI355X that cache belongs in HBM (60,000 MNIST images are
// 188 MB of 288 GB): the host keeps only the shuffle / repeat / shard / batch algebra on index streams
// (csrc/data/pipeline.cpp) and ships S x B int32 row indices per execution; this kernel gathers the rows
// into the training program's input ring.  dst[i] = src[idx[i]] for rows of `row_bytes` bytes.
#include "tde_common.h"

namespace tde {

template <typename V>
__global__ __launch_bounds__(256) void gather_rows_kernel(const V* __restrict__ src, int row_vecs, long long nrows,
                                                          const int* __restrict__ idx, long long n,
                                                          V* __restrict__ dst, int* __restrict__ bad) {
  const long long total = n * row_vecs;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long r = i / row_vecs;
    const int v = (int)(i - r * row_vecs);
    const int s = idx[r];
    if ((unsigned long long)s >= (unsigned long long)nrows) {  // never read out of the cache
      if (v == 0) atomicOr(bad, 1);
      continue;
    }
    dst[i] = src[(long long)s * row_vecs + v];
  }
}

}  // namespace tde

using namespace tde;

// dst[i, :] = src[idx[i], :] for i < n (row_bytes each; idx int32).  `bad` (device int, may be null) gets
// bit 0 set for an index outside [0, nrows).  16-byte vectors when rows and pointers allow, else 4-byte.
TDE_API int tde_gather_rows_dev(const void* src, long long row_bytes, long long nrows, const int* idx, long long n,
                                void* dst, int* bad, hipStream_t stream) {
  if (n <= 0) return 0;
  if (row_bytes <= 0 || row_bytes % 4 || !bad) return -1;
  const bool v16 = row_bytes % 16 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0;
  const long long vecs = row_bytes / (v16 ? 16 : 4);
  if (vecs >= (1LL << 30)) return -2;
  long long blocks = (n * vecs + 255) / 256;
  blocks = blocks > 4096 ? 4096 : blocks;
  if (v16)
    gather_rows_kernel<float4><<<(int)blocks, 256, 0, stream>>>((const float4*)src, (int)vecs, nrows, idx, n,
                                                                (float4*)dst, bad);
  else
    gather_rows_kernel<int><<<(int)blocks, 256, 0, stream>>>((const int*)src, (int)vecs, nrows, idx, n, (int*)dst,
                                                             bad);
  TDE_LAUNCH_CHECK();
  return 0;
}
