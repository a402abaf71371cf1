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

// The per-execution staging of a device-resident batch group (x and y of every step) into the program's input
// ring as ONE launch instead of one copy launch per tensor: up to kCopyPairs (src, dst, bytes) pairs; each pair
// moves 16-byte vectors when its size and pointers allow, 4-byte words otherwise.
namespace tde {
constexpr int kCopyPairs = 4;
struct CopyPairs {
  const char* src[kCopyPairs];
  char* dst[kCopyPairs];
  long long bytes[kCopyPairs];
  long long beg[kCopyPairs + 1];   // prefix offsets in 16-byte units over the pairs (each pair rounded up)
  int v16[kCopyPairs];
  int n;
};
__global__ __launch_bounds__(256) void copy_pairs_kernel(CopyPairs c) {
  const long long total = c.beg[c.n];
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    int j = 0;
    while (j + 1 < c.n && i >= c.beg[j + 1]) ++j;
    const long long o = (i - c.beg[j]) * 16;   // byte offset of this thread's 16-byte unit in pair j
    if (c.v16[j]) {
      *reinterpret_cast<float4*>(c.dst[j] + o) = *reinterpret_cast<const float4*>(c.src[j] + o);
    } else {
      for (long long b = o; b < o + 16 && b < c.bytes[j]; b += 4)
        *reinterpret_cast<int*>(c.dst[j] + b) = *reinterpret_cast<const int*>(c.src[j] + b);
    }
  }
}
}  // namespace tde

TDE_API int tde_copy_pairs(int n, const void* const* src, void* const* dst, const long long* bytes, hipStream_t stream) {
  if (n < 1 || n > kCopyPairs) return -1;
  CopyPairs c{};
  c.n = n;
  long long units = 0;
  for (int j = 0; j < n; ++j) {
    if (bytes[j] < 0 || bytes[j] % 4 || ((uintptr_t)src[j] & 3) || ((uintptr_t)dst[j] & 3)) return -2;
    c.src[j] = (const char*)src[j];
    c.dst[j] = (char*)dst[j];
    c.bytes[j] = bytes[j];
    c.v16[j] = bytes[j] % 16 == 0 && ((uintptr_t)src[j] & 15) == 0 && ((uintptr_t)dst[j] & 15) == 0;
    c.beg[j] = units;
    units += (bytes[j] + 15) / 16;
  }
  c.beg[n] = units;
  if (units == 0) return 0;
  long long blocks = (units + 255) / 256;
  blocks = blocks > 2048 ? 2048 : blocks;
  copy_pairs_kernel<<<(int)blocks, 256, 0, stream>>>(c);
  TDE_LAUNCH_CHECK();
  return 0;
}
