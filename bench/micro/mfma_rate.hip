// MFMA issue-rate probe: one 256-thread workgroup per CU, each wave runs N steps of K independent
// v_mfma_f32_16x16x32_bf16 on register operands (no memory in the loop), optionally with one ds_read_b128
// per MFMA.  Prints cycles per MFMA measured with s_memtime.  hipcc --offload-arch=gfx950 -O3 mfma_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// 32x32x16 variant: K independent 16-float accumulators
template <int K>
__global__ __launch_bounds__(256) void probe32(float* out, long long* cyc, int steps) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.001f * (lane + j)); b[j] = (__bf16)(0.002f * (lane - j)); }
  f32x16 acc[K];
  for (int k = 0; k < K; ++k) for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[k], 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int k = 0; k < K; ++k) r += acc[k][0] + acc[k][15];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K, bool LDS>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc, int steps) {
  __shared__ __attribute__((aligned(16))) bf16x8 sm[1024];
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.001f * (lane + j)); b[j] = (__bf16)(0.002f * (lane - j)); }
  sm[threadIdx.x] = a;
  sm[threadIdx.x + 256] = b;
  __syncthreads();
  f32x4 acc[K];
  for (int k = 0; k < K; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 f[2][K];
  for (int k = 0; k < K; ++k) { f[0][k] = a; f[1][k] = b; }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < steps; s += 2) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[0][k], b, acc[k], 0, 0, 0);
      if (LDS) f[1][k] = sm[(threadIdx.x + 64 * k + s) & 1023];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[1][k], b, acc[k], 0, 0, 0);
      if (LDS) f[0][k] = sm[(threadIdx.x + 64 * k + s + 1) & 1023];
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float r = 0.f;
  for (int k = 0; k < K; ++k) r += acc[k][0] + acc[k][3];
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K, bool LDS>
void run(float* out, long long* cyc, int grid) {
  const int steps = 200;
  hipLaunchKernelGGL((probe<K, LDS>), dim3(grid), dim3(256), 0, 0, out, cyc, steps);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<K, LDS>), dim3(grid), dim3(256), 0, 0, out, cyc, steps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c[1024];
  hipMemcpy(c, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0; for (int i = 0; i < grid; ++i) mean += c[i]; mean /= grid;
  const double n = (double)steps * K;
  printf("K=%2d lds=%d grid=%d: %.1f memtime-cycles/MFMA, wall %.1f us, %.1f ns/MFMA -> %.0f TF/s\n", K, (int)LDS,
         grid, mean / n, ms * 1e3, ms * 1e6 / n, 16384.0 * n * grid * 4 / (ms * 1e-3) / 1e12);
}

template <int K>
void run32(float* out, long long* cyc, int grid) {
  const int steps = 200;
  hipLaunchKernelGGL((probe32<K>), dim3(grid), dim3(256), 0, 0, out, cyc, steps);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe32<K>), dim3(grid), dim3(256), 0, 0, out, cyc, steps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  long long c[1024];
  hipMemcpy(c, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double mean = 0; for (int i = 0; i < grid; ++i) mean += c[i]; mean /= grid;
  const double n = (double)steps * K;
  printf("32x32x16 K=%2d grid=%d: %.1f memtime-cycles/MFMA, wall %.1f us, %.1f ns/MFMA -> %.0f TF/s\n", K, grid,
         mean / n, ms * 1e3, ms * 1e6 / n, 32768.0 * n * grid * 4 / (ms * 1e-3) / 1e12);
}

int main() {
  float* out; long long* cyc;
  hipMalloc(&out, 1024 * 256 * 4); hipMalloc(&cyc, 1024 * 8);
  run<14, false>(out, cyc, 256);
  run<14, true>(out, cyc, 256);
  run<8, false>(out, cyc, 256);
  run<4, false>(out, cyc, 256);
  run<14, false>(out, cyc, 1024);
  run<14, false>(out, cyc, 512);
  run32<4>(out, cyc, 256);
  run32<7>(out, cyc, 256);
  run32<4>(out, cyc, 512);
  run32<4>(out, cyc, 1024);
  return 0;
}
