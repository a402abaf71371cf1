// Probe: do device-scope f64 / f32 atomics from many workgroups (spread over all XCDs) onto a few
// addresses ever lose updates?  Every workgroup adds 1.0 to each of `naddr` counters `reps` times.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void add_f64(double* acc, int naddr, int reps) {
  for (int r = 0; r < reps; ++r)
    if ((int)threadIdx.x < naddr) atomicAdd(acc + threadIdx.x, 1.0);
}
__global__ void add_f32(float* acc, int naddr, int reps) {
  for (int r = 0; r < reps; ++r)
    if ((int)threadIdx.x < naddr) atomicAdd(acc + threadIdx.x, 1.0f);
}
__global__ void zero(double* a, float* b, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) { a[i] = 0.0; b[i] = 0.f; }
}

int main() {
  const int naddr = 48, blocks = 512, reps = 4, iters = 200;
  double* d; float* f;
  hipMalloc(&d, naddr * sizeof(double));
  hipMalloc(&f, naddr * sizeof(float));
  std::vector<double> hd(naddr);
  std::vector<float> hf(naddr);
  int bad64 = 0, bad32 = 0;
  double worst64 = 0;
  for (int it = 0; it < iters; ++it) {
    zero<<<1, 64>>>(d, f, naddr);
    add_f64<<<blocks, 64>>>(d, naddr, reps);
    add_f32<<<blocks, 64>>>(f, naddr, reps);
    hipMemcpy(hd.data(), d, naddr * sizeof(double), hipMemcpyDeviceToHost);
    hipMemcpy(hf.data(), f, naddr * sizeof(float), hipMemcpyDeviceToHost);
    for (int i = 0; i < naddr; ++i) {
      if (hd[i] != blocks * reps) { ++bad64; worst64 = std::max(worst64, blocks * reps - hd[i]); }
      if (hf[i] != blocks * reps) ++bad32;
    }
  }
  printf("{\"probe\": \"atomics\", \"iters\": %d, \"bad_f64\": %d, \"worst_f64_missing\": %g, \"bad_f32\": %d}\n",
         iters, bad64, worst64, bad32);
  return 0;
}
