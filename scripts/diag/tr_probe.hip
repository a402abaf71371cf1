// Probe of ds_read_b64_tr_b16 semantics: lane j supplies the address of 4 consecutive 16-bit
// elements 4j..4j+3 of an LDS array holding lds[e] = e; each lane prints the 4 elements it receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short v4i16 __attribute__((ext_vector_type(4)));
__global__ void probe(short* out) {
  __shared__ short lds[512];
  for (int e = threadIdx.x; e < 512; e += 64) lds[e] = (short)e;
  __syncthreads();
  const int j = threadIdx.x;
  v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(lds + 4 * j));
  for (int e = 0; e < 4; ++e) out[j * 4 + e] = v[e];
}
int main() {
  short* d;
  hipMalloc(&d, 256 * sizeof(short));
  probe<<<1, 64>>>(d);
  short h[256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int j = 0; j < 32; ++j) printf("lane %2d: %3d %3d %3d %3d\n", j, h[4 * j], h[4 * j + 1], h[4 * j + 2], h[4 * j + 3]);
  return 0;
}
