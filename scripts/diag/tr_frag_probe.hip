// Probe: write a [32][128] bf16 image with the kernel's swizzled 16-byte stores (value = 1000*k + n as
// short) and read fragments back with the kernel's tr_frag; print what lanes 0..3,16,17 receive.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short s8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
__device__ __forceinline__ int swz(int row, int ch) { return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))); }
__device__ __forceinline__ s8 tr_frag(const short* img, int mb, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int ch = (mb >> 3) + (pp >> 1);
  const char* base = reinterpret_cast<const char*>(img);
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + swz(8 * g + q, ch) + 8 * (pp & 1)));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + swz(8 * g + 4 + q, ch) + 8 * (pp & 1)));
  s8 r;
  for (int j = 0; j < 4; ++j) { r[j] = lo[j]; r[4 + j] = hi[j]; }
  return r;
}
__global__ void probe(short* out, int mb) {
  __shared__ __attribute__((aligned(16))) short smem[2 * 32 * 128];
  short* img = smem + 32 * 128;  // second buffer, like buf=1
  const int tid = threadIdx.x;
  for (int s = tid; s < 512; s += 256) {
    const int row = s >> 4, ch = s & 15;
    s8 v;
    for (int e = 0; e < 8; ++e) v[e] = (short)(100 * row + ch * 8 + e);
    *reinterpret_cast<s8*>(reinterpret_cast<char*>(img) + swz(row, ch)) = v;
  }
  __syncthreads();
  s8 f = tr_frag(img, mb, tid & 63);
  if (tid < 64)
    for (int e = 0; e < 8; ++e) out[tid * 8 + e] = f[e];
}
int main() {
  short* d;
  (void)hipMalloc(&d, 64 * 8 * sizeof(short));
  for (int mb : {0, 16}) {
    probe<<<1, 256>>>(d, mb);
    short h[512];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l : {0, 1, 2, 3, 4, 15, 16, 17, 33})
      printf("mb %2d lane %2d: %5d %5d %5d %5d %5d %5d %5d %5d\n", mb, l, h[8 * l], h[8 * l + 1], h[8 * l + 2],
             h[8 * l + 3], h[8 * l + 4], h[8 * l + 5], h[8 * l + 6], h[8 * l + 7]);
  }
  return 0;
}
