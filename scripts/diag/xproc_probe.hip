// Cross-process co-scheduling probe: do the grids of two processes that share ONE
// GPU run at the same time?  Each process launches `blocks` workgroups; workgroup c raises its flag c in a
// shared IPC buffer and then waits (bounded, s_memrealtime) for the OTHER process's flag c — the wait
// pattern of the xGMI all-reduce's cross-process phases.  Every workgroup records (start, arrival, end)
// on the device clock, which both processes share, so the two grids' lifetimes can be compared directly.
//
//   xproc_probe A <dir> <blocks> <extra_streams> <timeout_ms> <epochs>    (allocates, writes the handle)
//   xproc_probe B <dir> <blocks> <extra_streams> <timeout_ms> <epochs>    (maps the handle)
// extra_streams: streams created (and given one tiny kernel each) before the probe, like the per-group /
// side / comm streams of the framework's eager path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                \
    }                                                                         \
  } while (0)

constexpr int kMaxBlocks = 1024;

__global__ void noop_kernel(int* p) {
  if (threadIdx.x == 0 && p) p[blockIdx.x] = 1;
}

// flags: [2][kMaxBlocks] u32 (side 0 = A, 1 = B); rec: [blocks][4] u64 (start, arrived, end, ok)
__global__ void __launch_bounds__(256) probe_kernel(uint32_t* flags, int side, uint32_t epoch, long long timeout,
                                                    unsigned long long* rec) {
  const int c = blockIdx.x;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(flags + side * kMaxBlocks + c, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* other = flags + (1 - side) * kMaxBlocks + c;
    bool ok = true;
    while (__hip_atomic_load(other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout) {
        ok = false;
        break;
      }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    rec[c * 4 + 0] = t0;
    rec[c * 4 + 1] = t1;
    rec[c * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    rec[c * 4 + 3] = ok ? 1 : 0;
  }
  __syncthreads();
}

static void wait_file(const char* path) {
  for (int i = 0; i < 30000; ++i) {
    if (access(path, F_OK) == 0) return;
    usleep(1000);
  }
  fprintf(stderr, "timed out waiting for %s\n", path);
  exit(3);
}

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s A|B dir blocks extra_streams timeout_ms epochs\n", argv[0]);
    return 1;
  }
  const bool isA = argv[1][0] == 'A';
  const char* dir = argv[2];
  const int blocks = atoi(argv[3]), extra = atoi(argv[4]), epochs = atoi(argv[6]);
  const long long timeout = (long long)atoi(argv[5]) * 100000LL;   // 100 MHz ticks
  if (blocks < 1 || blocks > kMaxBlocks) return 1;
  char hpath[512], rA[512], rB[512];
  snprintf(hpath, sizeof(hpath), "%s/handle.bin", dir);
  snprintf(rA, sizeof(rA), "%s/ready_A", dir);
  snprintf(rB, sizeof(rB), "%s/ready_B", dir);
  CK(hipSetDevice(0));
  uint32_t* flags = nullptr;
  hipIpcMemHandle_t h;
  if (isA) {
    CK(hipExtMallocWithFlags((void**)&flags, 2 * kMaxBlocks * 4, hipDeviceMallocUncached));
    CK(hipMemset(flags, 0, 2 * kMaxBlocks * 4));
    CK(hipDeviceSynchronize());
    CK(hipIpcGetMemHandle(&h, flags));
    FILE* f = fopen(hpath, "wb");
    fwrite(&h, sizeof(h), 1, f);
    fclose(f);
  } else {
    wait_file(hpath);
    usleep(20000);
    FILE* f = fopen(hpath, "rb");
    if (fread(&h, sizeof(h), 1, f) != 1) return 4;
    fclose(f);
    CK(hipIpcOpenMemHandle((void**)&flags, h, hipIpcMemLazyEnablePeerAccess));
  }
  // extra streams with a little work each (the framework's eager path uses several per process)
  hipStream_t* ss = (hipStream_t*)calloc(extra + 1, sizeof(hipStream_t));
  int* scratch = nullptr;
  CK(hipMalloc((void**)&scratch, 4096));
  for (int i = 0; i < extra; ++i) {
    CK(hipStreamCreate(&ss[i]));
    noop_kernel<<<4, 64, 0, ss[i]>>>(scratch);
  }
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreate(&s));
  unsigned long long* rec = nullptr;
  CK(hipHostMalloc((void**)&rec, (size_t)blocks * 4 * 8, hipHostMallocMapped | hipHostMallocCoherent));
  // rendezvous: both processes launch within a few ms of each other
  FILE* f = fopen(isA ? rA : rB, "w");
  fclose(f);
  wait_file(isA ? rB : rA);
  int bad_total = 0;
  for (int ep = 1; ep <= epochs; ++ep) {
    memset(rec, 0, (size_t)blocks * 4 * 8);
    probe_kernel<<<blocks, 256, 0, s>>>(flags, isA ? 0 : 1, (uint32_t)ep, timeout, rec);
    CK(hipStreamSynchronize(s));
    unsigned long long smin = ~0ull, smax = 0, amax = 0, emax = 0;
    int bad = 0;
    for (int c = 0; c < blocks; ++c) {
      smin = rec[c * 4] < smin ? rec[c * 4] : smin;
      smax = rec[c * 4] > smax ? rec[c * 4] : smax;
      amax = rec[c * 4 + 1] > amax ? rec[c * 4 + 1] : amax;
      emax = rec[c * 4 + 2] > emax ? rec[c * 4 + 2] : emax;
      bad += rec[c * 4 + 3] ? 0 : 1;
    }
    bad_total += bad;
    printf("[probe %c] blocks=%d extra_streams=%d epoch=%d start=[%.1f, %.1f] us arrived<=%.1f us end<=%.1f us "
           "timed_out_blocks=%d\n",
           isA ? 'A' : 'B', blocks, extra, ep, smin / 100.0, smax / 100.0, amax / 100.0, emax / 100.0, bad);
    fflush(stdout);
  }
  if (!isA) CK(hipIpcCloseMemHandle(flags));
  return bad_total ? 5 : 0;
}
