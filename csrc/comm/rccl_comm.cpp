// RCCL (NCCL API over xGMI on MI355X) communicator wrapper with a C ABI.
//
// Data plane for MirroredStrategy / MultiWorkerMirroredStrategy gradient
// all-reduce, initial-variable broadcast and metric/BN-stat reductions
// (SURVEY.md §2.6 C1-C5, §5.8).  Every collective is enqueued on the caller's
// HIP stream so it is ordered with the producing/consuming kernels by stream
// order alone and can be captured into a hipGraph together with the training
// step (RCCL supports stream capture).
//
//  * multi-process: one rank per GPU, ncclUniqueId distributed by the C++ TCP
//    store (csrc/comm/tcp_store.cpp) or torch's store; ncclCommInitRank.
//  * in-process multi-GPU (MirroredStrategy(devices=[...])): ncclCommInitAll and
//    grouped per-device launches (ncclGroupStart/End).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#define TDE_API extern "C" __attribute__((visibility("default")))

static ncclDataType_t to_dtype(int d) {
  switch (d) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
    case 6: return ncclFloat64;
    default: return ncclFloat32;
  }
}

static ncclRedOp_t to_op(int o) {
  switch (o) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
    default: return ncclSum;
  }
}

TDE_API int tde_nccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

TDE_API const char* tde_nccl_error_string(int r) { return ncclGetErrorString((ncclResult_t)r); }

TDE_API int tde_nccl_get_unique_id(char* out128) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return (int)r;
  memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

TDE_API int tde_nccl_unique_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

TDE_API int tde_nccl_comm_init_rank(void** comm, int nranks, const char* id128, int rank,
                                    int device) {
  if (hipSetDevice(device) != hipSuccess) return -100;
  ncclUniqueId id;
  memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  *comm = (void*)c;
  return (int)r;
}

// Several local GPUs of one process joining one multi-process clique
// (MWMS with N GPUs per worker): ranks rank0 .. rank0+ndev-1.
TDE_API int tde_nccl_comm_init_ranks_grouped(void** comms, int nranks, const char* id128,
                                             int rank0, const int* devices, int ndev) {
  ncclUniqueId id;
  memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return (int)r;
  for (int i = 0; i < ndev; ++i) {
    hipSetDevice(devices[i]);
    ncclComm_t c = nullptr;
    r = ncclCommInitRank(&c, nranks, id, rank0 + i);
    comms[i] = (void*)c;
    if (r != ncclSuccess) break;
  }
  ncclResult_t r2 = ncclGroupEnd();
  return r != ncclSuccess ? (int)r : (int)r2;
}

TDE_API int tde_nccl_comm_init_all(void** comms, int ndev, const int* devices) {
  return (int)ncclCommInitAll((ncclComm_t*)comms, ndev, devices);
}

TDE_API int tde_nccl_comm_destroy(void* comm) { return (int)ncclCommDestroy((ncclComm_t)comm); }
TDE_API int tde_nccl_comm_abort(void* comm) { return (int)ncclCommAbort((ncclComm_t)comm); }

TDE_API int tde_nccl_comm_async_error(void* comm) {
  ncclResult_t e = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError((ncclComm_t)comm, &e);
  return r != ncclSuccess ? (int)r : (int)e;
}

TDE_API int tde_nccl_group_start() { return (int)ncclGroupStart(); }
TDE_API int tde_nccl_group_end() { return (int)ncclGroupEnd(); }

TDE_API int tde_nccl_all_reduce(const void* send, void* recv, size_t count, int dtype, int op,
                                void* comm, hipStream_t stream) {
  return (int)ncclAllReduce(send, recv, count, to_dtype(dtype), to_op(op), (ncclComm_t)comm,
                            stream);
}

TDE_API int tde_nccl_broadcast(const void* send, void* recv, size_t count, int dtype, int root,
                               void* comm, hipStream_t stream) {
  return (int)ncclBroadcast(send, recv, count, to_dtype(dtype), root, (ncclComm_t)comm, stream);
}

TDE_API int tde_nccl_all_gather(const void* send, void* recv, size_t count, int dtype,
                                void* comm, hipStream_t stream) {
  return (int)ncclAllGather(send, recv, count, to_dtype(dtype), (ncclComm_t)comm, stream);
}

TDE_API int tde_nccl_reduce_scatter(const void* send, void* recv, size_t count, int dtype, int op,
                                    void* comm, hipStream_t stream) {
  return (int)ncclReduceScatter(send, recv, count, to_dtype(dtype), to_op(op), (ncclComm_t)comm,
                                stream);
}

TDE_API int tde_nccl_send(const void* buf, size_t count, int dtype, int peer, void* comm,
                          hipStream_t stream) {
  return (int)ncclSend(buf, count, to_dtype(dtype), peer, (ncclComm_t)comm, stream);
}

TDE_API int tde_nccl_recv(void* buf, size_t count, int dtype, int peer, void* comm,
                          hipStream_t stream) {
  return (int)ncclRecv(buf, count, to_dtype(dtype), peer, (ncclComm_t)comm, stream);
}
