// Native RCCL communicator (libfls_comm.so): the data-parallel weight all-gather issued straight
// from C on the caller's HIP stream, one rcclComm per gather group.
//
// torch.distributed's "nccl" backend (RCCL on ROCm) stays the default for every collective
// (parallel/comm.py); this wrapper is the --dp_gather_comm native path of the weight fan-out, where
// each call is a fixed-size byte all-gather into an HBM slot on the copy stream, ordered by the
// stream itself (no torch Work object, no stream-sync bookkeeping).  The ranks bootstrap with one
// ncclUniqueId that rank 0 creates and the default process group broadcasts
// (parallel/native_comm.py).  Reference counterpart: the threads + shared dict of
// /root/reference/utils.py:24-75 (DeviceManager's host cache), which has no collective at all.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>

extern "C" {

int fls_rccl_version(void) {
  int v = 0;
  return ncclGetVersion(&v) == ncclSuccess ? v : -1;
}

int fls_rccl_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

// a fresh unique id into out (fls_rccl_id_bytes() bytes); 0 on success
int fls_rccl_unique_id(void* out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  std::memcpy(out, &id, sizeof id);
  return 0;
}

// a communicator of `nranks` ranks on HIP device `device` (collective: every rank calls it with the
// same id); nullptr on failure
void* fls_rccl_init(int nranks, int rank, const void* id, int device) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  ncclComm_t comm = nullptr;
  if (ncclCommInitRank(&comm, nranks, uid, rank) != ncclSuccess) return nullptr;
  return comm;
}

// recv[r * bytes .. (r + 1) * bytes) = rank r's send buffer, for every rank r; enqueued on `stream`
int fls_rccl_all_gather(void* comm, const void* send, void* recv, uint64_t bytes, void* stream) {
  if (!comm) return -2;
  return ncclAllGather(send, recv, (size_t)bytes, ncclUint8, (ncclComm_t)comm, (hipStream_t)stream) == ncclSuccess
             ? 0
             : -1;
}

// in-place fp32 all-reduce: op 0 sum, 1 max, 2 min
int fls_rccl_all_reduce_f32(void* comm, float* buf, uint64_t n, int op, void* stream) {
  if (!comm) return -2;
  const ncclRedOp_t o = op == 1 ? ncclMax : op == 2 ? ncclMin : ncclSum;
  return ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, o, (ncclComm_t)comm, (hipStream_t)stream) == ncclSuccess
             ? 0
             : -1;
}

int fls_rccl_destroy(void* comm) {
  if (!comm) return 0;
  return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? 0 : -1;
}

}  // extern "C"
