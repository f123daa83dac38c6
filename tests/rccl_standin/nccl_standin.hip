// nccl_standin.hip -- test-only stand-in for librccl.so.1 (tests/test_dp_standin_gpu.py).
//
// libmaddpg_hip.so dlopens RCCL at run time (mdp_api.cpp rccl()); with
// MDP_RCCL_LIB=<this library> it loads this one instead.  It gives the native
// data-parallel path a world > 1 on ONE GPU: a communicator of `nranks` ranks
// whose every peer holds exactly this rank's data, so the sum all-reduce is
// an in-place multiply by nranks (exact in fp32 for a power of two) -- the
// collective the library would run across nranks identical replicas.  Every
// call is logged (element count, buffer, op, dtype, communicator size) for the
// test to check the exchange pattern of the reference's update order
// (maddpg.py:188-194: 2N all-reduces per round in strict mode, one per round
// in throughput mode).  Not a product path: nothing under maddpg_amd/ names it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <vector>

struct ncclComm {
  int nranks, rank;
};

namespace {
struct Call {
  int64_t count;
  uint64_t recv, send;
  int32_t op, dtype, nranks, captured;
};
std::mutex mu;
std::vector<Call> calls;

__global__ void k_scale(const float* __restrict__ s, float* __restrict__ r, int64_t n, float f) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    r[i] = s[i] * f;
}
}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id, 0, sizeof(*id));
  std::memcpy(id->internal, "mdp-standin", 11);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (std::memcmp(id.internal, "mdp-standin", 11) != 0) return ncclInvalidArgument;
  if (nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  *comm = new ncclComm{nranks, rank};
  return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype,
                           ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
  if (!comm || datatype != ncclFloat32 || op != ncclSum) return ncclInvalidArgument;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream, &cs);
  {
    std::lock_guard<std::mutex> g(mu);
    calls.push_back(Call{(int64_t)count, (uint64_t)(uintptr_t)recvbuff, (uint64_t)(uintptr_t)sendbuff, (int32_t)op,
                         (int32_t)datatype, comm->nranks, cs == hipStreamCaptureStatusActive ? 1 : 0});
  }
  if (count == 0) return ncclSuccess;
  const int64_t n = (int64_t)count;
  const int grid = (int)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
  hipLaunchKernelGGL(k_scale, dim3(grid), dim3(256), 0, stream, (const float*)sendbuff, (float*)recvbuff, n,
                     (float)comm->nranks);
  return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  delete comm;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  if (!comm) return ncclInvalidArgument;
  *count = comm->nranks;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "stand-in error"; }

// the call log: up to `max` entries as [count, recv, send, op, dtype, nranks,
// captured] int64 rows; returns the number of calls logged; reset != 0 clears it
int64_t mdp_standin_calls(int64_t* out, int64_t max, int32_t reset) {
  std::lock_guard<std::mutex> g(mu);
  const int64_t n = (int64_t)calls.size();
  for (int64_t i = 0; i < n && i < max; ++i) {
    const Call& c = calls[(size_t)i];
    int64_t* o = out + 7 * i;
    o[0] = c.count;
    o[1] = (int64_t)c.recv;
    o[2] = (int64_t)c.send;
    o[3] = c.op;
    o[4] = c.dtype;
    o[5] = c.nranks;
    o[6] = c.captured;
  }
  if (reset) calls.clear();
  return n;
}

}  // extern "C"
