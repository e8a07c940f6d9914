// TEST INFRASTRUCTURE ONLY — a stand-in collective library for psgd_comm.cpp (never shipped,
// never loaded by the product unless a test sets PSGD_RCCL_LIB_FORCE to this file).
//
// It lets ONE process on ONE GPU run psgd_aggregate_comm as world size W: the communicator
// reports the world it was created with, and ncclAllReduce(SUM) writes W x the send buffer into
// the receive buffer on the given stream — exactly the SUM over W ranks that all hold the same
// buffer. Reference semantics being exercised: powersgd.py:204-219 (SUM of the out-factor, then
// x 1/W in the output) and utils.py:43-47 (flat tail divided by W, then SUM).
//
// Negative controls (read at every call, so one process can run several modes):
//   PSGD_STUB_MODE=sum    (default) recv = W * send
//   PSGD_STUB_MODE=twice  recv = W * W * send      (a collective applied twice)
//   PSGD_STUB_MODE=skip   the call with index PSGD_STUB_SKIP_AT (0-based, process-wide counter)
//                         leaves recv untouched (a collective that never happened)
// psgd_stub_calls() returns the number of ncclAllReduce calls so far (tests count them).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

struct ncclComm {
    int world = 1, rank = 0;
};

namespace {

std::atomic<long long> g_calls{0};

__global__ void __launch_bounds__(256) k_stub_scale(const float* __restrict__ src, float* __restrict__ dst,
                                                     size_t n, float f) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i] * f;
}

}  // namespace

extern "C" {

long long psgd_stub_calls(void) { return g_calls.load(); }

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof(*id));
    std::memcpy(id->internal, "psgd-rccl-stub", 14);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    auto* c = new ncclComm();
    c->world = nranks;
    c->rank = rank;
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "stub: success" : "stub: error"; }

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
    if (!comm || dt != ncclFloat32 || op != ncclSum) return ncclInvalidArgument;
    const long long idx = g_calls.fetch_add(1);
    const char* mode = std::getenv("PSGD_STUB_MODE");
    float f = float(comm->world);
    if (mode && std::strcmp(mode, "twice") == 0) f *= float(comm->world);
    if (mode && std::strcmp(mode, "skip") == 0) {
        const char* at = std::getenv("PSGD_STUB_SKIP_AT");
        if (at && std::atoll(at) == idx) {
            if (send != recv && count)
                return hipMemcpyAsync(recv, send, count * sizeof(float), hipMemcpyDeviceToDevice, stream) == hipSuccess
                           ? ncclSuccess : ncclUnhandledCudaError;
            return ncclSuccess;
        }
    }
    if (count == 0) return ncclSuccess;
    const unsigned blocks = unsigned(std::min<size_t>((count + 255) / 256, 4096));
    hipLaunchKernelGGL(k_stub_scale, dim3(blocks), dim3(256), 0, stream, static_cast<const float*>(send),
                       static_cast<float*>(recv), count, f);
    return hipGetLastError() == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

}  // extern "C"
