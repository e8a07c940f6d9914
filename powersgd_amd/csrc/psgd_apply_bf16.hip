// Instantiations of the fused residual/output kernels for bf16_t gradients (see psgd_stream.cuh).
#include "psgd_stream.cuh"

namespace psgd {
hipError_t launch_apply_bf16(int R, int nterms, bool shared, const ApplyArgs& a, int ntiles, hipStream_t s) {
    return dispatch_apply<bf16_t>(R, nterms, shared, a, ntiles, s);
}
}  // namespace psgd
