// Instantiations of the fused residual/output kernels for float gradients (see psgd_stream.cuh).
#include "psgd_stream.cuh"

namespace psgd {
hipError_t launch_apply_f32(int R, int nterms, bool shared, const ApplyArgs& a, int ntiles, hipStream_t s) {
    return dispatch_apply<float>(R, nterms, shared, a, ntiles, s);
}
}  // namespace psgd
