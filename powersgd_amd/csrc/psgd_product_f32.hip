// Instantiations of the product kernels for float gradients (see psgd_stream.cuh).
#include "psgd_stream.cuh"

namespace psgd {
hipError_t launch_product_f32(int R, bool even, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_product<float>(R, even, nres, a, ntiles, s);
}
hipError_t launch_odd_mfma_f32(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_odd_mfma<float>(R, nres, a, ntiles, s);
}
}  // namespace psgd
