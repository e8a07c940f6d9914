// Instantiations of the product kernels for bf16_t gradients (see psgd_stream.cuh).
#include "psgd_stream.cuh"

namespace psgd {
hipError_t launch_product_bf16(int R, bool even, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_product<bf16_t>(R, even, nres, a, ntiles, s);
}
hipError_t launch_odd_mfma_bf16(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_odd_mfma<bf16_t>(R, nres, a, ntiles, s);
}
}  // namespace psgd
