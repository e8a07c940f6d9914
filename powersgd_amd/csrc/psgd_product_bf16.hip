// Instantiations of the product kernels for bf16_t gradients (psgd_even.cuh, psgd_stream.cuh).
#include "psgd_even.cuh"

namespace psgd {
hipError_t launch_even_bf16(int R, int nres, const ProductArgs& a, int nwg, hipStream_t s) {
    return dispatch_even<bf16_t>(R, nres, a, nwg, s);
}
hipError_t launch_product_odd_bf16(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_odd<bf16_t>(R, nres, a, ntiles, s);
}
hipError_t launch_odd_mfma_bf16(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_odd_mfma<bf16_t>(R, nres, a, ntiles, s);
}
int even_resident_bf16(int R) { return even_resident<bf16_t>(R); }
}  // namespace psgd
