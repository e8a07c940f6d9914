// Instantiations of the product kernels for float gradients (psgd_even.cuh, psgd_stream.cuh).
#include "psgd_even.cuh"

namespace psgd {
hipError_t launch_even_f32(int R, int nres, const ProductArgs& a, int nwg, hipStream_t s) {
    return dispatch_even<float>(R, nres, a, nwg, s);
}
hipError_t launch_product_odd_f32(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_odd<float>(R, nres, a, ntiles, s);
}
hipError_t launch_odd_mfma_f32(int R, int nres, const ProductArgs& a, int ntiles, hipStream_t s) {
    return dispatch_odd_mfma<float>(R, nres, a, ntiles, s);
}
int even_resident_f32(int R) { return even_resident<float>(R); }
}  // namespace psgd
