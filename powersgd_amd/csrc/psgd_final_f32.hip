// Instantiations of the fused final-pass kernels for float gradients (see psgd_final.cuh).
#include "psgd_final.cuh"

namespace psgd {
hipError_t launch_final_odd_f32(int R, int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s,
                               int* waves) {
    return dispatch_final<float>(R, nres, smax, a, ntiles, s, waves);
}
hipError_t launch_final_oe_f32(int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    return dispatch_final_oe<float>(nres, smax, a, ntiles, s, waves);
}
hipError_t launch_lowrank_out_f32(int R, int nterms, const ApplyArgs& a, int ntiles, hipStream_t s) {
    return dispatch_lowrank<float>(R, nterms, a, ntiles, s);
}
}  // namespace psgd
