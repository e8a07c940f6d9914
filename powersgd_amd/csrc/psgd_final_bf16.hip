// Instantiations of the fused final-pass kernels for bf16_t gradients (see psgd_final.cuh).
#include "psgd_final.cuh"

namespace psgd {
hipError_t launch_final_odd_bf16(int R, int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s,
                               int* waves) {
    return dispatch_final<bf16_t>(R, nres, smax, a, ntiles, s, waves);
}
hipError_t launch_final_oe_bf16(int nres, int smax, const FinalArgs& a, int ntiles, hipStream_t s, int* waves) {
    return dispatch_final_oe<bf16_t>(nres, smax, a, ntiles, s, waves);
}
hipError_t launch_lowrank_out_bf16(int R, int nterms, const ApplyArgs& a, int ntiles, hipStream_t s) {
    return dispatch_lowrank<bf16_t>(R, nterms, a, ntiles, s);
}
}  // namespace psgd
