// Diagnostic: lane-movement semantics of permlane swaps / DPP, and the product kernels'
// reduce-scatter (every lane should hold item lane >> SH: sum over lanes of (lane + 64 item)).
#include "../powersgd_amd/csrc/psgd_internal.h"
#include "../powersgd_amd/csrc/psgd_stream.cuh"
#include <cstdio>
using namespace psgd;
template <int NV>
__global__ void k(float* o) {
    const int l = threadIdx.x;
    float v[NV];
#pragma unroll
    for (int t = 0; t < NV; ++t) v[t] = float(l + 64 * t);
    o[l] = reduce_scatter<NV>(v, l);
}
int main() {
    float *d, h[64];
    (void)hipMalloc(&d, sizeof(h));
    k<16><<<1, 64>>>(d);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("NV=16 item per lane:");
    for (int l = 0; l < 64; ++l) printf(" %.2f", (h[l] - 2016.f) / 4096.f);
    printf("\n");
    k<32><<<1, 64>>>(d);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("NV=32 item per lane:");
    for (int l = 0; l < 64; ++l) printf(" %.2f", (h[l] - 2016.f) / 4096.f);
    printf("\n");
    return 0;
}
