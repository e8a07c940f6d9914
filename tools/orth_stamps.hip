// Diagnostic build: the orthonormalisation kernels with s_memtime phase stamps
// (psgd_small.hip, PSGD_STAMPS; rank-4 panels through launch_orth, i.e. k_orth_wy).
// Prints shader-clock cycles per phase and the hipEvent duration of one launch.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPSGD_STAMPS -I include -I powersgd_amd/csrc \
//         tools/orth_stamps.hip -o tools/orth_stamps
#include "../powersgd_amd/csrc/psgd_small.hip"

#include <cstdio>
#include <vector>

using namespace psgd;

int main(int argc, char** argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 2048;
    const int nunits = argc > 2 ? atoi(argv[2]) : 54;
    const int r = 4;
    const size_t panel = size_t(k) * r;
    std::vector<float> h(panel * nunits);
    for (size_t i = 0; i < h.size(); ++i) h[i] = float((i * 2654435761u) % 1000) / 500.f - 1.f;
    std::vector<OrthUnit> units(nunits);
    for (int u = 0; u < nunits; ++u) units[u] = OrthUnit{int64_t(u) * int64_t(panel), k, r, 1};
    const int rr = argc > 3 ? atoi(argv[3]) : 4;
    (void)rr;
    float *st, *hx;
    OrthUnit* du;
    (void)hipMalloc(&st, h.size() * 4);
    (void)hipMalloc(&hx, h.size() * 4);
    (void)hipMalloc(&du, units.size() * sizeof(OrthUnit));
    (void)hipMemcpy(du, units.data(), units.size() * sizeof(OrthUnit), hipMemcpyHostToDevice);
    OrthArgs a{};
    a.units = du;
    a.state = st;
    a.hx = hx;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e9f;
    for (int rep = 0; rep < 20; ++rep) {
        (void)hipMemcpy(st, h.data(), h.size() * 4, hipMemcpyHostToDevice);
        (void)hipEventRecord(e0, 0);
        (void)launch_orth(a, nunits, r, k, false, 0);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    unsigned long long s[64];
    (void)hipMemcpyFromSymbol(s, HIP_SYMBOL(g_stamps), sizeof(s));
    printf("k=%d units=%d best launch %.2f us\n", k, nunits, best * 1e3);
    printf("loads %llu | geqr2 %llu | slarft+Q+stores %llu | total %llu cycles\n", s[1] - s[0], s[40] - s[1],
           s[42] - s[40], s[42] - s[0]);
    return 0;
}
