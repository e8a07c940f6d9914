// Diagnostic build: k_orth_chol<4> with s_memtime phase stamps (psgd_small.hip, PSGD_STAMPS):
// workgroup 0 takes a k-row panel, the other units are ResNet-50-like Q panels.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPSGD_STAMPS -I include -I powersgd_amd/csrc \
//         tools/chol_stamps.hip -o tools/chol_stamps
#include "../powersgd_amd/csrc/psgd_small.hip"

#include <cstdio>
#include <vector>

using namespace psgd;

int main(int argc, char** argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 4608;
    const int nunits = argc > 2 ? atoi(argv[2]) : 54;
    const int r = 4;
    std::vector<int> len(nunits);
    size_t total = 0;
    for (int u = 0; u < nunits; ++u) {
        len[u] = u == 0 ? k : 64 << (u % 6);
        total += size_t(len[u]) * r;
    }
    std::vector<float> h(total);
    for (size_t i = 0; i < h.size(); ++i) h[i] = float((i * 2654435761u) % 1000) / 500.f - 1.f;
    std::vector<OrthUnit> units(nunits);
    size_t off = 0;
    for (int u = 0; u < nunits; ++u) {
        units[u] = OrthUnit{int64_t(off), len[u], r, 1};
        off += size_t(len[u]) * r;
    }
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
    unsigned long long s[64], bs[64];
    for (int rep = 0; rep < 30; ++rep) {
        (void)hipMemcpy(st, h.data(), h.size() * 4, hipMemcpyHostToDevice);
        (void)hipEventRecord(e0, 0);
        (void)launch_orth(a, nunits, r, k, true, 0);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpyFromSymbol(s, HIP_SYMBOL(g_stamps), sizeof(s));
        if (ms < best) {
            best = ms;
            for (int i = 0; i < 64; ++i) bs[i] = s[i];
        }
    }
    printf("k=%d units=%d best launch %.2f us (s_memtime ticks)\n", k, nunits, best * 1e3);
    printf("unit load %llu | gram pass %llu | block sum %llu | chain %llu | apply %llu | total %llu\n",
           bs[10] - bs[9], bs[11] - bs[10], bs[12] - bs[11], bs[13] - bs[12], bs[14] - bs[13], bs[14] - bs[9]);
    return 0;
}

// the f64 flat pack lives in psgd_f64.hip (not part of this probe)
namespace psgd {
hipError_t launch_flat_pack_f64(const FlatArgs&, hipStream_t) { return hipErrorNotSupported; }
}
