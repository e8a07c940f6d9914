// Host-side cost of one kernel launch, by launch API (diagnostic tool, not part of the library):
// the world-size > 1 path of small plans (cfg5) is host-enqueue-bound (profiles/r06/w_gt1: 4-9 us
// of hipLaunchKernel per 3-5 us kernel). N launches of an empty kernel are enqueued back to back
// (no synchronisation in between) and the host time per enqueue is reported, for:
//   chevron-small   k<<<>>>(int)
//   chevron-struct  k<<<>>>(a 640-byte argument struct, the size of the codec's launch arguments)
//   module-params   hipModuleLaunchKernel on the hipFunction_t of hipGetFuncBySymbol, kernelParams
//   module-extra    the same with a packed argument buffer (HIP_LAUNCH_PARAM_BUFFER_POINTER)
//   ext             hipExtLaunchKernel (no events)
// and then the device time per launch of the same chain (events around it).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_cost.hip -o tools/launch_cost
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

struct Big {
    const void* p[64];
    long long n[16];
};

__global__ void k_small(int) {}
__global__ void k_big(Big b) {
    if (b.n[0] == 12345 && threadIdx.x == 1000) *(int*)b.p[0] = 1;  // keeps the argument live
}

int main() {
    constexpr int N = 400, REPS = 5;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Big big{};
    hipFunction_t f;
    CK(hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&k_big)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 50; ++w) launch();
        CK(hipStreamSynchronize(s));
        double best_host = 1e30, best_dev = 1e30;
        for (int rep = 0; rep < REPS; ++rep) {
            CK(hipEventRecord(e0, s));
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < N; ++i) launch();
            const auto t1 = std::chrono::steady_clock::now();
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double host = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
            best_host = host < best_host ? host : best_host;
            best_dev = ms * 1e3 / N < best_dev ? ms * 1e3 / N : best_dev;
        }
        std::printf("%-16s host %6.2f us per enqueue, device %6.2f us per launch (best of %d x %d)\n", name, best_host,
                    best_dev, REPS, N);
    };
    run("chevron-small", [&] { k_small<<<256, 256, 0, s>>>(1); });
    run("chevron-struct", [&] { k_big<<<256, 256, 0, s>>>(big); });
    run("module-params", [&] {
        void* args[] = {&big};
        CK(hipModuleLaunchKernel(f, 256, 1, 1, 256, 1, 1, 0, s, args, nullptr));
    });
    run("module-extra", [&] {
        size_t sz = sizeof(big);
        void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &big, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        CK(hipModuleLaunchKernel(f, 256, 1, 1, 256, 1, 1, 0, s, nullptr, extra));
    });
    run("ext", [&] {
        void* args[] = {&big};
        CK(hipExtLaunchKernel(reinterpret_cast<const void*>(&k_big), dim3(256), dim3(256), args, 0, s, nullptr,
                              nullptr, 0));
    });
    std::printf("sizeof(Big) = %zu\n", sizeof(Big));
    return 0;
}
