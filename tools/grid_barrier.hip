// Cost of an in-launch grid barrier vs a kernel boundary on this GPU (why the
// small plans keep one launch per power-iteration phase instead of one resident launch).
//
//   k_bar:   256 workgroups (one per CU, 256 threads) run B XCD-hierarchical grid barriers
//            (per-XCD arrival counter, the XCD's last arriver bumps a top counter, the last XCD
//            publishes a generation; every spin bounded) -> (t(B) - t(0)) / B per barrier.
//   k_empty: the same grid, no work, launched N times back to back on one stream
//            -> t(N) / N per dependent kernel boundary.
// build: hipcc -O3 --offload-arch=gfx950 tools/grid_barrier.hip -o tools/grid_barrier
#include <hip/hip_runtime.h>

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

constexpr int kXcd = 8;
constexpr unsigned kSpin = 1u << 22;

struct Bar {
    unsigned* xcd;  // [kXcd] arrivals per XCD (monotonic)
    unsigned* top;  // XCD leaders' arrivals (monotonic)
    unsigned* gen;  // [kXcd + 1] published generation per XCD, [kXcd] = top generation
    unsigned* err;
};

__device__ __forceinline__ unsigned ld_acq(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void grid_barrier(const Bar& b, unsigned epoch) {
    __syncthreads();
    if (threadIdx.x == 0) {
        // workgroups are dispatched round robin over the XCDs: block i runs on XCD i % 8
        const int x = blockIdx.x % kXcd;
        const unsigned per = (gridDim.x + kXcd - 1 - x) / kXcd;
        __atomic_thread_fence(__ATOMIC_RELEASE);
        const unsigned old = __hip_atomic_fetch_add(&b.xcd[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        if (old + 1 == epoch * per) {  // this XCD's last arriver
            const unsigned t = __hip_atomic_fetch_add(b.top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t + 1 == epoch * kXcd) {
                __hip_atomic_store(&b.gen[kXcd], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                while (ld_acq(&b.gen[kXcd]) < epoch && ++spins < kSpin) __builtin_amdgcn_s_sleep(1);
            }
            __hip_atomic_store(&b.gen[x], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (ld_acq(&b.gen[x]) < epoch && ++spins < kSpin) __builtin_amdgcn_s_sleep(1);
        }
        if (spins >= kSpin) __hip_atomic_store(b.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_bar(Bar b, unsigned base, int nbar) {
    for (int i = 1; i <= nbar; ++i) grid_barrier(b, base + unsigned(i));
}

__global__ __launch_bounds__(256) void k_empty() {}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int nwg = cus;  // one workgroup per CU: every one resident, the barrier can complete
    Bar b{};
    unsigned* mem;
    CK(hipMalloc(&mem, 64 * sizeof(unsigned)));
    CK(hipMemset(mem, 0, 64 * sizeof(unsigned)));
    b.xcd = mem;
    b.top = mem + 16;
    b.gen = mem + 32;
    b.err = mem + 48;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    unsigned epoch = 0;
    auto time_bar = [&](int nbar, int reps) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            k_bar<<<nwg, 256>>>(b, epoch, nbar);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            epoch += unsigned(nbar);
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        return best * 1e3f;  // us
    };
    auto time_empty = [&](int n, int reps) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < n; ++i) k_empty<<<nwg, 256>>>();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        return best * 1e3f;
    };
    time_bar(10, 3);
    time_empty(10, 3);  // warm-up
    const float t0 = time_bar(0, 20), t1 = time_bar(100, 20);
    const float e1_ = time_empty(1, 20), e100 = time_empty(101, 20);
    unsigned err = 0;
    CK(hipMemcpy(&err, b.err, sizeof(err), hipMemcpyDeviceToHost));
    std::printf("workgroups %d (one per CU), 256 threads\n", nwg);
    std::printf("grid barrier (XCD-hierarchical): %.2f us per barrier (t(100) %.1f us, t(0) %.1f us)%s\n",
                (t1 - t0) / 100.f, t1, t0, err ? "  [a spin TIMED OUT: invalid]" : "");
    std::printf("kernel boundary (empty %d-WG kernels back to back): %.2f us per launch (t(101) %.1f, t(1) %.1f)\n",
                nwg, (e100 - e1_) / 100.f, e100, e1_);
    CK(hipFree(mem));
    return err ? 2 : 0;
}
