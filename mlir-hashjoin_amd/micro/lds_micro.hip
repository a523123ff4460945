// lds_micro.hip -- LDS access costs of the join's build and probe shapes on
// gfx950: 64-bit CAS with return (the build's insert), 32-bit CAS, plain
// 64-bit stores, 64-bit reads, 32-bit adds with return, each to random slots
// of a 4096-slot table (32 KiB), 768-thread workgroups, 2 per CU (the fast
// join's shape).  Every wave-instruction's result feeds the next address, so
// the figure is a dependent chain per wave, as in the join's walks; INDEP
// variants issue 3 per lane before using any result (the build's 3 rows).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o lds_micro lds_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;

__device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

// OP: 0 CAS64, 1 CAS32, 2 store64, 3 read64, 4 add32 ret, 5 add32 no-ret, 6 exch64 ret,
// 7 exch32 ret, 8 add64 ret, 9 or32 ret
template <int OP, int IND>
__global__ __launch_bounds__(768, 6) void k_lds(int iters, u64 *sink) {
    __shared__ u64 t[4096];
    for (int j = threadIdx.x; j < 4096; j += 768) t[j] = 0;
    __syncthreads();
    unsigned h[IND], seed[IND];
#pragma unroll
    for (int k = 0; k < IND; ++k) {
        seed[k] = mix32(threadIdx.x * 7919u + blockIdx.x * 104729u + k * 31u);
        h[k] = seed[k] & 4095u;
    }
    u64 acc = 0;
    for (int it = 0; it < iters; ++it) {
        u64 r[IND];
#pragma unroll
        for (int k = 0; k < IND; ++k) {
            if constexpr (OP == 0) r[k] = atomicCAS(&t[h[k]], (u64)it, (u64)it + h[k]);
            else if constexpr (OP == 1) r[k] = atomicCAS((unsigned *)t + h[k] * 2, (unsigned)it, (unsigned)it + h[k]);
            else if constexpr (OP == 2) { t[h[k]] = (u64)it + h[k]; r[k] = 0; }
            else if constexpr (OP == 3) r[k] = t[h[k]];
            else if constexpr (OP == 4) r[k] = atomicAdd((unsigned *)t + h[k] * 2, 1u);
            else if constexpr (OP == 5) { atomicAdd((unsigned *)t + h[k] * 2, 1u); r[k] = 0; }
            else if constexpr (OP == 6) r[k] = atomicExch(&t[h[k]], (u64)it + h[k]);
            else if constexpr (OP == 7) r[k] = atomicExch((unsigned *)t + h[k] * 2, (unsigned)it + h[k]);
            else if constexpr (OP == 8) r[k] = atomicAdd(&t[h[k]], 1ull);
            else r[k] = atomicOr((unsigned *)t + h[k] * 2, 1u << (h[k] & 31));
        }
#pragma unroll
        for (int k = 0; k < IND; ++k) {
            // a fresh random slot per lane and step (lane-distinct seeds: the
            // lanes never converge onto one address); r >> 63 is 0 but keeps
            // the next access dependent on this one's result
            acc += r[k];
            h[k] = (mix32(seed[k] + (unsigned)it * 0x9E3779B9u) + (unsigned)(r[k] >> 63)) & 4095u;
        }
    }
    __syncthreads();
    if (acc == 0x123456789ull) sink[0] = t[threadIdx.x & 4095];
}

int main() {
    int cus = 256, dev = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    u64 *sink;
    CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 4096;
    auto run = [&](const char *name, int ind, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 3;
        const double ops = (double)iters * ind * 768 * 2 * cus;
        const double waveinstr_per_cu = (double)iters * ind * 12 * 2;
        printf("%-28s %8.3f ms  %7.2f Gops/s  %6.1f cycles per wave-instruction per CU (2.4 GHz)\n", name, ms,
               ops / ms / 1e6, ms * 1e-3 * 2.4e9 / waveinstr_per_cu);
    };
#define R(OP, IND, NAME) run(NAME, IND, [&] { hipLaunchKernelGGL((k_lds<OP, IND>), dim3(2 * cus), dim3(768), 0, 0, iters, sink); })
    R(0, 1, "CAS64 dependent");
    R(0, 3, "CAS64 x3 independent");
    R(1, 1, "CAS32 dependent");
    R(1, 3, "CAS32 x3 independent");
    R(2, 1, "store64");
    R(2, 3, "store64 x3");
    R(3, 1, "read64 dependent");
    R(3, 3, "read64 x3 independent");
    R(4, 1, "add32 ret dependent");
    R(4, 3, "add32 ret x3");
    R(5, 3, "add32 no-ret x3");
    R(6, 1, "exch64 dependent");
    R(6, 3, "exch64 x3");
    R(7, 3, "exch32 x3");
    R(8, 3, "add64 ret x3");
    R(9, 3, "or32 ret x3");
    return 0;
}
