// dpp_micro.hip -- checks the DPP wave scans of hj_internal.h (wave64
// inclusive prefix sum / max by row shifts + row broadcasts) against the
// host, for u32 and u64, and times them against __shfl_up (ds_bpermute).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o dpp_micro dpp_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hj_internal.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;

__global__ void k_check(const unsigned *in, const u64 *in64, unsigned *sum, unsigned *mx, u64 *sum64) {
    const int t = blockIdx.x * 64 + threadIdx.x;
    sum[t] = hj::wave_incl_add(in[t]);
    mx[t] = hj::wave_max_all(in[t]);
    sum64[t] = hj::wave_incl_add64(in64[t]);
}

template <bool DPP>
__global__ void k_time(unsigned *out, int iters) {
    unsigned x = threadIdx.x + blockIdx.x;
    for (int i = 0; i < iters; ++i) {
        if constexpr (DPP) {
            x = hj::wave_incl_add(x) ^ i;
        } else {
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned y = __shfl_up(x, o, 64);
                if ((int)(threadIdx.x & 63) >= o) x += y;
            }
            x ^= i;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    const int waves = 1024, n = waves * 64;
    std::vector<unsigned> h(n);
    std::vector<u64> h64(n);
    srand(3);
    for (int i = 0; i < n; ++i) {
        h[i] = (unsigned)rand() % 100000u;
        h64[i] = ((u64)(unsigned)rand() << 20) ^ (u64)rand();
    }
    unsigned *in, *sum, *mx;
    u64 *in64, *sum64;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&sum, n * 4));
    CK(hipMalloc(&mx, n * 4));
    CK(hipMalloc(&in64, n * 8));
    CK(hipMalloc(&sum64, n * 8));
    CK(hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(in64, h64.data(), n * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_check, dim3(waves), dim3(64), 0, 0, in, in64, sum, mx, sum64);
    CK(hipDeviceSynchronize());
    std::vector<unsigned> s(n), m(n);
    std::vector<u64> s64(n);
    CK(hipMemcpy(s.data(), sum, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m.data(), mx, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s64.data(), sum64, n * 8, hipMemcpyDeviceToHost));
    long bad = 0;
    for (int w = 0; w < waves; ++w) {
        unsigned acc = 0, best = 0;
        u64 acc64 = 0;
        for (int l = 0; l < 64; ++l) best = h[w * 64 + l] > best ? h[w * 64 + l] : best;
        for (int l = 0; l < 64; ++l) {
            const int i = w * 64 + l;
            acc += h[i];
            acc64 += h64[i];
            bad += (s[i] != acc) + (m[i] != best) + (s64[i] != acc64);
        }
    }
    printf("dpp scans: %ld mismatches over %d waves -> %s\n", bad, waves, bad ? "FAIL" : "OK");
    unsigned *o;
    CK(hipMalloc(&o, 256 * 256 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int v = 0; v < 2; ++v) {
        float best = 1e9f;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(e0));
            if (v) hipLaunchKernelGGL(k_time<true>, dim3(256), dim3(256), 0, 0, o, 4096);
            else hipLaunchKernelGGL(k_time<false>, dim3(256), dim3(256), 0, 0, o, 4096);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("%s wave scan: %.1f ns per scan per wave (4096 dependent scans, 4 waves per CU)\n",
               v ? "DPP      " : "shfl_up  ", best * 1e6 / 4096);
    }
    return bad ? 1 : 0;
}
