// offset_micro.hip -- does the persistent copy's speed depend on where the
// destination sits relative to the source?  The persistent shape (bench.py's
// copy floor, the partition passes) varies 1.35-1.58 ms per 4 GiB copy from
// process to process and box to box while the flat copy never varies
// (profiles/r05/r05l_*); the grid order and a rotated start change nothing,
// so the remaining suspect is the physical distance between the read and the
// write streams (HBM channel / bank interleave).  One 8.25 GiB allocation;
// source = its start, destination = 4 GiB + delta, for a set of deltas.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o offset_micro offset_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
typedef __attribute__((ext_vector_type(2))) unsigned long long v2;
constexpr int NT = 1024, IT = 4;
constexpr u64 T = (u64)NT * IT;

__device__ __forceinline__ v2 ld(const v2 *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(v2 *p, v2 v) { __builtin_nontemporal_store(v, p); }

__global__ __launch_bounds__(256) void k_flat(const v2 *in, v2 *out, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) st(out + i, ld(in + i));
}

__global__ __launch_bounds__(NT) void k_pers(const v2 *in, v2 *out, u64 n) {
    const u64 tiles = n / T, G = gridDim.x, b = blockIdx.x;
    const u64 t0 = b * tiles / G, t1 = (b + 1) * tiles / G;
    v2 r[IT], q[IT];
    if (t0 < t1)
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = ld(in + t0 * T + (u64)i * NT + threadIdx.x);
    for (u64 t = t0; t < t1; ++t) {
        if (t + 1 < t1)
#pragma unroll
            for (int i = 0; i < IT; ++i) q[i] = ld(in + (t + 1) * T + (u64)i * NT + threadIdx.x);
#pragma unroll
        for (int i = 0; i < IT; ++i) st(out + t * T + (u64)i * NT + threadIdx.x, r[i]);
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = q[i];
    }
}

int main() {
    const u64 n = 1ull << 28;   // 4 GiB of 16-B rows
    const u64 span = (n * 16) * 2 + (256ull << 20);
    char *base;
    CK(hipMalloc(&base, span));
    CK(hipMemset(base, 1, span));
    int dev, cus;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const v2 *src = (const v2 *)base;
    const u64 deltas[] = {0,        256,        4096,       65536,      1ull << 18, 1ull << 20, 2ull << 20,
                          3ull << 20, 4ull << 20, 8ull << 20, 16ull << 20, 32ull << 20, 64ull << 20,
                          (1ull << 20) + 4096, (5ull << 20) + 65536, (37ull << 20) + 8192, 128ull << 20,
                          (200ull << 20) + 12345ull * 256};
    printf("base %p  cus %d\n", (void *)base, cus);
    for (int round = 0; round < 2; ++round)
        for (u64 d : deltas) {
            v2 *dst = (v2 *)(base + n * 16 + d);
            float v[2][5];
            for (int shape = 0; shape < 2; ++shape)
                for (int rep = 0; rep < 5; ++rep) {
                    CK(hipEventRecord(e0));
                    if (shape == 0) hipLaunchKernelGGL(k_pers, dim3(cus), dim3(NT), 0, 0, src, dst, n);
                    else hipLaunchKernelGGL(k_flat, dim3(n / 256), dim3(256), 0, 0, src, dst, n);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&v[shape][rep], e0, e1));
                }
            for (int s = 0; s < 2; ++s)
                for (int i = 1; i < 5; ++i)
                    for (int j = i; j > 0 && v[s][j] < v[s][j - 1]; --j) { float t = v[s][j]; v[s][j] = v[s][j - 1]; v[s][j - 1] = t; }
            printf("delta %12llu B (%9.3f MiB)  persistent %7.4f ms  flat %7.4f ms\n", d, d / 1048576.0, v[0][2], v[1][2]);
        }
    return 0;
}
