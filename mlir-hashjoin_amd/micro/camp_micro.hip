// camp_micro.hip -- is the persistent shape's box/process variance a
// placement effect?  The passes and bench.py's persistent copy floor both give
// each CU one contiguous 1/256 of the input (streams 2^28 x 16 B / 256 = 16 MiB
// apart, advancing in step); the flat copy touches neighbouring addresses from
// every CU at once and never varies (1.32-1.33 ms on every box), while the
// persistent copy runs 1.35-1.58 ms depending on the box AND on the process
// (profiles/r05/r05k_*).  Same 4 GiB -> 4 GiB copy, five shapes:
//   flat          one row per thread, 256-thread workgroups
//   contiguous    one 1024-thread workgroup per CU, its own contiguous tile range (the passes)
//   grid-stride   one workgroup per CU, tiles b, b + G, b + 2G, ...
//   rotated       contiguous ranges, each workgroup starting at a different point of its range
//   contig-read / contig-write   the contiguous shape's loads / stores alone
// argv[1] = MiB to allocate (and keep) before the buffers, so separate runs see
// different physical placements.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o camp_micro camp_micro.hip
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

// MODE 0 contiguous, 1 grid-stride, 2 rotated, 3 contiguous loads only, 4 contiguous stores only
template <int MODE>
__global__ __launch_bounds__(NT) void k_pers(const v2 *in, v2 *out, u64 n, u64 *sink) {
    const u64 tiles = n / T, G = gridDim.x, b = blockIdx.x;
    const u64 t0 = b * tiles / G, t1 = (b + 1) * tiles / G, len = t1 - t0;
    const u64 cnt = MODE == 1 ? (tiles - b + G - 1) / G : len;
    const u64 rot = MODE == 2 && len ? (b * 7919u) % len : 0;
    auto tile = [&](u64 k) -> u64 {
        if (MODE == 1) return b + k * G;
        u64 j = k + rot;
        if (j >= len) j -= len;
        return t0 + j;
    };
    v2 r[IT], q[IT], acc = {0, 0};
    if (cnt && MODE != 4)
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = ld(in + tile(0) * T + (u64)i * NT + threadIdx.x);
    for (u64 k = 0; k < cnt; ++k) {
        const u64 t = tile(k);
        if (k + 1 < cnt && MODE != 4) {
            const u64 tn = tile(k + 1);
#pragma unroll
            for (int i = 0; i < IT; ++i) q[i] = ld(in + tn * T + (u64)i * NT + threadIdx.x);
        }
        if (MODE == 3) {
#pragma unroll
            for (int i = 0; i < IT; ++i) acc += r[i];
        } else {
#pragma unroll
            for (int i = 0; i < IT; ++i) st(out + t * T + (u64)i * NT + threadIdx.x, MODE == 4 ? v2{t, b} : r[i]);
        }
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = q[i];
    }
    if (MODE == 3 && acc.x == 0x123456789ull) sink[0] = acc.y;
}

int main(int argc, char **argv) {
    const u64 pre = argc > 1 ? strtoull(argv[1], nullptr, 10) : 0;
    void *hold = nullptr;
    if (pre) CK(hipMalloc(&hold, pre << 20));
    const u64 n = 1ull << 28;
    v2 *a, *b;
    u64 *sink;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, n * 16));
    CK(hipMemset(b, 2, n * 16));
    int dev, cus;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *what, auto launch) {
        float v[7];
        for (int rep = 0; rep < 7; ++rep) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&v[rep], e0, e1));
        }
        for (int i = 1; i < 7; ++i)
            for (int j = i; j > 0 && v[j] < v[j - 1]; --j) { float t = v[j]; v[j] = v[j - 1]; v[j - 1] = t; }
        printf("pre %6llu MiB  %-14s median %7.4f ms  min %7.4f  max %7.4f\n", pre, what, v[3], v[0], v[6]);
    };
    for (int round = 0; round < 2; ++round) {
        run("flat", [&] { hipLaunchKernelGGL(k_flat, dim3(n / 256), dim3(256), 0, 0, a, b, n); });
        run("contiguous", [&] { hipLaunchKernelGGL(k_pers<0>, dim3(cus), dim3(NT), 0, 0, a, b, n, sink); });
        run("grid-stride", [&] { hipLaunchKernelGGL(k_pers<1>, dim3(cus), dim3(NT), 0, 0, a, b, n, sink); });
        run("rotated", [&] { hipLaunchKernelGGL(k_pers<2>, dim3(cus), dim3(NT), 0, 0, a, b, n, sink); });
        run("contig-read", [&] { hipLaunchKernelGGL(k_pers<3>, dim3(cus), dim3(NT), 0, 0, a, b, n, sink); });
        run("contig-write", [&] { hipLaunchKernelGGL(k_pers<4>, dim3(cus), dim3(NT), 0, 0, a, b, n, sink); });
    }
    printf("pre %6llu MiB  a %p b %p\n", pre, (void *)a, (void *)b);
    return 0;
}
