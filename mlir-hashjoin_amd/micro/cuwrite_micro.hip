// cuwrite_micro.hip -- how fast can ONE CU write (and read)?  The partition
// pass issues a tile's 64 KiB of line stores in one phase and they drain at
// ~10.5 B/clk per CU (micro/pass_micro.hip, synthetic rows) -- the same
// 26 GB/s per CU that a full-chip write-only copy averages.  A per-CU cap
// would make the store phase a fixed cost that only overlap with the LDS
// phases can hide; a chip-level cap would not.  Streams 2 GiB of 16-B rows
// with G persistent 1024-thread workgroups (one per CU, G = 256 .. 16),
// 4 / 8 / 16 rows per thread per step, write-only (nt) and read-only (nt).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o cuwrite_micro cuwrite_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
typedef __attribute__((ext_vector_type(2))) unsigned long long v2;

template <int U>
__global__ __launch_bounds__(1024) void k_write(v2 *out, u64 n) {
    const u64 per = n / gridDim.x, lo = (u64)blockIdx.x * per, hi = lo + per;
    const v2 val = {(u64)blockIdx.x, 7ull};
    for (u64 b = lo; b + (u64)U * 1024 <= hi; b += (u64)U * 1024)
#pragma unroll
        for (int i = 0; i < U; ++i) __builtin_nontemporal_store(val, out + b + (u64)i * 1024 + threadIdx.x);
}
template <int U>
__global__ __launch_bounds__(1024) void k_read(const v2 *in, u64 n, u64 *sink) {
    const u64 per = n / gridDim.x, lo = (u64)blockIdx.x * per, hi = lo + per;
    u64 acc = 0;
    for (u64 b = lo; b + (u64)U * 1024 <= hi; b += (u64)U * 1024) {
        v2 r[U];
#pragma unroll
        for (int i = 0; i < U; ++i) r[i] = __builtin_nontemporal_load(in + b + (u64)i * 1024 + threadIdx.x);
#pragma unroll
        for (int i = 0; i < U; ++i) acc += r[i].x;
    }
    if (acc == 0x1234567ull) sink[0] = acc;
}

int main() {
    const u64 n = 1ull << 27;   // 2 GiB of 16-B rows
    v2 *buf;
    u64 *sink;
    CK(hipMalloc(&buf, n * 16));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, n * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *what, int G, auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipEventRecord(e0));
            launch(G);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const double gbs = n * 16.0 / (best * 1e6);
        printf("%-22s G %3d  %8.3f ms  %7.1f GB/s chip  %6.1f GB/s per CU  %5.1f B/clk per CU @2.4GHz\n", what, G, best,
               gbs, gbs / G, gbs / G / 2.4);
    };
    for (int G : {256, 128, 64, 32, 16}) {
        run("write nt, 4 rows/thr", G, [&](int g) { hipLaunchKernelGGL(k_write<4>, dim3(g), dim3(1024), 0, 0, buf, n); });
        run("write nt, 16 rows/thr", G, [&](int g) { hipLaunchKernelGGL(k_write<16>, dim3(g), dim3(1024), 0, 0, buf, n); });
        run("read nt, 4 rows/thr", G, [&](int g) { hipLaunchKernelGGL(k_read<4>, dim3(g), dim3(1024), 0, 0, buf, n, sink); });
        run("read nt, 16 rows/thr", G, [&](int g) { hipLaunchKernelGGL(k_read<16>, dim3(g), dim3(1024), 0, 0, buf, n, sink); });
    }
    return 0;
}
