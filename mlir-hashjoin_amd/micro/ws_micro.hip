// ws_micro.hip -- can a partition pass overlap its stream reads with its
// scattered bucket writes?  2^28 16-B rows, tiles of 8192 rows, one
// 1024-thread workgroup per CU; writes reproduce k_pass's pattern (512 bins,
// 16-row = 256-B runs per bin and tile into 512-row buckets).
//   MODE 0 read only, 1 write only, 2 every wave reads then writes its rows
//   (the k_pass order), 3 waves 0-7 read / waves 8-15 write (their own vmcnt)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o ws_micro ws_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
constexpr int kTile = 8192, kNT = 1024, kBins = 512, kRun = kTile / kBins, kBucket = 512;

// SPREAD 0: a workgroup's 512 open buckets are adjacent (4 MiB);
// SPREAD 1: they are G buckets (2 MiB at G = 256) apart -- as far apart as
// buckets from one global counter end up -- with the same 1 GiB window;
// SPREAD 2: as 0, but bin b's runs start (b * 5) % 8 rows into the bin's
// space, so every run is unaligned and each tile leaves partial 128-B lines
// that the next tile's run completes (k_pass's pattern); SPREAD 3 / 4: runs
// start on 64-B / 32-B boundaries only
template <int SPREAD = 0>
__device__ __forceinline__ u64 dest_row(unsigned t_local, unsigned wg, unsigned G, unsigned j) {
    constexpr int RUN = SPREAD == 5 ? 8 : SPREAD == 6 ? 32 : kRun;   // 5 / 6: aligned 128-B / 512-B runs
    constexpr int BINS = kTile / RUN;
    const unsigned b = j / RUN;                           // bin of staged row j
    const unsigned per = kBucket / RUN;                   // tiles per bucket
    const u64 bucket = SPREAD == 1 ? ((u64)(t_local / per) * BINS + b) * G + wg
                                   : ((u64)(t_local / per) * G + wg) * BINS + b;
    const unsigned shift = SPREAD == 2 ? (b * 5) % 8 : SPREAD == 3 ? (b & 1) * 4 : SPREAD == 4 ? (b & 1) * 2 : 0;
    return bucket * kBucket + shift + (t_local % per) * RUN + (j % RUN);
}

template <int MODE, int SPREAD = 0>
__global__ __launch_bounds__(kNT) void k_ws(const ulonglong2 *in, ulonglong2 *out, u64 n, u64 *sink) {
    const unsigned T = (unsigned)(n / kTile), G = gridDim.x;
    const unsigned t0 = (unsigned)((u64)blockIdx.x * T / G), t1 = (unsigned)((u64)(blockIdx.x + 1) * T / G);
    const unsigned wave = threadIdx.x / 64;
    u64 acc = 0;
    for (unsigned t = t0; t < t1; ++t) {
        const ulonglong2 *src = in + (u64)t * kTile;
        if constexpr (MODE == 0 || MODE == 2) {
            ulonglong2 r[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = src[i * kNT + threadIdx.x];
#pragma unroll
            for (int i = 0; i < 8; ++i) acc += r[i].x ^ r[i].y;
            if constexpr (MODE == 2) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const unsigned j = i * kNT + threadIdx.x;
                    out[dest_row<SPREAD>(t - t0, blockIdx.x, G, j)] = make_ulonglong2(acc + i, j);
                }
            }
        } else if constexpr (MODE == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const unsigned j = i * kNT + threadIdx.x;
                out[dest_row<SPREAD>(t - t0, blockIdx.x, G, j)] = make_ulonglong2(t, j);
            }
        } else {
            const unsigned lt = threadIdx.x & 511;
            if (wave < 8) {
                ulonglong2 r[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) r[i] = src[i * 512 + lt];
#pragma unroll
                for (int i = 0; i < 16; ++i) acc += r[i].x ^ r[i].y;
            } else if (t > t0) {   // the previous tile's rows
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const unsigned j = i * 512 + lt;
                    out[dest_row<SPREAD>(t - 1 - t0, blockIdx.x, G, j)] = make_ulonglong2(t, j);
                }
            }
        }
        __syncthreads();
    }
    if (acc == 0x123456789ull) *sink = acc;
}

int main() {
    const u64 n = 1ull << 28;
    ulonglong2 *in, *out;
    u64 *sink;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned G = (unsigned)cus;
    const u64 tiles_per = (n / kTile + G - 1) / G + 1;
    const u64 out_rows = (tiles_per / (kBucket / 32) + 1) * G * (kTile / 8) * kBucket + 8;
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, out_rows * 16));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 1, n * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-44s %7.3f ms  %7.1f GB/s (32 B/row)\n", name, ms, 32.0 * n / ms / 1e6);
    };
    run("read only", [&] { hipLaunchKernelGGL(k_ws<0>, dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("scattered write only", [&] { hipLaunchKernelGGL(k_ws<1>, dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("every wave: read then write (k_pass order)", [&] { hipLaunchKernelGGL(k_ws<2>, dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("waves 0-7 read, 8-15 write (prev tile)", [&] { hipLaunchKernelGGL(k_ws<3>, dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("scattered write only, buckets 2 MiB apart", [&] { hipLaunchKernelGGL((k_ws<1, 1>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("read then write, buckets 2 MiB apart", [&] { hipLaunchKernelGGL((k_ws<2, 1>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("scattered write only, unaligned runs", [&] { hipLaunchKernelGGL((k_ws<1, 2>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("read then write, unaligned runs", [&] { hipLaunchKernelGGL((k_ws<2, 2>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("scattered write only, aligned 128-B runs", [&] { hipLaunchKernelGGL((k_ws<1, 5>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("read then write, aligned 128-B runs", [&] { hipLaunchKernelGGL((k_ws<2, 5>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("read then write, aligned 512-B runs", [&] { hipLaunchKernelGGL((k_ws<2, 6>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("scattered write only, 64-B aligned runs", [&] { hipLaunchKernelGGL((k_ws<1, 3>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    run("scattered write only, 32-B aligned runs", [&] { hipLaunchKernelGGL((k_ws<1, 4>), dim3(G), dim3(kNT), 0, 0, in, out, n, sink); });
    return 0;
}
