// place_micro.hip -- is the partition pass's speed a property of where its
// DESTINATION buffer landed in physical memory?  The same pass (same source,
// same kernel) runs 1.43-1.47 or 1.75-1.79 ms depending on the bucket set it
// writes, bimodally, and the same allocation sequence gives the same times in
// a second process (profiles/r05/r05s_*).  Here: twelve 4.5 GiB buffers, and
// on each (a) the pass's write pattern alone -- every persistent 1024-thread
// workgroup writes, per 4096-row tile, one 128-B line into each of 512 open
// 16-KiB buckets of its own id range (pass 1's shape, rows synthetic) -- and
// (b) a flat sequential write of the same 4 GiB, and (c) a flat read.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o place_micro place_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
typedef __attribute__((ext_vector_type(2))) unsigned long long v2;

// pass-shaped writes: G workgroups, each TPW tiles; tile t writes one line of
// each of its 512 bins' open buckets.  V: 0 = line (t & 127) of bucket
// wbase + (t >> 7) * 512 + j (16-KiB buckets, every bin at the same line);
// 1 = bin j runs (7 j mod 128) lines ahead (bins at different lines, as a
// real pass's fills drift apart); 2 = 8-KiB buckets; 3 = 32-KiB buckets; 4 =
// bucket ids interleaved across workgroups (id * G + w).  Every store is
// bounds-checked against the buffer (nrows).
template <int V>
__global__ __launch_bounds__(1024) void k_passwrite(v2 *out, unsigned tpw, unsigned per_wg_buckets, u64 nrows) {
    const unsigned w = blockIdx.x, tid = threadIdx.x;
    const u64 wbase = (u64)w * per_wg_buckets;
    const v2 val = {w, 1};
    for (unsigned t = 0; t < tpw; ++t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const unsigned j = i * 128 + (tid >> 3);
            u64 row;
            if (V == 0) row = (wbase + (u64)(t >> 7) * 512 + j) * 1024 + (t & 127) * 8;
            if (V == 1) {
                const unsigned tt = t + ((j * 7) & 127);
                row = (wbase + (u64)(tt >> 7) * 512 + j) * 1024 + (tt & 127) * 8;
            }
            if (V == 2) row = (wbase * 2 + (u64)(t >> 6) * 512 + j) * 512 + (t & 63) * 8;
            if (V == 3) row = ((u64)w * (per_wg_buckets / 2) + j) * 2048 + (t & 255) * 8;
            if (V == 4) row = (((u64)(t >> 7) * 512 + j) * gridDim.x + w) * 1024 + (t & 127) * 8;
            if (row + 8 <= nrows) __builtin_nontemporal_store(val, out + row + (tid & 7));
        }
    }
}

__global__ __launch_bounds__(256) void k_flatwrite(v2 *out, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(v2{i, 2}, out + i);
}

__global__ __launch_bounds__(256) void k_flatread(const v2 *in, u64 n, u64 *sink) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) {
        const v2 v = __builtin_nontemporal_load(in + i);
        if (v.x == 0x1234567ull) sink[0] = v.y;
    }
}

int main(int argc, char **argv) {
    const int nbuf = argc > 1 ? atoi(argv[1]) : 12;
    // argv[2]: hipExtMallocWithFlags flags for the buffers (-1: hipMalloc);
    // argv[3] = 1: V0 + flat write only (for counter runs)
    const int flags = argc > 2 ? atoi(argv[2]) : -1;
    const bool quick = argc > 3 && atoi(argv[3]) == 1;
    const u64 n = 1ull << 28;            // rows written per test (4 GiB)
    const unsigned G = 256, tpw = (unsigned)(n / 4096 / G);   // 256 tiles per workgroup
    const unsigned per_wg = ((tpw + 127) / 128) * 512 + 512;  // buckets per workgroup range
    const u64 bytes = (u64)G * per_wg * 1024 * 16;
    const u64 nrows = bytes / 16;
    u64 *sink;
    CK(hipMalloc(&sink, 64));
    v2 *buf[64];
    for (int b = 0; b < nbuf; ++b) {
        if (flags < 0) CK(hipMalloc(&buf[b], bytes));
        else CK(hipExtMallocWithFlags((void **)&buf[b], bytes, (unsigned)flags));
        CK(hipMemset(buf[b], 0, bytes));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        float v[5];
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&v[rep], e0, e1));
        }
        for (int i = 1; i < 5; ++i)
            for (int j = i; j > 0 && v[j] < v[j - 1]; --j) { float t = v[j]; v[j] = v[j - 1]; v[j - 1] = t; }
        return v[2];
    };
    printf("buffers of %.2f GiB; pass-shaped write = %u workgroups x %u tiles x 64 KiB\n", bytes / 1073741824.0, G, tpw);
    for (int round = 0; round < 2; ++round)
        for (int b = 0; b < nbuf; ++b) {
            float pv[5] = {0, 0, 0, 0, 0};
            if (quick) {
                pv[0] = timeit([&] { hipLaunchKernelGGL(k_passwrite<0>, dim3(G), dim3(1024), 0, 0, buf[b], tpw, per_wg, nrows); });
                const float fw = timeit([&] { hipLaunchKernelGGL(k_flatwrite, dim3(n / 256), dim3(256), 0, 0, buf[b], n); });
                printf("buf %2d %p  pass-shaped write V0 %6.3f ms  flat write %6.3f\n", b, (void *)buf[b], pv[0], fw);
                continue;
            }
            pv[0] = timeit([&] { hipLaunchKernelGGL(k_passwrite<0>, dim3(G), dim3(1024), 0, 0, buf[b], tpw, per_wg, nrows); });
            pv[1] = timeit([&] { hipLaunchKernelGGL(k_passwrite<1>, dim3(G), dim3(1024), 0, 0, buf[b], tpw, per_wg, nrows); });
            pv[2] = timeit([&] { hipLaunchKernelGGL(k_passwrite<2>, dim3(G), dim3(1024), 0, 0, buf[b], tpw, per_wg, nrows); });
            pv[3] = timeit([&] { hipLaunchKernelGGL(k_passwrite<3>, dim3(G), dim3(1024), 0, 0, buf[b], tpw, per_wg, nrows); });
            pv[4] = timeit([&] { hipLaunchKernelGGL(k_passwrite<4>, dim3(G), dim3(1024), 0, 0, buf[b], tpw, per_wg, nrows); });
            const float fw = timeit([&] { hipLaunchKernelGGL(k_flatwrite, dim3(n / 256), dim3(256), 0, 0, buf[b], n); });
            const float fr = timeit([&] { hipLaunchKernelGGL(k_flatread, dim3(n / 256), dim3(256), 0, 0, buf[b], n, sink); });
            printf("buf %2d %p  pass-shaped write V0 %6.3f V1 %6.3f V2 %6.3f V3 %6.3f V4 %6.3f ms  flat write %6.3f  read %6.3f\n",
                   b, (void *)buf[b], pv[0], pv[1], pv[2], pv[3], pv[4], fw, fr);
        }
    return 0;
}
