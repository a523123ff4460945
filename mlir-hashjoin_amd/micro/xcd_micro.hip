// xcd_micro.hip -- does XCD-local slicing of a 32 MiB probe table pay?
// Random 16-B slot reads, 2^30 probes: (a) any slot from any workgroup;
// (b) workgroup b reads only slice b % 8 (4 MiB = one XCD's L2), relying on
// the round-robin block -> XCD deal (speed only, never correctness).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;

__device__ u64 mixd(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <bool SLICED, int ITEMS, int ATOMIC = 0>
__global__ __launch_bounds__(256) void k_probe(const ulonglong2 *t, int bits, u64 n, u64 *sink) {
    const u64 mask = (1ull << bits) - 1, smask = (1ull << (bits - 3)) - 1;
    const u64 slice = (u64)(blockIdx.x & 7) << (bits - 3);
    u64 acc = 0;
    for (u64 i = (u64)blockIdx.x * 256 * ITEMS + threadIdx.x; i < n; i += (u64)gridDim.x * 256 * ITEMS) {
        ulonglong2 v[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const u64 h = mixd(i + j * 256);
            const u64 s = SLICED ? (slice | (h & smask)) : (h & mask);
            v[j] = t[s];
        }
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) acc += v[j].x ^ v[j].y;
        if constexpr (ATOMIC == 1) {   // one returning atomic on ONE counter per 256*ITEMS rows
            __shared__ u64 sb;
            if (threadIdx.x == 0) sb = atomicAdd(sink + 1, (u64)(acc & 1) + 2048);
            __syncthreads();
            acc += sb;
        } else if constexpr (ATOMIC == 2) {   // same, spread over 64 counters
            __shared__ u64 sb;
            if (threadIdx.x == 0) sb = atomicAdd(sink + 8 + (blockIdx.x & 63) * 16, (u64)(acc & 1) + 2048);
            __syncthreads();
            acc += sb;
        }
    }
    if (acc == 0x1234567) *sink = acc;
}

int main() {
    const int bits = 21;   // 2^21 slots x 16 B = 32 MiB
    const u64 n = 1ull << 30;
    ulonglong2 *t;
    u64 *sink;
    CK(hipMalloc(&t, (16ull << bits)));
    CK(hipMalloc(&sink, 64 * 1024));
    CK(hipMemset(t, 1, 16ull << bits));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto fn) {
        fn(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 3; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 3;
        printf("%-36s %8.3f ms  %6.1f G probes/s\n", name, ms, n / ms / 1e6);
    };
    run("XCD slice + 1 atomic/2048 rows", [&] { hipLaunchKernelGGL((k_probe<true, 8, 1>), dim3(cus * 8), dim3(256), 0, 0, t, bits, n, sink); });
    run("XCD slice + atomic on 64 counters", [&] { hipLaunchKernelGGL((k_probe<true, 8, 2>), dim3(cus * 8), dim3(256), 0, 0, t, bits, n, sink); });
    run("any slot + 1 atomic/2048 rows", [&] { hipLaunchKernelGGL((k_probe<false, 8, 1>), dim3(cus * 8), dim3(256), 0, 0, t, bits, n, sink); });
    for (int wpc : {8}) {
        char a[64], b[64];
        snprintf(a, sizeof a, "any slot, %d wg/cu", wpc);
        snprintf(b, sizeof b, "XCD slice, %d wg/cu", wpc);
        run(a, [&] { hipLaunchKernelGGL((k_probe<false, 8>), dim3(cus * wpc), dim3(256), 0, 0, t, bits, n, sink); });
        run(b, [&] { hipLaunchKernelGGL((k_probe<true, 8>), dim3(cus * wpc), dim3(256), 0, 0, t, bits, n, sink); });
    }
    return 0;
}
