// micro.hip -- design microbenchmarks for the hash-join kernels (gfx950).
// Measures the primitive rates the table design depends on:
//   * random 64-bit CAS into a table of size T (agent vs workgroup scope)
//   * random 16-B slot reads from a table of size T (HBM / MALL / L2)
//   * streaming copy (HBM reference)
//   * LDS 64-bit CAS inserts
// Build: hipcc --offload-arch=gfx950 -O3 -o micro micro.hip ; run: ./micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int SCOPE>
__global__ __launch_bounds__(256) void k_cas(unsigned long long *t, unsigned long long mask, long long n, unsigned long long salt) {
    long long i = (long long)blockIdx.x * 1024 + threadIdx.x;
    unsigned long long h[4], o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = (mix((i + j * 256) ^ salt) & mask) * 2;   // key word of a 16-B slot
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (i + j * 256 < n) {
            unsigned long long exp = 0;
            if (SCOPE == 0) o[j] = atomicCAS(&t[h[j]], 0ull, (unsigned long long)(i + j * 256 + 1));
            else {
                __hip_atomic_compare_exchange_strong(&t[h[j]], &exp, (unsigned long long)(i + j * 256 + 1),
                                                     __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                o[j] = exp;
            }
        } else o[j] = 0;
    }
    unsigned long long x = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) x += o[j];
    if (x == 0x1234567ull) t[0] = x;
}

// workgroup-private regions: each block CASes inside its own region of R slots
template <int SCOPE>
__global__ __launch_bounds__(256) void k_cas_region(unsigned long long *t, unsigned long long rmask, int ops) {
    unsigned long long *base = t + (unsigned long long)blockIdx.x * (rmask + 1) * 2;
    unsigned long long acc = 0;
    for (int k = 0; k < ops; ++k) {
        unsigned long long h = (mix(((unsigned long long)blockIdx.x << 32) ^ (k * 256 + threadIdx.x)) & rmask) * 2;
        unsigned long long exp = 0;
        if (SCOPE == 0) acc += atomicCAS(&base[h], 0ull, 1ull + k);
        else {
            __hip_atomic_compare_exchange_strong(&base[h], &exp, 1ull + k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            acc += exp;
        }
    }
    if (acc == 0x1234567ull) t[0] = acc;
}

__global__ __launch_bounds__(256) void k_read(const ulonglong2 *t, unsigned long long mask, long long n, unsigned long long salt,
                                              unsigned long long *sink) {
    long long i = (long long)blockIdx.x * 1024 + threadIdx.x;
    unsigned long long acc = 0;
    ulonglong2 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        unsigned long long h = mix((i + j * 256) ^ salt) & mask;
        v[j] = (i + j * 256 < n) ? t[h] : make_ulonglong2(0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc += v[j].x ^ v[j].y;
    if (acc == 0x1234567ull) *sink = acc;
}

__global__ __launch_bounds__(256) void k_copy(const ulonglong2 *a, ulonglong2 *b, long long n) {
    long long i = (long long)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (i + j * 256 < n) b[i + j * 256] = a[i + j * 256];
}

// LDS insert: each block builds a 8192-slot (128 KB) table from 4096 keys, R rounds
__global__ __launch_bounds__(1024) void k_lds(int rounds, unsigned long long *sink) {
    __shared__ unsigned long long tab[8192 * 2];
    unsigned long long acc = 0;
    for (int r = 0; r < rounds; ++r) {
        for (int i = threadIdx.x; i < 8192 * 2; i += 1024) tab[i] = 0;
        __syncthreads();
        for (int k = threadIdx.x; k < 4096; k += 1024) {
            unsigned long long key = mix(((unsigned long long)blockIdx.x << 40) ^ (r << 20) ^ k) | 1;
            unsigned h = (unsigned)(key >> 51);
            while (true) {
                unsigned long long o = atomicCAS(&tab[h * 2], 0ull, key);
                if (o == 0) { tab[h * 2 + 1] = k; break; }
                h = (h + 1) & 8191;
            }
        }
        __syncthreads();
        for (int k = threadIdx.x; k < 4096; k += 1024) {
            unsigned long long key = mix(((unsigned long long)blockIdx.x << 40) ^ (r << 20) ^ (k * 7)) | 1;
            unsigned h = (unsigned)(key >> 51);
            while (tab[h * 2] != 0) { acc += (tab[h * 2] == key); h = (h + 1) & 8191; }
        }
        __syncthreads();
    }
    if (acc == 0x1234567ull) *sink = acc;
}

int main() {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const size_t maxbytes = 8ull << 30;
    void *buf, *buf2;
    CK(hipMalloc(&buf, maxbytes));
    CK(hipMalloc(&buf2, 4ull << 30));
    unsigned long long *sink;
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, maxbytes));
    auto time = [&](auto fn, int reps) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        return ms / reps;
    };
    const long long nops = 1ll << 26;
    unsigned grid = (unsigned)((nops + 1023) / 1024);
    // streaming copy reference: 2 GiB -> 2 GiB
    {
        long long n = (2ll << 30) / 16;
        float ms = time([&] { hipLaunchKernelGGL(k_copy, dim3((n + 1023) / 1024), dim3(256), 0, 0, (const ulonglong2 *)buf, (ulonglong2 *)buf2, n); }, 5);
        printf("copy 2GiB->2GiB: %.3f ms  %.1f GB/s (read+write)\n", ms, 2.0 * n * 16 / ms / 1e6);
    }
    for (int lg = 20; lg <= 29; ++lg) {   // table of 2^lg 16-B slots: 16 MiB .. 8 GiB
        unsigned long long slots = 1ull << lg, mask = slots - 1;
        float mr = time([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const ulonglong2 *)buf, mask, nops, 77ull, sink); }, 5);
        CK(hipMemset(buf, 0, slots * 16));
        float mc = time([&] { CK(hipMemsetAsync(buf, 0, slots * 16)); hipLaunchKernelGGL(k_cas<0>, dim3(grid), dim3(256), 0, 0, (unsigned long long *)buf, mask, nops, 99ull); }, 3);
        float mm = time([&] { CK(hipMemsetAsync(buf, 0, slots * 16)); }, 3);
        float mw = time([&] { CK(hipMemsetAsync(buf, 0, slots * 16)); hipLaunchKernelGGL(k_cas<1>, dim3(grid), dim3(256), 0, 0, (unsigned long long *)buf, mask, nops, 99ull); }, 3);
        printf("table %7.1f MiB: rand16B read %.2f Gops/s (%.3f ms) | CAS agent %.2f Gops/s | CAS wg-scope %.2f Gops/s (memset %.3f ms)\n",
               slots * 16 / 1048576.0, nops / mr / 1e6, mr, nops / (mc - mm) / 1e6, nops / (mw - mm) / 1e6, mm);
    }
    // per-workgroup private regions (2048 blocks), agent vs workgroup scope
    for (int lg = 12; lg <= 17; lg += 1) {
        unsigned long long rs = 1ull << lg;
        int ops = 64;
        unsigned blocks = 2048;
        if (rs * 16 * blocks > maxbytes) break;
        float m0 = time([&] { hipLaunchKernelGGL(k_cas_region<0>, dim3(blocks), dim3(256), 0, 0, (unsigned long long *)buf, rs - 1, ops); }, 3);
        float m1 = time([&] { hipLaunchKernelGGL(k_cas_region<1>, dim3(blocks), dim3(256), 0, 0, (unsigned long long *)buf, rs - 1, ops); }, 3);
        double n = (double)blocks * 256 * ops;
        printf("private region %6.0f KiB/block (2048 blocks): CAS agent %.2f Gops/s | wg-scope %.2f Gops/s\n",
               rs * 16 / 1024.0, n / m0 / 1e6, n / m1 / 1e6);
    }
    {
        int rounds = 16;
        unsigned blocks = 256 * 4;
        float ms = time([&] { hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(1024), 0, 0, rounds, sink); }, 3);
        double ins = (double)blocks * rounds * 4096;
        printf("LDS 8192-slot tables: %.2f G inserts+probes/s (%.3f ms)\n", ins / ms / 1e6, ms);
    }
    return 0;
}
