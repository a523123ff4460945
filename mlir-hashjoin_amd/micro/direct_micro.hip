// direct_micro.hip -- a partition pass WITHOUT the LDS stage: every row is
// stored straight from its lane to its bin's position (per-lane 16-B stores,
// a wave's 64 lanes on ~64 different lines), only the per-bin line tails in
// LDS.  The question: does the memory system assemble lines written by 8
// different store instructions of one CU as well as it takes k_pass's
// coalesced 128-B runs?  Without the 64 KiB stage a workgroup needs ~64 KiB
// of LDS, so two fit per CU.
//   2^28 random 16-B rows; bins = top bits of radix_hash; (workgroup, bin)
//   owns a contiguous region (no bucket chaining: the write pattern only).
//   Checked: every row lands once (count + xor checksum over the regions).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o direct_micro direct_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "hj_internal.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
using hj::fmix64;
using hj::radix_hash;

__global__ void k_fill(ulonglong2 *r, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) r[i] = make_ulonglong2(fmix64(i * 7 + 1), i);
}

// MODE 0: direct per-lane stores + LDS tails (the candidate)
// MODE 1: as 0 without stores (loads + LDS work only)
// MODE 2: loads + count only (no stores, no tails)
template <int NT, int IT, int FB, int MODE>
__global__ __launch_bounds__(NT) void k_direct(const ulonglong2 *in, ulonglong2 *out, u64 n, u64 cap, unsigned *fills) {
    constexpr unsigned F = 1u << FB, L = 8, T = NT * IT;
    __shared__ ulonglong2 tail[F * (L - 1)];
    __shared__ unsigned cnt[F], fill[F];
    const unsigned tiles = (unsigned)((n + T - 1) / T);
    const unsigned t0 = (unsigned)((u64)blockIdx.x * tiles / gridDim.x);
    const unsigned t1 = (unsigned)((u64)(blockIdx.x + 1) * tiles / gridDim.x);
    for (unsigned b = threadIdx.x; b < F; b += NT) cnt[b] = fill[b] = 0u;
    ulonglong2 *reg = out + (u64)blockIdx.x * F * cap;   // bin b: reg + b * cap
    ulonglong2 row[IT], nrow[IT];
    unsigned br[IT];
    auto load = [&](unsigned t, ulonglong2 (&r)[IT]) {
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const u64 x = (u64)t * T + (u64)i * NT + threadIdx.x;
            r[i] = x < n ? in[x] : make_ulonglong2(0ull, ~0ull);
        }
    };
    if (t0 < t1) load(t0, row);
    __syncthreads();
    for (unsigned t = t0; t < t1; ++t) {
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            if (row[i].y == ~0ull) { br[i] = ~0u; continue; }
            const unsigned b = (unsigned)(radix_hash(row[i].x) >> (64 - FB));
            br[i] = (b << 16) | atomicAdd(&cnt[b], 1u);
        }
        __syncthreads();
        if (t + 1 < t1) load(t + 1, nrow);
        if constexpr (MODE != 2) {
            // rows below their bin's last complete line go out now; the rest
            // wait (new tail) until the old tails are read
#pragma unroll
            for (int i = 0; i < IT; ++i) {
                if (br[i] == ~0u) continue;
                const unsigned b = br[i] >> 16, p = fill[b] + (br[i] & 0xffffu);
                const unsigned e = (fill[b] + cnt[b]) & ~(L - 1);
                if (p < e) {
                    if constexpr (MODE == 0) reg[(u64)b * cap + p] = row[i];
                    br[i] = ~0u;
                } else {
                    br[i] = (b << 16) | (p - e);
                }
            }
            for (unsigned q = threadIdx.x; q < F * (L - 1); q += NT) {
                const unsigned b = q / (L - 1), i = q - b * (L - 1);
                const unsigned f = fill[b], tl = f & (L - 1);
                if (i >= tl) continue;
                const unsigned p = f - tl + i;
                if (p >= ((f + cnt[b]) & ~(L - 1))) continue;
                if constexpr (MODE == 0) reg[(u64)b * cap + p] = tail[q];
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < IT; ++i)
                if (br[i] != ~0u) tail[(br[i] >> 16) * (L - 1) + (br[i] & 0xffffu)] = row[i];
        }
        for (unsigned b = threadIdx.x; b < F; b += NT) {
            fill[b] += cnt[b];
            cnt[b] = 0u;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < IT; ++i) row[i] = nrow[i];
    }
    // close: the last partial lines
    if constexpr (MODE == 0)
        for (unsigned q = threadIdx.x; q < F * (L - 1); q += NT) {
            const unsigned b = q / (L - 1), i = q - b * (L - 1);
            const unsigned f = fill[b], tl = f & (L - 1);
            if (i < tl) reg[(u64)b * cap + (f - tl + i)] = tail[q];
        }
    for (unsigned b = threadIdx.x; b < F; b += NT) fills[blockIdx.x * F + b] = fill[b];
}

__global__ void k_check(const ulonglong2 *out, u64 cap, const unsigned *fills, unsigned regions, u64 *res) {
    const unsigned r = blockIdx.x;
    if (r >= regions) return;
    u64 x = 0, c = 0;
    for (unsigned i = threadIdx.x; i < fills[r]; i += 256) {
        const ulonglong2 v = out[(u64)r * cap + i];
        x ^= fmix64(v.x + 3 * v.y);
        ++c;
    }
    atomicXor(&res[0], x);
    atomicAdd(&res[1], c);
}

__global__ void k_ref(const ulonglong2 *in, u64 n, u64 *res) {
    u64 x = 0;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) x ^= fmix64(in[i].x + 3 * in[i].y);
    atomicXor(&res[2], x);
}

// coalesced reference: read, then write the tile in aligned 128-B runs (ws_micro SPREAD 5 shape)
template <int NT, int IT>
__global__ __launch_bounds__(NT) void k_coal(const ulonglong2 *in, ulonglong2 *out, u64 n) {
    constexpr unsigned T = NT * IT;
    const unsigned tiles = (unsigned)(n / T);
    const unsigned t0 = (unsigned)((u64)blockIdx.x * tiles / gridDim.x);
    const unsigned t1 = (unsigned)((u64)(blockIdx.x + 1) * tiles / gridDim.x);
    for (unsigned t = t0; t < t1; ++t) {
        ulonglong2 r[IT];
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = in[(u64)t * T + (u64)i * NT + threadIdx.x];
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const unsigned j = i * NT + threadIdx.x, b = j / 8;
            out[(((u64)(t - t0) * gridDim.x + blockIdx.x) * (T / 8) + b) * 8 + (j & 7)] = r[i];
        }
    }
}

// contiguous copy with the next tile's loads issued before this tile's stores
template <int NT, int IT, bool NTS>
__global__ __launch_bounds__(NT) void k_copy_pf(const ulonglong2 *in, ulonglong2 *out, u64 n) {
    constexpr unsigned T = NT * IT;
    const unsigned tiles = (unsigned)(n / T);
    const unsigned t0 = (unsigned)((u64)blockIdx.x * tiles / gridDim.x);
    const unsigned t1 = (unsigned)((u64)(blockIdx.x + 1) * tiles / gridDim.x);
    ulonglong2 r[IT], q[IT];
    if (t0 < t1)
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = in[(u64)t0 * T + (u64)i * NT + threadIdx.x];
    for (unsigned t = t0; t < t1; ++t) {
        if (t + 1 < t1)
#pragma unroll
            for (int i = 0; i < IT; ++i) q[i] = in[(u64)(t + 1) * T + (u64)i * NT + threadIdx.x];
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            ulonglong2 *d = out + (u64)t * T + (u64)i * NT + threadIdx.x;
            if constexpr (NTS) __builtin_nontemporal_store(r[i].x, &d->x), __builtin_nontemporal_store(r[i].y, &d->y);
            else *d = r[i];
        }
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = q[i];
    }
}

int main() {
    const u64 n = 1ull << 28;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    ulonglong2 *in, *out;
    unsigned *fills;
    u64 *res;
    const u64 out_rows = 3ull << 28;
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, out_rows * 16));
    CK(hipMalloc(&fills, 4u << 20));
    CK(hipMalloc(&res, 64));
    hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, in, n);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-52s %7.3f ms  %7.1f GB/s (32 B/row)\n", name, ms, 32.0 * n / ms / 1e6);
    };
    auto check = [&](const char *name, unsigned regions, u64 cap) {
        CK(hipMemset(res, 0, 64));
        hipLaunchKernelGGL(k_check, dim3(regions), dim3(256), 0, 0, out, cap, fills, regions, res);
        hipLaunchKernelGGL(k_ref, dim3(4096), dim3(256), 0, 0, in, n, res);
        u64 h[3];
        CK(hipMemcpy(h, res, 24, hipMemcpyDeviceToHost));
        printf("  check %-44s rows %llu/%llu  %s\n", name, h[1], n, (h[1] == n && h[0] == h[2]) ? "OK" : "MISMATCH");
    };
#define RUN(NT, IT, FB, MODE, WPC, NAME)                                                                       \
    {                                                                                                         \
        const unsigned G = (unsigned)cus * WPC;                                                               \
        const u64 cap = ((n / G) >> FB) * 3 / 2 / 8 * 8 + 64;                                                 \
        if ((u64)G * (1u << FB) * cap > out_rows) { printf("skip %s\n", NAME); }                             \
        else {                                                                                                \
            timeit(NAME, [&] { hipLaunchKernelGGL((k_direct<NT, IT, FB, MODE>), dim3(G), dim3(NT), 0, 0, in, out, n, cap, fills); }); \
            if (MODE == 0) check(NAME, G << FB, cap);                                                         \
        }                                                                                                     \
    }
    timeit("coalesced 128-B runs, 1024 x 8, 1/CU", [&] { hipLaunchKernelGGL((k_coal<1024, 8>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
    timeit("coalesced 128-B runs, 512 x 8, 2/CU", [&] { hipLaunchKernelGGL((k_coal<512, 8>), dim3(2 * cus), dim3(512), 0, 0, in, out, n); });
    timeit("hipMemcpyAsync D2D 4 GiB", [&] { CK(hipMemcpyAsync(out, in, n * 16, hipMemcpyDeviceToDevice, 0)); });
    timeit("copy, next tile prefetched, 1024 x 4, 1/CU", [&] { hipLaunchKernelGGL((k_copy_pf<1024, 4, false>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
    timeit("copy, next tile prefetched, 512 x 4, 2/CU", [&] { hipLaunchKernelGGL((k_copy_pf<512, 4, false>), dim3(2 * cus), dim3(512), 0, 0, in, out, n); });
    timeit("copy, next tile prefetched, 256 x 4, 4/CU", [&] { hipLaunchKernelGGL((k_copy_pf<256, 4, false>), dim3(4 * cus), dim3(256), 0, 0, in, out, n); });
    timeit("copy, next tile prefetched, 256 x 8, 4/CU", [&] { hipLaunchKernelGGL((k_copy_pf<256, 8, false>), dim3(4 * cus), dim3(256), 0, 0, in, out, n); });
    timeit("copy, next tile prefetched, 256 x 4, 8/CU", [&] { hipLaunchKernelGGL((k_copy_pf<256, 4, false>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
    timeit("copy, prefetched, nt stores, 256 x 4, 4/CU", [&] { hipLaunchKernelGGL((k_copy_pf<256, 4, true>), dim3(4 * cus), dim3(256), 0, 0, in, out, n); });
    timeit("copy, prefetched, nt stores, 1024 x 4, 1/CU", [&] { hipLaunchKernelGGL((k_copy_pf<1024, 4, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
    RUN(1024, 4, 9, 0, 1, "direct 512 bins, 1024 x 4, 1/CU");
    RUN(512, 4, 9, 0, 2, "direct 512 bins, 512 x 4, 2/CU");

    return 0;
}
