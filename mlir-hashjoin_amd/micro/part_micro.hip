// part_micro.hip -- what limits a radix-partition pass on gfx950?
// n = 2^28 packed 16-B rows.  Variants (each timed with hipEvents):
//   copy          : row-for-row 16-B copy (streaming roofline)
//   keys          : read the key half of each row, reduce (read-only roofline)
//   hist_lds      : + LDS atomic histogram (512 bins), one count row per tile
//   sort_local    : full tile counting sort in LDS, rows written back into the
//                   tile's own region (LDS cost, perfect write locality)
//   scatter_runs  : same sort, rows written as runs of ~8 into 512 far-apart
//                   bin regions (the real partition write pattern)
//   direct_runs   : no LDS staging: each lane writes its row straight to
//                   (bin region + tile slot + rank)  (L2 write combining)
//   *_t2048       : the same with 2048-row tiles / 256 threads (more WGs/CU)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;

__global__ __launch_bounds__(256) void k_copy(const ulonglong2 *a, ulonglong2 *b, u64 n) {
    u64 i = (u64)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (i + j * 256 < n) b[i + j * 256] = a[i + j * 256];
}

__global__ __launch_bounds__(512) void k_keys(const ulonglong2 *a, u64 n, u64 *sink) {
    u64 base = (u64)blockIdx.x * 4096 + threadIdx.x;
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (base + j * 512 < n) acc += a[base + j * 512].x;
    if (acc == 0x1234567ull) *sink = acc;
}

template <int TILE, int NT>
__global__ __launch_bounds__(NT) void k_hist_lds(const ulonglong2 *a, u64 n, unsigned *hist) {
    __shared__ unsigned cnt[512];
    for (int b = threadIdx.x; b < 512; b += NT) cnt[b] = 0;
    __syncthreads();
    u64 base = (u64)blockIdx.x * TILE + threadIdx.x;
#pragma unroll
    for (int j = 0; j < TILE / NT; ++j)
        if (base + j * NT < n) atomicAdd(&cnt[(a[base + j * NT].x * 0x9E3779B97F4A7C15ull) >> 55], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < 512; b += NT) hist[(u64)blockIdx.x * 512 + b] = cnt[b];
}

// MODE 0: write back into the tile region; 1: runs into bin regions via LDS staging;
// MODE 2: direct from registers to bin regions (no staging)
template <int TILE, int NT, int MODE>
__global__ __launch_bounds__(NT) void k_sort(const ulonglong2 *a, ulonglong2 *out, u64 n) {
    constexpr int IT = TILE / NT;
    __shared__ ulonglong2 stage[MODE == 2 ? 1 : TILE];
    __shared__ unsigned short sb[MODE == 2 ? 1 : TILE];
    __shared__ unsigned cnt[512];
    __shared__ unsigned start[512];
    const u64 tile = blockIdx.x;
    const u64 ntiles = gridDim.x;
    for (int b = threadIdx.x; b < 512; b += NT) cnt[b] = 0;
    __syncthreads();
    ulonglong2 row[IT];
    unsigned br[IT];
    u64 base = tile * TILE + threadIdx.x;
#pragma unroll
    for (int j = 0; j < IT; ++j) row[j] = a[base + j * NT];
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        unsigned b = (unsigned)((row[j].x * 0x9E3779B97F4A7C15ull) >> 55);
        br[j] = (b << 16) | atomicAdd(&cnt[b], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        unsigned c[8], s = 0;
        for (int j = 0; j < 8; ++j) { c[j] = cnt[threadIdx.x * 8 + j]; s += c[j]; }
        unsigned x = s;
        for (int o = 1; o < 64; o <<= 1) { unsigned y = __shfl_up(x, o, 64); if ((int)threadIdx.x >= o) x += y; }
        unsigned run = x - s;
        for (int j = 0; j < 8; ++j) { start[threadIdx.x * 8 + j] = run; run += c[j]; }
    }
    __syncthreads();
    // bin region b: rows [b * n/512, (b+1) * n/512); this tile's slot: tile * (TILE/512) rows (+ rank)
    const u64 region = n / 512, slot = TILE / 512;
    if constexpr (MODE == 2) {
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned b = br[j] >> 16, r = br[j] & 0xffff;
            u64 dst = (u64)b * region + tile * slot + (r < slot ? r : slot - 1);
            out[dst] = row[j];
        }
    } else {
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned b = br[j] >> 16;
            unsigned pos = start[b] + (br[j] & 0xffff);
            stage[pos] = row[j];
            sb[pos] = (unsigned short)b;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned i = j * NT + threadIdx.x;
            if (MODE == 0) {
                out[tile * TILE + i] = stage[i];
            } else {
                unsigned b = sb[i], r = i - start[b];
                out[(u64)b * region + tile * slot + (r < slot ? r : slot - 1)] = stage[i];
            }
        }
    }
    (void)ntiles;
}

// Stripe variant: a workgroup sorts K consecutive tiles; each bin's rows from
// the whole stripe are contiguous in the output (per-bin running cursor), so
// tile k+1's run continues tile k's partial line in the same XCD's L2.
template <int TILE, int NT, int K, int FB>
__global__ __launch_bounds__(NT) void k_stripe(const ulonglong2 *a, ulonglong2 *out, u64 n) {
    constexpr int IT = TILE / NT;
    constexpr int F = 1 << FB;
    __shared__ ulonglong2 stage[TILE];
    __shared__ unsigned short sb[TILE];
    __shared__ unsigned cnt[F];
    __shared__ unsigned start[F];
    __shared__ unsigned cur[F];
    const u64 stripe = blockIdx.x;
    const u64 region = n / F, sslot = (u64)K * TILE / F;
    for (int b = threadIdx.x; b < F; b += NT) cur[b] = 0;
    for (int k = 0; k < K; ++k) {
        for (int b = threadIdx.x; b < F; b += NT) cnt[b] = 0;
        __syncthreads();
        ulonglong2 row[IT];
        unsigned br[IT];
        u64 base = (stripe * K + k) * TILE + threadIdx.x;
#pragma unroll
        for (int j = 0; j < IT; ++j) row[j] = a[base + j * NT];
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned b = (unsigned)((row[j].x * 0x9E3779B97F4A7C15ull) >> (64 - FB));
            br[j] = (b << 16) | atomicAdd(&cnt[b], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            constexpr int PL = (F + 63) / 64;
            unsigned c[PL], s = 0;
            for (int j = 0; j < PL; ++j) { int b = threadIdx.x * PL + j; c[j] = b < F ? cnt[b] : 0; s += c[j]; }
            unsigned x = s;
            for (int o = 1; o < 64; o <<= 1) { unsigned y = __shfl_up(x, o, 64); if ((int)threadIdx.x >= o) x += y; }
            unsigned run = x - s;
            for (int j = 0; j < PL; ++j) { int b = threadIdx.x * PL + j; if (b < F) start[b] = run; run += c[j]; }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned b = br[j] >> 16;
            unsigned pos = start[b] + (br[j] & 0xffff);
            stage[pos] = row[j];
            sb[pos] = (unsigned short)b;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned i = j * NT + threadIdx.x;
            unsigned b = sb[i];
            u64 r = cur[b] + (i - start[b]);
            out[(u64)b * region + stripe * sslot + (r < sslot ? r : sslot - 1)] = stage[i];
        }
        __syncthreads();
        for (int b = threadIdx.x; b < F; b += NT) cur[b] += cnt[b];
    }
}

int main() {
    const u64 n = 1ull << 28;
    ulonglong2 *a, *b;
    unsigned *hist;
    u64 *sink;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&hist, (n / 2048) * 512 * 4));
    CK(hipMalloc(&sink, 64));
    // random keys
    {
        ulonglong2 *h = (ulonglong2 *)malloc(1 << 24);
        u64 x = 88172645463325252ull;
        for (int i = 0; i < (1 << 20); ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = make_ulonglong2(x, i); }
        for (u64 o = 0; o < n; o += (1 << 20)) CK(hipMemcpy(a + o, h, 1 << 24, hipMemcpyHostToDevice));
        free(h);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, double bytes, auto fn) {
        fn(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
        printf("%-22s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    const double rw = 2.0 * n * 16, rd = n * 16.0;
    run("copy", rw, [&] { hipLaunchKernelGGL(k_copy, dim3(n / 1024), dim3(256), 0, 0, a, b, n); });
    run("keys (16B rows)", rd, [&] { hipLaunchKernelGGL(k_keys, dim3(n / 4096), dim3(512), 0, 0, a, n, sink); });
    run("hist_lds t4096", rd, [&] { hipLaunchKernelGGL((k_hist_lds<4096, 512>), dim3(n / 4096), dim3(512), 0, 0, a, n, hist); });
    run("hist_lds t2048", rd, [&] { hipLaunchKernelGGL((k_hist_lds<2048, 256>), dim3(n / 2048), dim3(256), 0, 0, a, n, hist); });
    run("sort_local t4096", rw, [&] { hipLaunchKernelGGL((k_sort<4096, 512, 0>), dim3(n / 4096), dim3(512), 0, 0, a, b, n); });
    run("scatter_runs t4096", rw, [&] { hipLaunchKernelGGL((k_sort<4096, 512, 1>), dim3(n / 4096), dim3(512), 0, 0, a, b, n); });
    run("direct_runs t4096", rw, [&] { hipLaunchKernelGGL((k_sort<4096, 512, 2>), dim3(n / 4096), dim3(512), 0, 0, a, b, n); });
    run("sort_local t2048", rw, [&] { hipLaunchKernelGGL((k_sort<2048, 256, 0>), dim3(n / 2048), dim3(256), 0, 0, a, b, n); });
    run("scatter_runs t2048", rw, [&] { hipLaunchKernelGGL((k_sort<2048, 256, 1>), dim3(n / 2048), dim3(256), 0, 0, a, b, n); });
    run("direct_runs t2048", rw, [&] { hipLaunchKernelGGL((k_sort<2048, 256, 2>), dim3(n / 2048), dim3(256), 0, 0, a, b, n); });
    run("sort_local t1024", rw, [&] { hipLaunchKernelGGL((k_sort<1024, 256, 0>), dim3(n / 1024), dim3(256), 0, 0, a, b, n); });
    run("scatter_runs t8192", rw, [&] { hipLaunchKernelGGL((k_sort<8192, 1024, 1>), dim3(n / 8192), dim3(1024), 0, 0, a, b, n); });
    run("stripe t4096 K8 F512", rw, [&] { hipLaunchKernelGGL((k_stripe<4096, 512, 8, 9>), dim3(n / 4096 / 8), dim3(512), 0, 0, a, b, n); });
    run("stripe t4096 K16 F512", rw, [&] { hipLaunchKernelGGL((k_stripe<4096, 512, 16, 9>), dim3(n / 4096 / 16), dim3(512), 0, 0, a, b, n); });
    run("stripe t4096 K32 F512", rw, [&] { hipLaunchKernelGGL((k_stripe<4096, 512, 32, 9>), dim3(n / 4096 / 32), dim3(512), 0, 0, a, b, n); });
    run("stripe t4096 K16 F256", rw, [&] { hipLaunchKernelGGL((k_stripe<4096, 512, 16, 8>), dim3(n / 4096 / 16), dim3(512), 0, 0, a, b, n); });
    run("stripe t4096 K32 F256", rw, [&] { hipLaunchKernelGGL((k_stripe<4096, 512, 32, 8>), dim3(n / 4096 / 32), dim3(512), 0, 0, a, b, n); });
    run("stripe t2048 K32 F256", rw, [&] { hipLaunchKernelGGL((k_stripe<2048, 256, 32, 8>), dim3(n / 2048 / 32), dim3(256), 0, 0, a, b, n); });
    run("stripe t4096 K64 F128", rw, [&] { hipLaunchKernelGGL((k_stripe<4096, 512, 64, 7>), dim3(n / 4096 / 64), dim3(512), 0, 0, a, b, n); });
    return 0;
}
