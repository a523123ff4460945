// frontier_micro.hip -- does the partition pass's write pattern cost it the
// gap between the persistent copy (5.4-5.5 TB/s) and the flat copy (6.3)?
// The pass writes whole 128-B lines to one frontier per (workgroup, bin):
// 256 workgroups x 512 bins = 131k frontiers across the whole output, each
// advancing one line per tile.  Model write streams of 2^28 16-B rows (4 GiB)
// by persistent 1024-thread workgroups, one line per 8 lanes, 8 lines per
// wave store instruction, one line per bin per tile (4096 rows = 512 lines):
//   own     per-(workgroup, bin) regions (the pass's layout)
//   shared  one region per bin, the workgroups' lines of a tile adjacent
//           (line (k * G + w) of bin b: what a line claim on a shared
//           bucket per bin would give)
//   seq     the workgroup's lines contiguous (a streamed write)
// each write-only and with a streamed read of 4 GiB beside it (the pass's
// read side), plus the flat one-row-per-thread copy for reference.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o frontier_micro frontier_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
typedef ulonglong2 row_t;

constexpr int NT = 1024, IT = 4, TILE = NT * IT, LINES = TILE / 8, BINS = 512;

__device__ __forceinline__ void st_nt(row_t *p, row_t v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
}
__device__ __forceinline__ row_t ld_nt(const row_t *p) {
    return make_ulonglong2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
}

// MODE 0 own, 1 shared, 2 seq; RD: also stream-read a tile per tile
template <int MODE, bool RD>
__global__ __launch_bounds__(NT) void k_front(const row_t *in, row_t *out, u64 n, u64 *res) {
    const unsigned G = gridDim.x, w = blockIdx.x;
    const u64 tiles = n / TILE, tpw = tiles / G;   // tiles per workgroup (n a multiple of G * TILE)
    const unsigned lane8 = threadIdx.x & 7u, slot = threadIdx.x >> 3;   // 128 lines per instruction round
    u64 acc = 0;
    for (u64 k = 0; k < tpw; ++k) {
        row_t r[IT];
        if constexpr (RD) {
            const u64 t = (u64)w * tpw + k;
#pragma unroll
            for (int i = 0; i < IT; ++i) r[i] = ld_nt(in + t * TILE + (u64)i * NT + threadIdx.x);
        }
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const unsigned b = (unsigned)i * (NT / 8) + slot;   // this tile's line of bin b
            u64 line;
            if constexpr (MODE == 0) line = ((u64)w * BINS + b) * tpw + k;
            else if constexpr (MODE == 1) line = (u64)b * (tpw * G) + k * G + w;
            else line = ((u64)w * tpw + k) * LINES + b;
            const row_t v = RD ? r[i] : make_ulonglong2(line, k);
            st_nt(out + line * 8 + lane8, v);
        }
        if constexpr (RD) acc += r[0].x;
    }
    if (acc == 0x123456789ull) res[0] = acc;
}

__global__ __launch_bounds__(256) void k_flat(const row_t *in, row_t *out, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) st_nt(out + i, in[i]);
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const u64 n = 1ull << 28;
    if (n % ((u64)cus * TILE) != 0 && (n / TILE) % (u64)cus != 0) printf("note: %d CUs, n not a multiple\n", cus);
    const unsigned G = (unsigned)cus;
    const u64 nn = (n / TILE / G) * G * TILE;   // rows the persistent kernels cover
    row_t *in, *out;
    u64 *res;
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, n * 16));
    CK(hipMalloc(&res, 64));
    CK(hipMemset(in, 1, n * 16));
    CK(hipMemset(out, 0, n * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, u64 rows, double bpr, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 10;
        printf("%-44s %8.3f ms  %7.1f GB/s\n", name, ms, bpr * rows / ms / 1e6);
    };
    for (int rep = 0; rep < 2; ++rep) {
        timeit("write only, own frontiers (pass layout)", nn, 16, [&] { hipLaunchKernelGGL((k_front<0, false>), dim3(G), dim3(NT), 0, 0, in, out, nn, res); });
        timeit("write only, shared frontiers", nn, 16, [&] { hipLaunchKernelGGL((k_front<1, false>), dim3(G), dim3(NT), 0, 0, in, out, nn, res); });
        timeit("write only, sequential", nn, 16, [&] { hipLaunchKernelGGL((k_front<2, false>), dim3(G), dim3(NT), 0, 0, in, out, nn, res); });
        timeit("read + write, own frontiers (pass layout)", nn, 32, [&] { hipLaunchKernelGGL((k_front<0, true>), dim3(G), dim3(NT), 0, 0, in, out, nn, res); });
        timeit("read + write, shared frontiers", nn, 32, [&] { hipLaunchKernelGGL((k_front<1, true>), dim3(G), dim3(NT), 0, 0, in, out, nn, res); });
        timeit("read + write, sequential", nn, 32, [&] { hipLaunchKernelGGL((k_front<2, true>), dim3(G), dim3(NT), 0, 0, in, out, nn, res); });
        timeit("flat copy, 1 row per thread", n, 32, [&] { hipLaunchKernelGGL(k_flat, dim3(n / 256), dim3(256), 0, 0, in, out, n); });
    }
    CK(hipDeviceSynchronize());
    return 0;
}
