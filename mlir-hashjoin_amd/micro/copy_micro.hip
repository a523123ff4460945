// copy_micro.hip -- how fast can this chip stream a copy?  The partition
// passes run within 2 % of a streamed copy of their bytes (1.553 ms per
// 2 x 4 GiB, 5.53 TB/s: direct_micro.hip); MI355X_MICROARCH.md quotes
// 6.29 TB/s for a float4 copy.  Variants: one 16-B row per thread over a
// full grid, grid-stride with U rows per thread in flight, persistent tiles
// with the next tile prefetched; plain / non-temporal loads and stores;
// 4 GiB and 1 GiB; plus read-only and write-only rates.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o copy_micro copy_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
typedef ulonglong2 row_t;

template <bool NTL>
__device__ __forceinline__ row_t ld(const row_t *p) {
    if constexpr (NTL) return make_ulonglong2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
    else return *p;
}
template <bool NTS>
__device__ __forceinline__ void st(row_t *p, row_t v) {
    if constexpr (NTS) __builtin_nontemporal_store(v.x, &p->x), __builtin_nontemporal_store(v.y, &p->y);
    else *p = v;
}

__global__ void k_fill(row_t *r, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) r[i] = make_ulonglong2(i * 0x9E3779B97F4A7C15ull, i);
}

// one row per thread, the whole grid (n / 256 workgroups)
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_flat(const row_t *in, row_t *out, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) st<NTS>(out + i, ld<NTL>(in + i));
}

// U rows per thread, the whole grid (n / (NT * U) workgroups), a workgroup's
// rows contiguous
template <int NT, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_flatu(const row_t *in, row_t *out, u64 n) {
    const u64 base = (u64)blockIdx.x * NT * U;
    row_t r[U];
#pragma unroll
    for (int i = 0; i < U; ++i) r[i] = ld<NTL>(in + base + (u64)i * NT + threadIdx.x);
#pragma unroll
    for (int i = 0; i < U; ++i) st<NTS>(out + base + (u64)i * NT + threadIdx.x, r[i]);
}

// persistent, tiles interleaved over workgroups (tile t = blockIdx + k * grid),
// the next tile's loads issued before this tile's stores
template <int NT, int IT, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_pfi(const row_t *in, row_t *out, u64 n) {
    constexpr u64 T = (u64)NT * IT;
    const u64 tiles = n / T;
    row_t r[IT], q[IT];
    u64 t = blockIdx.x;
    if (t < tiles)
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = ld<NTL>(in + t * T + (u64)i * NT + threadIdx.x);
    for (; t < tiles; t += gridDim.x) {
        const u64 tn = t + gridDim.x;
        if (tn < tiles)
#pragma unroll
            for (int i = 0; i < IT; ++i) q[i] = ld<NTL>(in + tn * T + (u64)i * NT + threadIdx.x);
#pragma unroll
        for (int i = 0; i < IT; ++i) st<NTS>(out + t * T + (u64)i * NT + threadIdx.x, r[i]);
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = q[i];
    }
}

// flat write-only / read-only: one row per thread, the whole grid
template <bool NTS>
__global__ __launch_bounds__(256) void k_flat_w(row_t *out, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) st<NTS>(out + i, make_ulonglong2(i, ~i));
}
template <bool NTL>
__global__ __launch_bounds__(256) void k_flat_r(const row_t *in, u64 n, u64 *res) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    const row_t r = ld<NTL>(in + i);
    if ((r.x ^ r.y) == 0x123456789ull) res[0] = i;
}

// U rows per thread per step, workgroup-contiguous chunks, grid-stride
template <int NT, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_gs(const row_t *in, row_t *out, u64 n) {
    constexpr u64 T = (u64)NT * U;
    for (u64 base = (u64)blockIdx.x * T; base < n; base += (u64)gridDim.x * T) {
        row_t r[U];
#pragma unroll
        for (int i = 0; i < U; ++i) r[i] = ld<NTL>(in + base + (u64)i * NT + threadIdx.x);
#pragma unroll
        for (int i = 0; i < U; ++i) st<NTS>(out + base + (u64)i * NT + threadIdx.x, r[i]);
    }
}

// persistent: a contiguous range of tiles per workgroup, next tile's loads
// issued before this tile's stores (the pass's loop shape)
template <int NT, int IT, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_pf(const row_t *in, row_t *out, u64 n) {
    constexpr u64 T = (u64)NT * IT;
    const u64 tiles = n / T;
    const u64 t0 = (u64)blockIdx.x * tiles / gridDim.x, t1 = (u64)(blockIdx.x + 1) * tiles / gridDim.x;
    row_t r[IT], q[IT];
    if (t0 < t1)
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = ld<NTL>(in + t0 * T + (u64)i * NT + threadIdx.x);
    for (u64 t = t0; t < t1; ++t) {
        if (t + 1 < t1)
#pragma unroll
            for (int i = 0; i < IT; ++i) q[i] = ld<NTL>(in + (t + 1) * T + (u64)i * NT + threadIdx.x);
#pragma unroll
        for (int i = 0; i < IT; ++i) st<NTS>(out + t * T + (u64)i * NT + threadIdx.x, r[i]);
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = q[i];
    }
}

// two 8-B columns in, one 16-B row out (pass 1's shape)
template <int NT, int U, bool NTS>
__global__ __launch_bounds__(NT) void k_cols(const u64 *k, const u64 *p, row_t *out, u64 n) {
    constexpr u64 T = (u64)NT * U * 2;   // rows per step: 2 per thread per slot (16-B column loads)
    for (u64 base = (u64)blockIdx.x * T; base < n; base += (u64)gridDim.x * T) {
        ulonglong2 a[U], b[U];
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const u64 x = base + ((u64)i * NT + threadIdx.x) * 2;
            a[i] = *(const ulonglong2 *)(k + x);
            b[i] = *(const ulonglong2 *)(p + x);
        }
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const u64 x = base + ((u64)i * NT + threadIdx.x) * 2;
            st<NTS>(out + x, make_ulonglong2(a[i].x, b[i].x));
            st<NTS>(out + x + 1, make_ulonglong2(a[i].y, b[i].y));
        }
    }
}

template <int NT, int U, bool NTL>
__global__ __launch_bounds__(NT) void k_read(const row_t *in, u64 n, u64 *res) {
    constexpr u64 T = (u64)NT * U;
    u64 s = 0;
    for (u64 base = (u64)blockIdx.x * T; base < n; base += (u64)gridDim.x * T) {
        row_t r[U];
#pragma unroll
        for (int i = 0; i < U; ++i) r[i] = ld<NTL>(in + base + (u64)i * NT + threadIdx.x);
#pragma unroll
        for (int i = 0; i < U; ++i) s += r[i].x ^ r[i].y;
    }
    if (s == 0x123456789ull) res[0] = s;   // keeps the loads
}

template <int NT, int U, bool NTS>
__global__ __launch_bounds__(NT) void k_write(row_t *out, u64 n) {
    constexpr u64 T = (u64)NT * U;
    for (u64 base = (u64)blockIdx.x * T; base < n; base += (u64)gridDim.x * T)
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const u64 x = base + (u64)i * NT + threadIdx.x;
            st<NTS>(out + x, make_ulonglong2(x, ~x));
        }
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const u64 nmax = 1ull << 28;   // 4 GiB of 16-B rows
    row_t *in, *out;
    u64 *res;
    CK(hipMalloc(&in, nmax * 16));
    CK(hipMalloc(&out, nmax * 16));
    CK(hipMalloc(&res, 64));
    hipLaunchKernelGGL(k_fill, dim3(nmax / 256), dim3(256), 0, 0, in, nmax);
    hipLaunchKernelGGL(k_fill, dim3(nmax / 256), dim3(256), 0, 0, out, nmax);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, u64 n, double bytes_per_row, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) fn();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 10;
        printf("%-56s n=2^%d %8.3f ms  %7.1f GB/s\n", name, 63 - __builtin_clzll(n), ms, bytes_per_row * n / ms / 1e6);
    };
    for (u64 n : {nmax}) {
        const unsigned gflat = (unsigned)(n / 256);
        timeit("flatu 256 x 2, nt store", n, 32, [&] { hipLaunchKernelGGL((k_flatu<256, 2, false, true>), dim3(n / 512), dim3(256), 0, 0, in, out, n); });
        timeit("flatu 256 x 4, nt store", n, 32, [&] { hipLaunchKernelGGL((k_flatu<256, 4, false, true>), dim3(n / 1024), dim3(256), 0, 0, in, out, n); });
        timeit("flatu 1024 x 1, nt store", n, 32, [&] { hipLaunchKernelGGL((k_flatu<1024, 1, false, true>), dim3(n / 1024), dim3(1024), 0, 0, in, out, n); });
        timeit("flatu 1024 x 4, nt store", n, 32, [&] { hipLaunchKernelGGL((k_flatu<1024, 4, false, true>), dim3(n / 4096), dim3(1024), 0, 0, in, out, n); });
        timeit("flatu 64 x 1, nt store", n, 32, [&] { hipLaunchKernelGGL((k_flatu<64, 1, false, true>), dim3(n / 64), dim3(64), 0, 0, in, out, n); });
        timeit("gs 256 x 1, 8/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 1, false, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("gs 256 x 1, 8/CU, nt load + store", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 1, true, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("gs 256 x 2, 8/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 2, false, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("gs 64 x 1, 32/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<64, 1, false, true>), dim3(32 * cus), dim3(64), 0, 0, in, out, n); });
        timeit("pf 256 x 1, 8/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pf<256, 1, false, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("pfi 1024 x 4, 1/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pfi<1024, 4, false, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("pfi 1024 x 2, 1/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pfi<1024, 2, false, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("pfi 1024 x 1, 1/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pfi<1024, 1, false, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("pfi 1024 x 4, 1/CU, nt load + store", n, 32, [&] { hipLaunchKernelGGL((k_pfi<1024, 4, true, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("pfi 256 x 1, 8/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pfi<256, 1, false, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("flat write only, nt", n, 16, [&] { hipLaunchKernelGGL((k_flat_w<true>), dim3(gflat), dim3(256), 0, 0, out, n); });
        timeit("flat write only, plain", n, 16, [&] { hipLaunchKernelGGL((k_flat_w<false>), dim3(gflat), dim3(256), 0, 0, out, n); });
        timeit("flat read only, nt", n, 16, [&] { hipLaunchKernelGGL((k_flat_r<true>), dim3(gflat), dim3(256), 0, 0, in, n, res); });
        timeit("flat read only, plain", n, 16, [&] { hipLaunchKernelGGL((k_flat_r<false>), dim3(gflat), dim3(256), 0, 0, in, n, res); });
        timeit("flat 1 row/thread, plain", n, 32, [&] { hipLaunchKernelGGL((k_flat<false, false>), dim3(gflat), dim3(256), 0, 0, in, out, n); });
        timeit("flat 1 row/thread, nt store", n, 32, [&] { hipLaunchKernelGGL((k_flat<false, true>), dim3(gflat), dim3(256), 0, 0, in, out, n); });
        timeit("flat 1 row/thread, nt load + store", n, 32, [&] { hipLaunchKernelGGL((k_flat<true, true>), dim3(gflat), dim3(256), 0, 0, in, out, n); });
        timeit("gs 256 x 4, 8/CU, plain", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 4, false, false>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("gs 256 x 4, 8/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 4, false, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("gs 256 x 8, 8/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 8, false, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("gs 256 x 4, 16/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 4, false, true>), dim3(16 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("gs 512 x 4, 4/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<512, 4, false, true>), dim3(4 * cus), dim3(512), 0, 0, in, out, n); });
        timeit("gs 1024 x 4, 2/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<1024, 4, false, true>), dim3(2 * cus), dim3(1024), 0, 0, in, out, n); });
        timeit("gs 1024 x 4, 1/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_gs<1024, 4, false, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("gs 256 x 4, 8/CU, nt load + store", n, 32, [&] { hipLaunchKernelGGL((k_gs<256, 4, true, true>), dim3(8 * cus), dim3(256), 0, 0, in, out, n); });
        timeit("pf 1024 x 4, 1/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pf<1024, 4, false, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("pf 1024 x 4, 1/CU, nt load + store", n, 32, [&] { hipLaunchKernelGGL((k_pf<1024, 4, true, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("pf 512 x 4, 2/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pf<512, 4, false, true>), dim3(2 * cus), dim3(512), 0, 0, in, out, n); });
        timeit("pf 1024 x 2, 1/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pf<1024, 2, false, true>), dim3(cus), dim3(1024), 0, 0, in, out, n); });
        timeit("pf 1024 x 4, 2/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_pf<1024, 4, false, true>), dim3(2 * cus), dim3(1024), 0, 0, in, out, n); });
        timeit("cols 256 x 2 (2 rows/slot), 8/CU, nt store", n, 32, [&] { hipLaunchKernelGGL((k_cols<256, 2, true>), dim3(8 * cus), dim3(256), 0, 0, (const u64 *)in, (const u64 *)in + n, out, n); });
        timeit("read only, gs 256 x 4, 8/CU", n, 16, [&] { hipLaunchKernelGGL((k_read<256, 4, false>), dim3(8 * cus), dim3(256), 0, 0, in, n, res); });
        timeit("read only, gs 256 x 8, 8/CU, nt", n, 16, [&] { hipLaunchKernelGGL((k_read<256, 8, true>), dim3(8 * cus), dim3(256), 0, 0, in, n, res); });
        timeit("write only, gs 256 x 4, 8/CU, plain", n, 16, [&] { hipLaunchKernelGGL((k_write<256, 4, false>), dim3(8 * cus), dim3(256), 0, 0, out, n); });
        timeit("write only, gs 256 x 4, 8/CU, nt", n, 16, [&] { hipLaunchKernelGGL((k_write<256, 4, true>), dim3(8 * cus), dim3(256), 0, 0, out, n); });
        timeit("hipMemcpyAsync D2D", n, 32, [&] { CK(hipMemcpyAsync(out, in, n * 16, hipMemcpyDeviceToDevice, 0)); });
    }
    CK(hipDeviceSynchronize());
    return 0;
}
