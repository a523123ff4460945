// mall_micro.hip -- does the 256 MiB Infinity Cache absorb a write -> read
// hand-off between two kernels?  The question behind fusing S's second
// partition pass into the join (profiles/r02_probe_floor_analysis.md 4):
// pass 2 would write each chunk of its output into a small ring that the
// join reads back at once, instead of 4 GiB that go to HBM and back.
//
// Per chunk c of X bytes (4 GiB in all):
//   k_copy:    src[c]            -> mid(c)        (pass 2: read HBM, write)
//   k_combine: mid(c) ^ rr[c]    -> out[c]        (join: read mid + R, write pairs)
// MODE ring: mid(c) = ring + (c % 2) * X (reused, 2X bytes)
// MODE flat: mid(c) = big + c * X        (4 GiB, every line once)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o mall_micro mall_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
constexpr int kNT = 256, kUn = 4;

__global__ __launch_bounds__(kNT) void k_copy(const uint4 *src, uint4 *dst, u64 n) {
    const u64 stride = (u64)gridDim.x * kNT * kUn;
    for (u64 b = (u64)blockIdx.x * kNT * kUn + threadIdx.x; b < n; b += stride) {
        uint4 v[kUn];
#pragma unroll
        for (int i = 0; i < kUn; ++i) v[i] = b + i * kNT < n ? src[b + i * kNT] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < kUn; ++i)
            if (b + i * kNT < n) dst[b + i * kNT] = v[i];
    }
}

__global__ __launch_bounds__(kNT) void k_combine(const uint4 *a, const uint4 *r, uint4 *out, u64 n) {
    const u64 stride = (u64)gridDim.x * kNT * kUn;
    for (u64 b = (u64)blockIdx.x * kNT * kUn + threadIdx.x; b < n; b += stride) {
        uint4 x[kUn], y[kUn];
#pragma unroll
        for (int i = 0; i < kUn; ++i) {
            const bool ok = b + i * kNT < n;
            x[i] = ok ? a[b + i * kNT] : make_uint4(0, 0, 0, 0);
            y[i] = ok ? r[b + i * kNT] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < kUn; ++i)
            if (b + i * kNT < n)
                out[b + i * kNT] = make_uint4(x[i].x ^ y[i].x, x[i].y ^ y[i].y, x[i].z ^ y[i].z, x[i].w ^ y[i].w);
    }
}

int main(int argc, char **argv) {
    const u64 total = 4ull << 30;   // bytes per array
    const u64 n16 = total / 16;
    uint4 *src, *rr, *out, *big, *ring;
    CK(hipMalloc(&src, total));
    CK(hipMalloc(&rr, total));
    CK(hipMalloc(&out, total));
    CK(hipMalloc(&big, total));
    CK(hipMalloc(&ring, 512ull << 20));
    CK(hipMemset(src, 1, total));
    CK(hipMemset(rr, 2, total));
    CK(hipMemset(out, 0, total));
    CK(hipMemset(big, 0, total));
    CK(hipMemset(ring, 0, 512ull << 20));
    const int grid = 1024;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // whole-array baselines (one launch each)
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_copy, dim3(grid), dim3(kNT), 0, 0, src, big, n16);
        hipLaunchKernelGGL(k_combine, dim3(grid), dim3(kNT), 0, 0, big, rr, out, n16);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("whole   copy+combine 4 GiB: %.3f ms (20 GiB moved: %.2f TB/s)\n", ms, 20.0 * (1 << 30) / ms / 1e9);
    }
    const u64 xs[] = {8ull << 20, 16ull << 20, 32ull << 20, 64ull << 20, 128ull << 20, 256ull << 20};
    for (u64 X : xs) {
        const u64 nc = total / X, x16 = X / 16;
        for (int mode = 0; mode < 2; ++mode) {
            float best = 1e9f;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(e0));
                for (u64 c = 0; c < nc; ++c) {
                    uint4 *mid = mode == 0 ? ring + (c & 1) * x16 : big + c * x16;
                    hipLaunchKernelGGL(k_copy, dim3(grid), dim3(kNT), 0, 0, src + c * x16, mid, x16);
                    hipLaunchKernelGGL(k_combine, dim3(grid), dim3(kNT), 0, 0, mid, rr + c * x16, out + c * x16, x16);
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("chunk %4llu MiB %s: %.3f ms (%llu chunks, %llu launches)\n", X >> 20, mode == 0 ? "ring" : "flat", best,
                   nc, 2 * nc);
        }
    }
    return 0;
}
