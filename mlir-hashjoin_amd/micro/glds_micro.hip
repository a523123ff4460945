// glds_micro.hip -- semantics check of the gfx950 LDS-DMA load
// (__builtin_amdgcn_global_load_lds, 16 B per lane) as the join's staging
// would use it: a wave loads one run (<= 64 rows of 16 B) from per-lane
// global addresses into a contiguous LDS block; lanes past the run's end are
// switched off (EXEC).  Checks: (1) lane i lands at base + 16 i, (2) an
// inactive lane writes nothing (the sentinel survives), (3) a counted
// s_waitcnt vmcnt + barrier makes the rows visible to every wave.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o glds_micro glds_micro.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
constexpr int kNT = 256, kRuns = 8;   // 8 runs per block, 2 per wave

__global__ __launch_bounds__(kNT) void k_glds(const uint4 *g, const unsigned *cnt, const unsigned *src, uint4 *out) {
    __shared__ uint4 buf[kRuns * 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kRuns * 64; i += kNT) buf[i] = make_uint4(0xdeadbeef, 0xdeadbeef, 0xdeadbeef, 0xdeadbeef);
    __syncthreads();
    for (int r = w; r < kRuns; r += kNT / 64) {
        const unsigned run = blockIdx.x * kRuns + r;
        const unsigned c = cnt[run];
        if ((unsigned)lane < c)
            __builtin_amdgcn_global_load_lds((const void *)(g + src[run] + lane), (void *)(buf + r * 64), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < kRuns * 64; i += kNT) out[(size_t)blockIdx.x * kRuns * 64 + i] = buf[i];
}

int main() {
    const int blocks = 64, runs = blocks * kRuns, rows = 1 << 20;
    std::vector<uint4> hg(rows);
    for (int i = 0; i < rows; ++i) hg[i] = make_uint4(i, i * 3u + 1, ~i, i ^ 0x5a5a5a5a);
    std::vector<unsigned> hc(runs), hs(runs);
    srand(7);
    for (int r = 0; r < runs; ++r) {
        hc[r] = r % 5 == 0 ? 64 : (unsigned)(rand() % 65);
        hs[r] = (unsigned)(rand() % (rows - 64));
    }
    uint4 *g, *out;
    unsigned *c, *s;
    CK(hipMalloc(&g, rows * sizeof(uint4)));
    CK(hipMalloc(&out, (size_t)runs * 64 * sizeof(uint4)));
    CK(hipMalloc(&c, runs * 4));
    CK(hipMalloc(&s, runs * 4));
    CK(hipMemcpy(g, hg.data(), rows * sizeof(uint4), hipMemcpyHostToDevice));
    CK(hipMemcpy(c, hc.data(), runs * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(s, hs.data(), runs * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_glds, dim3(blocks), dim3(kNT), 0, 0, g, c, s, out);
    CK(hipDeviceSynchronize());
    std::vector<uint4> ho((size_t)runs * 64);
    CK(hipMemcpy(ho.data(), out, ho.size() * sizeof(uint4), hipMemcpyDeviceToHost));
    long bad_rows = 0, bad_sentinel = 0;
    for (int r = 0; r < runs; ++r)
        for (unsigned l = 0; l < 64; ++l) {
            const uint4 v = ho[(size_t)r * 64 + l];
            if (l < hc[r]) {
                const uint4 e = hg[hs[r] + l];
                bad_rows += (v.x != e.x || v.y != e.y || v.z != e.z || v.w != e.w);
            } else {
                bad_sentinel += (v.x != 0xdeadbeef || v.w != 0xdeadbeef);
            }
        }
    printf("glds: %d runs, rows wrong %ld, inactive lanes that wrote %ld -> %s\n", runs, bad_rows, bad_sentinel,
           (bad_rows || bad_sentinel) ? "FAIL" : "OK");
    return (bad_rows || bad_sentinel) ? 1 : 0;
}
