// pass_micro.hip -- ablation of the partition pass kernel (k_pass) on 2^28
// packed 16-B rows, first pass (512 bins) and a 256-bin pass.
// (The ablation of the earlier kernel is kept in
// profiles/r01_micro_pass_ablation.txt; micro/ws_micro.hip isolates the
// write pattern.)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o pass_micro pass_micro.hip
#include "../csrc/hj_radix.hip"

#include <cstdio>
#include <vector>
#ifndef PHASE_ABL
#define PHASE_ABL 8
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

__global__ void k_fill(ulonglong2 *r, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) r[i] = make_ulonglong2(fmix64(i * 7 + 1), i);
}

int main() {
    const u64 n = 1ull << 28;
    ulonglong2 *in, *out;
    unsigned *bbin, *bfill, *nb;
    const u64 maxb = n / 256 + (1u << 20);
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, maxb * 512 * 16));
    CK(hipMalloc(&bbin, maxb * 4));
    CK(hipMalloc(&bfill, maxb * 4));
    CK(hipMalloc(&nb, 64));
    hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, in, n);
    CK(hipDeviceSynchronize());
    PassArgs a{};
    a.in.key = in;
    a.in.pay = nullptr;
    a.in.n = (long long)n;
    a.in.form = kPacked64;
    a.n = n;
    a.nseg = 1;
    a.out_rows = out;
    a.bbin = bbin;
    a.bfill = bfill;
    a.nb = nb;
    a.max_buckets = (unsigned)maxb;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned grid = pass_grid(n);
    auto run = [&](const char *name, auto launch) {
        CK(hipMemset(nb, 0, 4));
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 5; ++i) {
            CK(hipMemsetAsync(nb, 0, 4));
            launch();
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-40s %7.3f ms  %7.1f GB/s (32 B/row)\n", name, ms, 32.0 * n / ms / 1e6);
    };
    for (int fb : {9}) {
        a.fbits = fb;
        a.shift = 64 - fb;
        for (int pbl : {9}) {
            a.out_pbl = pbl;
            char nm[64];
            snprintf(nm, sizeof nm, "F%d PB%d k_pass", 1 << fb, 1 << pbl);
            run(nm, [&] { hipLaunchKernelGGL((k_pass<true, kPackedRow>), dim3(grid), dim3(kPassThreads), 0, 0, a); });
#define P(ABL, TXT)                                                                                       \
    snprintf(nm, sizeof nm, "F%d PB%d %s", 1 << fb, 1 << pbl, TXT);                                       \
    run(nm, [&] { hipLaunchKernelGGL((k_pass<true, kPackedRow, ABL>), dim3(grid), dim3(kPassThreads), 0, 0, a); })
            P(1, "no bucket atomic");
            P(2, "synthetic rows");
            P(4, "no row stores");
            P(6, "synthetic rows, no stores");
#undef P
            // phase times (cycles of s_memtime, summed over a workgroup's tiles, mean over workgroups)
            u64 *prof;
            CK(hipMalloc(&prof, grid * 8 * sizeof(u64)));
            CK(hipMemset(prof, 0, grid * 8 * sizeof(u64)));
            a.prof = prof;
            CK(hipMemset(nb, 0, 4));
            hipLaunchKernelGGL((k_pass<true, kPackedRow, PHASE_ABL>), dim3(grid), dim3(kPassThreads), 0, 0, a);
            CK(hipDeviceSynchronize());
            std::vector<u64> h(grid * 8);
            CK(hipMemcpy(h.data(), prof, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
            const char *names[6] = {"load wait + hash + LDS count", "scan + bucket atomic", "LDS scatter",
                                    "next loads issued + stores + tails", "new tails + bookkeeping", "-"};
            double tot = 0;
            double m[6];
            for (int k = 0; k < 5; ++k) {
                double acc = 0;
                for (unsigned g = 0; g < grid; ++g) acc += (double)h[g * 8 + k];
                m[k] = acc / grid;
                tot += m[k];
            }
            for (int k = 0; k < 5; ++k) printf("  phase %-38s %10.0f cycles  %5.1f %%\n", names[k], m[k], 100.0 * m[k] / tot);
            a.prof = nullptr;
            CK(hipFree(prof));
        }
    }
    return 0;
}
