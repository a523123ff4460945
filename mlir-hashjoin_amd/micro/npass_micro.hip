// npass_micro.hip -- the i32 (reference-types) first partition pass as the
// product runs it on REF-B's 1e8 keys: k_pass<false, kCol32> in the
// half-size variant (512 threads, 256 bins, 8 rows per thread), with the
// ABL knobs of k_pass (2 synthetic rows, 4 no row stores, 8 phase times).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o npass_micro npass_micro.hip
#include "../csrc/hj_radix.hip"

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

__global__ void k_fill32(int *k, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) k[i] = (int)(1 + fmix64(i * 7 + 1) % 1000000000ull);
}

int main() {
    const u64 n = 100000000ull;
    constexpr int NT = kSmallPassThreads, FM = kSmallFan, IT = kSmallNarrowRows;
    int *keys;
    u64 *out;
    unsigned *bbin, *bfill, *nb, *wst;
    const int fb = 8, pbl = kPassPbl;
    const u64 maxb = n / (1u << pbl) + (1u << 20);
    CK(hipMalloc(&keys, n * 4));
    CK(hipMalloc(&out, (maxb << pbl) * 8));
    CK(hipMalloc(&bbin, maxb * 4));
    CK(hipMalloc(&bfill, maxb * 4));
    CK(hipMalloc(&nb, 64));
    CK(hipMalloc(&wst, 1025 * 4));
    hipLaunchKernelGGL(k_fill32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, keys, n);
    CK(hipDeviceSynchronize());
    PassArgs a{};
    a.in.key = keys;
    a.in.pay = nullptr;
    a.in.n = (long long)n;
    a.in.row_base = 0;
    a.in.form = kCol32;
    a.n = n;
    a.nseg = 1;
    a.out_rows = out;
    a.bbin = bbin;
    a.bfill = bfill;
    a.nb = nb;
    a.max_buckets = (unsigned)maxb;
    a.wstart = wst;
    a.fbits = fb;
    a.shift = 64 - fb;
    a.out_pbl = pbl;
    a.tile_rows = pass_tile_rows(fb, false);
    const unsigned grid = pass_grid(n, fb, false);
    printf("n %llu, grid %u, tile rows %u, PB %u\n", n, grid, a.tile_rows, 1u << pbl);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 10; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 10;
        printf("%-36s %7.4f ms  %7.1f GB/s (12 B/row)\n", name, ms, 12.0 * n / ms / 1e6);
    };
#define P(ABL, TXT)                                                                                           \
    run(TXT, [&] {                                                                                             \
        hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, a, false, grid, wst, (u64 *)nullptr,         \
                           (u64 *)nullptr, 0ull);                                                              \
        hipLaunchKernelGGL((k_pass<false, kCol32, ABL, false, NT, FM, IT>), dim3(grid), dim3(NT), 0, 0, a);   \
    })
    P(0, "product");
    P(2, "synthetic rows (no loads)");
    P(4, "no row stores");
    P(6, "synthetic rows, no stores");
#undef P
    u64 *prof;
    CK(hipMalloc(&prof, grid * 8 * sizeof(u64)));
    CK(hipMemset(prof, 0, grid * 8 * sizeof(u64)));
    a.prof = prof;
    hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, a, false, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);
    hipLaunchKernelGGL((k_pass<false, kCol32, 8, false, NT, FM, IT>), dim3(grid), dim3(NT), 0, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<u64> h(grid * 8);
    CK(hipMemcpy(h.data(), prof, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
    const char *names[5] = {"load wait + hash + LDS count", "scan + bucket ids", "LDS scatter + line map",
                            "next loads issued + stores", "new tails + bookkeeping"};
    double m[5], tot = 0;
    for (int k = 0; k < 5; ++k) {
        double acc = 0;
        for (unsigned g = 0; g < grid; ++g) acc += (double)h[g * 8 + k];
        m[k] = acc / grid;
        tot += m[k];
    }
    for (int k = 0; k < 5; ++k) printf("  phase %-36s %10.0f cycles  %5.1f %%\n", names[k], m[k], 100.0 * m[k] / tot);
    return 0;
}
