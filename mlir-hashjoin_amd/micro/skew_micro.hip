// skew_micro.hip -- why is C4's S pass 2 (2.05 ms) slower than R's (1.55)?
// The product's 8-bit bucketed pass (k_pass small variant: 512 threads,
// 2048-row tiles, 2 workgroups per CU) over the bucketed output of a 9-bit
// first pass of 2^28 packed rows, uniform keys vs C4-like skew (about 3 % of
// the rows on three hot keys: 1.6 / 0.9 / 0.6 %, the top of Zipf(0.9) at
// 2^28).  Prints the pass time, per-workgroup phase totals (s_memtime, ABL 8)
// and the slowest workgroups' tiles and phases.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o skew_micro skew_micro.hip
#include "../csrc/hj_radix.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

__global__ void k_fill(ulonglong2 *r, u64 n, int skew) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    u64 k = fmix64(i * 7 + 1);
    if (skew) {
        const unsigned j = (unsigned)(fmix64(i ^ 0x5EED) % 1000u);
        if (j < 31) k = j < 16 ? 11ull : (j < 25 ? 22ull : 33ull);
    }
    r[i] = make_ulonglong2(k, i);
}

int main() {
    const u64 n = 1ull << 28;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    ulonglong2 *in, *out;
    unsigned *bbin, *bfill, *nb, *wst;
    const u64 maxb = n / 256 + (1u << 20);
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, maxb * 512 * 16));
    CK(hipMalloc(&bbin, maxb * 4));
    CK(hipMalloc(&bfill, maxb * 4));
    CK(hipMalloc(&nb, 64));
    CK(hipMalloc(&wst, 1025 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    RadixPlan p1{};
    p1.passes = 1;
    p1.bits[0] = 9;
    p1.pbl[0] = kPassPbl;
    p1.total_bits = 9;
    const int P1 = 512, P2 = P1 << 8;
    RadixNeed nd = radix_need((long long)n, p1, true);
    BucketSet b1;
    CK(hipMalloc(&b1.rows, nd.rows * 16));
    CK(hipMalloc(&b1.bbin, nd.buckets * 4));
    CK(hipMalloc(&b1.bfill, nd.buckets * 4));
    CK(hipMalloc(&b1.rstart, (P1 + 1) * 8));
    b1.max_buckets = (unsigned)nd.buckets;
    b1.max_rows = nd.rows;
    b1.max_runs = (nd.rows >> kRunLog) + nd.buckets;
    CK(hipMalloc(&b1.runs, (b1.max_runs + kRunPad) * 8));
    RadixWork ws{};
    CK(hipMalloc(&ws.nb, 64));
    CK(hipMalloc(&ws.pcur, (P2 + 1) * 8));
    CK(hipMalloc(&ws.rcur, (P2 + 1) * 8));
    CK(hipMalloc(&ws.tile_start, (P2 + 1) * 4));
    CK(hipMalloc(&ws.tile_owner, radix_tiles((long long)n, P2) * 4));
    CK(hipMalloc(&ws.tdesc, radix_tiles((long long)n, P2) * 16));
    CK(hipMalloc(&ws.wstart, 1025 * 4));
    CK(hipMalloc(&ws.scan_sums, (P2 / 8192 + 2) * 8));
    CK(hipMalloc(&ws.scan_state, (P2 / 1024 + 4) * 8));
    constexpr int NT = kSmallPassThreads, FM = kSmallFan, IT = kPassRows, TR = NT * IT;
    const unsigned grid = 2u * (unsigned)cus;
    u64 *prof;
    CK(hipMalloc(&prof, grid * 8 * sizeof(u64)));
    for (int skew : {0, 1}) {
        hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, in, n, skew);
        CK(hipMemset(ws.scan_state, 0, (P2 / 1024 + 4) * 8));
        SrcDev src{};
        src.form = kPacked64;
        src.key = in;
        src.n = (long long)n;
        CK(radix_partition(src, true, p1, ws, b1, 0));
        chunk_map(b1.rstart, nullptr, P1, (unsigned)(TR >> kRunLog), ws.tile_start, ws.tile_owner, ws.pcur,
                  ws.scan_sums, 0);
        const u64 tb = radix_tiles((long long)n, P1);
        hipLaunchKernelGGL(k_tile_desc, dim3(blocks_for(tb, 256)), dim3(256), 0, 0, (const unsigned *)ws.tile_start,
                           (const unsigned *)ws.tile_owner, (const u64 *)b1.rstart, P1, (unsigned)tb,
                           (TileDesc *)ws.tdesc, (unsigned)(TR >> kRunLog));
        CK(hipDeviceSynchronize());
        unsigned ntiles = 0;
        CK(hipMemcpy(&ntiles, ws.tile_start + P1, 4, hipMemcpyDeviceToHost));
        std::vector<u64> rs(P1 + 1);
        CK(hipMemcpy(rs.data(), b1.rstart, (P1 + 1) * 8, hipMemcpyDeviceToHost));
        u64 mx = 0;
        for (int p = 0; p < P1; ++p) mx = std::max(mx, rs[p + 1] - rs[p]);
        printf("== skew %d: pass-1 segments 512, largest %llu runs (mean %.0f); %u pass-2 tiles of %d rows\n", skew, mx,
               rs[P1] / 512.0, ntiles, TR);
        PassArgs b{};
        b.n = n;
        b.in_rows = b1.rows;
        b.in_runs = b1.runs;
        b.in_rstart = b1.rstart;
        b.in_max_rows = b1.max_rows;
        b.in_max_runs = b1.max_runs;
        b.tile_start = ws.tile_start;
        b.tdesc = (const TileDesc *)ws.tdesc;
        b.nseg = P1;
        b.out_rows = out;
        b.bbin = bbin;
        b.bfill = bfill;
        b.nb = nb;
        b.max_buckets = (unsigned)maxb;
        b.wstart = wst;
        b.out_pbl = kFinalPbl;
        b.fbits = 8;
        b.shift = 64 - 17;
        b.tile_rows = TR;
        auto launch = [&](bool profd) {
            hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, b, true, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);
            if (profd) hipLaunchKernelGGL((k_pass<true, kBucketed, 8, false, NT, FM>), dim3(grid), dim3(NT), 0, 0, b);
            else hipLaunchKernelGGL((k_pass<true, kBucketed, 0, false, NT, FM>), dim3(grid), dim3(NT), 0, 0, b);
        };
        launch(false);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 5; ++i) launch(false);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("pass 2 (product shape: %d threads, %d bins, %d-row tiles, %u workgroups): %.3f ms\n", NT, FM, TR, grid,
               ms / 5);
        CK(hipMemset(prof, 0, grid * 8 * sizeof(u64)));
        b.prof = prof;
        launch(true);
        CK(hipDeviceSynchronize());
        b.prof = nullptr;
        std::vector<u64> h(grid * 8);
        CK(hipMemcpy(h.data(), prof, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
        std::vector<unsigned> ts(P1 + 1);
        CK(hipMemcpy(ts.data(), ws.tile_start, (P1 + 1) * 4, hipMemcpyDeviceToHost));
        const char *names[5] = {"count", "scan", "scatter", "stores", "bookkeeping"};
        std::vector<std::pair<double, unsigned>> wt(grid);
        double mean[5] = {0, 0, 0, 0, 0};
        for (unsigned g = 0; g < grid; ++g) {
            double t = 0;
            for (int k = 0; k < 5; ++k) {
                t += (double)h[g * 8 + k];
                mean[k] += (double)h[g * 8 + k] / grid;
            }
            wt[g] = {t, g};
        }
        std::sort(wt.begin(), wt.end());
        printf("  mean phases:");
        for (int k = 0; k < 5; ++k) printf(" %s %.0f", names[k], mean[k]);
        printf("\n  workgroup totals (cycles): min %.0f median %.0f p90 %.0f max %.0f\n", wt[0].first, wt[grid / 2].first,
               wt[grid * 9 / 10].first, wt[grid - 1].first);
        for (unsigned r = grid - 6; r < grid; ++r) {
            const unsigned g = wt[r].second;
            const unsigned t0 = (unsigned)((u64)g * ntiles / grid), t1 = (unsigned)((u64)(g + 1) * ntiles / grid);
            const int seg0 = (int)(std::upper_bound(ts.begin(), ts.end(), t0) - ts.begin()) - 1;
            printf("  wg %4u (tiles %u-%u, first segment %d):", g, t0, t1, seg0);
            for (int k = 0; k < 5; ++k) printf(" %s %llu", names[k], h[g * 8 + k]);
            printf("\n");
        }
    }
    return 0;
}
