// pass_micro.hip -- ablation of the partition pass kernel (k_pass) on 2^28
// (round 4: the product's 1024-thread variant; the ABL knobs still apply)
// packed 16-B rows, first pass (512 bins) and a 256-bin pass.
// (The ablation of the earlier kernel is kept in
// profiles/r01_micro_pass_ablation.txt; micro/ws_micro.hip isolates the
// write pattern.)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o pass_micro pass_micro.hip
#include "../csrc/hj_radix.hip"

#include <cstdio>
#include <algorithm>
#include <vector>
#ifndef PHASE_ABL
#define PHASE_ABL 8
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

// skew: about 3 % of the rows carry one of three hot keys (1.6 / 0.9 /
// 0.6 %), the top of C4's Zipf(0.9) foreign keys
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

int main(int argc, char **argv) {
    const int skew = argc > 1;   // any argument: skewed keys
    const u64 n = 1ull << 28;
    ulonglong2 *in, *out;
    unsigned *bbin, *bfill, *nb;
    const u64 maxb = n / 256 + (1u << 20);
    CK(hipMalloc(&in, n * 16));
    CK(hipMalloc(&out, maxb * 512 * 16));
    CK(hipMalloc(&bbin, maxb * 4));
    CK(hipMalloc(&bfill, maxb * 4));
    CK(hipMalloc(&nb, 64));
    hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, in, n, skew);
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
    unsigned *wst;
    CK(hipMalloc(&wst, 1025 * 4));
    a.wstart = wst;
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
    for (int fb : {8, 9}) {
        a.fbits = fb;
        a.shift = 64 - fb;
        for (int pbl : {9, 10}) {
            a.out_pbl = pbl;
            char nm[64];
            snprintf(nm, sizeof nm, "F%d PB%d k_pass", 1 << fb, 1 << pbl);
            run(nm, [&] {
                hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, a, false, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);
                hipLaunchKernelGGL((k_pass<true, kPackedRow>), dim3(grid), dim3(kPassThreads), 0, 0, a);
            });
#define P(ABL, TXT)                                                                                       \
    snprintf(nm, sizeof nm, "F%d PB%d %s", 1 << fb, 1 << pbl, TXT);                                       \
    run(nm, [&] {                                                                                          \
        hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, a, false, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);                    \
        hipLaunchKernelGGL((k_pass<true, kPackedRow, ABL>), dim3(grid), dim3(kPassThreads), 0, 0, a);     \
    })
            P(2, "synthetic rows");
            P(4, "no row stores");
            P(6, "synthetic rows, no stores");
#undef P
            // phase times (cycles of s_memtime, summed over a workgroup's tiles, mean over workgroups)
            u64 *prof;
            CK(hipMalloc(&prof, grid * 8 * sizeof(u64)));
            CK(hipMemset(prof, 0, grid * 8 * sizeof(u64)));
            a.prof = prof;
            hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, a, false, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);
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
    // ---- a real second pass: the bucketed output of a 512-bin first pass
    // (512-row buckets, listed as runs) partitioned by the next 8 bits into
    // 256-row buckets, as radix_partition's pass 2 at |R| = 2^28
    {
        RadixPlan p1{};
        p1.passes = 1;
        p1.bits[0] = 9;
        p1.pbl[0] = kPassPbl;
        p1.total_bits = 9;
        const int P1 = 512;
        RadixNeed nd = radix_need((long long)n, p1, true);
        BucketSet b1;
        CK(hipMalloc(&b1.rows, nd.rows * 16));
        CK(hipMalloc(&b1.bbin, nd.buckets * 4));
        CK(hipMalloc(&b1.bfill, nd.buckets * 4));
        CK(hipMalloc(&b1.rstart, (P1 + 1) * 8));
        b1.max_buckets = (unsigned)nd.buckets;
        b1.max_rows = nd.rows;
        b1.max_runs = (nd.rows >> kRunLog) + nd.buckets;
        CK(hipMalloc(&b1.runs, b1.max_runs * 8));
        const int P2 = P1 << 8;
        RadixWork ws{};
        CK(hipMalloc(&ws.nb, 64));
        CK(hipMalloc(&ws.pcur, (P2 + 1) * 8));
        CK(hipMalloc(&ws.rcur, (P2 + 1) * 8));
        CK(hipMalloc(&ws.tile_start, (P2 + 1) * 4));
        CK(hipMalloc(&ws.tile_owner, radix_tiles((long long)n, P2) * 4));
        CK(hipMalloc(&ws.tdesc, radix_tiles((long long)n, P2) * 16));
        CK(hipMalloc(&ws.wstart, 1025 * 4));
        CK(hipMalloc(&ws.scan_sums, (P2 / 8192 + 2) * 8));
        CK(hipMalloc(&ws.scan_state, (P2 / 1024 + 4) * 8));   // (one-launch scans: zero between calls)
        CK(hipMemset(ws.scan_state, 0, (P2 / 1024 + 4) * 8));
        SrcDev src{};
        src.form = kPacked64;
        src.key = in;
        src.n = (long long)n;
        CK(radix_partition(src, true, p1, ws, b1, 0));
        chunk_map(b1.rstart, nullptr, P1, (unsigned)(kTile >> kRunLog), ws.tile_start, ws.tile_owner, ws.pcur,
                  ws.scan_sums, 0);
        {
            const u64 tb = radix_tiles((long long)n, P1);
            hipLaunchKernelGGL(k_tile_desc, dim3(blocks_for(tb, 256)), dim3(256), 0, 0, (const unsigned *)ws.tile_start,
                               (const unsigned *)ws.tile_owner, (const u64 *)b1.rstart, P1, (unsigned)tb,
                               (TileDesc *)ws.tdesc, (unsigned)(kTile >> kRunLog));
        }
        CK(hipDeviceSynchronize());
        unsigned ntiles = 0;
        u64 nruns = 0;
        CK(hipMemcpy(&ntiles, ws.tile_start + P1, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&nruns, b1.rstart + P1, 8, hipMemcpyDeviceToHost));
        printf("pass-1 set: %llu runs (%.3f x n/64), %u pass-2 tiles (%.3f x n/4096)\n", nruns,
               nruns / (double)(n >> 6), ntiles, ntiles / (double)(n >> 12));
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
        {
            // correctness: every row must land in the pass-2 output exactly once
            hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, b, true, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);
            hipLaunchKernelGGL((k_pass<true, kBucketed>), dim3(grid), dim3(kPassThreads), 0, 0, b);
            CK(hipDeviceSynchronize());
            unsigned nbh = 0;
            CK(hipMemcpy(&nbh, nb, 4, hipMemcpyDeviceToHost));
            std::vector<unsigned> bb(nbh), bf(nbh);
            CK(hipMemcpy(bb.data(), bbin, nbh * 4ull, hipMemcpyDeviceToHost));
            CK(hipMemcpy(bf.data(), bfill, nbh * 4ull, hipMemcpyDeviceToHost));
            u64 rows = 0, used = 0;
            for (unsigned j = 0; j < nbh; ++j)
                if (bb[j] != kNoBucket) {
                    rows += bf[j];
                    ++used;
                }
            std::vector<ulonglong2> td(ntiles);
            CK(hipMemcpy(td.data(), ws.tdesc, ntiles * 16ull, hipMemcpyDeviceToHost));
            u64 druns = 0;
            for (unsigned t = 0; t < ntiles; ++t) druns += (unsigned)td[t].y;
            printf("pass-2 check: %u bucket ids, %llu used, %llu rows out of %llu (%s); descriptors cover %llu runs of %llu\n",
                   nbh, used, rows, n, rows == n ? "ok" : "MISMATCH", druns, nruns);
        }
        auto p2 = [&] {
            hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, b, true, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);
            hipLaunchKernelGGL((k_pass<true, kBucketed>), dim3(grid), dim3(kPassThreads), 0, 0, b);
        };
        run("pass 2 (F256 PB256, runs) k_pass", p2);
#define P2X(ABL, TXT)                                                                                  \
    run("pass 2 " TXT, [&] {                                                                             \
        hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, b, true, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);                    \
        hipLaunchKernelGGL((k_pass<true, kBucketed, ABL>), dim3(grid), dim3(kPassThreads), 0, 0, b);     \
    })
        P2X(2, "synthetic rows");
        P2X(4, "no row stores");
        P2X(6, "synthetic rows, no stores");
#undef P2X
        b.out_pbl = kPassPbl;
        run("pass 2 with 512-row output buckets", p2);
        b.out_pbl = kFinalPbl;
        u64 *prof;
        CK(hipMalloc(&prof, grid * 8 * sizeof(u64)));
        CK(hipMemset(prof, 0, grid * 8 * sizeof(u64)));
        b.prof = prof;
        hipLaunchKernelGGL(k_id_plan, dim3(1), dim3(1024), 0, 0, b, true, grid, wst, (u64 *)nullptr, (u64 *)nullptr, 0ull);
        hipLaunchKernelGGL((k_pass<true, kBucketed, PHASE_ABL>), dim3(grid), dim3(kPassThreads), 0, 0, b);
        CK(hipDeviceSynchronize());
        std::vector<u64> h(grid * 8);
        CK(hipMemcpy(h.data(), prof, h.size() * sizeof(u64), hipMemcpyDeviceToHost));
        const char *names[5] = {"load wait + hash + LDS count", "scan + bucket atomic", "LDS scatter",
                                "next loads issued + stores + tails", "new tails + bookkeeping"};
        double m[5], tot = 0;
        for (int k = 0; k < 5; ++k) {
            double acc = 0;
            for (unsigned g = 0; g < grid; ++g) acc += (double)h[g * 8 + k];
            m[k] = acc / grid;
            tot += m[k];
        }
        for (int k = 0; k < 5; ++k) printf("  pass 2 phase %-38s %10.0f cycles  %5.1f %%\n", names[k], m[k], 100.0 * m[k] / tot);
        // the slowest workgroups and their phases (stragglers under skew)
        std::vector<std::pair<double, unsigned>> wt(grid);
        for (unsigned g = 0; g < grid; ++g) {
            double t = 0;
            for (int k = 0; k < 5; ++k) t += (double)h[g * 8 + k];
            wt[g] = {t, g};
        }
        std::sort(wt.begin(), wt.end());
        printf("  workgroup totals: min %.0f median %.0f max %.0f cycles\n", wt[0].first, wt[grid / 2].first,
               wt[grid - 1].first);
        for (unsigned r = grid - 4; r < grid; ++r) {
            const unsigned g = wt[r].second;
            printf("  wg %4u:", g);
            for (int k = 0; k < 5; ++k) printf(" %10llu", h[g * 8 + k]);
            printf("\n");
        }
    }
    return 0;
}
