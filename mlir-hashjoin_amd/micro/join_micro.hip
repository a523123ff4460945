// join_micro.hip -- ablation of the radix join kernel (k_join) on the real
// partition layout: |R| = |S| = 2^28 PK-FK rows are partitioned by the
// product's radix_partition (bucket sets), then only the join is timed.
// ABL bits switch phases off: 1 cursor atomic, 2 output writes, 4 probe,
// 8 build.  Also reports the bucket-fill statistics of the final sets.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o join_micro join_micro.hip
#include "../csrc/hj_radix.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

__device__ u64 mixd(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// mode 0: PK-FK (every S row matches once); 1: keys uniform in [1, 2^32]
// on both sides (C1-ref's distribution scaled to 2^28 rows: repeated build
// keys, 1/16 of the probes match); 2: PK-FK with 1/16 of the probes matching
__global__ void k_gen(ulonglong2 *r, ulonglong2 *s, u64 n, int mode) {
    u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (mode == 1) {
        r[i] = make_ulonglong2((mixd(i) & 0xFFFFFFFFull) + 1, i);
        s[i] = make_ulonglong2((mixd(i ^ 0x5555555555ull) & 0xFFFFFFFFull) + 1, i);
        return;
    }
    r[i] = make_ulonglong2(mixd(i), i);
    const u64 j = mixd(i ^ 0xabcdef) % n;
    s[i] = make_ulonglong2(mode == 2 && (mixd(i ^ 0x777) & 15) ? mixd(j + n) : mixd(j), i);
}

template <typename T>
T *dalloc(u64 n) {
    T *p;
    CK(hipMalloc(&p, n * sizeof(T) + 16));
    return p;
}

BucketSet make_set(RadixNeed nd, int P) {
    BucketSet b;
    b.rows = dalloc<ulonglong2>(nd.rows);
    b.bbin = dalloc<unsigned>(nd.buckets);
    b.bfill = dalloc<unsigned>(nd.buckets);
    b.rstart = dalloc<u64>((u64)P + 1);
    b.max_buckets = (unsigned)nd.buckets;
    b.max_rows = nd.rows;
    b.max_runs = (nd.rows >> kRunLog) + nd.buckets;
    b.runs = dalloc<u64>(b.max_runs);
    return b;
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const u64 n = 1ull << 28;
    ulonglong2 *r = dalloc<ulonglong2>(n), *s = dalloc<ulonglong2>(n);
    hipLaunchKernelGGL(k_gen, dim3(n / 256), dim3(256), 0, 0, r, s, n, mode);
    const RadixPlan pl = radix_plan((long long)n);
    const int P = 1 << pl.total_bits;
    printf("plan: %d passes, bits %d/%d/%d, P=%d\n", pl.passes, pl.bits[0], pl.bits[1], pl.bits[2], P);
    RadixWork ws;
    ws.tmp = make_set(radix_need((long long)n, pl, false), P);
    ws.nb = dalloc<unsigned>(4);
    ws.pcur = dalloc<u64>(P + 1);
    ws.rcur = dalloc<u64>(P + 1);
    ws.tile_start = dalloc<unsigned>(P + 1);
    ws.tile_owner = dalloc<unsigned>(radix_tiles((long long)n, P));
    ws.tdesc = dalloc<char>(radix_tiles((long long)n, P) * 16);
    ws.wstart = dalloc<unsigned>(1025);
    ws.scan_sums = dalloc<u64>(P / 8192 + 2);
    const RadixNeed nd = radix_need((long long)n, pl, true);
    BucketSet rs = make_set(nd, P), ss = make_set(nd, P);
    SrcDev src;
    src.form = kPacked64;
    src.pay = nullptr;
    src.row_base = 0;
    src.n = (long long)n;
    src.key = r;
    CK(radix_partition(src, true, pl, ws, rs, 0));
    src.key = s;
    CK(radix_partition(src, true, pl, ws, ss, 0));
    CK(hipDeviceSynchronize());
    // run statistics of the final sets
    for (int side = 0; side < 2; ++side) {
        const BucketSet &b = side ? ss : rs;
        std::vector<u64> ps(P + 1);
        CK(hipMemcpy(ps.data(), b.rstart, (P + 1) * 8, hipMemcpyDeviceToHost));
        std::vector<u64> lst(ps[P]);
        CK(hipMemcpy(lst.data(), b.runs, ps[P] * 8, hipMemcpyDeviceToHost));
        u64 rows = 0, part = 0, maxr = 0, maxrows = 0;
        for (int p = 0; p < P; ++p) {
            u64 pr = 0;
            for (u64 i = ps[p]; i < ps[p + 1]; ++i) {
                const unsigned f = (unsigned)(lst[i] & 127u);
                pr += f;
                part += f < 64;
            }
            rows += pr;
            const u64 nr = ps[p + 1] - ps[p];
            maxr = nr > maxr ? nr : maxr;
            maxrows = pr > maxrows ? pr : maxrows;
        }
        printf("%s: runs %llu rows %llu partial runs %llu (%.2f/partition) max runs %llu max rows %llu\n",
               side ? "S" : "R", ps[P], rows, part, (double)part / P, maxr, maxrows);
    }
    unsigned *work = dalloc<unsigned>(radix_work_words(pl, ss.max_runs));
    void *desc = dalloc<char>(radix_join_items(pl, ss.max_runs) * radix_item_desc_bytes());
    u64 *out_r = dalloc<u64>(n + (1 << 20)), *out_s = dalloc<u64>(n + (1 << 20)), *cnt = dalloc<u64>(8),
        *dup = dalloc<u64>(8);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // the product launch, then hand-rolled ablation launches with the same args
    auto run = [&](const char *name, auto launch) {
        CK(hipMemset(cnt, 0, 8));
        launch();
        CK(hipDeviceSynchronize());
        u64 m = 0;
        CK(hipMemcpy(&m, cnt, 8, hipMemcpyDeviceToHost));
        CK(hipEventRecord(e0));
        for (int i = 0; i < 5; ++i) {
            CK(hipMemsetAsync(cnt, 0, 8));
            launch();
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-34s %7.3f ms  %7.1f GB/s  M=%llu\n", name, ms, (3.0 * n * 16) / ms / 1e6, m);
    };
    run("radix_join (product)", [&] {
        CK(radix_join(true, pl, ws, rs, ss, ss.max_runs, work, desc, out_r, out_s, (long long)n, cnt, dup, false, 0, nullptr, false));
    });
    // work map of the product call stays in `work`
    JoinArgs a;
    a.r = rs.rows; a.s = ss.rows; a.r_runs = rs.runs; a.s_runs = ss.runs; a.r_rstart = rs.rstart;
    a.s_rstart = ss.rstart; a.P = P; a.work_start = work; a.desc = (const ItemDesc *)desc;
    a.out_r = out_r; a.out_s = out_s; a.cap = (long long)n; a.counter = cnt; a.dup_flag = dup;
    const int cus = cu_count();
#define J(TSL, NT, PER_CU, WR, ABL, NAME)                                                                  \
    run(NAME, [&] {                                                                                       \
        a.tshift = 64 - pl.total_bits - TSL;                                                              \
        hipLaunchKernelGGL((k_join<true, WR, TSL, NT, ABL>), dim3(PER_CU * cus), dim3(NT), 0, 0, a);      \
    })
    J(12, 512, 2, true, 0, "full");
    J(12, 512, 2, false, 0, "count only");
    J(12, 512, 2, true, 1, "no atomic");
    J(12, 512, 2, true, 2, "no writes");
    J(12, 512, 2, true, 3, "no atomic, no writes");
    J(12, 512, 2, true, 19, "no atomic/writes, 1st-slot probe");
    J(12, 512, 2, true, 11, "no atomic/writes/build");
    J(12, 512, 2, true, 7, "no probe/atomic/writes");
    J(12, 512, 2, true, 15, "loads + init only");
    return 0;
}
