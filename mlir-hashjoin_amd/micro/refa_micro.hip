// refa_micro.hip -- where k_join spends the reference's headline workload
// (join-performances.md:3-6: 10M x 10M i32 keys uniform in [1, 100k], ~1e9
// result pairs, ~100 per probe row).  Narrow (key << 32 | row id) rows are
// partitioned by the product's radix_partition; only the join is timed, with
// ABL bits switching phases off: 1 cursor atomic, 2 output writes, 4 probe,
// 8 build.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o refa_micro refa_micro.hip
#include "../csrc/hj_radix.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

__global__ void k_gen_ref(u64 *r, u64 *s, u64 n, unsigned range) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    r[i] = ((fmix64(i * 2 + 1) % range + 1) << 32) | i;
    s[i] = ((fmix64(i * 2 + 2) % range + 1) << 32) | i;
}

template <typename T>
T *dalloc(u64 n) {
    T *p;
    CK(hipMalloc(&p, n * sizeof(T) + 16));
    return p;
}

BucketSet make_set(RadixNeed nd, int P) {
    BucketSet b;
    b.rows = dalloc<u64>(nd.rows);
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
    const u64 n = argc > 1 ? strtoull(argv[1], nullptr, 0) : 10000000ull;
    const unsigned range = argc > 2 ? (unsigned)strtoul(argv[2], nullptr, 0) : 100000u;
    u64 *r = dalloc<u64>(n), *s = dalloc<u64>(n);
    hipLaunchKernelGGL(k_gen_ref, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, r, s, n, range);
    const RadixPlan pl = radix_plan((long long)n);
    const int P = 1 << pl.total_bits;
    printf("n=%llu keys in [1, %u]: %d passes, bits %d/%d, P=%d\n", n, range, pl.passes, pl.bits[0], pl.bits[1], P);
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
    CK(radix_partition(src, false, pl, ws, rs, 0));
    src.key = s;
    CK(radix_partition(src, false, pl, ws, ss, 0));
    CK(hipDeviceSynchronize());
    const u64 cap = 1200000000ull;
    unsigned *work = dalloc<unsigned>(radix_work_words(pl, ss.max_runs));
    void *desc = dalloc<char>(radix_join_items(pl, ss.max_runs) * radix_item_desc_bytes());
    unsigned *out_r = dalloc<unsigned>(cap), *out_s = dalloc<unsigned>(cap);
    u64 *cnt = dalloc<u64>(8), *dup = dalloc<u64>(8);
    // a build-side sample that says "most keys repeat": the grouped join over every item
    unsigned long long *stats = dalloc<unsigned long long>(2);
    {
        const unsigned long long most[2] = {1, 1};
        CK(hipMemcpy(stats, most, sizeof(most), hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
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
        printf("%-34s %7.3f ms  M=%llu  (%.2f TB/s of 8-B pairs written)\n", name, ms, m, 8.0 * m / ms / 1e9);
    };
    // the general kernel over every item (what the product runs once the
    // fast path has deferred most items)
    CK(radix_join(false, pl, ws, rs, ss, ss.max_runs, work, desc, out_r, out_s, (long long)cap, cnt, dup, false, 0,
                  stats, false));
    CK(hipDeviceSynchronize());
    run("product general path (k_join_grp)", [&] {
        CK(radix_join(false, pl, ws, rs, ss, ss.max_runs, work, desc, out_r, out_s, (long long)cap, cnt, dup, false, 0,
                      stats, false));
    });
    run("product general, count only", [&] {
        CK(radix_join(false, pl, ws, rs, ss, ss.max_runs, work, desc, out_r, out_s, 0, cnt, dup, true, 0, stats, false));
    });
    JoinArgs a;
    a.r = rs.rows; a.s = ss.rows; a.r_runs = rs.runs; a.s_runs = ss.runs; a.r_rstart = rs.rstart;
    a.s_rstart = ss.rstart; a.P = P; a.work_start = work; a.desc = (const ItemDesc *)desc;
    a.out_r = out_r; a.out_s = out_s; a.cap = (long long)cap; a.counter = cnt; a.dup_flag = dup;
    a.tshift = 64 - pl.total_bits - 12;
    const int cus = cu_count();
#define J(WR, ABL, NAME) \
    run(NAME, [&] { hipLaunchKernelGGL((k_join<false, WR, 12, 512, ABL>), dim3(2 * cus), dim3(512), 0, 0, a); })
    J(true, 0, "k_join full");
    J(false, 0, "count only");
    J(true, 1, "no atomic");
    J(true, 2, "no writes");
    J(true, 3, "no atomic, no writes");
    J(true, 7, "no probe/atomic/writes");
    J(true, 15, "loads + init only");
    return 0;
}
