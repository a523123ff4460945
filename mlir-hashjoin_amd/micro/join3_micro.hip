// join3_micro.hip -- does a third fast-join workgroup per CU pay?  Narrow
// PK-FK rows (key << 32 | row id, |R| = |S| = 2^28, every S row matches once)
// are partitioned by the product's radix_partition and joined by the product
// call; then k_join_u is launched directly in other shapes and workgroups per
// CU over the same work map (narrow rows: a 32 KiB table, so LDS allows 3-4
// workgroups; the waves per SIMD bound the VGPRs).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o join3_micro join3_micro.hip
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

// distinct 32-bit build keys (odd multiplier: a bijection on 32 bits);
// wide rows: C3's distinct 64-bit keys + row-id payloads
__global__ void k_gen(u64 *r, u64 *s, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const u64 kr = (i * 0x9E3779B1ull) & 0xFFFFFFFFull;
    const u64 j = mixd(i ^ 0xabcdef) % n;
    const u64 ks = (j * 0x9E3779B1ull) & 0xFFFFFFFFull;
    r[i] = (kr << 32) | i;
    s[i] = (ks << 32) | i;
}
__global__ void k_gen_w(ulonglong2 *r, ulonglong2 *s, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    r[i] = make_ulonglong2(mixd(i), i);
    s[i] = make_ulonglong2(mixd(mixd(i ^ 0xabcdef) % n), i);
}

template <typename T>
T *dalloc(u64 n) {
    T *p;
    CK(hipMalloc(&p, n * sizeof(T) + 16));
    return p;
}

template <bool W>
BucketSet make_set(RadixNeed nd, int P) {
    BucketSet b;
    b.rows = dalloc<u64>(nd.rows * (W ? 2 : 1));
    b.bbin = dalloc<unsigned>(nd.buckets);
    b.bfill = dalloc<unsigned>(nd.buckets);
    b.rstart = dalloc<u64>((u64)P + 1);
    b.max_buckets = (unsigned)nd.buckets;
    b.max_rows = nd.rows;
    b.max_runs = (nd.rows >> kRunLog) + nd.buckets;
    b.runs = dalloc<u64>(b.max_runs);
    return b;
}

template <bool W>
int body(int lg) {
    const u64 n = 1ull << lg;
    u64 *r = dalloc<u64>(n * (W ? 2 : 1)), *s = dalloc<u64>(n * (W ? 2 : 1));
    if (W) hipLaunchKernelGGL(k_gen_w, dim3((unsigned)(n / 256)), dim3(256), 0, 0, (ulonglong2 *)r, (ulonglong2 *)s, n);
    else hipLaunchKernelGGL(k_gen, dim3((unsigned)(n / 256)), dim3(256), 0, 0, r, s, n);
    const RadixPlan pl = radix_plan((long long)n);
    const int P = 1 << pl.total_bits;
    printf("%s PK-FK n=2^%d: %d passes, bits %d/%d, P=%d\n", W ? "wide" : "narrow", lg, pl.passes, pl.bits[0], pl.bits[1], P);
    RadixWork ws;
    ws.tmp = make_set<W>(radix_need((long long)n, pl, false), P);
    ws.nb = dalloc<unsigned>(4);
    ws.pcur = dalloc<u64>(P + 1);
    ws.rcur = dalloc<u64>(P + 1);
    ws.tile_start = dalloc<unsigned>(P + 1);
    ws.tile_owner = dalloc<unsigned>(radix_tiles((long long)n, P));
    ws.tdesc = dalloc<char>(radix_tiles((long long)n, P) * 16);
    ws.wstart = dalloc<unsigned>(1025);
    ws.scan_sums = dalloc<u64>(P / 8192 + 2);
    const RadixNeed nd = radix_need((long long)n, pl, true);
    BucketSet rs = make_set<W>(nd, P), ss = make_set<W>(nd, P);
    SrcDev src;
    src.form = kPacked64;
    src.pay = nullptr;
    src.row_base = 0;
    src.n = (long long)n;
    src.key = r;
    CK(radix_partition(src, W, pl, ws, rs, 0));
    src.key = s;
    CK(radix_partition(src, W, pl, ws, ss, 0));
    CK(hipDeviceSynchronize());
    unsigned *work = dalloc<unsigned>(radix_work_words(pl, ss.max_runs));
    void *desc = dalloc<char>(radix_join_items(pl, ss.max_runs) * radix_item_desc_bytes());
    u64 *out_r = dalloc<u64>(n + (1 << 20)), *out_s = dalloc<u64>(n + (1 << 20));
    u64 *cnt = dalloc<u64>(8), *dup = dalloc<u64>(8);
    unsigned *defer = dalloc<unsigned>(radix_join_items(pl, ss.max_runs) + 8), *defer_n = dalloc<unsigned>(4);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        CK(hipMemset(cnt, 0, 8));
        CK(hipMemset(defer_n, 0, 4));
        CK(hipMemset(dup, 0, 8));
        launch();
        CK(hipDeviceSynchronize());
        u64 m = 0, df = 0;
        unsigned dn = 0;
        CK(hipMemcpy(&df, dup, 8, hipMemcpyDeviceToHost));
        if (df) printf("  (dup flag set)\n");
        CK(hipMemcpy(&m, cnt, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&dn, defer_n, 4, hipMemcpyDeviceToHost));
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
        printf("%-40s %7.3f ms  %7.1f GB/s  M=%llu deferred=%u\n", name, ms, (3.0 * n * (W ? 16 : 8)) / ms / 1e6, m, dn);
    };
    run("radix_join (product)", [&] {
        CK(radix_join(W, pl, ws, rs, ss, ss.max_runs, work, desc, out_r, out_s, (long long)n, cnt, dup, false, 0, nullptr, false));
    });
    JoinArgs a;
    a.r = rs.rows; a.s = ss.rows; a.r_runs = rs.runs; a.s_runs = ss.runs; a.r_rstart = rs.rstart;
    a.s_rstart = ss.rstart; a.P = P; a.work_start = work; a.desc = (const ItemDesc *)desc;
    a.out_r = out_r; a.out_s = out_s; a.cap = (long long)n; a.counter = cnt; a.dup_flag = dup;
    a.defer = defer; a.defer_n = defer_n;
    a.tshift = 64 - pl.total_bits - 12;
    const int cus = cu_count();
#define U(NT, RI, SI, WPS, PER_CU, NAME) \
    run(NAME, [&] { hipLaunchKernelGGL((k_join_u<W, true, 12, NT, RI, SI, WPS>), dim3(PER_CU * cus), dim3(NT), 0, 0, a); })
    U(768, 3, 3, 6, 2, "768 thr 3+3, 2/CU (product shape)");
    U(768, 3, 3, 6, 1, "768 thr 3+3, 1/CU");
    U(1024, 3, 3, 8, 2, "1024 thr 3+3 (8 waves/SIMD), 2/CU");
    U(1024, 2, 2, 8, 2, "1024 thr 2+2, 2/CU");
    U(768, 2, 2, 8, 2, "768 thr 2+2, 2/CU");
    U(512, 4, 4, 6, 3, "512 thr 4+4, 3/CU");
#define UA(ABL, NAME) \
    run(NAME, [&] { hipLaunchKernelGGL((k_join_u<W, true, 12, 768, 3, 3, 6, true, ABL>), dim3(2 * cus), dim3(768), 0, 0, a); })
    if (!W) {   // i32 rows: an 8192-slot table is 64 KiB, still 2 workgroups per CU
        a.tshift = 64 - pl.total_bits - 13;
        run("768 thr 3+3, 8192 slots", [&] { hipLaunchKernelGGL((k_join_u<W, true, 13, 768, 3, 3, 6>), dim3(2 * cus), dim3(768), 0, 0, a); });
        a.tshift = 64 - pl.total_bits - 12;
    }
    {
        run("k_join_b", [&] { hipLaunchKernelGGL((k_join_b<W, true, 768, 3, 3, 6>), dim3(2 * cus), dim3(768), 0, 0, a); });
        run("k_join_b DETECT (repeat check only)", [&] { hipLaunchKernelGGL((k_join_b<W, false, 768, 3, 3, 6, true>), dim3(2 * cus), dim3(768), 0, 0, a); });
    }
    UA(1, "product shape, no cursor atomic");
    UA(2, "product shape, no output stores");
    UA(3, "product shape, no atomic, no stores");
    UA(7, "no atomic/stores/probe");
    UA(11, "no atomic/stores/build (empty-table probe)");
    UA(7 + 16, "no atomic/stores/probe/collision walks");
    UA(7 + 32, "no atomic/stores/probe/tpay");
    UA(7 + 48, "no atomic/stores/probe/walks/tpay");
    UA(3 + 16, "no atomic/stores/collision walks");
    return 0;
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int wide = argc > 2 ? atoi(argv[2]) : 0;
    return wide ? body<true>(lg) : body<false>(lg);
}
