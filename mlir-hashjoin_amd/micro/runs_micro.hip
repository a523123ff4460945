// runs_micro.hip -- how many runs (<= 64 rows of one bucket) do the final
// partitions of a radix_partition hold?  The join takes an item's R side in
// build rounds of NW * RI runs and its S chunk in sub-chunks of NW * SI runs
// (k_join_b: 36 for int64 rows, 48 for i32 rows); every round or sub-chunk
// past the first costs the item one more dependent load latency.  Runs the
// product's partition (same pass variants) on 2^28 int64 rows (C3's R) and
// 1e8 i32 rows (REF-B's) and prints the distribution of runs per partition.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../csrc -I../../include -o runs_micro runs_micro.hip
#include "../csrc/hj_radix.hip"

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

__global__ void k_fill64(u64 *k, u64 *p, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) { k[i] = fmix64(i * 7 + 1); p[i] = i; }
}
__global__ void k_fill32(int *k, u64 n) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) k[i] = (int)(fmix64(i * 3 + 5) % 1000000000ull) + 1;
}

template <class T> T *dalloc(u64 n) { T *p; CK(hipMalloc(&p, n * sizeof(T) + 64)); return p; }

void run(bool wide, u64 n, int lim_a, int lim_b) {
    const RadixPlan pl = radix_plan((long long)n, 0, wide);
    const int P = 1 << pl.total_bits;
    const size_t esz = wide ? 16 : 8;
    RadixNeed nf = radix_need((long long)n, pl, true), nt = radix_need((long long)n, pl, false);
    auto mkset = [&](RadixNeed nd, int parts) {
        BucketSet b{};
        b.rows = dalloc<char>(nd.rows * esz);
        b.bbin = dalloc<unsigned>(nd.buckets);
        b.bfill = dalloc<unsigned>(nd.buckets);
        b.rstart = dalloc<u64>((u64)parts + 1);
        b.max_buckets = (unsigned)nd.buckets;
        b.max_rows = nd.rows;
        b.max_runs = (nd.rows >> kRunLog) + nd.buckets;
        b.runs = dalloc<u64>(b.max_runs);
        return b;
    };
    BucketSet fin = mkset(nf, P);
    RadixWork ws{};
    ws.tmp = mkset(nt, P);
    ws.nb = dalloc<unsigned>(16);
    ws.pcur = dalloc<u64>(P + 1);
    ws.rcur = dalloc<u64>(P + 1);
    ws.tile_start = dalloc<unsigned>(P + 1);
    ws.tile_owner = dalloc<unsigned>(radix_tiles((long long)n, P));
    ws.tdesc = dalloc<char>(radix_tiles((long long)n, P) * 16);
    ws.wstart = dalloc<unsigned>(1025);
    ws.scan_sums = dalloc<u64>(P / 8192 + 2);
    ws.scan_state = dalloc<u64>(P / 1024 + 4);
    CK(hipMemset(ws.scan_state, 0, (P / 1024 + 4) * 8));
    SrcDev src{};
    src.n = (long long)n;
    if (wide) {
        u64 *k = dalloc<u64>(n), *p = dalloc<u64>(n);
        hipLaunchKernelGGL(k_fill64, dim3((n + 255) / 256), dim3(256), 0, 0, k, p, n);
        src.key = k;
        src.pay = p;
        src.form = kCols64;
    } else {
        int *k = dalloc<int>(n);
        hipLaunchKernelGGL(k_fill32, dim3((n + 255) / 256), dim3(256), 0, 0, k, n);
        src.key = k;
        src.form = kCol32;
    }
    CK(radix_partition(src, wide, pl, ws, fin, 0));
    CK(hipDeviceSynchronize());
    std::vector<u64> rs(P + 1);
    CK(hipMemcpy(rs.data(), fin.rstart, (P + 1) * 8ull, hipMemcpyDeviceToHost));
    std::vector<u64> hist(257, 0);
    u64 over_a = 0, over_b = 0, mx = 0;
    for (int p = 0; p < P; ++p) {
        const u64 r = rs[p + 1] - rs[p];
        hist[r < 256 ? r : 256]++;
        over_a += r > (u64)lim_a;
        over_b += r > (u64)lim_b;
        mx = r > mx ? r : mx;
    }
    printf("%s n=%llu plan %d passes (%d+%d bits), %d partitions, %.1f rows/partition, %llu runs (%.3f x n/64), max %llu\n",
           wide ? "int64" : "i32", n, pl.passes, pl.bits[0], pl.bits[1], P, (double)n / P, rs[P],
           rs[P] / (double)(n >> 6), mx);
    printf("  partitions over %d runs: %.2f %%, over %d runs: %.2f %%\n", lim_a, 100.0 * over_a / P, lim_b,
           100.0 * over_b / P);
    printf("  runs: count\n");
    for (int r = 0; r <= 256; ++r)
        if (hist[r] * 1000 > (u64)P) printf("  %3d: %6.2f %%\n", r, 100.0 * hist[r] / P);
}

int main() {
    run(true, 1ull << 28, 36, 48);
    run(false, 100000000ull, 48, 64);
    return 0;
}
