// join_micro.hip -- ablation of the radix join kernel (k_join) on synthetic,
// already-partitioned PK-FK data: 2^17 partitions x 2048 R rows and 2048 S
// rows (the C3 shape after partitioning).  ABL bits switch phases off:
// 1 cursor atomic, 2 output writes, 4 probe, 8 build.
// Build: hipcc --offload-arch=gfx950 -O3 -I../csrc -I../../include -o join_micro join_micro.hip
#include "../csrc/hj_radix.hip"

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
using namespace hj;
typedef unsigned long long u64;

__device__ u64 mixd(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_gen(ulonglong2 *r, ulonglong2 *s, u64 per, int bits, u64 ginv, u64 n) {
    u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    u64 p = i / per;
    u64 h = (p << (64 - bits)) | (mixd(i) >> bits);
    r[i] = make_ulonglong2(h * ginv, i);
    u64 j = p * per + mixd(i ^ 0xabcdef) % per;
    u64 hj = (p << (64 - bits)) | (mixd(j) >> bits);
    s[i] = make_ulonglong2(hj * ginv, i);
}

__global__ void k_maps(u64 *r_off, u64 *s_off, unsigned *ws, unsigned *wo, u64 per, int P) {
    int p = blockIdx.x * 256 + threadIdx.x;
    if (p > P) return;
    r_off[p] = (u64)p * per;
    s_off[p] = (u64)p * per;
    ws[p] = p;
    if (p < P) wo[p] = p;
}

int main() {
    const int bits = 17, P = 1 << bits;
    const u64 per = 2048, n = (u64)P * per;
    u64 ginv = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 6; ++i) ginv *= 2 - 0x9E3779B97F4A7C15ull * ginv;
    ulonglong2 *r, *s;
    u64 *r_off, *s_off, *out_r, *out_s, *cnt, *dup;
    unsigned *ws, *wo;
    CK(hipMalloc(&r, n * 16)); CK(hipMalloc(&s, n * 16));
    CK(hipMalloc(&r_off, (P + 1) * 8)); CK(hipMalloc(&s_off, (P + 1) * 8));
    CK(hipMalloc(&ws, (P + 1) * 4)); CK(hipMalloc(&wo, P * 4));
    CK(hipMalloc(&out_r, n * 8)); CK(hipMalloc(&out_s, n * 8)); CK(hipMalloc(&cnt, 64)); CK(hipMalloc(&dup, 64));
    hipLaunchKernelGGL(k_gen, dim3(n / 256), dim3(256), 0, 0, r, s, per, bits, ginv, n);
    hipLaunchKernelGGL(k_maps, dim3(P / 256 + 1), dim3(256), 0, 0, r_off, s_off, ws, wo, per, P);
    CK(hipDeviceSynchronize());
    JoinArgs a;
    a.r = r; a.s = s; a.r_off = r_off; a.s_off = s_off; a.P = P; a.work_start = ws; a.work_owner = wo;
    a.tshift = 64 - bits - 12; a.out_r = out_r; a.out_s = out_s; a.cap = (long long)n; a.counter = cnt; a.dup_flag = dup;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int cus = cu_count();
    auto run = [&](const char *name, auto launch) {
        CK(hipMemset(cnt, 0, 8)); launch(); CK(hipDeviceSynchronize());
        u64 m = 0; CK(hipMemcpy(&m, cnt, 8, hipMemcpyDeviceToHost));
        CK(hipEventRecord(e0));
        for (int i = 0; i < 5; ++i) { CK(hipMemsetAsync(cnt, 0, 8)); launch(); }
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
        printf("%-34s %7.3f ms  %7.1f GB/s  M=%llu\n", name, ms, (3.0 * n * 16) / ms / 1e6, m);
    };
#define J(TSL, NT, PER_CU, WR, ABL, NAME)                                                                       \
    run(NAME, [&] { hipLaunchKernelGGL((k_join<true, WR, TSL, NT, ABL>), dim3(PER_CU * cus), dim3(NT), 0, 0, a); })
    J(12, 512, 2, true, 0, "full");
    J(12, 512, 2, false, 0, "count only");
    J(12, 512, 2, true, 1, "no atomic");
    J(12, 512, 2, true, 2, "no writes");
    J(12, 512, 2, true, 3, "no atomic, no writes");
    J(12, 512, 2, true, 7, "no probe/atomic/writes");
    J(12, 512, 2, true, 15, "loads + init only");
    J(12, 512, 3, true, 0, "full, 3 WG/CU grid");
    J(12, 512, 4, true, 0, "full, 4 WG/CU grid (non-resident)");
    a.tshift = 64 - bits - 11;
    J(11, 256, 4, true, 0, "tsl11 full (4 WG/CU)");
    J(11, 256, 4, true, 15, "tsl11 loads + init only");
    a.tshift = 64 - bits - 13;
    J(13, 1024, 1, true, 0, "tsl13 full (1 WG/CU)");
    return 0;
}
