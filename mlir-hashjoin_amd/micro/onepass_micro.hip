// onepass_micro.hip -- VERDICT r04 item 2: can S be partitioned in ONE pass
// into 2^14-2^15 bins if each bin's rows are assembled in 128-B line buffers
// that live in a global (L2 / Infinity-Cache resident) array, and only whole
// lines are copied (nt) to the bins' HBM regions?
//
// At 2^14-2^15 bins a 4096-row tile holds 0.12-0.25 rows per bin, so an LDS
// counting sort of the tile aggregates nothing: every row needs its own slot
// claim on its bin (one returning device atomic), and a line buffer shared by
// all workgroups needs a second atomic per row to learn when its 8 rows have
// landed (the writers are on different XCDs: row stores are sc1 write-through
// and ordered before the count by vmcnt(0), the copier reads sc1).
// Modes, over 2^28 16-B rows with uniform random keys (bin = top bits of a
// multiplicative hash), persistent 1024-thread workgroups, 4 rows per thread:
//   0 full design: claim atomic -> row into line buffer (2 lines per bin,
//     by line parity) -> done-count atomic -> the 8th row's lane copies the
//     line to HBM with nt stores and resets the count
//   1 claims + rows straight to their HBM slot (no line buffers: 16-B
//     scattered stores into 2^B frontiers, partial lines)
//   2 claims only (the atomic stream alone: a lower bound of modes 0 and 1)
//   3 the streamed read alone (the input side every mode has)
// Every mode is checked: mode 0/1 rebuild the key checksum of the input from
// the output regions (+ mode 0's lines still in their buffers).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o onepass_micro onepass_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;
typedef ulonglong2 row_t;

constexpr int NT = 1024, IT = 4, TILE = NT * IT;

__device__ __forceinline__ u64 mix(u64 x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
__global__ void k_fill(row_t *r, u64 n, u64 seed) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) r[i] = make_ulonglong2(mix(i ^ seed), i);
}
__device__ __forceinline__ row_t ld_nt(const row_t *p) {
    return make_ulonglong2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
}
__device__ __forceinline__ void st_nt(row_t *p, row_t v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
}
// write-through (sc1) 16-B row store / load: visible to a reader on another XCD
__device__ __forceinline__ void st_wt(row_t *p, row_t v) {
    __hip_atomic_store(&p->x, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&p->y, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ row_t ld_wt(const row_t *p) {
    return make_ulonglong2(__hip_atomic_load(&p->x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __hip_atomic_load(&p->y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

struct Args {
    const row_t *in;
    u64 n;
    int bits;          // bins = 2^bits
    u64 cap;           // rows per bin region
    row_t *out;        // bins x cap
    u64 *fill;         // bins: rows claimed
    unsigned *done;    // bins x 2: rows landed in line buffer (bin, parity)
    row_t *lbuf;       // bins x 2 x 8 rows
    u64 *sink;
};

template <int MODE>
__global__ __launch_bounds__(NT) void k_onepass(Args a) {
    const u64 tiles = a.n / TILE;
    const u64 t0 = (u64)blockIdx.x * tiles / gridDim.x, t1 = (u64)(blockIdx.x + 1) * tiles / gridDim.x;
    u64 acc = 0;
    for (u64 t = t0; t < t1; ++t) {
        row_t r[IT];
#pragma unroll
        for (int i = 0; i < IT; ++i) r[i] = ld_nt(a.in + t * TILE + (u64)i * NT + threadIdx.x);
        if constexpr (MODE == 3) {
#pragma unroll
            for (int i = 0; i < IT; ++i) acc += r[i].x;
            continue;
        }
        u64 pos[IT];
        unsigned bin[IT];
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            bin[i] = (unsigned)((r[i].x * 0x9E3779B97F4A7C15ull) >> (64 - a.bits));
            pos[i] = atomicAdd(&a.fill[bin[i]], 1ull);
        }
        if constexpr (MODE == 2) {
#pragma unroll
            for (int i = 0; i < IT; ++i) acc += pos[i];
            continue;
        }
        if constexpr (MODE == 1) {
#pragma unroll
            for (int i = 0; i < IT; ++i)
                if (pos[i] < a.cap) st_nt(a.out + (u64)bin[i] * a.cap + pos[i], r[i]);
            continue;
        }
        // MODE 0: line buffers
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const u64 L = pos[i] >> 3;
            const unsigned slot = (unsigned)(pos[i] & 7u), par = (unsigned)(L & 1u);
            st_wt(a.lbuf + ((u64)bin[i] * 2 + par) * 8 + slot, r[i]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every row store complete before its count
        unsigned d[IT];
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const unsigned par = (unsigned)((pos[i] >> 3) & 1u);
            d[i] = atomicAdd(&a.done[bin[i] * 2 + par], 1u);
        }
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            if (d[i] == 7u) {   // this row completed its line: copy it out whole
                const u64 L = pos[i] >> 3;
                const unsigned par = (unsigned)(L & 1u);
                const row_t *src = a.lbuf + ((u64)bin[i] * 2 + par) * 8;
                if ((L + 1) * 8 <= a.cap)
                    for (int k = 0; k < 8; ++k) st_nt(a.out + (u64)bin[i] * a.cap + L * 8 + k, ld_wt(src + k));
                __hip_atomic_store(&a.done[bin[i] * 2 + par], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (acc == 0x123456789ull) a.sink[0] = acc;
}

// checksum of keys over every bin's region rows [0, min(fill, cap)) -- whole
// lines only in mode 0 (the partial last line is still in its buffer)
__global__ void k_sum(const row_t *out, const u64 *fill, u64 cap, int bins, int whole_lines, const row_t *lbuf,
                      u64 *res) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= bins) return;
    const unsigned lane = threadIdx.x & 63u;
    u64 f = fill[b] < cap ? fill[b] : cap;
    u64 s = 0, c = 0;
    const u64 hi = whole_lines ? (f & ~7ull) : f;
    for (u64 i = lane; i < hi; i += 64) s += out[(u64)b * cap + i].x, ++c;
    if (whole_lines) {   // rows of the open (partial) line, still in its buffer
        const u64 L = f >> 3;
        for (u64 i = L * 8 + lane; i < f; i += 64) s += lbuf[((u64)b * 2 + (L & 1)) * 8 + (i & 7)].x, ++c;
    }
    atomicAdd(&res[0], s);
    atomicAdd(&res[1], c);
}
__global__ void k_sum_in(const row_t *in, u64 n, u64 *res) {
    u64 s = 0;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += (u64)gridDim.x * 256) s += in[i].x;
    atomicAdd(&res[2], s);
}

int main(int argc, char **argv) {
    const int log2n = argc > 1 ? atoi(argv[1]) : 28;
    const u64 n = 1ull << log2n;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    row_t *in, *out, *lbuf;
    u64 *fill, *res, *sink;
    unsigned *done;
    CK(hipMalloc(&in, n * 16));
    const int maxbits = 15;
    // bin regions: mean n / bins rows, +25 % + 256 (the largest over both bin counts)
    CK(hipMalloc(&out, (n + n / 4 + ((u64)1 << maxbits) * 256) * 16));
    CK(hipMalloc(&lbuf, (u64)(1 << maxbits) * 2 * 8 * 16));
    CK(hipMalloc(&fill, (u64)(1 << maxbits) * 8));
    CK(hipMalloc(&done, (u64)(1 << maxbits) * 2 * 4));
    CK(hipMalloc(&res, 64));
    CK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(k_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, in, n, 0x5eedull);
    CK(hipMemset(res, 0, 64));
    hipLaunchKernelGGL(k_sum_in, dim3(4096), dim3(256), 0, 0, in, n, res);
    u64 hres[3];
    CK(hipMemcpy(hres, res, 24, hipMemcpyDeviceToHost));
    const u64 insum = hres[2];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[4] = {"line buffers (claim + sc1 row + done count + whole-line nt copy)",
                            "claims + rows straight to HBM slots (partial lines)",
                            "claim atomics only", "streamed read only"};
    printf("one S pass, 2^%d 16-B rows, %d workgroups x %d threads, %d rows per thread per tile\n", log2n, cus, NT, IT);
    for (int bits : {14, 15}) {
        const int bins = 1 << bits;
        const u64 cap = (n >> bits) + (n >> (bits + 2)) + 256;
        for (int mode : {3, 2, 1, 0}) {
            float best = 1e30f;
            bool ok = true;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipMemset(fill, 0, (u64)bins * 8));
                CK(hipMemset(done, 0, (u64)bins * 2 * 4));
                Args a{in, n, bits, cap, out, fill, done, lbuf, sink};
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(k_onepass<0>, dim3(cus), dim3(NT), 0, 0, a);
                if (mode == 1) hipLaunchKernelGGL(k_onepass<1>, dim3(cus), dim3(NT), 0, 0, a);
                if (mode == 2) hipLaunchKernelGGL(k_onepass<2>, dim3(cus), dim3(NT), 0, 0, a);
                if (mode == 3) hipLaunchKernelGGL(k_onepass<3>, dim3(cus), dim3(NT), 0, 0, a);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
                if (mode <= 1) {
                    CK(hipMemset(res, 0, 16));
                    hipLaunchKernelGGL(k_sum, dim3((bins + 3) / 4), dim3(256), 0, 0, out, fill, cap, bins,
                                       mode == 0 ? 1 : 0, lbuf, res);
                    CK(hipMemcpy(hres, res, 16, hipMemcpyDeviceToHost));
                    ok = ok && hres[0] == insum && hres[1] == n;
                }
            }
            const double gbs = (mode == 3 ? 16.0 : mode == 2 ? 16.0 : 32.0) * n / (best * 1e6);
            printf("bins 2^%d  %-66s %8.3f ms  (%.0f GB/s of %s)%s\n", bits, names[mode], best, gbs,
                   mode >= 2 ? "reads" : "reads + writes", mode <= 1 ? (ok ? "  checksum ok" : "  CHECKSUM MISMATCH") : "");
        }
    }
    return 0;
}
