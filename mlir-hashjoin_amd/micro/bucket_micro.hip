// bucket_micro.hip -- histogram-free radix partition pass (bucket chaining).
//
// A persistent workgroup counting-sorts each 4096-row tile by bin in LDS and
// appends every bin's run to that workgroup's current fixed-size bucket for
// the bin; full buckets are replaced by fresh ones from one global atomic
// counter.  No histogram pass, no global scan: the input is read once.
// Compared against the two-phase pass (LDS histogram + scatter into exact
// bin offsets).  n = 2^28 packed 16-B rows, 512 and 256 bins.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef unsigned long long u64;

constexpr unsigned kNone = 0xffffffffu;

template <int TILE, int NT, int FB, int PB, int NTM = 0>
__global__ __launch_bounds__(NT) void k_bucket(const ulonglong2 *__restrict__ a, u64 n, ulonglong2 *__restrict__ out,
                                                  unsigned *__restrict__ bucket_bin, unsigned *__restrict__ bucket_fill,
                                                  unsigned *__restrict__ next_bucket) {
    constexpr int IT = TILE / NT;
    constexpr int F = 1 << FB;
    __shared__ ulonglong2 stage[TILE];
    __shared__ unsigned short sb[TILE];
    __shared__ unsigned cnt[F], start[F], cur[F], fill[F], nbase[F];
    for (int b = threadIdx.x; b < F; b += NT) { cur[b] = kNone; fill[b] = PB; }
    const u64 ntiles = (n + TILE - 1) / TILE;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int b = threadIdx.x; b < F; b += NT) cnt[b] = 0;
        __syncthreads();
        ulonglong2 row[IT];
        unsigned br[IT];
        const u64 base = tile * TILE + threadIdx.x;
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            if (base + j * NT < n) {
                if constexpr (NTM & 1) {
                    row[j].x = __builtin_nontemporal_load(&a[base + j * NT].x);
                    row[j].y = __builtin_nontemporal_load(&a[base + j * NT].y);
                } else {
                    row[j] = a[base + j * NT];
                }
            } else {
                row[j] = make_ulonglong2(0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            if (base + j * NT < n) {
                unsigned b = (unsigned)((row[j].x * 0x9E3779B97F4A7C15ull) >> (64 - FB));
                br[j] = (b << 16) | atomicAdd(&cnt[b], 1u);
            } else {
                br[j] = 0xffffffffu;
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            constexpr int PL = (F + 63) / 64;
            unsigned c[PL], s = 0;
            for (int j = 0; j < PL; ++j) { int b = threadIdx.x * PL + j; c[j] = b < F ? cnt[b] : 0; s += c[j]; }
            unsigned x = s;
            for (int o = 1; o < 64; o <<= 1) { unsigned y = __shfl_up(x, o, 64); if ((int)threadIdx.x >= o) x += y; }
            unsigned run = x - s;
            for (int j = 0; j < PL; ++j) { int b = threadIdx.x * PL + j; if (b < F) start[b] = run; run += c[j]; }
        }
        // bucket bookkeeping: one thread per bin
        for (int b = threadIdx.x; b < F; b += NT) {
            const unsigned c = cnt[b];
            if (c == 0) continue;
            const unsigned f = fill[b];
            const unsigned k = (f + c - 1) / PB;              // fresh buckets needed
            if (k) {
                const unsigned nb = atomicAdd(next_bucket, k);
                nbase[b] = nb;
                if (cur[b] != kNone) bucket_fill[cur[b]] = PB;
                for (unsigned i = 0; i < k; ++i) {
                    bucket_bin[nb + i] = b;
                    if (i + 1 < k) bucket_fill[nb + i] = PB;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            if (br[j] == 0xffffffffu) continue;
            unsigned b = br[j] >> 16;
            unsigned pos = start[b] + (br[j] & 0xffff);
            stage[pos] = row[j];
            sb[pos] = (unsigned short)b;
        }
        __syncthreads();
        const unsigned tn = (unsigned)min<u64>(TILE, n - tile * TILE);
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned i = j * NT + threadIdx.x;
            if (i >= tn) continue;
            unsigned b = sb[i];
            unsigned p = fill[b] + (i - start[b]);
            unsigned k = p / PB;
            unsigned bk = k == 0 ? cur[b] : nbase[b] + k - 1;
            if constexpr (NTM & 2) {
                __builtin_nontemporal_store(stage[i].x, &out[(u64)bk * PB + (p % PB)].x);
                __builtin_nontemporal_store(stage[i].y, &out[(u64)bk * PB + (p % PB)].y);
            } else {
                out[(u64)bk * PB + (p % PB)] = stage[i];
            }
        }
        __syncthreads();
        for (int b = threadIdx.x; b < F; b += NT) {
            const unsigned c = cnt[b];
            if (c == 0) continue;
            const unsigned f = fill[b];
            const unsigned k = (f + c - 1) / PB;
            if (k) { cur[b] = nbase[b] + k - 1; fill[b] = f + c - k * PB; }
            else fill[b] = f + c;
        }
        // next iteration's cnt reset is ordered after this by the barrier below
        __syncthreads();
    }
    for (int b = threadIdx.x; b < F; b += NT)
        if (cur[b] != kNone) bucket_fill[cur[b]] = fill[b];
}


// Write-combining variant: rows reach a bucket only as whole 128-B lines
// (8 rows); up to 7 leftover rows per bin wait in an LDS carry buffer.  Bucket
// fills stay multiples of 8 until the final flush, so every store is a full,
// aligned line.
template <int TILE, int NT, int FB, int PB>
__global__ __launch_bounds__(NT) void k_bucket_wc(const ulonglong2 *__restrict__ a, u64 n, ulonglong2 *__restrict__ out,
                                                  unsigned *__restrict__ bucket_bin, unsigned *__restrict__ bucket_fill,
                                                  unsigned *__restrict__ next_bucket) {
    constexpr int IT = TILE / NT;
    constexpr int F = 1 << FB;
    constexpr int L = 8;
    __shared__ ulonglong2 stage[TILE];
    __shared__ ulonglong2 carry[F * L];
    __shared__ unsigned short sb[TILE];
    __shared__ unsigned cnt[F], start[F], cur[F], fill[F], nbase[F];
    __shared__ unsigned char cc[F], fl[F];        // carried rows, lines flushed this tile
    for (int b = threadIdx.x; b < F; b += NT) { cur[b] = kNone; fill[b] = PB; cc[b] = 0; }
    const u64 ntiles = (n + TILE - 1) / TILE;
    for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        for (int b = threadIdx.x; b < F; b += NT) cnt[b] = 0;
        __syncthreads();
        ulonglong2 row[IT];
        unsigned br[IT];
        const u64 base = tile * TILE + threadIdx.x;
#pragma unroll
        for (int j = 0; j < IT; ++j) row[j] = base + j * NT < n ? a[base + j * NT] : make_ulonglong2(0, 0);
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            if (base + j * NT < n) {
                unsigned b = (unsigned)((row[j].x * 0x9E3779B97F4A7C15ull) >> (64 - FB));
                br[j] = (b << 16) | atomicAdd(&cnt[b], 1u);
            } else {
                br[j] = 0xffffffffu;
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            constexpr int PL = (F + 63) / 64;
            unsigned c[PL], s = 0;
            for (int j = 0; j < PL; ++j) { int b = threadIdx.x * PL + j; c[j] = b < F ? cnt[b] : 0; s += c[j]; }
            unsigned x = s;
            for (int o = 1; o < 64; o <<= 1) { unsigned y = __shfl_up(x, o, 64); if ((int)threadIdx.x >= o) x += y; }
            unsigned run = x - s;
            for (int j = 0; j < PL; ++j) { int b = threadIdx.x * PL + j; if (b < F) start[b] = run; run += c[j]; }
        }
        for (int b = threadIdx.x; b < F; b += NT) {
            const unsigned c = cnt[b] + cc[b];
            const unsigned w = c / L * L;                    // rows leaving as whole lines
            fl[b] = (unsigned char)(w / L);
            if (w == 0) continue;
            const unsigned f = fill[b];
            const unsigned k = (f + w - 1) / PB;
            if (k) {
                const unsigned nb = atomicAdd(next_bucket, k);
                nbase[b] = nb;
                if (cur[b] != kNone) bucket_fill[cur[b]] = PB;
                for (unsigned i = 0; i < k; ++i) {
                    bucket_bin[nb + i] = b;
                    if (i + 1 < k) bucket_fill[nb + i] = PB;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            if (br[j] == 0xffffffffu) continue;
            unsigned b = br[j] >> 16;
            unsigned pos = start[b] + (br[j] & 0xffff);
            stage[pos] = row[j];
            sb[pos] = (unsigned short)b;
        }
        __syncthreads();
        const unsigned tn = (unsigned)min<u64>(TILE, n - tile * TILE);
        auto dst = [&](unsigned b, unsigned v) {
            unsigned p = fill[b] + v, k = p / PB;
            unsigned bk = k == 0 ? cur[b] : nbase[b] + k - 1;
            return (u64)bk * PB + (p % PB);
        };
        // carried rows lead their bin's sequence
        for (unsigned t = threadIdx.x; t < F * L; t += NT) {
            unsigned b = t / L, j = t % L;
            if (j < cc[b] && j < fl[b] * L) out[dst(b, j)] = carry[t];
        }
        ulonglong2 keep[IT];
        int kslot[IT];
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            unsigned i = j * NT + threadIdx.x;
            kslot[j] = -1;
            if (i >= tn) continue;
            unsigned b = sb[i];
            unsigned v = cc[b] + (i - start[b]);
            if (v < fl[b] * L) out[dst(b, v)] = stage[i];
            else { keep[j] = stage[i]; kslot[j] = b * L + (v - fl[b] * L); }
        }
        // carried rows that do not leave shift down behind nothing (fl == 0 keeps them in place)
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j)
            if (kslot[j] >= 0) carry[kslot[j]] = keep[j];
        for (int b = threadIdx.x; b < F; b += NT) {
            const unsigned c = cnt[b] + cc[b];
            const unsigned w = fl[b] * L;
            cc[b] = (unsigned char)(c - w);
            if (w == 0) continue;
            const unsigned f = fill[b];
            const unsigned k = (f + w - 1) / PB;
            if (k) { cur[b] = nbase[b] + k - 1; fill[b] = f + w - k * PB; }
            else fill[b] = f + w;
        }
        __syncthreads();
    }
    // final flush of the carried rows (partial lines)
    for (int b = threadIdx.x; b < F; b += NT) {
        const unsigned c = cc[b];
        if (c == 0) { if (cur[b] != kNone) bucket_fill[cur[b]] = fill[b]; continue; }
        unsigned f = fill[b];
        if (f + c > PB) {
            if (cur[b] != kNone) bucket_fill[cur[b]] = f;
            const unsigned nb = atomicAdd(next_bucket, 1u);
            bucket_bin[nb] = b;
            cur[b] = nb; f = 0;
        }
        for (unsigned j = 0; j < c; ++j) out[(u64)cur[b] * PB + f + j] = carry[b * L + j];
        bucket_fill[cur[b]] = f + c;
    }
}

// two-phase reference pass: per-tile LDS histogram then exact-offset scatter
template <int TILE, int NT, int FB>
__global__ __launch_bounds__(NT) void k_hist(const ulonglong2 *a, u64 n, unsigned *hist) {
    constexpr int F = 1 << FB;
    __shared__ unsigned cnt[F];
    for (int b = threadIdx.x; b < F; b += NT) cnt[b] = 0;
    __syncthreads();
    u64 base = (u64)blockIdx.x * TILE + threadIdx.x;
#pragma unroll
    for (int j = 0; j < TILE / NT; ++j)
        if (base + j * NT < n) atomicAdd(&cnt[(a[base + j * NT].x * 0x9E3779B97F4A7C15ull) >> (64 - FB)], 1u);
    __syncthreads();
    for (int b = threadIdx.x; b < F; b += NT) hist[(u64)blockIdx.x * F + b] = cnt[b];
}

int main() {
    const u64 n = 1ull << 28;
    ulonglong2 *a, *b;
    unsigned *bbin, *bfill, *nextb, *hist;
    const u64 maxb = (n / 64) + 4096ull * 512;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, (n + 4096ull * 512 * 256) * 16));
    CK(hipMalloc(&bbin, maxb * 4));
    CK(hipMalloc(&bfill, maxb * 4));
    CK(hipMalloc(&nextb, 64));
    CK(hipMalloc(&hist, (n / 4096) * 512 * 4));
    {
        ulonglong2 *h = (ulonglong2 *)malloc(1 << 24);
        u64 x = 88172645463325252ull;
        for (int i = 0; i < (1 << 20); ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = make_ulonglong2(x, i); }
        for (u64 o = 0; o < n; o += (1 << 20)) CK(hipMemcpy(a + o, h, 1 << 24, hipMemcpyHostToDevice));
        free(h);
    }
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](const char *name, double bytes, auto fn) {
        fn(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 5; ++r) fn();
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
        printf("%-34s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    const double rw = 2.0 * n * 16, rd = n * 16.0;
    run("hist t4096 F512 (read only)", rd, [&] { hipLaunchKernelGGL((k_hist<4096, 512, 9>), dim3(n / 4096), dim3(512), 0, 0, a, n, hist); });
#define BUCKETT(T, NT, FB, PB, WPC)                                                                     \
    run("bucket t" #T " F" #FB " PB" #PB " wg/cu" #WPC, rw, [&] {                                        \
        CK(hipMemsetAsync(nextb, 0, 4));                                                                 \
        hipLaunchKernelGGL((k_bucket<T, NT, FB, PB>), dim3(cus * WPC), dim3(NT), 0, 0, a, n, b, bbin, bfill, nextb); \
    });
#define BUCKET(FB, PB, WPC) BUCKETT(4096, 512, FB, PB, WPC)
    BUCKET(9, 256, 2)
    BUCKET(9, 512, 2)
    BUCKET(9, 1024, 2)
    BUCKET(8, 256, 2)
    BUCKET(8, 512, 2)
    BUCKET(9, 256, 1)
    BUCKET(9, 256, 4)
    BUCKETT(8192, 1024, 9, 512, 1)
    BUCKETT(8192, 1024, 9, 1024, 1)
    BUCKETT(8192, 1024, 8, 512, 1)
    BUCKETT(8192, 512, 9, 512, 1)
    BUCKETT(2048, 256, 9, 512, 4)
#define BNT(T, NT, FB, PB, M)                                                                                \
    run("bucket t" #T " F" #FB " PB" #PB " ntmode" #M, rw, [&] {                                        \
        CK(hipMemsetAsync(nextb, 0, 4));                                                                 \
        hipLaunchKernelGGL((k_bucket<T, NT, FB, PB, M>), dim3(cus), dim3(NT), 0, 0, a, n, b, bbin, bfill, nextb); \
    });
    BNT(8192, 1024, 9, 512, 1)
    BNT(8192, 1024, 9, 512, 2)
    BNT(8192, 1024, 9, 512, 3)
    BNT(8192, 1024, 8, 512, 3)
#define WC(T, NT, FB, PB)                                                                                \
    run("wc t" #T " F" #FB " PB" #PB, rw, [&] {                                                         \
        CK(hipMemsetAsync(nextb, 0, 4));                                                                 \
        hipLaunchKernelGGL((k_bucket_wc<T, NT, FB, PB>), dim3(cus), dim3(NT), 0, 0, a, n, b, bbin, bfill, nextb); \
    });
    // verify: every row landed once in a bucket of its bin
    {
        CK(hipMemsetAsync(nextb, 0, 4));
        hipLaunchKernelGGL((k_bucket_wc<4096, 1024, 9, 256>), dim3(cus), dim3(1024), 0, 0, a, n, b, bbin, bfill, nextb);
        CK(hipDeviceSynchronize());
        unsigned nb;
        CK(hipMemcpy(&nb, nextb, 4, hipMemcpyDeviceToHost));
        std::vector<unsigned> hb(nb), hf(nb);
        CK(hipMemcpy(hb.data(), bbin, nb * 4ull, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hf.data(), bfill, nb * 4ull, hipMemcpyDeviceToHost));
        std::vector<ulonglong2> rows((u64)nb * 256);
        CK(hipMemcpy(rows.data(), b, rows.size() * 16, hipMemcpyDeviceToHost));
        u64 tot = 0, bad = 0, xs = 0;
        for (unsigned j = 0; j < nb; ++j) {
            tot += hf[j];
            for (unsigned i = 0; i < hf[j]; ++i) {
                const ulonglong2 r = rows[(u64)j * 256 + i];
                if ((unsigned)((r.x * 0x9E3779B97F4A7C15ull) >> 55) != hb[j]) ++bad;
                xs += r.y;
            }
        }
        const u64 want = (n / (1 << 20)) * ((1ull << 20) * ((1 << 20) - 1) / 2);
        printf("verify: buckets %u (%.1f%% slack) rows %llu/%llu wrong-bin %llu payload-sum %s\n", nb,
               100.0 * ((double)nb * 256 - n) / n, tot, n, bad, xs == want ? "ok" : "MISMATCH");
    }
    return 0;
}
