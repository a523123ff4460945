// hj_radix.hip -- radix-partitioned hash join for large build sides (gfx950).
//
// Why (profiles/r01_micro_primitives.txt): on MI355X a random 16-B read from
// a table far larger than the caches costs a 64-B HBM line (~50 G/s chip-wide)
// and a device-scope CAS executes at the memory side (~17 G/s), so a
// global-table build of 2^28 rows is CAS-bound (32 ms) and its probe is
// line-bound.  Partitioning both relations by the top bits of the key hash
// until a partition's build side fits one workgroup's LDS turns every HBM
// access into a streaming, coalesced one; the hash table lives only in LDS.
//
//   pass k (1..3): tile histogram  ->  exclusive scan  ->  scatter (counting
//                  sort of a 4096-row tile in LDS, then runs of rows written
//                  contiguously to their partition)  ->  next segment offsets
//   join:          one workgroup per (partition, S chunk of 8192 rows): build
//                  the partition's R rows into an LDS table (8192 slots,
//                  <= 5120 rows per round), probe the chunk's S rows, count,
//                  block-scan, reserve the block's output with ONE global
//                  atomic, and write every pair at its exact position.
//
// The reference's count -> prefix -> probe protocol (join_v1.mlir:288-521) is
// kept, but per workgroup and on LDS, so the output needs no staging buffer
// and has no overflow path.
#include "hj_internal.h"

namespace hj {
namespace {

typedef unsigned long long u64;
constexpr u64 kGold = 0x9E3779B97F4A7C15ull;
constexpr int kTile = 4096;        // rows per partition-pass tile
constexpr int kPassThreads = 512;  // 8 rows per thread
constexpr int kJoinThreads = 1024;
constexpr int kJoinItems = 8;      // S rows per thread -> 8192-row chunk
constexpr int kChunk = kJoinThreads * kJoinItems;
constexpr int kTSlots = 8192;      // LDS table slots (128 KiB wide)
constexpr int kRCap = 5120;        // build rows per round (load factor <= 0.625)

__device__ __forceinline__ u64 rhash(u64 k) { return k * kGold; }

// --------------------------------------------------------------- helpers
// Largest s in [0, nseg) with start[s] <= w (start[nseg] > w): segment of
// work item / tile w.  Empty segments are skipped automatically.
__device__ __forceinline__ int find_seg(const unsigned *start, int nseg, unsigned w) {
    int lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (start[mid] <= w) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Block-wide exclusive scan of one u64 per thread.  All NT threads must call.
template <int NT>
__device__ __forceinline__ u64 block_excl_scan(u64 v, u64 *wsum, u64 *total) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u64 x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const u64 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
        u64 t = lane < NW ? wsum[lane] : 0ull;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            const u64 y = __shfl_up(t, o, 64);
            if (lane >= o) t += y;
        }
        if (lane < NW) wsum[lane] = t;
    }
    __syncthreads();
    const u64 before = w ? wsum[w - 1] : 0ull;
    *total = wsum[NW - 1];
    __syncthreads();   // wsum reusable after return
    return before + x - v;
}

// Row loaders of the partition passes' first input.
template <class KT, class PT, int FORM>
__device__ __forceinline__ void load_row(const void *key, const void *pay, long long row_base, long long row, KT &k,
                                         PT &p) {
    if constexpr (FORM == kPacked64) {
        const ulonglong2 v = ((const ulonglong2 *)key)[row];
        k = (KT)v.x;
        p = (PT)v.y;
    } else if constexpr (FORM == kCol32) {
        k = (KT)(unsigned)((const int *)key)[row];
        p = (PT)(row_base + row);
    } else {
        k = ((const KT *)key)[row];
        p = ((const PT *)pay)[row];
    }
}

template <class KT, int FORM>
__device__ __forceinline__ KT load_key(const void *key, long long row) {
    if constexpr (FORM == kPacked64) return (KT)((const u64 *)key)[2 * row];
    else if constexpr (FORM == kCol32) return (KT)(unsigned)((const int *)key)[row];
    else return ((const KT *)key)[row];
}

// --------------------------------------------------------------- maps
// start[s] = sum over s' < s of count(s'), count(s) = ceil(len_a(s) / chunk),
// or 0 when off_b is given and segment s of b is empty (no build rows ->
// nothing to join).  One block of 1024 threads.
__global__ __launch_bounds__(1024) void k_chunk_map(const u64 *off_a, const u64 *off_b, int nseg, unsigned chunk,
                                                    unsigned *start) {
    __shared__ u64 wsum[16];
    const int per = (nseg + 1023) / 1024;
    const int s0 = threadIdx.x * per;
    u64 local = 0;
    for (int s = s0; s < s0 + per && s < nseg; ++s) {
        const u64 len = off_a[s + 1] - off_a[s];
        const bool live = off_b ? (off_b[s + 1] > off_b[s]) : true;
        local += live ? (len + chunk - 1) / chunk : 0ull;
    }
    u64 total;
    u64 run = block_excl_scan<1024>(local, wsum, &total);
    for (int s = s0; s < s0 + per && s < nseg; ++s) {
        start[s] = (unsigned)run;
        const u64 len = off_a[s + 1] - off_a[s];
        const bool live = off_b ? (off_b[s + 1] > off_b[s]) : true;
        run += live ? (len + chunk - 1) / chunk : 0ull;
    }
    if (threadIdx.x == 0) start[nseg] = (unsigned)total;
}

__global__ void k_set_off(u64 *off, u64 n) {
    if (threadIdx.x == 0) {
        off[0] = 0;
        off[1] = n;
    }
}

// --------------------------------------------------------------- scan
// In-place exclusive scan of a u64 array (3 kernels: block scan, scan of
// block sums, add).  8192 elements per block.
constexpr int kScanPer = 8;
constexpr int kScanBlock = 1024 * kScanPer;

__global__ __launch_bounds__(1024) void k_scan_blocks(u64 *a, u64 n, u64 *sums) {
    __shared__ u64 wsum[16];
    const u64 base = (u64)blockIdx.x * kScanBlock + (u64)threadIdx.x * kScanPer;
    u64 v[kScanPer], s = 0;
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        v[i] = (base + i < n) ? a[base + i] : 0ull;
        s += v[i];
    }
    u64 total;
    u64 run = block_excl_scan<1024>(s, wsum, &total);
#pragma unroll
    for (int i = 0; i < kScanPer; ++i) {
        if (base + i < n) a[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_scan_sums(u64 *sums, unsigned nb) {
    __shared__ u64 wsum[16];
    u64 carry = 0;
    for (unsigned b0 = 0; b0 < nb; b0 += 1024) {
        const unsigned i = b0 + threadIdx.x;
        const u64 v = i < nb ? sums[i] : 0ull;
        u64 total;
        const u64 ex = block_excl_scan<1024>(v, wsum, &total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(1024) void k_scan_add(u64 *a, u64 n, const u64 *sums) {
    const u64 add = sums[blockIdx.x];
    const u64 base = (u64)blockIdx.x * kScanBlock;
    for (int i = threadIdx.x; i < kScanBlock; i += 1024)
        if (base + i < n) a[base + i] += add;
}

// --------------------------------------------------------------- partition pass
struct PassArgs {
    const void *in_key;
    const void *in_pay;
    long long row_base;
    const u64 *seg_off;       // nseg + 1
    int nseg;
    const unsigned *tile_start;  // nseg + 1
    u64 *hist;                // [seg][bin][tile] counts, then exclusive offsets
    void *out_key;
    void *out_pay;
    u64 *next_off;            // nseg * F + 1
    int shift;                // bin = (hash >> shift) & (F - 1)
    int fbits;
};

__device__ __forceinline__ void tile_of(const PassArgs &a, unsigned wg, int &seg, unsigned &t, unsigned &ntiles,
                                        u64 &lo, u64 &hi) {
    seg = a.nseg == 1 ? 0 : find_seg(a.tile_start, a.nseg, wg);
    t = wg - a.tile_start[seg];
    ntiles = a.tile_start[seg + 1] - a.tile_start[seg];
    lo = a.seg_off[seg] + (u64)t * kTile;
    const u64 e = a.seg_off[seg + 1];
    hi = lo + kTile < e ? lo + kTile : e;
}

template <class KT, int FORM>
__global__ __launch_bounds__(kPassThreads) void k_hist(PassArgs a) {
    __shared__ unsigned cnt[256];
    const unsigned wg = blockIdx.x;
    if (wg >= a.tile_start[a.nseg]) return;   // upper-bound grid
    int seg;
    unsigned t, ntiles;
    u64 lo, hi;
    tile_of(a, wg, seg, t, ntiles, lo, hi);
    const unsigned F = 1u << a.fbits;
    for (unsigned b = threadIdx.x; b < F; b += kPassThreads) cnt[b] = 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kTile / kPassThreads; ++i) {
        const u64 row = lo + (u64)i * kPassThreads + threadIdx.x;
        if (row < hi) {
            const KT k = load_key<KT, FORM>(a.in_key, (long long)row);
            atomicAdd(&cnt[(unsigned)(rhash((u64)k) >> a.shift) & (F - 1)], 1u);
        }
    }
    __syncthreads();
    const u64 base = (u64)a.tile_start[seg] * F;
    for (unsigned b = threadIdx.x; b < F; b += kPassThreads) a.hist[base + (u64)b * ntiles + t] = cnt[b];
}

template <class KT, class PT, int FORM>
__global__ __launch_bounds__(kPassThreads) void k_scatter(PassArgs a) {
    constexpr int IT = kTile / kPassThreads;
    __shared__ KT sk[kTile];
    __shared__ PT sp[kTile];
    __shared__ unsigned char sb[kTile];
    __shared__ unsigned cnt[256];
    __shared__ long long dst_base[256];
    const unsigned wg = blockIdx.x;
    if (wg >= a.tile_start[a.nseg]) return;
    int seg;
    unsigned t, ntiles;
    u64 lo, hi;
    tile_of(a, wg, seg, t, ntiles, lo, hi);
    const unsigned F = 1u << a.fbits;
    for (unsigned b = threadIdx.x; b < F; b += kPassThreads) cnt[b] = 0u;
    __syncthreads();
    KT k[IT];
    PT p[IT];
    unsigned bin[IT], rank[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const u64 row = lo + (u64)i * kPassThreads + threadIdx.x;
        if (row < hi) {
            load_row<KT, PT, FORM>(a.in_key, a.in_pay, a.row_base, (long long)row, k[i], p[i]);
            bin[i] = (unsigned)(rhash((u64)k[i]) >> a.shift) & (F - 1);
            rank[i] = atomicAdd(&cnt[bin[i]], 1u);
        } else {
            bin[i] = 0xFFFFFFFFu;
        }
    }
    __syncthreads();
    // exclusive scan of the F bin counts (first wave, 4 bins per lane) and
    // the destination base of each bin's run: scanned global offset - local start
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        unsigned c[4], s = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned b = lane * 4 + j;
            c[j] = b < F ? cnt[b] : 0u;
            s += c[j];
        }
        unsigned x = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        unsigned run = x - s;
        const u64 hb = (u64)a.tile_start[seg] * F;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned b = lane * 4 + j;
            if (b < F) {
                cnt[b] = run;   // now the local start of bin b
                dst_base[b] = (long long)a.hist[hb + (u64)b * ntiles + t] - (long long)run;
            }
            run += c[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        if (bin[i] != 0xFFFFFFFFu) {
            const unsigned pos = cnt[bin[i]] + rank[i];
            sk[pos] = k[i];
            sp[pos] = p[i];
            sb[pos] = (unsigned char)bin[i];
        }
    }
    __syncthreads();
    const unsigned n = (unsigned)(hi - lo);
    KT *ok = (KT *)a.out_key;
    PT *op = (PT *)a.out_pay;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const unsigned j = (unsigned)i * kPassThreads + threadIdx.x;
        if (j < n) {
            const u64 dst = (u64)(dst_base[sb[j]] + (long long)j);
            ok[dst] = sk[j];
            op[dst] = sp[j];
        }
    }
}

__global__ __launch_bounds__(256) void k_next_off(PassArgs a) {
    const unsigned F = 1u << a.fbits;
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    const u64 tot = (u64)a.nseg * F;
    if (i < tot) {
        const int seg = (int)(i >> a.fbits);
        const unsigned b = (unsigned)(i & (F - 1));
        const unsigned nt = a.tile_start[seg + 1] - a.tile_start[seg];
        a.next_off[i] = nt ? a.hist[(u64)a.tile_start[seg] * F + (u64)b * nt] : a.seg_off[seg];
    }
    if (i == 0) a.next_off[tot] = a.seg_off[a.nseg];
}

// --------------------------------------------------------------- join
struct JoinArgs {
    const void *rk, *rp, *sk, *sp;   // partitioned SoA relations
    const u64 *r_off, *s_off;        // P + 1 each
    int P;
    const unsigned *work_start;      // P + 1: S chunks per partition (0 if no R rows)
    int tshift;                      // LDS slot = (hash >> tshift) & (kTSlots - 1)
    void *out_r, *out_s;
    long long cap;
    u64 *counter;
    u64 *dup_flag;                   // set to 1 if any partition's build rows repeat a key
};

struct JWide {
    typedef u64 KT;
    typedef u64 PT;
    static constexpr bool kNullKeys = true;
};
struct JNarrow {
    typedef unsigned KT;
    typedef unsigned PT;
    static constexpr bool kNullKeys = false;
};

template <class J, bool WRITE>
__global__ __launch_bounds__(kJoinThreads) void k_join(JoinArgs a) {
    typedef typename J::KT KT;
    typedef typename J::PT PT;
    constexpr u64 kEmpty = J::kNullKeys ? kEmptyKey64 : ~0ull;
    constexpr unsigned kMask = kTSlots - 1;
    // wide: tkey/tpay; narrow: tkey holds packed (key << 32 | row id)
    __shared__ u64 tkey[kTSlots];
    __shared__ PT tpay[J::kNullKeys ? kTSlots : 1];
    __shared__ u64 wsum[16];
    __shared__ u64 s_base;
    __shared__ unsigned s_dup;

    const unsigned w = blockIdx.x;
    if (w >= a.work_start[a.P]) return;   // upper-bound grid
    const int p = find_seg(a.work_start, a.P, w);
    const unsigned c = w - a.work_start[p];
    const u64 s_lo = a.s_off[p] + (u64)c * kChunk;
    const u64 s_end = a.s_off[p + 1];
    const u64 s_hi = s_lo + kChunk < s_end ? s_lo + kChunk : s_end;
    const u64 r_lo = a.r_off[p], r_hi = a.r_off[p + 1];

    KT k[kJoinItems];
    PT pv[kJoinItems];
    unsigned h0[kJoinItems];
    bool v[kJoinItems];
    bool has_null_s = false;
#pragma unroll
    for (int i = 0; i < kJoinItems; ++i) {
        const u64 row = s_lo + (u64)i * kJoinThreads + threadIdx.x;
        v[i] = row < s_hi;
        k[i] = v[i] ? ((const KT *)a.sk)[row] : (KT)0;
        pv[i] = v[i] ? ((const PT *)a.sp)[row] : (PT)0;
        h0[i] = (unsigned)(rhash((u64)k[i]) >> a.tshift) & kMask;
        if (J::kNullKeys && v[i] && (u64)k[i] == kEmptyKey64) {
            has_null_s = true;
            v[i] = false;   // matched by the null pass below
        }
    }
    u64 n_null_r = 0;
    const KT *rk = (const KT *)a.rk;
    const PT *rp = (const PT *)a.rp;

    for (u64 r0 = r_lo; r0 < r_hi; r0 += kRCap) {
        const u64 r1 = r0 + kRCap < r_hi ? r0 + kRCap : r_hi;
        // ---- init: every slot EMPTY (16-B LDS stores)
        for (int j = threadIdx.x; j < kTSlots / 2; j += kJoinThreads)
            ((ulonglong2 *)tkey)[j] = make_ulonglong2(kEmpty, kEmpty);
        if (threadIdx.x == 0) s_dup = 0u;
        __syncthreads();
        // ---- build this round's rows
        bool dup = false;
        for (u64 row = r0 + threadIdx.x; row < r1; row += kJoinThreads) {
            const KT key = rk[row];
            const PT pay = rp[row];
            if (J::kNullKeys && (u64)key == kEmptyKey64) {
                ++n_null_r;
                continue;
            }
            unsigned h = (unsigned)(rhash((u64)key) >> a.tshift) & kMask;
            const u64 val = J::kNullKeys ? (u64)key : (((u64)key << 32) | (u64)pay);
            while (true) {
                const u64 old = atomicCAS(&tkey[h], kEmpty, val);
                if (old == kEmpty) break;
                dup |= J::kNullKeys ? (old == (u64)key) : ((old >> 32) == (u64)key);
                h = (h + 1) & kMask;
            }
            if constexpr (J::kNullKeys) tpay[h] = pay;
        }
        if (dup) s_dup = 1u;
        __syncthreads();
        const bool unique = s_dup == 0u;
        if (!unique && threadIdx.x == 0)
            __hip_atomic_store(a.dup_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // ---- count (and remember the matched slot when build keys are unique)
        unsigned m[kJoinItems];
        u64 cnt = 0;
#pragma unroll
        for (int i = 0; i < kJoinItems; ++i) {
            m[i] = 0xFFFFFFFFu;
            if (!v[i]) continue;
            unsigned h = h0[i];
            while (true) {
                const u64 sv = tkey[h];
                if (sv == kEmpty) break;
                const bool hit = J::kNullKeys ? (sv == (u64)k[i]) : ((sv >> 32) == (u64)k[i]);
                if (hit) {
                    ++cnt;
                    if (unique) {
                        m[i] = h;
                        break;
                    }
                }
                h = (h + 1) & kMask;
            }
        }
        u64 total;
        const u64 pre = block_excl_scan<kJoinThreads>(cnt, wsum, &total);
        if constexpr (!WRITE) {
            if (threadIdx.x == 0 && total) atomicAdd(a.counter, total);
        } else if (total) {
            if (threadIdx.x == 0) s_base = atomicAdd(a.counter, total);
            __syncthreads();
            u64 pos = s_base + pre;
            PT *orr = (PT *)a.out_r;
            PT *oss = (PT *)a.out_s;
#pragma unroll
            for (int i = 0; i < kJoinItems; ++i) {
                if (!v[i]) continue;
                if (unique) {
                    if (m[i] != 0xFFFFFFFFu) {
                        if (pos < (u64)a.cap) {
                            orr[pos] = J::kNullKeys ? tpay[m[i]] : (PT)(tkey[m[i]] & 0xffffffffull);
                            oss[pos] = pv[i];
                        }
                        ++pos;
                    }
                } else {
                    unsigned h = h0[i];
                    while (true) {
                        const u64 sv = tkey[h];
                        if (sv == kEmpty) break;
                        const bool hit = J::kNullKeys ? (sv == (u64)k[i]) : ((sv >> 32) == (u64)k[i]);
                        if (hit) {
                            if (pos < (u64)a.cap) {
                                orr[pos] = J::kNullKeys ? tpay[h] : (PT)(sv & 0xffffffffull);
                                oss[pos] = pv[i];
                            }
                            ++pos;
                        }
                        h = (h + 1) & kMask;
                    }
                }
            }
        }
        __syncthreads();   // table reused by the next round
    }

    // ---- INT64_MIN keys (the wide EMPTY sentinel): matched outside the table.
    if constexpr (J::kNullKeys) {
        if (__syncthreads_or(has_null_s ? 1 : 0)) {
            u64 nn;
            (void)block_excl_scan<kJoinThreads>(n_null_r, wsum, &nn);   // null R rows of this partition
            u64 cnt = 0;
            if (has_null_s) {
#pragma unroll
                for (int i = 0; i < kJoinItems; ++i) {
                    const u64 row = s_lo + (u64)i * kJoinThreads + threadIdx.x;
                    if (row < s_hi && (u64)k[i] == kEmptyKey64) cnt += nn;
                }
            }
            u64 total;
            const u64 pre = block_excl_scan<kJoinThreads>(cnt, wsum, &total);
            if constexpr (!WRITE) {
                if (threadIdx.x == 0 && total) atomicAdd(a.counter, total);
            } else if (total) {
                if (threadIdx.x == 0) s_base = atomicAdd(a.counter, total);
                __syncthreads();
                u64 pos = s_base + pre;
                if (has_null_s) {
                    for (int i = 0; i < kJoinItems; ++i) {
                        const u64 row = s_lo + (u64)i * kJoinThreads + threadIdx.x;
                        if (!(row < s_hi && (u64)k[i] == kEmptyKey64)) continue;
                        for (u64 r = r_lo; r < r_hi; ++r) {
                            if ((u64)rk[r] != kEmptyKey64) continue;
                            if (pos < (u64)a.cap) {
                                ((PT *)a.out_r)[pos] = rp[r];
                                ((PT *)a.out_s)[pos] = pv[i];
                            }
                            ++pos;
                        }
                    }
                }
            }
        }
    }
}

inline unsigned blocks_for(u64 n, u64 per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

// ----------------------------------------------------------------- planning
RadixPlan radix_plan(long long n_build, int force_bits) {
    RadixPlan pl;
    int bits = 1;
    while (bits < 24 && ((unsigned long long)n_build >> bits) > 4096ull) ++bits;   // avg build rows per partition <= 4096
    if (force_bits > 0) bits = force_bits < 24 ? force_bits : 24;
    pl.total_bits = bits;
    pl.passes = bits <= 8 ? 1 : (bits <= 16 ? 2 : 3);
    int left = bits;
    for (int i = 0; i < pl.passes; ++i) {
        pl.bits[i] = (left + (pl.passes - i) - 1) / (pl.passes - i);
        left -= pl.bits[i];
    }
    for (int i = pl.passes; i < 3; ++i) pl.bits[i] = 0;
    return pl;
}

size_t radix_hist_elems(long long n, int max_nseg) {
    return ((size_t)n / kTile + (size_t)max_nseg + 2) * 256;
}

int radix_chunk_rows() { return kChunk; }

// Partition one relation into the plan's 2^total_bits partitions.
// Output: out_key/out_pay (SoA, element size esz each) grouped by partition,
// out_off (P + 1 offsets).  Uses ws.tmp_* as the ping buffer for multi-pass
// plans.  Asynchronous; no allocation.
hipError_t radix_partition(const SrcDev &src, bool wide, const RadixPlan &pl, const RadixWork &ws, void *out_key,
                           void *out_pay, unsigned long long *out_off, hipStream_t st) {
    const u64 n = (u64)src.n;
    hipLaunchKernelGGL(k_set_off, dim3(1), dim3(64), 0, st, ws.off_a, n);
    int nseg = 1;
    int shift = 64;
    const void *in_k = src.key, *in_p = src.pay;
    int form = src.form;
    u64 *seg_off = ws.off_a;
    for (int pass = 0; pass < pl.passes; ++pass) {
        const int fb = pl.bits[pass];
        shift -= fb;
        const bool last = pass == pl.passes - 1;
        // destination of this pass: final buffers on the last pass, else ping/pong
        void *dk, *dp;
        if (last) {
            dk = out_key;
            dp = out_pay;
        } else {
            const bool to_tmp = ((pl.passes - 1 - pass) % 2) == 1;
            dk = to_tmp ? ws.tmp_key : out_key;
            dp = to_tmp ? ws.tmp_pay : out_pay;
        }
        u64 *next_off = last ? out_off : (seg_off == ws.off_a ? ws.off_b : ws.off_a);
        PassArgs a;
        a.in_key = in_k;
        a.in_pay = in_p;
        a.row_base = src.row_base;
        a.seg_off = seg_off;
        a.nseg = nseg;
        a.tile_start = ws.tile_start;
        a.hist = ws.hist;
        a.out_key = dk;
        a.out_pay = dp;
        a.next_off = next_off;
        a.shift = shift;
        a.fbits = fb;
        const unsigned F = 1u << fb;
        hipLaunchKernelGGL(k_chunk_map, dim3(1), dim3(1024), 0, st, (const u64 *)seg_off, (const u64 *)nullptr, nseg,
                           (unsigned)kTile, ws.tile_start);
        const unsigned grid = (unsigned)(n / kTile + nseg + 1);
        const u64 hlen = (u64)grid * F;
        hipError_t e = hipMemsetAsync(ws.hist, 0, hlen * sizeof(u64), st);
        if (e != hipSuccess) return e;
#define HJ_HIST(KT, FORM) hipLaunchKernelGGL((k_hist<KT, FORM>), dim3(grid), dim3(kPassThreads), 0, st, a)
#define HJ_SCAT(KT, PT, FORM) hipLaunchKernelGGL((k_scatter<KT, PT, FORM>), dim3(grid), dim3(kPassThreads), 0, st, a)
        if (wide) {
            if (form == kPacked64) HJ_HIST(u64, kPacked64);
            else HJ_HIST(u64, kCols64);
        } else {
            if (form == kCol32) HJ_HIST(unsigned, kCol32);
            else HJ_HIST(unsigned, kCols64);
        }
        // exclusive scan of the [seg][bin][tile] counts -> output offsets
        const unsigned nb = blocks_for(hlen, kScanBlock);
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, st, ws.hist, hlen, ws.scan_sums);
        if (nb > 1) {
            hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, st, ws.scan_sums, nb);
            hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(1024), 0, st, ws.hist, hlen, (const u64 *)ws.scan_sums);
        }
        if (wide) {
            if (form == kPacked64) HJ_SCAT(u64, u64, kPacked64);
            else HJ_SCAT(u64, u64, kCols64);
        } else {
            if (form == kCol32) HJ_SCAT(unsigned, unsigned, kCol32);
            else HJ_SCAT(unsigned, unsigned, kCols64);
        }
#undef HJ_HIST
#undef HJ_SCAT
        hipLaunchKernelGGL(k_next_off, dim3(blocks_for((u64)nseg * F + 1, 256)), dim3(256), 0, st, a);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        // next pass reads what this one wrote, as SoA
        in_k = dk;
        in_p = dp;
        form = kCols64;
        seg_off = next_off;
        nseg *= (int)F;
    }
    return hipSuccess;
}

hipError_t radix_join(bool wide, const RadixPlan &pl, const void *rk, const void *rp, const unsigned long long *r_off,
                      const void *sk, const void *sp, const unsigned long long *s_off, long long n_s,
                      unsigned *work_start, void *out_r, void *out_s, long long cap, unsigned long long *counter,
                      unsigned long long *dup_flag, bool count_only, hipStream_t st) {
    const int P = 1 << pl.total_bits;
    hipLaunchKernelGGL(k_chunk_map, dim3(1), dim3(1024), 0, st, s_off, r_off, P, (unsigned)kChunk, work_start);
    JoinArgs a;
    a.rk = rk;
    a.rp = rp;
    a.sk = sk;
    a.sp = sp;
    a.r_off = r_off;
    a.s_off = s_off;
    a.P = P;
    a.work_start = work_start;
    a.tshift = 64 - pl.total_bits - 13;   // 13 = log2(kTSlots): the bits right below the partition bits
    a.out_r = out_r;
    a.out_s = out_s;
    a.cap = cap;
    a.counter = counter;
    a.dup_flag = dup_flag;
    const unsigned grid = (unsigned)((u64)n_s / kChunk + (u64)P + 1);
    if (wide) {
        if (count_only) hipLaunchKernelGGL((k_join<JWide, false>), dim3(grid), dim3(kJoinThreads), 0, st, a);
        else hipLaunchKernelGGL((k_join<JWide, true>), dim3(grid), dim3(kJoinThreads), 0, st, a);
    } else {
        if (count_only) hipLaunchKernelGGL((k_join<JNarrow, false>), dim3(grid), dim3(kJoinThreads), 0, st, a);
        else hipLaunchKernelGGL((k_join<JNarrow, true>), dim3(grid), dim3(kJoinThreads), 0, st, a);
    }
    return hipGetLastError();
}

}  // namespace hj
