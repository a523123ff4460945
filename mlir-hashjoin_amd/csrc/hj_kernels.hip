// hj_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the hash join.
//
// Reference kernels replaced (kernel inventory):
//   initializeHT  join_v1.mlir:180-202  -> k_init    (slot fill, 16 B/lane)
//   build         join_v1.mlir:213-277  -> k_build   (linear probing, 64-bit CAS)
//   count         join_v1.mlir:288-425  -> k_probe<WRITE=false>
//   probe v1/v2   join_v1.mlir:436-521, join_v2.mlir:450-604
//                                       -> k_probe<WRITE=true>: ILP slot
//                                          reads, ballot-compacted output,
//                                          one global cursor add per block
// plus the radix partition used by the multi-GPU exchange and the
// counter-based generators of the benchmark inputs.
//
// Wave64 throughout: 256-thread blocks (4 waves), all per-lane work
// independent, no warp-32 idioms.  Integer/byte work: no MFMA.
#include "hj_internal.h"
#include "hj_gen.h"

namespace hj {
namespace {

constexpr int kBlock = 256;
constexpr int kBuildItems = 4;   // rows per thread in build (CAS ILP)
constexpr int kProbeItems = 8;   // rows per thread in probe (tile = 2048 rows)
constexpr int kPartItems = 8;    // rows per thread in partition

__device__ __forceinline__ unsigned long long slot_of(unsigned long long k, int shift) {
    return (k * 0x9E3779B97F4A7C15ull) >> shift;   // Fibonacci hashing, top bits
}

// ------------------------------------------------------------------ sources
struct Tuple {
    unsigned long long k, p;
};

template <int FORM>
__device__ __forceinline__ Tuple load_src(const SrcDev &s, long long row);

template <>
__device__ __forceinline__ Tuple load_src<kCols64>(const SrcDev &s, long long row) {
    return {((const unsigned long long *)s.key)[row], ((const unsigned long long *)s.pay)[row]};
}
template <>
__device__ __forceinline__ Tuple load_src<kPacked64>(const SrcDev &s, long long row) {
    const ulonglong2 v = ((const ulonglong2 *)s.key)[row];
    return {v.x, v.y};
}
template <>
__device__ __forceinline__ Tuple load_src<kCol32>(const SrcDev &s, long long row) {
    return {(unsigned long long)(unsigned)((const int *)s.key)[row],
            (unsigned long long)(s.row_base + row)};
}

// ------------------------------------------------------------------ layouts
template <int L>
struct Lay;

template <>
struct Lay<kWide> {
    using slot_t = Slot64;
    using out_t = long long;
    static constexpr unsigned long long kEmptyWord = kEmptyKey64;
    static __device__ __forceinline__ unsigned long long *word(slot_t *sl, unsigned long long h) { return &sl[h].key; }
    static __device__ __forceinline__ unsigned long long cas_val(unsigned long long k, unsigned long long) { return k; }
    static __device__ __forceinline__ unsigned long long word_key(unsigned long long w) { return w; }
    static __device__ __forceinline__ void after_claim(slot_t *sl, unsigned long long h, unsigned long long p) { sl[h].pay = p; }
    static __device__ __forceinline__ bool empty(const slot_t &s) { return s.key == kEmptyKey64; }
    static __device__ __forceinline__ unsigned long long key(const slot_t &s) { return s.key; }
    static __device__ __forceinline__ unsigned long long pay(const slot_t &s) { return s.pay; }
    static __device__ __forceinline__ bool null_key(unsigned long long k) { return k == kEmptyKey64; }
};

template <>
struct Lay<kNarrow> {
    using slot_t = unsigned long long;
    using out_t = int;
    static constexpr unsigned long long kEmptyWord = kEmptySlot32;
    static __device__ __forceinline__ unsigned long long *word(slot_t *sl, unsigned long long h) { return &sl[h]; }
    static __device__ __forceinline__ unsigned long long cas_val(unsigned long long k, unsigned long long p) { return (k << 32) | (p & 0xffffffffull); }
    static __device__ __forceinline__ unsigned long long word_key(unsigned long long w) { return w >> 32; }
    static __device__ __forceinline__ void after_claim(slot_t *, unsigned long long, unsigned long long) {}
    static __device__ __forceinline__ bool empty(const slot_t &s) { return s == kEmptySlot32; }
    static __device__ __forceinline__ unsigned long long key(const slot_t &s) { return s >> 32; }
    static __device__ __forceinline__ unsigned long long pay(const slot_t &s) { return s & 0xffffffffull; }
    static __device__ __forceinline__ bool null_key(unsigned long long) { return false; }
};

template <int N, typename T>
__device__ __forceinline__ T pick(const T (&a)[N], int i) {   // static-index select: no scratch
    T r = a[0];
#pragma unroll
    for (int j = 1; j < N; ++j) r = (i == j) ? a[j] : r;
    return r;
}

// ------------------------------------------------------------------ init
// initializeHT (join_v2.mlir:203-225) sets heads[:] = -1; here every slot is
// set EMPTY with 16-B stores, and the side count / dup flag are reset.
template <int L>
__global__ __launch_bounds__(kBlock) void k_init(TableDev t, unsigned long long n16) {
    const ulonglong2 v = (L == kWide) ? make_ulonglong2(kEmptyKey64, 0ull)
                                      : make_ulonglong2(kEmptySlot32, kEmptySlot32);
    ulonglong2 *p = (ulonglong2 *)t.slots;
    const unsigned long long base = (unsigned long long)blockIdx.x * (kBlock * 4) + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const unsigned long long j = base + (unsigned long long)i * kBlock;
        if (j < n16) p[j] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x < 2) t.meta[threadIdx.x] = 0ull;
}

// ------------------------------------------------------------------ build
// build + @insertNodeInHashTable (join_v2.mlir:236-300): the reference takes
// a node with atomicAdd(freeIndex) -- one address hit by every thread -- and
// prepends it with atomicExch on the bucket head.  Here each row claims its
// own slot with one 64-bit CAS at its hash position (linear probing on
// failure).  The first CAS of all kBuildItems rows is issued before any
// result is consumed, so each lane has that many atomics in flight.
// A failed CAS that returns the row's own key proves the build side has a
// duplicate key (both rows walk the same probe sequence, so the later one
// must fail on the earlier one's slot); that sets meta[1], and probes then
// keep walking past matches.  Without duplicates a probe stops at its match.
template <int L, int FORM>
__global__ __launch_bounds__(kBlock) void k_build(TableDev t, SrcDev src) {
    using LY = Lay<L>;
    using slot_t = typename LY::slot_t;
    slot_t *sl = (slot_t *)t.slots;
    const long long base = (long long)blockIdx.x * (kBlock * kBuildItems) + threadIdx.x;
    unsigned long long k[kBuildItems], p[kBuildItems], h[kBuildItems], o[kBuildItems];
    bool v[kBuildItems];
#pragma unroll
    for (int i = 0; i < kBuildItems; ++i) {
        const long long row = base + (long long)i * kBlock;
        v[i] = row < src.n;
        Tuple tp = v[i] ? load_src<FORM>(src, row) : Tuple{0ull, 0ull};
        k[i] = tp.k;
        p[i] = tp.p;
    }
#pragma unroll
    for (int i = 0; i < kBuildItems; ++i) {
        if (v[i] && LY::null_key(k[i])) {   // wide only: INT64_MIN keys -> side list
            const unsigned long long idx = atomicAdd(&t.meta[0], 1ull);
            t.side[idx] = p[i];
            v[i] = false;
        }
        h[i] = slot_of(k[i], t.shift);
        o[i] = v[i] ? atomicCAS(LY::word(sl, h[i]), LY::kEmptyWord, LY::cas_val(k[i], p[i]))
                    : LY::kEmptyWord;
    }
    bool dup = false;
#pragma unroll
    for (int i = 0; i < kBuildItems; ++i) {
        if (!v[i]) continue;
        unsigned long long hh = h[i], old = o[i];
        while (old != LY::kEmptyWord) {
            dup |= (LY::word_key(old) == k[i]);
            hh = (hh + 1) & t.mask;
            old = atomicCAS(LY::word(sl, hh), LY::kEmptyWord, LY::cas_val(k[i], p[i]));
        }
        LY::after_claim(sl, hh, p[i]);
    }
    // one store per block: same-address stores from every thread that saw a
    // repeated key serialise at the memory side (the radix join's flag cost
    // 3.5 ms at 2^28 uniform keys before it was made per workgroup)
    if (__syncthreads_or(dup ? 1 : 0) && threadIdx.x == 0)
        __hip_atomic_store(&t.meta[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ probe tiles
// A probe tile is kProbeItems * kBlock rows: tile q = rows [q * kTile, ...).
constexpr int kProbeTile = kBlock * kProbeItems;
#ifndef HJ_LDS_TABLE_BYTES
#define HJ_LDS_TABLE_BYTES 65536
#endif
// global tables up to this size are probed from LDS (k_probe<..., LDS>);
// kLdsPerCu: the LDS the copies of one CU's workgroups may take together
constexpr int kLdsTableBytes = HJ_LDS_TABLE_BYTES;
constexpr int kLdsPerCu = 128 * 1024;

template <int L, int FORM>
__device__ __forceinline__ bool probe_row(const SrcDev &src, unsigned long long q, int i, Tuple &tp) {
    const long long row = (long long)q * kProbeTile + (long long)i * kBlock + threadIdx.x;
    if (row >= src.n) return false;
    tp = load_src<FORM>(src, row);
    return true;
}

// ------------------------------------------------------------------ probe
// count (join_v1.mlir:288-425, join_v2.mlir:311-439) and probe
// (join_v1.mlir:436-521, join_v2.mlir:450-604) in one kernel family.
//
// Each thread owns kProbeItems rows of a 2048-row tile (coalesced loads).
//
// Fast path (duplicate-free build side, no INT64_MIN probe key in the tile):
// every row's first slot load is issued before any is resolved, so a lane
// has kProbeItems random reads in flight (the table read is latency-bound:
// one dependent read per lane at a time left HBM idle); rows still open
// after their first slot walk the chain.  A row matches at most once, so
// the output is compacted with wave ballots in row-slot-major order: each
// store instruction writes one contiguous run per wave, after ONE global
// cursor add per tile.
//
// General path (duplicates or null keys): a flattened per-lane loop (one
// slot load per iteration; a lane moves to its next row when the current is
// resolved) with matches staged in LDS through a wave-aggregated cursor (the
// v2 idea, join_v2.mlir:525-538), one cursor add per tile and a coalesced
// flush; more than kStage matches spill straight to global (the v2 overflow
// path, :539-549).  The cursor counts every match, so a caller whose
// capacity was too small still learns the exact M (rows past cap dropped).
//
// LDS (small tables, <= kLdsTableBytes): each workgroup first copies the
// whole table into LDS and the fast path reads its slots there; the probes
// of a table that fits one XCD's L2 were random L2 reads (~82-96 G/s), well
// below the rate the probe side streams at (profiles/r06/r06sr_small_build_sides.txt).
template <int L, int FORM, bool WRITE, bool LDS = false>
__global__ __launch_bounds__(kBlock) void k_probe(TableDev t, SrcDev src, OutDev out, unsigned *slow,
                                                  unsigned long long slow_cap) {
    using LY = Lay<L>;
    using slot_t = typename LY::slot_t;
    using out_t = typename LY::out_t;
    constexpr int NW = kBlock / 64;
    __shared__ unsigned long long st_base;
    __shared__ unsigned long long wsum[NW];
    __shared__ unsigned s_cw[kProbeItems * NW];
    extern __shared__ ulonglong2 s_tab[];

    const slot_t *sl = (const slot_t *)t.slots;
    if constexpr (LDS) {
        const unsigned long long n16 = (t.mask + 1) * sizeof(slot_t) / 16;
        const ulonglong2 *g16 = (const ulonglong2 *)t.slots;
        for (unsigned long long j = threadIdx.x; j < n16; j += kBlock) s_tab[j] = g16[j];
        __syncthreads();
    }
    auto slot_at = [&](unsigned long long h) -> slot_t {
        if constexpr (LDS) return ((const slot_t *)s_tab)[h];
        else return sl[h];
    };
    const bool unique = (__hip_atomic_load(&t.meta[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const unsigned long long nt = (unsigned long long)((src.n + kProbeTile - 1) / kProbeTile);
    for (unsigned long long q = blockIdx.x; q < nt; q += gridDim.x) {
        unsigned long long K[kProbeItems], P[kProbeItems];
        bool V[kProbeItems];
        bool has_null = false;
#pragma unroll
        for (int i = 0; i < kProbeItems; ++i) {
            Tuple tp{0ull, 0ull};
            V[i] = probe_row<L, FORM>(src, q, i, tp);
            K[i] = tp.k;
            P[i] = tp.p;
            has_null |= V[i] && LY::null_key(K[i]);
        }
        // general path (k_probe_slow takes the tile): a null probe key, or
        // -- with repeated build keys -- a row with more than one match
        auto to_slow = [&]() {
            if (threadIdx.x == 0) {
                const unsigned long long j = atomicAdd(&t.meta[3], 1ull);
                if (j < slow_cap) slow[j] = (unsigned)q;   // (sized so it always is; else k_probe_slow flags the count)
            }
        };
        if (__syncthreads_or(has_null ? 1 : 0)) {
            to_slow();
            continue;
        }
        slot_t S[kProbeItems];
        unsigned long long H[kProbeItems];
#pragma unroll
        for (int i = 0; i < kProbeItems; ++i) {
            H[i] = slot_of(K[i], t.shift);
            if (V[i]) S[i] = slot_at(H[i]);
        }
        unsigned found = 0;
        unsigned long long RP[kProbeItems];
#pragma unroll
        for (int i = 0; i < kProbeItems; ++i) {
            RP[i] = 0;
            if (!V[i]) continue;
            // duplicate-free table: the chain ends at the match or at EMPTY
            // (a two-exit loop with nothing else in it)
            slot_t sv = S[i];
            unsigned long long hh = H[i];
            while (!LY::empty(sv) && LY::key(sv) != K[i]) {
                hh = (hh + 1) & t.mask;
                sv = slot_at(hh);
            }
            if (!LY::empty(sv)) {
                found |= 1u << i;
                RP[i] = LY::pay(sv);
            }
        }
        if (!unique) {
            // repeated build keys: a matched row walks on to EMPTY; a second
            // copy of its key sends the tile to the general path (a few
            // repeated keys used to send every tile there: i32 2^12 random
            // build keys, 3.2 ms against 0.6 without a repeat,
            // profiles/r06/r06lu_lds_table_probe_ab.txt)
            bool multi = false;
#pragma unroll
            for (int i = 0; i < kProbeItems; ++i) {
                if (!((found >> i) & 1u)) continue;
                unsigned long long hh = slot_of(K[i], t.shift);
                slot_t sv = slot_at(hh);
                while (!LY::empty(sv) && LY::key(sv) != K[i]) {   // (back to the first copy)
                    hh = (hh + 1) & t.mask;
                    sv = slot_at(hh);
                }
                hh = (hh + 1) & t.mask;
                sv = slot_at(hh);
                while (!LY::empty(sv) && !multi) {
                    multi = LY::key(sv) == K[i];
                    hh = (hh + 1) & t.mask;
                    sv = slot_at(hh);
                }
            }
            if (__syncthreads_or(multi ? 1 : 0)) {
                to_slow();
                continue;
            }
        }
        if constexpr (!WRITE) {
            unsigned long long c = (unsigned long long)__popc(found);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
            if (lane == 0) wsum[wv] = c;
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned long long tot = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) tot += wsum[w];
                if (tot) atomicAdd(out.counter, tot);
            }
        } else {
            const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
            unsigned lpre[kProbeItems];
#pragma unroll
            for (int i = 0; i < kProbeItems; ++i) {
                const unsigned long long bal = __ballot((found >> i) & 1u);
                lpre[i] = (unsigned)__popcll(bal & lt);
                if (lane == 0) s_cw[i * NW + wv] = (unsigned)__popcll(bal);
            }
            __syncthreads();
            if (wv == 0) {   // exclusive scan of the kProbeItems * NW runs (<= 64)
                static_assert(kProbeItems * NW <= 64, "one lane per run");
                const unsigned v = lane < kProbeItems * NW ? s_cw[lane] : 0u;
                unsigned x = v;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const unsigned y = __shfl_up(x, o, 64);
                    if (lane >= o) x += y;
                }
                if (lane < kProbeItems * NW) s_cw[lane] = x - v;
                if (lane == 63) st_base = x ? atomicAdd(out.counter, (unsigned long long)x) : 0ull;
            }
            __syncthreads();
            out_t *orr = (out_t *)out.r;
            out_t *oss = (out_t *)out.s;
#pragma unroll
            for (int i = 0; i < kProbeItems; ++i) {
                if (!((found >> i) & 1u)) continue;
                const unsigned long long gi = st_base + s_cw[i * NW + wv] + lpre[i];
                if (gi < (unsigned long long)out.cap) {
                    orr[gi] = (out_t)RP[i];
                    oss[gi] = (out_t)P[i];
                }
            }
        }
        __syncthreads();   // s_cw / st_base / wsum reused by the next tile
    }
}

// General path over the tiles k_probe handed over (slow[0 .. meta[3])):
// persistent workgroups, one tile at a time.
template <int L, int FORM, bool WRITE>
__global__ __launch_bounds__(kBlock) void k_probe_slow(TableDev t, SrcDev src, OutDev out, const unsigned *slow,
                                                       unsigned long long slow_cap) {
    using LY = Lay<L>;
    using slot_t = typename LY::slot_t;
    using out_t = typename LY::out_t;
    constexpr int kStage = 1024;
    constexpr int NW = kBlock / 64;
    __shared__ out_t st_r[WRITE ? kStage : 1];
    __shared__ out_t st_s[WRITE ? kStage : 1];
    __shared__ unsigned st_n;
    __shared__ unsigned long long st_base;
    __shared__ unsigned long long wsum[NW];

    const slot_t *sl = (const slot_t *)t.slots;
    const bool unique = (__hip_atomic_load(&t.meta[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0ull);
    const unsigned long long ntiles = t.meta[3] < slow_cap ? t.meta[3] : slow_cap;
    // an undersized slow list would drop tiles: report it through the count
    // (bit 63, never a real M) rather than return a short result
    if (blockIdx.x == 0 && threadIdx.x == 0 && t.meta[3] > slow_cap) atomicOr(out.counter, 1ull << 63);
    for (unsigned long long j = blockIdx.x; j < ntiles; j += gridDim.x) {
        if (threadIdx.x == 0) st_n = 0u;
        const unsigned id = slow[j];
        unsigned long long K[kProbeItems], P[kProbeItems];
        bool V[kProbeItems];
#pragma unroll
        for (int i = 0; i < kProbeItems; ++i) {
            Tuple tp{0ull, 0ull};
            V[i] = probe_row<L, FORM>(src, id, i, tp);
            K[i] = tp.k;
            P[i] = tp.p;
        }
        __syncthreads();   // st_n visible

        unsigned long long cnt = 0;
        auto emit = [&](unsigned long long rv, unsigned long long sv) {
            if constexpr (!WRITE) {
                ++cnt;
            } else {
                const unsigned idx = atomicAdd(&st_n, 1u);
                if (idx < (unsigned)kStage) {
                    st_r[idx] = (out_t)rv;
                    st_s[idx] = (out_t)sv;
                } else {
                    const unsigned long long g = atomicAdd(out.counter, 1ull);
                    if (g < (unsigned long long)out.cap) {
                        ((out_t *)out.r)[g] = (out_t)rv;
                        ((out_t *)out.s)[g] = (out_t)sv;
                    }
                }
            }
        };

        int it = -1;
        bool have = false;
        unsigned long long k = 0, p = 0, hh = 0;
        while (true) {
            while (!have) {
                if (++it >= kProbeItems) break;
                if (!pick(V, it)) continue;
                k = pick(K, it);
                p = pick(P, it);
                if (LY::null_key(k)) {   // wide: INT64_MIN probe key matches every side row
                    const unsigned long long ns = t.meta[0];
                    for (unsigned long long q = 0; q < ns; ++q) emit(t.side[q], p);
                    continue;
                }
                hh = slot_of(k, t.shift);
                have = true;
            }
            if (!have) break;
            const slot_t s = sl[hh];
            if (LY::empty(s)) {
                have = false;
            } else {
                if (LY::key(s) == k) {
                    emit(LY::pay(s), p);
                    if (unique) have = false;
                }
                hh = (hh + 1) & t.mask;
            }
        }

        if constexpr (WRITE) {
            __syncthreads();
            const unsigned nb = st_n;
            const unsigned nl = nb < (unsigned)kStage ? nb : (unsigned)kStage;
            if (threadIdx.x == 0) st_base = nl ? atomicAdd(out.counter, (unsigned long long)nl) : 0ull;
            __syncthreads();
            const unsigned long long gb = st_base;
            out_t *orr = (out_t *)out.r;
            out_t *oss = (out_t *)out.s;
            for (unsigned q = threadIdx.x; q < nl; q += kBlock) {
                const unsigned long long g = gb + q;
                if (g < (unsigned long long)out.cap) {
                    orr[g] = st_r[q];
                    oss[g] = st_s[q];
                }
            }
        } else {
            unsigned long long c = cnt;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
            if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
            __syncthreads();
            if (threadIdx.x == 0) {
                unsigned long long tot = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) tot += wsum[w];
                if (tot) atomicAdd(out.counter, tot);
            }
        }
        __syncthreads();   // st_n / staging reused by the next tile
    }
}

// ------------------------------------------------------------------ partition
// Radix partition by a hash independent of the slot hash (fmix64 top word,
// multiply-shift onto [0, P)), so a partition's keys still spread over its
// local table.  Used to route R and S rows to their owning GPU.  rbits > 0:
// the top rbits of the radix join's own key hash instead (P = 2^rbits) --
// the folded routing, whose parts are (owner, first-pass bin) pairs.
__device__ __forceinline__ unsigned part_of(unsigned long long k, unsigned P, int rbits) {
    if (rbits > 0) return (unsigned)(radix_hash(k) >> (64 - rbits));
    return (unsigned)(((fmix64(k) >> 32) * (unsigned long long)P) >> 32);
}

// Parts at most this many: LDS counter updates are aggregated per wave (one
// atomic per distinct part and wave instead of one per lane: with 1-8 parts
// every lane of a wave hits the same few counters).
constexpr unsigned kAggParts = 16;

// Wave-aggregated cnt[d] += 1 for every lane with `valid`; returns the lane's
// rank among the lanes of its wave and part, offset by the counter's old
// value.  All 64 lanes must call it (ballots).
__device__ __forceinline__ unsigned agg_add(unsigned *cnt, unsigned d, bool valid) {
    const unsigned lane = threadIdx.x & 63u;
    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    unsigned long long todo = __ballot(valid);
    unsigned rank = 0u;
    while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const unsigned dl = __shfl(d, leader, 64);
        const bool mine = valid && d == dl;
        const unsigned long long m = __ballot(mine);
        unsigned b = 0u;
        if ((int)lane == leader) b = atomicAdd(&cnt[dl], (unsigned)__popcll(m));
        b = __shfl(b, leader, 64);
        if (mine) rank = b + (unsigned)__popcll(m & lt);
        todo &= ~m;
    }
    return rank;
}

template <int FORM>
__global__ __launch_bounds__(kBlock) void k_part_hist(SrcDev src, unsigned P, int rbits, unsigned long long *counts) {
    extern __shared__ unsigned lds_hist[];
    for (unsigned i = threadIdx.x; i < P; i += kBlock) lds_hist[i] = 0u;
    __syncthreads();
    // grid-stride over 2048-row chunks: one flush of the block's counts at
    // the end (a flush per chunk put ~10^5 atomics on each part's counter)
    for (long long base = (long long)blockIdx.x * (kBlock * kPartItems) + threadIdx.x; base - threadIdx.x < src.n;
         base += (long long)gridDim.x * (kBlock * kPartItems)) {
#pragma unroll
        for (int i = 0; i < kPartItems; ++i) {
            const long long row = base + (long long)i * kBlock;
            const bool v = row < src.n;
            const unsigned d = v ? part_of(load_src<FORM>(src, row).k, P, rbits) : 0u;
            if (P <= kAggParts) (void)agg_add(lds_hist, d, v);
            else if (v) atomicAdd(&lds_hist[d], 1u);
        }
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < P; i += kBlock)
        if (lds_hist[i]) atomicAdd(&counts[i], (unsigned long long)lds_hist[i]);
}

__global__ void k_part_offsets(const unsigned long long *counts, unsigned P, unsigned long long *cursors) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        unsigned long long acc = 0;
        for (unsigned i = 0; i < P; ++i) {
            cursors[i] = acc;
            acc += counts[i];
        }
    }
}

template <int FORM>
__global__ __launch_bounds__(kBlock) void k_part_scatter(SrcDev src, unsigned P, int rbits, ulonglong2 *out,
                                                         unsigned long long *cursors) {
    extern __shared__ unsigned lds[];   // [0,P) local counts -> ranks, [P,3P) u64 bases
    unsigned *cnt = lds;
    unsigned long long *bases = (unsigned long long *)(lds + ((P + 1) & ~1u));
    for (unsigned i = threadIdx.x; i < P; i += kBlock) cnt[i] = 0u;
    __syncthreads();
    const long long base = (long long)blockIdx.x * (kBlock * kPartItems) + threadIdx.x;
    unsigned long long k[kPartItems], p[kPartItems];
    unsigned pid[kPartItems];
#pragma unroll
    for (int i = 0; i < kPartItems; ++i) {
        const long long row = base + (long long)i * kBlock;
        if (row < src.n) {
            Tuple tp = load_src<FORM>(src, row);
            k[i] = tp.k;
            p[i] = tp.p;
            pid[i] = part_of(tp.k, P, rbits);
            atomicAdd(&cnt[pid[i]], 1u);
        } else {
            pid[i] = ~0u;
            k[i] = p[i] = 0ull;
        }
    }
    __syncthreads();
    for (unsigned i = threadIdx.x; i < P; i += kBlock) {
        const unsigned c = cnt[i];
        bases[i] = c ? atomicAdd(&cursors[i], (unsigned long long)c) : 0ull;
        cnt[i] = 0u;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPartItems; ++i) {
        if (pid[i] == ~0u) continue;
        const unsigned r = atomicAdd(&cnt[pid[i]], 1u);
        out[bases[pid[i]] + r] = make_ulonglong2(k[i], p[i]);
    }
}

// Staged scatter for up to kRouteMaxParts parts: one 8192-row tile per
// workgroup is counting-sorted by part in LDS and every part's run is then
// written by consecutive lanes to consecutive addresses.  k_part_scatter
// writes each row to its own rank slot (lanes of a wave hit unrelated
// addresses and most 128-B lines are written in pieces, each a
// read-modify-write in HBM: profiles/r01_micro_write_alignment.txt).
// Two shapes: up to 512 parts, 8192-row tiles (152 KiB of LDS: one
// workgroup per CU, whose load and store phases then alternate on the CU);
// 4..64 parts (the multi-GPU owner routing: one part per rank), 2048-row
// tiles in 37 KiB, four workgroups per CU overlapping each other's phases:
// 8 parts 4.22 -> 2.78 ms and 64 parts 6.11 -> 3.33 ms per 2^28 rows
// (profiles/r02_route_tiles.txt).  1-2 parts keep the large tile (2-5 %
// faster there); a 128-part small tile (38 KiB) and a 4096-row tile for
// 65..256 parts measured no better than the large one.
constexpr int kRouteTile = 8192;
constexpr int kRouteThreads = 1024;
constexpr int kRouteMaxParts = 512;
constexpr int kRouteTileS = 2048;
constexpr int kRouteThreadsS = 256;
constexpr int kRouteMaxPartsS = 64;

template <int FORM, int TILE, int NT, int MAXP>
__global__ __launch_bounds__(NT) void k_route_scatter(SrcDev src, unsigned P, int rbits, ulonglong2 *out,
                                                      unsigned long long *cursors) {
    constexpr int IT = TILE / NT;
    static_assert(MAXP % 64 == 0 && TILE % NT == 0 && IT % 2 == 0, "route tile shape");
    __shared__ ulonglong2 stage[TILE];
    __shared__ unsigned short sp[TILE];
    __shared__ unsigned cnt[MAXP], start[MAXP];
    __shared__ unsigned long long base[MAXP];
    for (unsigned i = threadIdx.x; i < P; i += NT) cnt[i] = 0u;
    __syncthreads();
    const long long lo = (long long)blockIdx.x * TILE;
    ulonglong2 row[IT];
    unsigned pr[IT];   // part << 16 | rank, or ~0
    if constexpr (FORM == kCols64) {
        // two consecutive rows per lane: one 16-B load from each column
        const unsigned long long *kc = (const unsigned long long *)src.key, *pc = (const unsigned long long *)src.pay;
        const bool al = ((((uintptr_t)kc) | ((uintptr_t)pc)) & 15) == 0;
#pragma unroll
        for (int i = 0; i < IT / 2; ++i) {
            const long long r = lo + 2ll * (i * NT + threadIdx.x);
            if (al && r + 1 < src.n) {
                const ulonglong2 k2 = *(const ulonglong2 *)(kc + r), p2 = *(const ulonglong2 *)(pc + r);
                row[2 * i] = make_ulonglong2(k2.x, p2.x);
                row[2 * i + 1] = make_ulonglong2(k2.y, p2.y);
                pr[2 * i] = pr[2 * i + 1] = 0u;
            } else {
                const bool v0 = r < src.n, v1 = r + 1 < src.n;
                row[2 * i] = v0 ? make_ulonglong2(kc[r], pc[r]) : make_ulonglong2(0ull, 0ull);
                row[2 * i + 1] = v1 ? make_ulonglong2(kc[r + 1], pc[r + 1]) : make_ulonglong2(0ull, 0ull);
                pr[2 * i] = v0 ? 0u : ~0u;
                pr[2 * i + 1] = v1 ? 0u : ~0u;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const long long r = lo + (long long)i * NT + threadIdx.x;
            const bool v = r < src.n;
            const Tuple tp = v ? load_src<FORM>(src, r) : Tuple{0ull, 0ull};
            row[i] = make_ulonglong2(tp.k, tp.p);
            pr[i] = v ? 0u : ~0u;
        }
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const bool v = pr[i] != ~0u;
        const unsigned d = v ? part_of(row[i].x, P, rbits) : 0u;
        if (P <= kAggParts) {
            const unsigned r = agg_add(cnt, d, v);
            if (v) pr[i] = (d << 16) | r;
        } else if (v) {
            pr[i] = (d << 16) | atomicAdd(&cnt[d], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < 64) {   // wave 0: stage offsets; one cursor atomic per non-empty part
        const unsigned lane = threadIdx.x;
        constexpr int PER = MAXP / 64;
        unsigned c[PER], sum = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const unsigned d = lane * PER + j;
            c[j] = d < P ? cnt[d] : 0u;
            sum += c[j];
        }
        unsigned x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        unsigned run = x - sum;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const unsigned d = lane * PER + j;
            if (d < P) {
                start[d] = run;
                base[d] = c[j] ? atomicAdd(&cursors[d], (unsigned long long)c[j]) : 0ull;
            }
            run += c[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        if (pr[i] == ~0u) continue;
        const unsigned d = pr[i] >> 16, pos = start[d] + (pr[i] & 0xffffu);
        stage[pos] = row[i];
        sp[pos] = (unsigned short)d;
    }
    __syncthreads();
    const long long rem = src.n - lo;
    const unsigned tn = rem < TILE ? (unsigned)rem : (unsigned)TILE;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const unsigned j = (unsigned)i * NT + threadIdx.x;
        if (j >= tn) continue;
        const unsigned d = sp[j];
        out[base[d] + (j - start[d])] = stage[j];
    }
}

// ------------------------------------------------------------------ datagen
__global__ __launch_bounds__(kBlock) void k_gen_pkfk(unsigned long long seed, long long NR,
                                                     unsigned long long hit_thr, long long r0, long long nr,
                                                     long long *rkey, long long *rpay, long long s0, long long ns,
                                                     long long *skey, long long *spay) {
    const unsigned long long salt = pkfk_salt(seed);
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i < nr) {
        const unsigned long long g = (unsigned long long)(r0 + i);
        rkey[i] = pkfk_rkey(salt, g);
        rpay[i] = (long long)g;
    }
    if (i < ns) {
        const unsigned long long g = (unsigned long long)(s0 + i);
        skey[i] = pkfk_skey(seed, salt, NR, hit_thr, g);
        spay[i] = (long long)g;
    }
}

__global__ __launch_bounds__(kBlock) void k_gen_uniform_i64(unsigned long long seed, unsigned long long sid,
                                                            long long lo, long long hi, long long i0, long long n,
                                                            long long *key, long long *pay) {
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const unsigned long long range = (unsigned long long)(hi - lo) + 1ull;
    const unsigned long long g = (unsigned long long)(i0 + i);
    const unsigned long long r = rand64(seed, sid, g);
    key[i] = lo + (long long)(range ? r % range : r);
    if (pay) pay[i] = (long long)g;
}

__global__ __launch_bounds__(kBlock) void k_gen_uniform_i32(unsigned long long seed, unsigned long long sid,
                                                            int lo, int hi, long long i0, long long n, int *key) {
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const unsigned long long range = (unsigned long long)((long long)hi - (long long)lo) + 1ull;
    const unsigned long long r = rand64(seed, sid, (unsigned long long)(i0 + i));
    key[i] = (int)((long long)lo + (long long)(r % range));
}

__global__ __launch_bounds__(kBlock) void k_gen_zipf(unsigned long long seed, ZipfParams z, long long s0, long long ns,
                                                     long long *skey, long long *spay) {
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i >= ns) return;
    const unsigned long long g = (unsigned long long)(s0 + i);
    skey[i] = zipf_skey(seed, z, g);
    spay[i] = (long long)g;
}

// ------------------------------------------------------------------ rows
// nested-loop.mlir's result rows (:160-188) materialised from join pairs.
// Key column (column 0) of a row-major int32 table with row stride ld.
__global__ __launch_bounds__(kBlock) void k_key_col_i32(const int *t, long long rows, long long ld, int *out) {
    const long long i = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (i < rows) out[i] = t[i * ld];
}

// out[m] = [X[px[m]][0 .. cx), Y[py[m]][1 .. cy)] for m < min(*count, cap):
// one lane per output element, so the stores are coalesced and the row
// gathers are the only scattered accesses.
__global__ __launch_bounds__(kBlock) void k_gather_rows_i32(const int *x, long long ldx, int cx, const int *y,
                                                            long long ldy, int cy, const int *px, const int *py,
                                                            const unsigned long long *count, long long cap,
                                                            int *out, long long ldo) {
    const int oc = cx + cy - 1;
    const unsigned long long m_all = *count;
    const long long m = (long long)(m_all < (unsigned long long)cap ? m_all : (unsigned long long)cap);
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < m * oc; e += (long long)gridDim.x * kBlock) {
        const long long r = e / oc;
        const int c = (int)(e - r * oc);
        out[r * ldo + c] = c < cx ? x[(long long)px[r] * ldx + c] : y[(long long)py[r] * ldy + (c - cx + 1)];
    }
}

// ------------------------------------------------------------------ selection
// Experiments/selection.mlir (:34-155): keep the elements that pass
// `v <op> c`, compacted.  Order-preserving here (the reference orders blocks
// by an atomic): count per tile, exclusive scan of the counts, then each tile
// writes its survivors in element order.  A lane reads 16 B per load: slot j
// of lane t holds elements j*64*NW*W + t*W .. +W (W = 16 B / sizeof(V)), so
// element order is (slot, wave, lane, w) and positions come from per-lane
// counts, a wave prefix sum and one (slot, wave) scan per tile.
// Float compares are ordered (NaN never passes), like the reference's olt.
constexpr int kSelSlots = 4;

template <typename V>
__device__ __forceinline__ bool sel_pass(V v, int op, V c) {
    switch (op) {
        case 0: return v < c;
        case 1: return v <= c;
        case 2: return v > c;
        case 3: return v >= c;
        case 4: return v == c;
        default: return v < c || v > c;   // ordered not-equal
    }
}

template <typename V>
struct SelVec {
    static constexpr int W = 16 / sizeof(V);
    static constexpr long long kTile = (long long)kBlock * kSelSlots * W;
    V v[W];
};

// Slot j of this lane: W elements at e0 (vector load when whole and aligned).
template <typename V>
__device__ __forceinline__ void sel_load(const V *in, long long n, long long e0, bool vec_ok, SelVec<V> &x) {
    constexpr int W = SelVec<V>::W;
    if (vec_ok && e0 + W <= n) {
        const uint4 u = *(const uint4 *)(in + e0);
        __builtin_memcpy(x.v, &u, 16);
    } else {
#pragma unroll
        for (int w = 0; w < W; ++w) x.v[w] = e0 + w < n ? in[e0 + w] : V(0);
    }
}

template <typename V>
__global__ __launch_bounds__(kBlock) void k_sel_count(const V *in, long long n, int op, V c, bool vec_ok,
                                                      unsigned long long *tile_cnt) {
    constexpr int W = SelVec<V>::W;
    __shared__ unsigned ws[kBlock / 64];
    const long long base = (long long)blockIdx.x * SelVec<V>::kTile + (long long)threadIdx.x * W;
    unsigned k = 0;
#pragma unroll
    for (int j = 0; j < kSelSlots; ++j) {
        SelVec<V> x;
        const long long e0 = base + (long long)j * kBlock * W;
        sel_load(in, n, e0, vec_ok, x);
#pragma unroll
        for (int w = 0; w < W; ++w) k += (e0 + w < n && sel_pass(x.v[w], op, c)) ? 1u : 0u;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) k += __shfl_down(k, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = k;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned t = 0;
#pragma unroll
        for (int w = 0; w < kBlock / 64; ++w) t += ws[w];
        tile_cnt[blockIdx.x] = t;
    }
}

template <typename V>
__global__ __launch_bounds__(kBlock) void k_sel_write(const V *in, long long n, int op, V c, bool vec_ok,
                                                      const unsigned long long *tile_off, unsigned ntiles, V *out,
                                                      long long *out_row, long long cap,
                                                      unsigned long long *count) {
    constexpr int W = SelVec<V>::W;
    constexpr int NW = kBlock / 64;
    __shared__ unsigned s_cw[kSelSlots * NW];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long base = (long long)blockIdx.x * SelVec<V>::kTile + (long long)threadIdx.x * W;
    SelVec<V> x[kSelSlots];
    unsigned pass[kSelSlots], lpre[kSelSlots];
#pragma unroll
    for (int j = 0; j < kSelSlots; ++j) {
        const long long e0 = base + (long long)j * kBlock * W;
        sel_load(in, n, e0, vec_ok, x[j]);
        pass[j] = 0;
#pragma unroll
        for (int w = 0; w < W; ++w)
            if (e0 + w < n && sel_pass(x[j].v[w], op, c)) pass[j] |= 1u << w;
        // lane prefix within the wave for this slot
        const unsigned k = (unsigned)__popc(pass[j]);
        unsigned xs = k;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(xs, o, 64);
            if (lane >= o) xs += y;
        }
        lpre[j] = xs - k;
        if (lane == 63) s_cw[j * NW + wv] = xs;
    }
    __syncthreads();
    if (threadIdx.x == 0) {   // (slot, wave) runs in element order: kSelSlots * NW = 16 entries
        unsigned run = 0;
#pragma unroll
        for (int q = 0; q < kSelSlots * NW; ++q) {
            const unsigned v = s_cw[q];
            s_cw[q] = run;
            run += v;
        }
    }
    __syncthreads();
    const unsigned long long tb = tile_off[blockIdx.x];
#pragma unroll
    for (int j = 0; j < kSelSlots; ++j) {
        unsigned long long g = tb + s_cw[j * NW + wv] + lpre[j];
        const long long e0 = base + (long long)j * kBlock * W;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            if (!((pass[j] >> w) & 1u)) continue;
            if (g < (unsigned long long)cap) {
                out[g] = x[j].v[w];
                if (out_row) out_row[g] = e0 + w;
            }
            ++g;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *count = tile_off[ntiles];
}

inline unsigned grid_for(long long n, int per_block) {
    return (unsigned)((n + per_block - 1) / per_block);
}

}  // namespace

// ---------------------------------------------------------------- launchers
hipError_t launch_init(const TableDev &t, int layout, unsigned long long cap, hipStream_t st) {
    const unsigned long long bytes = cap * (layout == kWide ? 16ull : 8ull);
    const unsigned long long n16 = bytes / 16ull;
    const unsigned g = grid_for((long long)n16, kBlock * 4);
    if (layout == kWide) hipLaunchKernelGGL(k_init<kWide>, dim3(g), dim3(kBlock), 0, st, t, n16);
    else hipLaunchKernelGGL(k_init<kNarrow>, dim3(g), dim3(kBlock), 0, st, t, n16);
    return hipGetLastError();
}

hipError_t launch_build(const TableDev &t, int layout, const SrcDev &src, hipStream_t st) {
    if (src.n <= 0) return hipSuccess;
    const unsigned g = grid_for(src.n, kBlock * kBuildItems);
    if (layout == kWide) {
        if (src.form == kCols64) hipLaunchKernelGGL((k_build<kWide, kCols64>), dim3(g), dim3(kBlock), 0, st, t, src);
        else if (src.form == kPacked64) hipLaunchKernelGGL((k_build<kWide, kPacked64>), dim3(g), dim3(kBlock), 0, st, t, src);
        else return hipErrorInvalidValue;
    } else {
        if (src.form == kCol32) hipLaunchKernelGGL((k_build<kNarrow, kCol32>), dim3(g), dim3(kBlock), 0, st, t, src);
        else return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

size_t probe_tiles(long long n) {
    // plain tiles: one slow-list entry per 2048-row tile at most
    return (size_t)(n > 0 ? (n + kProbeTile - 1) / kProbeTile : 0) + 1;
}

hipError_t launch_probe(const TableDev &t, int layout, const SrcDev &src, const OutDev &out,
                        bool count_only, unsigned *slow, size_t slow_cap, hipStream_t st) {
    if (src.n <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(&t.meta[3], 0, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    const unsigned long long cap = slow_cap;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const unsigned tiles = grid_for(src.n, kProbeTile);
    const unsigned gs = tiles < (unsigned)(cus * 8) ? tiles : (unsigned)(cus * 8);
    // a table of <= kLdsTableBytes: every workgroup copies it into LDS once
    // and strides over the tiles (as many workgroups as LDS lets a CU hold)
    const size_t tbytes = (size_t)(t.mask + 1) * (layout == kWide ? 16 : 8);
    const bool lds = tbytes <= (size_t)kLdsTableBytes && tbytes >= 16;
    unsigned per_cu = lds ? (unsigned)(kLdsPerCu / tbytes) : 1u;
    if (per_cu > 8) per_cu = 8;
    if (per_cu < 1) per_cu = 1;
    const unsigned gl = tiles < (unsigned)cus * per_cu ? tiles : (unsigned)cus * per_cu;
    const unsigned g = lds ? gl : tiles;   // (global table: one block per tile)
#define HJ_PROBE(L, F)                                                                                        \
    do {                                                                                                      \
        if (count_only) {                                                                                     \
            if (lds)                                                                                          \
                hipLaunchKernelGGL((k_probe<L, F, false, true>), dim3(g), dim3(kBlock), tbytes, st, t, src,   \
                                   out, slow, cap);                                                           \
            else hipLaunchKernelGGL((k_probe<L, F, false>), dim3(g), dim3(kBlock), 0, st, t, src, out, slow, cap); \
            hipLaunchKernelGGL((k_probe_slow<L, F, false>), dim3(gs), dim3(kBlock), 0, st, t, src, out,       \
                               (const unsigned *)slow, cap);                                                  \
        } else {                                                                                              \
            if (lds)                                                                                          \
                hipLaunchKernelGGL((k_probe<L, F, true, true>), dim3(g), dim3(kBlock), tbytes, st, t, src,    \
                                   out, slow, cap);                                                           \
            else hipLaunchKernelGGL((k_probe<L, F, true>), dim3(g), dim3(kBlock), 0, st, t, src, out, slow, cap); \
            hipLaunchKernelGGL((k_probe_slow<L, F, true>), dim3(gs), dim3(kBlock), 0, st, t, src, out,        \
                               (const unsigned *)slow, cap);                                                  \
        }                                                                                                     \
    } while (0)
    if (layout == kWide) {
        if (src.form == kCols64) HJ_PROBE(kWide, kCols64);
        else if (src.form == kPacked64) HJ_PROBE(kWide, kPacked64);
        else return hipErrorInvalidValue;
    } else {
        if (src.form == kCol32) HJ_PROBE(kNarrow, kCol32);
        else return hipErrorInvalidValue;
    }
#undef HJ_PROBE
    return hipGetLastError();
}

hipError_t launch_partition(const SrcDev &src, int nparts, void *out_tuples,
                            unsigned long long *counts, unsigned long long *cursors, hipStream_t st, int rbits) {
    const unsigned P = (unsigned)nparts;
    if (rbits > 0 && (rbits > 13 || P != (1u << rbits))) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(counts, 0, sizeof(unsigned long long) * P, st);
    if (e != hipSuccess) return e;
    if (src.n > 0) {
        const unsigned g = grid_for(src.n, kBlock * kPartItems);
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const unsigned gh = g < (unsigned)cus * 8u ? g : (unsigned)cus * 8u;
        const size_t lds_h = sizeof(unsigned) * P;
        const size_t lds_s = sizeof(unsigned) * ((P + 1) & ~1u) + sizeof(unsigned long long) * P;
        if (src.form == kCols64) hipLaunchKernelGGL(k_part_hist<kCols64>, dim3(gh), dim3(kBlock), lds_h, st, src, P, rbits, counts);
        else if (src.form == kPacked64) hipLaunchKernelGGL(k_part_hist<kPacked64>, dim3(gh), dim3(kBlock), lds_h, st, src, P, rbits, counts);
        else return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_part_offsets, dim3(1), dim3(64), 0, st, counts, P, cursors);
        if (P >= 4u && P <= (unsigned)kRouteMaxPartsS) {
            const unsigned gt = grid_for(src.n, kRouteTileS);
            if (src.form == kCols64)
                hipLaunchKernelGGL((k_route_scatter<kCols64, kRouteTileS, kRouteThreadsS, kRouteMaxPartsS>), dim3(gt),
                                   dim3(kRouteThreadsS), 0, st, src, P, rbits, (ulonglong2 *)out_tuples, cursors);
            else
                hipLaunchKernelGGL((k_route_scatter<kPacked64, kRouteTileS, kRouteThreadsS, kRouteMaxPartsS>), dim3(gt),
                                   dim3(kRouteThreadsS), 0, st, src, P, rbits, (ulonglong2 *)out_tuples, cursors);
        } else if (P <= (unsigned)kRouteMaxParts) {
            const unsigned gt = grid_for(src.n, kRouteTile);
            if (src.form == kCols64)
                hipLaunchKernelGGL((k_route_scatter<kCols64, kRouteTile, kRouteThreads, kRouteMaxParts>), dim3(gt),
                                   dim3(kRouteThreads), 0, st, src, P, rbits, (ulonglong2 *)out_tuples, cursors);
            else
                hipLaunchKernelGGL((k_route_scatter<kPacked64, kRouteTile, kRouteThreads, kRouteMaxParts>), dim3(gt),
                                   dim3(kRouteThreads), 0, st, src, P, rbits, (ulonglong2 *)out_tuples, cursors);
        } else if (src.form == kCols64)
            hipLaunchKernelGGL(k_part_scatter<kCols64>, dim3(g), dim3(kBlock), lds_s, st, src, P, rbits, (ulonglong2 *)out_tuples, cursors);
        else
            hipLaunchKernelGGL(k_part_scatter<kPacked64>, dim3(g), dim3(kBlock), lds_s, st, src, P, rbits, (ulonglong2 *)out_tuples, cursors);
    }
    return hipGetLastError();
}

hipError_t launch_gen_pkfk(unsigned long long seed, long long NR, unsigned long long hit_thr,
                           long long r0, long long nr, long long *rkey, long long *rpay,
                           long long s0, long long ns, long long *skey, long long *spay, hipStream_t st) {
    const long long n = nr > ns ? nr : ns;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_pkfk, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, seed, NR, hit_thr, r0, nr,
                       rkey, rpay, s0, ns, skey, spay);
    return hipGetLastError();
}

hipError_t launch_gen_zipf(unsigned long long seed, const ZipfParams &z, long long s0, long long ns, long long *skey,
                           long long *spay, hipStream_t st) {
    if (ns <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_zipf, dim3(grid_for(ns, kBlock)), dim3(kBlock), 0, st, seed, z, s0, ns, skey, spay);
    return hipGetLastError();
}

hipError_t launch_gen_uniform_i64(unsigned long long seed, unsigned long long sid, long long lo, long long hi,
                                  long long i0, long long n, long long *key, long long *pay, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_uniform_i64, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, seed, sid, lo, hi, i0, n,
                       key, pay);
    return hipGetLastError();
}

hipError_t launch_gen_uniform_i32(unsigned long long seed, unsigned long long sid, int lo, int hi, long long i0,
                                  long long n, int *key, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_uniform_i32, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, st, seed, sid, lo, hi, i0, n,
                       key);
    return hipGetLastError();
}

hipError_t launch_key_col_i32(const int *t, long long rows, long long ld, int *out, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_key_col_i32, dim3(grid_for(rows, kBlock)), dim3(kBlock), 0, st, t, rows, ld, out);
    return hipGetLastError();
}

hipError_t launch_gather_rows_i32(const int *x, long long ldx, int cx, const int *y, long long ldy, int cy,
                                  const int *px, const int *py, const unsigned long long *count, long long cap,
                                  int *out, long long ldo, hipStream_t st) {
    if (cap <= 0) return hipSuccess;
    const long long elems = cap * (long long)(cx + cy - 1);
    unsigned g = grid_for(elems, kBlock * 4);
    if (g > 65536u) g = 65536u;   // grid-stride beyond
    hipLaunchKernelGGL(k_gather_rows_i32, dim3(g), dim3(kBlock), 0, st, x, ldx, cx, y, ldy, cy, px, py, count, cap,
                       out, ldo);
    return hipGetLastError();
}

static size_t select_tiles_of(long long n, long long tile) { return (size_t)(n > 0 ? (n + tile - 1) / tile : 0); }

size_t select_tiles(long long n) {   // upper bound over element types (int64 tiles hold fewer elements)
    return select_tiles_of(n, SelVec<long long>::kTile);
}

template <typename V>
static hipError_t launch_select_t(const V *in, long long n, int op, V c, V *out, long long *out_row, long long cap,
                                  unsigned long long *count, unsigned long long *tiles, unsigned long long *sums,
                                  hipStream_t st) {
    const unsigned nt = (unsigned)select_tiles_of(n, SelVec<V>::kTile);
    if (nt == 0) return hipMemsetAsync(count, 0, sizeof(unsigned long long), st);
    const bool vec_ok = (((uintptr_t)in) & 15) == 0;
    hipLaunchKernelGGL((k_sel_count<V>), dim3(nt), dim3(kBlock), 0, st, in, n, op, c, vec_ok, tiles);
    hipError_t e = hipMemsetAsync(tiles + nt, 0, sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    e = exclusive_scan_u64(tiles, (unsigned long long)nt + 1, sums, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_sel_write<V>), dim3(nt), dim3(kBlock), 0, st, in, n, op, c, vec_ok,
                       (const unsigned long long *)tiles, nt, out, out_row, cap, count);
    return hipGetLastError();
}

hipError_t launch_select_f32(const float *in, long long n, int op, float c, float *out, long long *out_row,
                             long long cap, unsigned long long *count, unsigned long long *tiles,
                             unsigned long long *sums, hipStream_t st) {
    return launch_select_t<float>(in, n, op, c, out, out_row, cap, count, tiles, sums, st);
}

hipError_t launch_select_i64(const long long *in, long long n, int op, long long c, long long *out,
                             long long *out_row, long long cap, unsigned long long *count, unsigned long long *tiles,
                             unsigned long long *sums, hipStream_t st) {
    return launch_select_t<long long>(in, n, op, c, out, out_row, cap, count, tiles, sums, st);
}

// ------------------------------------------------------------ copy floors
// The box's own streamed-copy rate, so a bench line can say how far each
// phase is from it.  16-B rows, non-temporal
// loads and stores (the partition passes' access flavour).
typedef unsigned long long cp_u64;
typedef __attribute__((ext_vector_type(2))) unsigned long long cp_v2;

__device__ __forceinline__ cp_v2 cp_ld(const cp_v2 *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void cp_st(cp_v2 *p, cp_v2 v) { __builtin_nontemporal_store(v, p); }

// one row per thread over the whole grid (n / 256 workgroups): the chip's
// best copy shape (6.2-6.4 TB/s, profiles/r04_copy_and_interleave.txt)
__global__ __launch_bounds__(256) void k_copy_flat(const cp_v2 *__restrict__ in, cp_v2 *__restrict__ out, cp_u64 n) {
    const cp_u64 i = (cp_u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) cp_st(out + i, cp_ld(in + i));
}

// the partition passes' loop shape: one 1024-thread workgroup per CU walks a
// contiguous range of 4096-row tiles with the next tile's loads in flight
// during this tile's stores
constexpr int kCpNT = 1024, kCpIT = 4;
__global__ __launch_bounds__(kCpNT) void k_copy_persistent(const cp_v2 *__restrict__ in, cp_v2 *__restrict__ out,
                                                           cp_u64 n) {
    constexpr cp_u64 T = (cp_u64)kCpNT * kCpIT;
    const cp_u64 tiles = n / T;
    const cp_u64 t0 = (cp_u64)blockIdx.x * tiles / gridDim.x, t1 = (cp_u64)(blockIdx.x + 1) * tiles / gridDim.x;
    cp_v2 r[kCpIT], q[kCpIT];
    if (t0 < t1)
#pragma unroll
        for (int i = 0; i < kCpIT; ++i) r[i] = cp_ld(in + t0 * T + (cp_u64)i * kCpNT + threadIdx.x);
    for (cp_u64 t = t0; t < t1; ++t) {
        if (t + 1 < t1)
#pragma unroll
            for (int i = 0; i < kCpIT; ++i) q[i] = cp_ld(in + (t + 1) * T + (cp_u64)i * kCpNT + threadIdx.x);
#pragma unroll
        for (int i = 0; i < kCpIT; ++i) cp_st(out + t * T + (cp_u64)i * kCpNT + threadIdx.x, r[i]);
#pragma unroll
        for (int i = 0; i < kCpIT; ++i) r[i] = q[i];
    }
    // rows past the last whole tile (n % T): the last workgroup, one per thread
    if (blockIdx.x == gridDim.x - 1)
        for (cp_u64 i = tiles * T + threadIdx.x; i < n; i += kCpNT) cp_st(out + i, cp_ld(in + i));
}

hipError_t launch_stream_copy(const void *in, void *out, long long rows, int shape, int cus, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    const cp_v2 *s = (const cp_v2 *)in;
    cp_v2 *d = (cp_v2 *)out;
    if (shape == 0)
        hipLaunchKernelGGL(k_copy_persistent, dim3(cus > 0 ? cus : 1), dim3(kCpNT), 0, st, s, d, (cp_u64)rows);
    else
        hipLaunchKernelGGL(k_copy_flat, dim3(grid_for(rows, 256)), dim3(256), 0, st, s, d, (cp_u64)rows);
    return hipGetLastError();
}

// ------------------------------------------------------- placement probe
// The partition passes write, per 4096-row tile, one 128-B line into each of
// ~512 open 1024-row buckets of the workgroup's own bucket range.  Into some
// physical placements of the destination buffer that pattern runs 25-35 %
// slower than a flat write of the same bytes; it is a property of the
// allocation (bimodal, reproducible per buffer, the flat write and flat read
// never vary, contiguous allocations are slow more often:
// profiles/r05/r05t_place_micro.txt, r05u_*).  placement_probe writes the
// pass's pattern (synthetic rows, every workgroup in its own range) and a flat
// stream of the same bytes into a fresh buffer; ratio = pattern / flat.
// (nb = 128 / 256 / 512 open buckets per workgroup: nb / 128 lines per
// thread group of 8 lanes per tile; buckets of 2^lpb_log 128-B lines)
__global__ __launch_bounds__(1024) void k_place_pattern(cp_v2 *__restrict__ out, unsigned tpw, cp_u64 wrows,
                                                        unsigned nb, unsigned lpb_log) {
    const unsigned w = blockIdx.x, tid = threadIdx.x;
    const cp_u64 base = (cp_u64)w * wrows;
    const cp_v2 val = {(cp_u64)w, 1ull};
    const unsigned lmask = (1u << lpb_log) - 1u;
    for (unsigned t = 0; t < tpw; ++t)
        for (unsigned i = 0; i < nb / 128u; ++i) {
            const unsigned j = i * 128u + (tid >> 3);   // the line's bin
            cp_st(out + base + ((((cp_u64)(t >> lpb_log) * nb + j) << lpb_log) + (t & lmask)) * 8u + (tid & 7u), val);
        }
}

__global__ __launch_bounds__(256) void k_place_flat(cp_v2 *__restrict__ out, cp_u64 n) {
    const cp_u64 i = (cp_u64)blockIdx.x * 256 + threadIdx.x;
    if (i < n) cp_st(out + i, cp_v2{i, 2ull});
}

hipError_t placement_probe(void *buf, size_t bytes, size_t bucket_bytes, int cus, float *ratio) {
    *ratio = 0.0f;
    if (cus <= 0 || !buf) return hipErrorInvalidValue;
    // 128-B lines per bucket (a power of two, 8 .. 128)
    unsigned lpb_log = 3;
    while (lpb_log < 7 && (size_t(128) << (lpb_log + 1)) <= bucket_bytes) ++lpb_log;
    const cp_u64 bv2 = (cp_u64)8 << lpb_log;   // 16-B units per bucket
    // every workgroup's range: whole buckets, >= two per bin (512 bins; 256 /
    // 128 in smaller buffers)
    const cp_u64 wrows = ((cp_u64)(bytes / 16) / (cp_u64)cus) / bv2 * bv2;
    const cp_u64 buckets = wrows / bv2;
    const unsigned nb = buckets >= 1024 ? 512u : buckets >= 512 ? 256u : 128u;
    if (buckets < 256) return hipErrorInvalidValue;
    // tiles per workgroup: a bin's buckets (t >> lpb_log) stay inside the range
    const cp_u64 tw = (buckets / nb - 1) << lpb_log;
    const unsigned tpw = (unsigned)(tw > 512 ? 512 : tw);
    const cp_u64 flat = (cp_u64)tpw * 8u * nb * (cp_u64)cus;   // the same rows, streamed
    cp_v2 *out = (cp_v2 *)buf;
    hipEvent_t e[4];
    hipError_t err = hipSuccess;
    int made = 0;
    for (; made < 4 && err == hipSuccess; ++made) err = hipEventCreate(&e[made]);
    float best_p = 1e30f, best_f = 1e30f;
    for (int rep = 0; rep < 3 && err == hipSuccess; ++rep) {
        // rep 0 warms up (first touch of the pages), reps 1-2 are kept
        err = hipEventRecord(e[0], 0);
        hipLaunchKernelGGL(k_place_pattern, dim3(cus), dim3(1024), 0, 0, out, tpw, wrows, nb, lpb_log);
        if (err == hipSuccess) err = hipEventRecord(e[1], 0);
        hipLaunchKernelGGL(k_place_flat, dim3((unsigned)((flat + 255) / 256)), dim3(256), 0, 0, out, flat);
        if (err == hipSuccess) err = hipEventRecord(e[2], 0);
        if (err == hipSuccess) err = hipGetLastError();
        if (err == hipSuccess) err = hipEventSynchronize(e[2]);
        float tp = 0.0f, tf = 0.0f;
        if (err == hipSuccess) err = hipEventElapsedTime(&tp, e[0], e[1]);
        if (err == hipSuccess) err = hipEventElapsedTime(&tf, e[1], e[2]);
        if (rep > 0 && err == hipSuccess) {
            if (tp < best_p) best_p = tp;
            if (tf < best_f) best_f = tf;
        }
    }
    for (int i = 0; i < made; ++i) (void)hipEventDestroy(e[i]);
    if (err == hipSuccess) *ratio = best_f > 0.0f ? best_p / best_f : 0.0f;
    return err;
}

}  // namespace hj
