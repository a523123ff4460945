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
//   join:          one work item per (partition, S chunk): build the
//                  partition's R rows into an LDS table, probe the chunk's S
//                  rows, count, block-scan, reserve the block's output with
//                  ONE global atomic, and write every pair at its position.
//
// Partitioned rows are packed: 16-B {key, payload} (64-bit keys) or 8-B
// (key << 32 | row id) (the reference's i32 types), so a row moves with one
// global load/store and an i32 row is already its own LDS table entry.
//
// Scatter and join are persistent (2 workgroups per CU) and software-
// pipelined: the next tile / work item is loaded into registers before the
// current one's LDS phase, so HBM latency hides behind LDS work.
//
// The reference's count -> prefix -> probe protocol (join_v1.mlir:288-521) is
// kept, but per workgroup and on LDS, so the output needs no staging buffer
// and has no overflow path.
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "hj_internal.h"

namespace hj {
namespace {

typedef unsigned long long u64;
constexpr u64 kGold = 0x9E3779B97F4A7C15ull;
constexpr int kTile = 4096;        // rows per partition-pass tile
constexpr int kPassThreads = 512;  // 8 rows per thread
constexpr int kPassRows = kTile / kPassThreads;
constexpr int kJoinItems = 4;      // S rows per thread per sub-chunk of the join kernel
constexpr int kJoinSub = 8;        // sub-chunks per work item (one table build serves all)
constexpr int kPackedRow = 3;      // SrcForm of partition-pass outputs (packed rows)

__device__ __forceinline__ u64 rhash(u64 k) { return k * kGold; }

// --------------------------------------------------------------- rows
template <bool WIDE>
struct Row;

template <>
struct Row<true> {   // 64-bit key / 64-bit payload
    typedef ulonglong2 T;
    static __device__ __forceinline__ u64 key(const T &r) { return r.x; }
    static __device__ __forceinline__ u64 pay(const T &r) { return r.y; }
    static __device__ __forceinline__ T make(u64 k, u64 p) { return make_ulonglong2(k, p); }
    static __device__ __forceinline__ T zero() { return make_ulonglong2(0ull, 0ull); }
};

template <>
struct Row<false> {   // i32 key (zero-extended) / i32 row id, packed key << 32 | row id
    typedef u64 T;
    static __device__ __forceinline__ u64 key(const T &r) { return r >> 32; }
    static __device__ __forceinline__ u64 pay(const T &r) { return r & 0xffffffffull; }
    static __device__ __forceinline__ T make(u64 k, u64 p) { return (k << 32) | (p & 0xffffffffull); }
    static __device__ __forceinline__ T zero() { return 0ull; }
};

// Row `row` of a pass input in form FORM.
template <bool WIDE, int FORM>
__device__ __forceinline__ typename Row<WIDE>::T load_row(const SrcDev &s, long long row) {
    typedef Row<WIDE> R;
    if constexpr (FORM == kPackedRow || FORM == kPacked64) {
        return ((const typename R::T *)s.key)[row];
    } else if constexpr (FORM == kCol32) {
        return R::make((u64)(unsigned)((const int *)s.key)[row], (u64)(s.row_base + row));
    } else {   // kCols64
        return R::make(((const u64 *)s.key)[row], ((const u64 *)s.pay)[row]);
    }
}

// --------------------------------------------------------------- helpers
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

// item -> segment list from a chunk map (start[] as written by k_chunk_map):
// one thread per segment writes its items' owner, so consumers need a single
// load instead of a log2(nseg)-step dependent binary search.
__global__ __launch_bounds__(256) void k_work_list(const unsigned *start, int nseg, unsigned *owner) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= nseg) return;
    for (unsigned w = start[s]; w < start[s + 1]; ++w) owner[w] = (unsigned)s;
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
    SrcDev in;                   // pass input (key/pay/row_base/form; n unused)
    const u64 *seg_off;          // nseg + 1
    int nseg;
    const unsigned *tile_start;  // nseg + 1
    const unsigned *tile_owner;  // tile -> segment (nseg > 1)
    u64 *hist;                   // [seg][bin][tile] counts, then exclusive offsets
    void *out;                   // packed rows
    u64 *next_off;               // nseg * F + 1
    int shift;                   // bin = (hash >> shift) & (F - 1)
    int fbits;
};

struct TileRange {
    int seg;
    unsigned t, ntiles;
    u64 lo, hi;
};

__device__ __forceinline__ TileRange tile_range(const PassArgs &a, unsigned wg) {
    TileRange r;
    r.seg = a.nseg == 1 ? 0 : (int)a.tile_owner[wg];
    r.t = wg - a.tile_start[r.seg];
    r.ntiles = a.tile_start[r.seg + 1] - a.tile_start[r.seg];
    r.lo = a.seg_off[r.seg] + (u64)r.t * kTile;
    const u64 e = a.seg_off[r.seg + 1];
    r.hi = r.lo + kTile < e ? r.lo + kTile : e;
    return r;
}

// Per-tile bin counts.  Keys are read 16 B per lane (two keys of a key
// column, or the key half of one packed row).
template <bool WIDE, int FORM>
__global__ __launch_bounds__(kPassThreads) void k_hist(PassArgs a) {
    typedef Row<WIDE> R;
    __shared__ unsigned cnt[512];
    const unsigned wg = blockIdx.x;
    if (wg >= a.tile_start[a.nseg]) return;   // upper-bound grid
    const TileRange tr = tile_range(a, wg);
    const unsigned F = 1u << a.fbits;
    for (unsigned b = threadIdx.x; b < F; b += kPassThreads) cnt[b] = 0u;
    __syncthreads();
    auto bin_of = [&](u64 k) { return (unsigned)(rhash(k) >> a.shift) & (F - 1); };
    if constexpr (FORM == kCols64) {
        // two consecutive keys per lane (one 16-B load): rows lo + 2*(i*NT + tid) + {0,1}
        const bool al = ((((uintptr_t)a.in.key) & 15) == 0) && ((tr.lo & 1) == 0);
#pragma unroll
        for (int i = 0; i < kPassRows / 2; ++i) {
            const u64 row = tr.lo + 2ull * ((u64)i * kPassThreads + threadIdx.x);
            if (al && row + 1 < tr.hi) {
                const ulonglong2 kk = *(const ulonglong2 *)((const u64 *)a.in.key + row);
                atomicAdd(&cnt[bin_of(kk.x)], 1u);
                atomicAdd(&cnt[bin_of(kk.y)], 1u);
            } else {
                if (row < tr.hi) atomicAdd(&cnt[bin_of(((const u64 *)a.in.key)[row])], 1u);
                if (row + 1 < tr.hi) atomicAdd(&cnt[bin_of(((const u64 *)a.in.key)[row + 1])], 1u);
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < kPassRows; ++i) {
            const u64 row = tr.lo + (u64)i * kPassThreads + threadIdx.x;
            if (row < tr.hi) atomicAdd(&cnt[bin_of(R::key(load_row<WIDE, FORM>(a.in, (long long)row)))], 1u);
        }
    }
    __syncthreads();
    const u64 base = (u64)a.tile_start[tr.seg] * F;
    for (unsigned b = threadIdx.x; b < F; b += kPassThreads) a.hist[base + (u64)b * tr.ntiles + tr.t] = cnt[b];
}

// Counting sort of each tile by bin in LDS, then contiguous runs written to
// the bins' scanned output offsets.  Persistent: a workgroup walks tiles
// wg, wg + grid, ... and loads the next tile's rows before sorting this one.
template <bool WIDE, int FORM>
__global__ __launch_bounds__(kPassThreads, 4) void k_scatter(PassArgs a) {   // 2 workgroups per CU: <= 128 VGPRs
    typedef Row<WIDE> R;
    typedef typename R::T T;
    constexpr int IT = kPassRows;
    __shared__ T stage[kTile];
    __shared__ unsigned short sb[kTile];
    __shared__ unsigned cnt[512];
    __shared__ long long dst_base[512];
    const unsigned total = a.tile_start[a.nseg];
    unsigned wg = blockIdx.x;
    if (wg >= total) return;
    const unsigned F = 1u << a.fbits;
    T *out = (T *)a.out;

    TileRange tr = tile_range(a, wg);
    T row[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
        const u64 r = tr.lo + (u64)i * kPassThreads + threadIdx.x;
        row[i] = r < tr.hi ? load_row<WIDE, FORM>(a.in, (long long)r) : R::zero();
    }
    while (true) {
        // prefetch the next tile
        const unsigned wn = wg + gridDim.x;
        const bool more = wn < total;
        TileRange tn;
        T nrow[IT];
        if (more) {
            tn = tile_range(a, wn);
#pragma unroll
            for (int i = 0; i < IT; ++i) {
                const u64 r = tn.lo + (u64)i * kPassThreads + threadIdx.x;
                nrow[i] = r < tn.hi ? load_row<WIDE, FORM>(a.in, (long long)r) : R::zero();
            }
        }
        // ---- sort this tile
        for (unsigned b = threadIdx.x; b < F; b += kPassThreads) cnt[b] = 0u;
        __syncthreads();
        unsigned br[IT];   // bin << 16 | rank within the tile's bin (bin < 512, rank < 4096)
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const u64 r = tr.lo + (u64)i * kPassThreads + threadIdx.x;
            if (r < tr.hi) {
                const unsigned b = (unsigned)(rhash(R::key(row[i])) >> a.shift) & (F - 1);
                br[i] = (b << 16) | atomicAdd(&cnt[b], 1u);
            } else {
                br[i] = 0xFFFFFFFFu;
            }
        }
        __syncthreads();
        // exclusive scan of the bin counts (first wave, 8 bins per lane) and each
        // bin's run destination base = scanned global offset - local start
        if (threadIdx.x < 64) {
            const int lane = threadIdx.x;
            unsigned c[8], s = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const unsigned b = lane * 8 + j;
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
            const u64 hb = (u64)a.tile_start[tr.seg] * F;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const unsigned b = lane * 8 + j;
                if (b < F) {
                    cnt[b] = run;
                    dst_base[b] = (long long)a.hist[hb + (u64)b * tr.ntiles + tr.t] - (long long)run;
                }
                run += c[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            if (br[i] != 0xFFFFFFFFu) {
                const unsigned b = br[i] >> 16;
                const unsigned pos = cnt[b] + (br[i] & 0xffffu);
                stage[pos] = row[i];
                sb[pos] = (unsigned short)b;
            }
        }
        __syncthreads();
        const unsigned n = (unsigned)(tr.hi - tr.lo);
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const unsigned j = (unsigned)i * kPassThreads + threadIdx.x;
            if (j < n) out[(u64)(dst_base[sb[j]] + (long long)j)] = stage[j];
        }
        if (!more) break;
        __syncthreads();   // stage/cnt reused by the next tile
        wg = wn;
        tr = tn;
#pragma unroll
        for (int i = 0; i < IT; ++i) row[i] = nrow[i];
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
    const void *r, *s;               // partitioned packed rows
    const u64 *r_off, *s_off;        // P + 1 each
    int P;
    const unsigned *work_start;      // P + 1: S chunks per partition (0 if no R rows)
    const unsigned *work_owner;      // work item -> partition
    int tshift;                      // LDS slot = (hash >> tshift) & (slots - 1)
    void *out_r, *out_s;
    long long cap;
    u64 *counter;
    u64 *dup_flag;                   // set to 1 if any partition's build rows repeat a key
};

struct Item {
    u64 s_lo, s_hi, r_lo, r_hi;
};

template <int CH>
__device__ __forceinline__ Item item_of(const JoinArgs &a, unsigned w) {
    const int p = (int)a.work_owner[w];
    const unsigned c = w - a.work_start[p];
    Item it;
    it.s_lo = a.s_off[p] + (u64)c * CH;
    const u64 e = a.s_off[p + 1];
    it.s_hi = it.s_lo + CH < e ? it.s_lo + CH : e;
    it.r_lo = a.r_off[p];
    it.r_hi = a.r_off[p + 1];
    return it;
}

// A persistent workgroup of NT threads walks work items w = wg, wg + grid, ...
// Work item = (partition, S chunk of up to kJoinSub * NT * SI rows): build
// the partition's R rows into a 2^TSL-slot LDS table (rounds of RCAP rows
// for oversized partitions), then probe the chunk in sub-chunks of NT * SI
// rows.  The next item's first S sub-chunk and R round are loaded into
// registers before this item's LDS phase.
// ABL (diagnostics only, micro/join_micro.hip; the product uses 0) switches
// phases off: 1 no cursor atomic, 2 no output writes, 4 no probe, 8 no build.
template <bool WIDE, bool WRITE, int TSL, int NT, int ABL = 0>
__global__ __launch_bounds__(NT, 4) void k_join(JoinArgs a) {   // 4 waves per SIMD: <= 128 VGPRs
    typedef Row<WIDE> R;
    typedef typename R::T T;
    typedef typename std::conditional<WIDE, u64, unsigned>::type PT;   // output element
    constexpr int TS = 1 << TSL;
    constexpr unsigned kMask = TS - 1;
    constexpr int SI = kJoinItems;            // S rows per thread per sub-chunk
    constexpr int RCAP = TS * 5 / 8;          // build rows per round (load factor <= 0.625)
    constexpr int RI = RCAP / NT;             // build rows per thread per round
    constexpr int SUBR = NT * SI;             // rows per sub-chunk
    constexpr int CH = kJoinSub * SUBR;       // rows per work item
    // wide: EMPTY key INT64_MIN (rows with that key take the null path);
    // narrow: the all-ones word (row ids < 2^31 never produce it)
    constexpr u64 kEmpty = WIDE ? kEmptyKey64 : ~0ull;
    __shared__ u64 tkey[TS];                  // wide: keys; narrow: packed rows
    __shared__ u64 tpay[WIDE ? TS : 1];
    __shared__ u64 wsum[16];
    __shared__ u64 s_base;
    __shared__ unsigned s_dup;

    const unsigned total = a.work_start[a.P];
    unsigned w = blockIdx.x;
    if (w >= total) return;
    const T *rrows = (const T *)a.r;
    const T *srows = (const T *)a.s;
    PT *orr = (PT *)a.out_r;
    PT *oss = (PT *)a.out_s;

    Item it = item_of<CH>(a, w);
    T sv_[SI], rv_[RI];
#pragma unroll
    for (int i = 0; i < RI; ++i) {
        const u64 row = it.r_lo + (u64)i * NT + threadIdx.x;
        rv_[i] = row < it.r_hi ? rrows[row] : R::zero();
    }

    while (true) {
        // this item's first S sub-chunk: issued before the table init / build
        // so its latency hides behind them
#pragma unroll
        for (int i = 0; i < SI; ++i) {
            const u64 row = it.s_lo + (u64)i * NT + threadIdx.x;
            sv_[i] = row < it.s_hi ? srows[row] : R::zero();
        }
        // ---- prefetch the next work item's build rows
        const unsigned wn = w + gridDim.x;
        const bool more = wn < total;
        Item nx;
        T nrv[RI];
        if (more) {
            nx = item_of<CH>(a, wn);
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                const u64 row = nx.r_lo + (u64)i * NT + threadIdx.x;
                nrv[i] = row < nx.r_hi ? rrows[row] : R::zero();
            }
        }

        u64 n_null_r = 0;
        bool any_null_s = false;
        for (u64 r0 = it.r_lo; r0 < it.r_hi; r0 += RCAP) {
            const u64 r1 = r0 + RCAP < it.r_hi ? r0 + RCAP : it.r_hi;
            if (r0 != it.r_lo) {   // later rounds (oversized partitions)
#pragma unroll
                for (int i = 0; i < RI; ++i) {
                    const u64 row = r0 + (u64)i * NT + threadIdx.x;
                    rv_[i] = row < r1 ? rrows[row] : R::zero();
                }
            }
            // ---- init: every slot EMPTY (16-B LDS stores)
            for (int j = threadIdx.x; j < TS / 2; j += NT) ((ulonglong2 *)tkey)[j] = make_ulonglong2(kEmpty, kEmpty);
            if (threadIdx.x == 0) s_dup = 0u;
            __syncthreads();
            // ---- build this round's rows: every row's first CAS is issued
            // before any result is used (RI independent LDS atomics in flight)
            bool dup = false;
            unsigned hb[RI];
            u64 ob[RI], vb[RI];
            bool act[RI];
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                const u64 row = r0 + (u64)i * NT + threadIdx.x;
                const u64 key = R::key(rv_[i]);
                act[i] = row < r1;
                if (WIDE && act[i] && key == kEmptyKey64) {
                    ++n_null_r;
                    act[i] = false;
                }
                if constexpr ((ABL & 8) != 0) act[i] = false;
                hb[i] = (unsigned)(rhash(key) >> a.tshift) & kMask;
                if constexpr (WIDE) vb[i] = key;
                else vb[i] = rv_[i];
                ob[i] = act[i] ? atomicCAS(&tkey[hb[i]], kEmpty, vb[i]) : kEmpty;
            }
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                if (!act[i]) continue;
                const u64 key = R::key(rv_[i]);
                unsigned h = hb[i];
                u64 old = ob[i];
                while (old != kEmpty) {
                    dup |= WIDE ? (old == key) : ((old >> 32) == key);
                    h = (h + 1) & kMask;
                    old = atomicCAS(&tkey[h], kEmpty, vb[i]);
                }
                if constexpr (WIDE) tpay[h] = R::pay(rv_[i]);
            }
            if (dup) s_dup = 1u;
            __syncthreads();
            const bool unique = s_dup == 0u;
            if (!unique && threadIdx.x == 0)
                __hip_atomic_store(a.dup_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

            // ---- probe the chunk, one sub-chunk of S rows at a time
            for (u64 sb = it.s_lo; sb < it.s_hi; sb += SUBR) {
                if (sb != it.s_lo || r0 != it.r_lo) {
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const u64 row = sb + (u64)i * NT + threadIdx.x;
                        sv_[i] = row < it.s_hi ? srows[row] : R::zero();
                    }
                }
                // first slot of every row read before any is resolved (SI
                // independent LDS reads in flight); most rows end there
                unsigned m[SI], hp[SI];
                u64 e0[SI];
                bool pa[SI];
                u64 cnt = 0;
#pragma unroll
                for (int i = 0; i < SI; ++i) {
                    m[i] = 0xFFFFFFFFu;
                    const u64 row = sb + (u64)i * NT + threadIdx.x;
                    const u64 key = R::key(sv_[i]);
                    pa[i] = row < it.s_hi;
                    if (WIDE && pa[i] && key == kEmptyKey64) {   // matched by the null pass below
                        any_null_s = true;
                        pa[i] = false;
                    }
                    if constexpr ((ABL & 4) != 0) {
                        cnt += pa[i] ? (key & 1) : 0;
                        pa[i] = false;
                    }
                    hp[i] = (unsigned)(rhash(key) >> a.tshift) & kMask;
                    e0[i] = pa[i] ? tkey[hp[i]] : kEmpty;
                }
#pragma unroll
                for (int i = 0; i < SI; ++i) {
                    if (!pa[i]) continue;
                    const u64 key = R::key(sv_[i]);
                    unsigned h = hp[i];
                    u64 e = e0[i];
                    while (e != kEmpty) {
                        if ((WIDE ? e : (e >> 32)) == key) {
                            ++cnt;
                            if (unique) {
                                m[i] = h;
                                break;
                            }
                        }
                        h = (h + 1) & kMask;
                        e = tkey[h];
                    }
                }
                u64 tot;
                const u64 pre = block_excl_scan<NT>(cnt, wsum, &tot);
                if constexpr (!WRITE) {
                    if (threadIdx.x == 0 && tot) atomicAdd(a.counter, tot);
                } else if (tot) {
                    if (threadIdx.x == 0) s_base = (ABL & 1) ? (u64)w * CH : atomicAdd(a.counter, tot);
                    __syncthreads();
                    u64 pos = s_base + pre;
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        if constexpr ((ABL & 2) != 0) break;
                        const PT spay = (PT)R::pay(sv_[i]);
                        if (unique) {
                            if (m[i] != 0xFFFFFFFFu) {
                                if (pos < (u64)a.cap) {
                                    orr[pos] = WIDE ? (PT)tpay[m[i]] : (PT)(tkey[m[i]] & 0xffffffffull);
                                    oss[pos] = spay;
                                }
                                ++pos;
                            }
                        } else {
                            const u64 row = sb + (u64)i * NT + threadIdx.x;
                            const u64 key = R::key(sv_[i]);
                            if (row >= it.s_hi || (WIDE && key == kEmptyKey64)) continue;
                            unsigned h = (unsigned)(rhash(key) >> a.tshift) & kMask;
                            while (true) {
                                const u64 e = tkey[h];
                                if (e == kEmpty) break;
                                if ((WIDE ? e : (e >> 32)) == key) {
                                    if (pos < (u64)a.cap) {
                                        orr[pos] = WIDE ? (PT)tpay[h] : (PT)(e & 0xffffffffull);
                                        oss[pos] = spay;
                                    }
                                    ++pos;
                                }
                                h = (h + 1) & kMask;
                            }
                        }
                    }
                    __syncthreads();   // s_base reused by the next sub-chunk
                }
            }
            __syncthreads();   // table reused by the next round / item
        }

        // ---- INT64_MIN keys (the wide EMPTY sentinel): matched outside the table
        if constexpr (WIDE) {
            if (__syncthreads_or(any_null_s ? 1 : 0)) {
                u64 nn;
                (void)block_excl_scan<NT>(n_null_r, wsum, &nn);   // null R rows of this partition
                for (u64 sb = it.s_lo; sb < it.s_hi; sb += SUBR) {
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const u64 row = sb + (u64)i * NT + threadIdx.x;
                        sv_[i] = row < it.s_hi ? srows[row] : R::zero();
                    }
                    u64 cnt = 0;
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const u64 row = sb + (u64)i * NT + threadIdx.x;
                        if (row < it.s_hi && R::key(sv_[i]) == kEmptyKey64) cnt += nn;
                    }
                    u64 tot;
                    const u64 pre = block_excl_scan<NT>(cnt, wsum, &tot);
                    if constexpr (!WRITE) {
                        if (threadIdx.x == 0 && tot) atomicAdd(a.counter, tot);
                    } else if (tot) {
                        if (threadIdx.x == 0) s_base = atomicAdd(a.counter, tot);
                        __syncthreads();
                        u64 pos = s_base + pre;
                        for (int i = 0; i < SI; ++i) {
                            const u64 row = sb + (u64)i * NT + threadIdx.x;
                            if (!(row < it.s_hi && R::key(sv_[i]) == kEmptyKey64)) continue;
                            for (u64 r = it.r_lo; r < it.r_hi; ++r) {
                                const T rr = rrows[r];
                                if (R::key(rr) != kEmptyKey64) continue;
                                if (pos < (u64)a.cap) {
                                    orr[pos] = (PT)R::pay(rr);
                                    oss[pos] = (PT)R::pay(sv_[i]);
                                }
                                ++pos;
                            }
                        }
                        __syncthreads();
                    }
                }
            }
        }

        if (!more) break;
        w = wn;
        it = nx;
#pragma unroll
        for (int i = 0; i < RI; ++i) rv_[i] = nrv[i];
    }
}

// Join kernel variant: log2 LDS slots and workgroup size.  HJ_JOIN_TSL
// (11 | 12 | 13) overrides the default for experiments.
struct JoinVariant {
    int tsl;
    int nt;
};
JoinVariant join_variant() {
    static int tsl = [] {
        const char *e = getenv("HJ_JOIN_TSL");
        const int v = e ? atoi(e) : 12;
        return (v == 11 || v == 12 || v == 13) ? v : 12;
    }();
    return JoinVariant{tsl, tsl == 13 ? 1024 : (tsl == 12 ? 512 : 256)};
}

int cu_count() {
    static int n = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return cus > 0 ? cus : 256;
    }();
    return n;
}

inline unsigned blocks_for(u64 n, u64 per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

// ----------------------------------------------------------------- planning
RadixPlan radix_plan(long long n_build, int force_bits) {
    // average build rows per partition <= half the join kernel's LDS slots
    const int tsl = join_variant().tsl;
    RadixPlan pl;
    int bits = 1;
    while (bits < 24 && ((unsigned long long)n_build >> bits) > (1ull << (tsl - 1))) ++bits;
    if (force_bits > 0) bits = force_bits < 24 ? force_bits : 24;
    pl.total_bits = bits;
    pl.passes = (bits + 8) / 9;   // <= 9 bits (512-way fan-out) per pass
    int left = bits;
    for (int i = 0; i < pl.passes; ++i) {
        pl.bits[i] = (left + (pl.passes - i) - 1) / (pl.passes - i);
        left -= pl.bits[i];
    }
    for (int i = pl.passes; i < 3; ++i) pl.bits[i] = 0;
    return pl;
}

size_t radix_hist_elems(long long n, int max_nseg) {
    return ((size_t)n / kTile + (size_t)max_nseg + 2) * 512;
}

int radix_chunk_rows() { return join_variant().nt * kJoinItems * kJoinSub; }

// Partition one relation into the plan's 2^total_bits partitions of packed
// rows (16 B wide, 8 B narrow) in `out`, with partition offsets in out_off
// (P + 1).  ws.tmp is the ping buffer of multi-pass plans.  Asynchronous; no
// allocation.
hipError_t radix_partition(const SrcDev &src, bool wide, const RadixPlan &pl, const RadixWork &ws, void *out,
                           unsigned long long *out_off, hipStream_t st) {
    const u64 n = (u64)src.n;
    hipLaunchKernelGGL(k_set_off, dim3(1), dim3(64), 0, st, ws.off_a, n);
    int nseg = 1;
    int shift = 64;
    SrcDev in = src;
    u64 *seg_off = ws.off_a;
    static const unsigned persist_env = [] {
        const char *e = getenv("HJ_SCATTER_WG_PER_CU");   // experiments: 0 = one tile per workgroup
        return e ? (unsigned)atoi(e) : 2u;
    }();
    const unsigned persist = persist_env ? persist_env * (unsigned)cu_count() : 0xFFFFFFFFu;
    for (int pass = 0; pass < pl.passes; ++pass) {
        const int fb = pl.bits[pass];
        shift -= fb;
        const bool last = pass == pl.passes - 1;
        // destination: final buffer on the last pass, else alternate so the
        // last pass lands in `out`
        void *dst = last ? out : ((((pl.passes - 1 - pass) % 2) == 1) ? ws.tmp : out);
        u64 *next_off = last ? out_off : (seg_off == ws.off_a ? ws.off_b : ws.off_a);
        PassArgs a;
        a.in = in;
        a.seg_off = seg_off;
        a.nseg = nseg;
        a.tile_start = ws.tile_start;
        a.tile_owner = ws.tile_owner;
        a.hist = ws.hist;
        a.out = dst;
        a.next_off = next_off;
        a.shift = shift;
        a.fbits = fb;
        const unsigned F = 1u << fb;
        hipLaunchKernelGGL(k_chunk_map, dim3(1), dim3(1024), 0, st, (const u64 *)seg_off, (const u64 *)nullptr, nseg,
                           (unsigned)kTile, ws.tile_start);
        const unsigned grid = (unsigned)(n / kTile + nseg + 1);
        if (nseg > 1)
            hipLaunchKernelGGL(k_work_list, dim3(blocks_for((u64)nseg, 256)), dim3(256), 0, st,
                               (const unsigned *)ws.tile_start, nseg, ws.tile_owner);
        const u64 hlen = (u64)grid * F;
        hipError_t e = hipMemsetAsync(ws.hist, 0, hlen * sizeof(u64), st);
        if (e != hipSuccess) return e;
        const unsigned sgrid = grid < persist ? grid : persist;
#define HJ_PASS(W, FORM)                                                                                  \
    do {                                                                                                  \
        hipLaunchKernelGGL((k_hist<W, FORM>), dim3(grid), dim3(kPassThreads), 0, st, a);                  \
        const unsigned nb = blocks_for(hlen, kScanBlock);                                                 \
        hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, st, ws.hist, hlen, ws.scan_sums);      \
        if (nb > 1) {                                                                                     \
            hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(1024), 0, st, ws.scan_sums, nb);                \
            hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(1024), 0, st, ws.hist, hlen,                    \
                               (const u64 *)ws.scan_sums);                                                \
        }                                                                                                 \
        hipLaunchKernelGGL((k_scatter<W, FORM>), dim3(sgrid), dim3(kPassThreads), 0, st, a);              \
    } while (0)
        if (wide) {
            if (in.form == kCols64) HJ_PASS(true, kCols64);
            else HJ_PASS(true, kPackedRow);   // kPacked64 input == packed row layout
        } else {
            if (in.form == kCol32) HJ_PASS(false, kCol32);
            else HJ_PASS(false, kPackedRow);
        }
#undef HJ_PASS
        hipLaunchKernelGGL(k_next_off, dim3(blocks_for((u64)nseg * F + 1, 256)), dim3(256), 0, st, a);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        // the next pass reads this pass's packed rows
        in.key = dst;
        in.pay = nullptr;
        in.form = kPackedRow;
        seg_off = next_off;
        nseg *= (int)F;
    }
    return hipSuccess;
}

hipError_t radix_join(bool wide, const RadixPlan &pl, const void *r_rows, const unsigned long long *r_off,
                      const void *s_rows, const unsigned long long *s_off, long long n_s, unsigned *work_start,
                      void *out_r, void *out_s, long long cap, unsigned long long *counter,
                      unsigned long long *dup_flag, bool count_only, hipStream_t st) {
    const int P = 1 << pl.total_bits;
    unsigned *work_owner = work_start + P + 1;
    const JoinVariant jv = join_variant();
    const unsigned chunk = (unsigned)(jv.nt * kJoinItems * kJoinSub);
    hipLaunchKernelGGL(k_chunk_map, dim3(1), dim3(1024), 0, st, s_off, r_off, P, chunk, work_start);
    hipLaunchKernelGGL(k_work_list, dim3(blocks_for((u64)P, 256)), dim3(256), 0, st, (const unsigned *)work_start, P,
                       work_owner);
    JoinArgs a;
    a.r = r_rows;
    a.s = s_rows;
    a.r_off = r_off;
    a.s_off = s_off;
    a.P = P;
    a.work_start = work_start;
    a.work_owner = work_owner;
    a.tshift = 64 - pl.total_bits - jv.tsl;   // the hash bits right below the partition bits
    a.out_r = out_r;
    a.out_s = out_s;
    a.cap = cap;
    a.counter = counter;
    a.dup_flag = dup_flag;
    const unsigned items = (unsigned)((u64)n_s / chunk + (u64)P + 1);
    // persistent grid: as many workgroups as fit at once (LDS-limited)
    const int per_cu = jv.tsl == 13 ? 1 : (jv.tsl == 12 ? 2 : 4);
    const unsigned pg = (unsigned)(per_cu * cu_count());
    const unsigned grid = items < pg ? items : pg;
#define HJ_JOIN(W, WR, TSL, NT) hipLaunchKernelGGL((k_join<W, WR, TSL, NT>), dim3(grid), dim3(NT), 0, st, a)
#define HJ_JOIN_V(W, WR)                              \
    do {                                              \
        if (jv.tsl == 13) HJ_JOIN(W, WR, 13, 1024);   \
        else if (jv.tsl == 12) HJ_JOIN(W, WR, 12, 512); \
        else HJ_JOIN(W, WR, 11, 256);                 \
    } while (0)
    if (wide) {
        if (count_only) HJ_JOIN_V(true, false);
        else HJ_JOIN_V(true, true);
    } else {
        if (count_only) HJ_JOIN_V(false, false);
        else HJ_JOIN_V(false, true);
    }
#undef HJ_JOIN_V
#undef HJ_JOIN
    return hipGetLastError();
}

}  // namespace hj
