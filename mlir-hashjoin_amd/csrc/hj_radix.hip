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
//   pass k (1..3): bucket chaining.  A workgroup owns a contiguous range of
//                  8192-row tiles; it counting-sorts each tile by bin in LDS
//                  and appends every bin's run to the workgroup's current
//                  bucket for that bin (2^pbl rows; a full bucket is replaced
//                  by fresh ids from the workgroup's own id range).  The input
//                  is read ONCE: no histogram pass and no global scan
//                  (profiles/r01_micro_bucket_pass.txt: 2.27 ms per 2^28-row
//                  pass vs 3.3 ms for histogram + exact-offset scatter).
//                  Then the buckets are listed per partition (two small
//                  kernels over ~n/512 bucket ids).
//   join:          one work item per (partition, S bucket chunk): build the
//                  partition's R buckets into an LDS table (rounds of RCAP
//                  rows for oversized partitions), probe the chunk, count,
//                  block-scan, reserve the block's output with ONE global
//                  atomic, and write every pair at its position.
//
// Partitioned rows are packed: 16-B {key, payload} (64-bit keys) or 8-B
// (key << 32 | row id) (the reference's i32 types), so a row moves with one
// global load/store and an i32 row is already its own LDS table entry.
//
// The reference's count -> prefix -> probe protocol (join_v1.mlir:288-521) is
// kept, but per workgroup and on LDS, so the output needs no staging buffer
// and has no overflow path.
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "hj.h"
#include "hj_internal.h"

namespace hj {
namespace {

typedef unsigned long long u64;
constexpr int kTile = 4096;        // rows per partition-pass tile (LDS staging: 64 KiB wide)
constexpr int kPassThreads = 1024; // one workgroup per CU
constexpr int kPassRows = kTile / kPassThreads;
constexpr int kMaxFan = 512;       // bins per pass (9 bits)
// passes of <= 8 bits: half-size workgroups (512 threads, 2048-row tiles,
// 256 bins' line tails: ~70 KiB of LDS), two per CU, so one workgroup's LDS
// phases overlap the other's loads and stores
constexpr int kSmallPassThreads = 512;
constexpr int kSmallFan = 256;
constexpr int kJoinItems = 5;      // S rows per thread per sub-chunk of the join kernel (2560 rows = 10 buckets)
constexpr int kJoinSub = 8;        // sub-chunks per work item (one table build serves all)
constexpr int kPackedRow = 3;      // SrcForm of packed-row inputs
constexpr int kBucketed = 4;       // SrcForm of a previous pass's bucket set
constexpr unsigned kNoBucket = 0xFFFFFFFFu;
// Join items of multi-chunk partitions first (k_item_desc): int64 rows only
// (profiles/r03_heavy_first.txt).
constexpr bool kHeavyFirst = true;

__device__ __forceinline__ u64 rhash(u64 k) { return radix_hash(k); }

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

// Streaming (non-temporal) loads/stores for data touched once per kernel.
// Measured (profiles/r01_nt_variants.txt): join loads + stores nt -2.7 %;
// pass loads nt +3 %.  Pass stores: nt cost +66 % while a line's old tail
// and new rows went out in two store instructions (nt bypasses the L2 that
// assembled them); since round 4 every line is one instruction's (k_pass's
// line stores) and nt stores are 0.3-2.6 % faster (profiles/r04_line_stores.txt).
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
template <bool NT, typename T>
__device__ __forceinline__ T ld_s(const T *p) {
    if constexpr (!NT) {
        return *p;
    } else if constexpr (sizeof(T) == 16) {
        const v2u64 x = __builtin_nontemporal_load((const v2u64 *)p);
        T r;
        r.x = x.x;
        r.y = x.y;
        return r;
    } else {
        return __builtin_nontemporal_load(p);
    }
}
template <bool NT, typename T>
__device__ __forceinline__ void st_s(T *p, const T &v) {
    if constexpr (!NT) {
        *p = v;
    } else if constexpr (sizeof(T) == 16) {
        v2u64 x;
        x.x = v.x;
        x.y = v.y;
        __builtin_nontemporal_store(x, (v2u64 *)p);
    } else {
        __builtin_nontemporal_store(v, p);
    }
}
// (nt loads in the passes: 1 % off C3's step since the stores are whole nt
// lines; with plain stores they lost 0.3 ms -- profiles/r04_pass_nt_loads.txt)
constexpr bool kNtPassLd = true, kNtPassSt = true;
constexpr bool kNtJoinLd = true, kNtJoinSt = true;

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
    const u64 x = wave_incl_add64(v);
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
        const u64 t = wave_incl_add64(lane < NW ? wsum[lane] : 0ull);
        if (lane < NW) wsum[lane] = t;
    }
    __syncthreads();
    const u64 before = w ? wsum[w - 1] : 0ull;
    *total = wsum[NW - 1];
    __syncthreads();   // wsum reusable after return
    return before + x - v;
}

// --------------------------------------------------------------- maps
// Chunk map of nseg segments: count(s) = ceil(len_a(s) / chunk), or 0 when
// off_b is given and segment s of b is empty (no build rows -> nothing to
// join); start = exclusive scan of count (scan_u64), and owner[w] = the
// segment of chunk w, so consumers need one load instead of a search.
// split: the high half of each count word also counts the chunks of
// segments with >= 2 of them (their scan: k_item_desc's heavy-first order).
__global__ __launch_bounds__(256) void k_chunk_count(const u64 *off_a, const u64 *off_b, int nseg, unsigned chunk,
                                                     u64 *cnt, bool split) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s > nseg) return;
    if (s == nseg) {
        cnt[s] = 0;
        return;
    }
    const u64 len = off_a[s + 1] - off_a[s];
    const bool live = off_b ? (off_b[s + 1] > off_b[s]) : true;
    const u64 c = live ? (len + chunk - 1) / chunk : 0ull;
    cnt[s] = split && c >= 2 ? c | (c << 32) : c;
}

// (2^tl threads per segment: many chunks per segment -- a pass's tiles --
// fill their owners side by side instead of one thread looping)
__global__ __launch_bounds__(256) void k_chunk_finish(const u64 *scan, int nseg, unsigned *start, unsigned *owner,
                                                      int tl) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int s = g >> tl, l = g & ((1 << tl) - 1);
    if (s > nseg) return;
    if (l == 0) start[s] = (unsigned)scan[s];
    if (s < nseg)
        for (u64 w = (unsigned)scan[s] + (u64)l; w < (unsigned)scan[s + 1]; w += (1u << tl)) owner[w] = (unsigned)s;
}

// --------------------------------------------------------------- scan
// In-place exclusive scan of a u64 array (2 kernels: block scan, then each
// block adds the sum of the block totals before it, reduced by the block
// itself).  8192 elements per block.
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

__global__ __launch_bounds__(1024) void k_scan_add(u64 *a, u64 n, const u64 *sums) {
    __shared__ u64 wsum[16];
    if (blockIdx.x == 0) return;   // (uniform: block 0 adds nothing)
    u64 v = 0;
    for (unsigned i = threadIdx.x; i < blockIdx.x; i += 1024) v += sums[i];
    u64 add;
    block_excl_scan<1024>(v, wsum, &add);
    const u64 base = (u64)blockIdx.x * kScanBlock;
    for (int i = threadIdx.x; i < kScanBlock; i += 1024)
        if (base + i < n) a[base + i] += add;
}

__device__ __forceinline__ unsigned runs_of(unsigned fill) { return (fill + (1u << kRunLog) - 1) >> kRunLog; }

// --------------------------------------------------------------- one-launch scan
// Exclusive scan in ONE launch (decoupled look-back) for the listings of the
// radix passes and the join's work map: tiles of kScanBlock elements are
// taken in ticket order; a tile publishes its aggregate, wave 0 looks back
// over its predecessors' words (aggregate, or inclusive prefix: stop there),
// then the tile publishes its inclusive prefix.  A word is flag << 62 |
// value; both sides use 8-B device-scope atomic RMWs (executed coherently
// across the XCDs' L2s).  Forward progress: a tile only waits on tiles
// whose tickets were drawn earlier, i.e. by running workgroups.
// state: one word per tile + ticket + done counter, zero on entry; the last
// workgroup to finish clears them for the next call (a kernel boundary
// orders that before any later launch).
constexpr u64 kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbVal = (1ull << 62) - 1;
// tiles of 1024 elements (256 threads x 4): 2^17 partitions spread over 129
// workgroups instead of 17 (the scan is latency-bound, not byte-bound)
constexpr int kLbThreads = 256, kLbPer = 4, kLbTile = kLbThreads * kLbPer;

// MAP (the join's work map, chunk_map's three launches in one): element p <
// nseg is the chunk count of segment p -- ceil(len_a(p) / chunk), 0 when
// off_b says segment p of b is empty -- and, with split, its heavy count
// (the count when >= 2) in bits 31..61; element nseg is 0.  The scan goes
// to scan[] as heavy << 32 | count (k_item_desc's split order), its low half
// to start[], and owner[w] = p for segment p's chunks.
struct ChunkMapArgs {
    const u64 *off_a, *off_b;
    unsigned chunk;
    bool split;
    unsigned *start, *owner;
};

template <bool MAP>
__global__ __launch_bounds__(kLbThreads) void k_scan_lb(u64 *a, u64 n, u64 *state, ChunkMapArgs mp) {
    __shared__ u64 wsum[16];
    __shared__ u64 s_pre;
    __shared__ unsigned s_tile;
    const unsigned nt = (unsigned)((n + kLbTile - 1) / kLbTile);
    if (threadIdx.x == 0) s_tile = (unsigned)atomicAdd(&state[nt], 1ull);
    __syncthreads();
    const unsigned t = s_tile;
    const u64 base = (u64)t * kLbTile + (u64)threadIdx.x * kLbPer;
    u64 v[kLbPer], s = 0;
#pragma unroll
    for (int i = 0; i < kLbPer; ++i) {
        const u64 e = base + i;
        if constexpr (MAP) {
            v[i] = 0ull;
            if (e + 1 < n) {   // (element n - 1 = nseg: 0)
                const u64 len = mp.off_a[e + 1] - mp.off_a[e];
                const bool live = mp.off_b ? (mp.off_b[e + 1] > mp.off_b[e]) : true;
                const u64 c = live ? (len + mp.chunk - 1) / mp.chunk : 0ull;
                v[i] = mp.split && c >= 2 ? c | (c << 31) : c;
            }
        } else {
            v[i] = e < n ? a[e] : 0ull;
        }
        s += v[i];
    }
    u64 total;
    u64 run = block_excl_scan<kLbThreads>(s, wsum, &total);
    if (threadIdx.x < 64) {
        const unsigned lane = threadIdx.x;
        u64 pre = 0;
        if (t == 0) {
            if (lane == 0) atomicExch(&state[0], kLbInc | total);
        } else {
            if (lane == 0) atomicExch(&state[t], kLbAgg | total);
            // wave 0 reads 64 predecessors at a time (lane j: tile w - 1 - j)
            for (unsigned w = t; w > 0;) {
                const u64 x = lane < w ? atomicOr(&state[w - 1 - lane], 0ull) : kLbInc;   // (past tile 0: a stop)
                const u64 inc = __ballot((x >> 62) == 2ull), none = __ballot((x >> 62) == 0ull);
                const u64 upto = inc ? (inc & (~inc + 1ull)) * 2ull - 1ull : ~0ull;   // lanes up to the nearest stop
                if (none & upto) {   // a predecessor has not published yet: read again
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                pre += wave_incl_add64((upto >> lane) & 1ull && lane < w ? (x & kLbVal) : 0ull);
                pre = __shfl(pre, 63);
                if (inc) break;
                w = w > 64u ? w - 64u : 0u;
            }
            if (lane == 0) atomicExch(&state[t], kLbInc | (pre + total));
        }
        if (lane == 0) s_pre = pre;
    }
    __syncthreads();
    run += s_pre;
#pragma unroll
    for (int i = 0; i < kLbPer; ++i) {
        const u64 e = base + i;
        if (e < n) {
            if constexpr (MAP) {
                const unsigned lo = (unsigned)(run & 0x7FFFFFFFull);
                a[e] = ((run >> 31) << 32) | lo;
                mp.start[e] = lo;
                const unsigned c = (unsigned)(v[i] & 0x7FFFFFFFull);
                for (unsigned k = 0; k < c; ++k) mp.owner[lo + k] = (unsigned)e;
            } else {
                a[e] = run;
            }
        }
        run += v[i];
    }
    __syncthreads();
    // The done count is what lets the last workgroup clear every word, so it
    // must not overtake this tile's own publishes (the atomicExch calls on
    // state[t] above): a release fence orders them, and the clearing thread's acquire fence
    // orders every tile's publish before its clears.  Two
    // fences per workgroup, once per scan.
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&state[nt + 1], 1ull) == (u64)nt - 1ull) {
            __threadfence();
            for (unsigned k = 0; k < nt + 2; ++k) atomicExch(&state[k], 0ull);
        }
    }
}

// --------------------------------------------------------------- partition pass
struct PassArgs {
    SrcDev in;                   // pass-1 source (FORM != kBucketed)
    u64 n;                       // pass-1 source rows
    bool cols_aligned;           // kCols64: both columns 16-B aligned
    // FORM == kBucketed: the previous pass's set, tiles of up to kTile rows
    // (kTile >> kRunLog runs) that never straddle two segments
    const void *in_rows;
    const u64 *in_runs;          // row << 7 | count
    const u64 *in_rstart;
    u64 in_max_rows, in_max_runs;   // capacities of the input set (loads are clamped to them)
    const unsigned *tile_start;  // nseg + 1
    const struct TileDesc *tdesc;   // per tile (k_tile_desc)
    int nseg;
    // output set
    void *out_rows;
    unsigned *bbin, *bfill, *nb;
    const unsigned *wstart;      // G + 1: workgroup w's bucket ids are [wstart[w], wstart[w + 1]) (k_id_plan)
    unsigned max_buckets;
    int out_pbl;
    int shift;                   // bin = (hash >> shift) & (F - 1)
    int fbits;
    u64 *prof = nullptr;         // diagnostics (ABL & 8): per workgroup, cycles per phase
    // the listing's per-partition run counts (zeroed by the plan kernel that
    // runs before the pass): a bucket adds its runs when it is full or closed
    // (k_bcount's count, done where the buckets are made); null: no listing
    u64 *rcnt = nullptr;
    // EXACT passes (the folded routing): workgroup w writes bin b's rows to
    // out rows [slot_base[b * G + w], ...) -- exact, contiguous per bin, no
    // buckets; out_max_rows bounds every write
    const u64 *slot_base = nullptr;
    u64 out_max_rows = 0;
    int hash_top = 0;   // EXACT: bin = the top fbits of the hash (shift = 64 - fbits)
    unsigned tile_rows = kTile;   // rows per tile of this pass's kernel variant (its threads x kPassRows)
};

// A bucketed pass's tile: runs [lo, lo + cnt) (cnt <= kTile / 64) of segment seg.
struct TileDesc {
    u64 lo;
    unsigned cnt, seg;
};

__global__ __launch_bounds__(256) void k_tile_desc(const unsigned *tile_start, const unsigned *tile_owner,
                                                   const u64 *rstart, int nseg, unsigned bound, TileDesc *desc,
                                                   unsigned rpt) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    if (t >= tile_start[nseg] || t >= bound) return;
    const unsigned seg = tile_owner[t];
    const u64 lo = rstart[seg] + (u64)(t - tile_start[seg]) * rpt;
    const u64 e = rstart[seg + 1];
    TileDesc d;
    d.lo = lo;
    d.cnt = (unsigned)(e - lo < (u64)rpt ? e - lo : (u64)rpt);
    d.seg = seg;
    desc[t] = d;
}

template <int FORM, int TILE = kTile>
__device__ __forceinline__ unsigned pass_tiles(const PassArgs &a) {
    if constexpr (FORM == kBucketed) return a.tile_start[a.nseg];
    else return (unsigned)((a.n + TILE - 1) / TILE);
}

// Row v (0 <= v < kTile) of the row-source tile starting at row lo; false
// if the source has no such row.
template <bool WIDE, int FORM>
__device__ __forceinline__ bool tile_row(const PassArgs &a, u64 lo, unsigned v, typename Row<WIDE>::T &out) {
    const u64 row = lo + v;
    if (row >= a.n) return false;
    out = load_row<WIDE, FORM>(a.in, (long long)row);
    return true;
}

// One partition pass (see the file header).  Workgroup w owns tiles
// [w*T/G, (w+1)*T/G); its open bucket per bin lives in LDS (cur, fill) and
// is closed (bfill written) when the workgroup moves to another segment or
// finishes, so at most (G + nseg) * F buckets are ever partly filled.
//
// Only whole 128-B lines are written.  A bin's run from one tile starts and
// ends inside lines, and a line stored in two parts costs the HBM a
// read-modify-write: 2.47 ms per 2^28-row pass with unaligned 256-B runs
// against 1.67 ms for the same traffic in aligned runs
// (profiles/r01_micro_write_alignment.txt, micro/ws_micro.hip).  So each bin
// keeps the rows of its last, incomplete line in LDS (tail, < L rows) and
// writes them with the line's remaining rows from a later tile; a bucket
// holds a whole number of lines, and only the final line of a workgroup's
// open bucket is ever written partly (at close).
// ABL (diagnostics only, micro/pass_micro.hip; the product uses 0): 1 fresh
// buckets from a fixed per-tile range instead of the global atomic, 2
// synthetic rows instead of loads, 4 no row stores (rows and tails), 8 time
// the phases (s_memtime after each barrier, summed into a.prof).
// EXACT: the same tiles, counting sort, line tails and pipelined loads, but
// each (workgroup, bin) writes one exact contiguous slot (k_slot_hist + scan
// give the bases): rows land grouped by bin with no holes, so a bin's rows
// can be sent as one message.  A slot's first line is shared with the slot
// before it (written partly, once); every other line is written whole.
template <bool WIDE, int FORM, int ABL = 0, bool EXACT = false, int NT = kPassThreads, int FMAX = kMaxFan,
          int IT = kPassRows>
__global__ __launch_bounds__(NT) void k_pass(PassArgs a) {
    typedef Row<WIDE> R;
    typedef typename R::T T;
    constexpr int kTile = NT * IT;          // (shadows the file's: this variant's tile)
    constexpr int kPassThreads = NT;
    constexpr int kMaxFan = FMAX;
    static_assert(FMAX == 256 || FMAX == 512, "wave 0 scans 4 or 8 bins per lane");
    constexpr unsigned L = 128 / sizeof(T);   // rows per line
    __shared__ T stage[kTile];
    __shared__ T tail[kMaxFan * (L - 1)];   // bin b: rows of positions [fill & ~(L-1), fill)
    __shared__ __attribute__((aligned(16))) unsigned cnt[kMaxFan], start[kMaxFan], cur[kMaxFan], fill[kMaxFan],
        nbase[kMaxFan], lstart[kMaxFan];
    // the tile's complete lines, bin by bin: line x of the tile is a line of
    // bin lbin[x] (its (x - lstart[b])-th), written by L lanes of ONE store
    // instruction (old tail rows + new rows), so no line is ever stored in
    // two parts
    constexpr int kLines = (kTile + kMaxFan * (L - 1)) / L;
    __shared__ unsigned short lbin[kLines];
    __shared__ unsigned s_nl;
    // EXACT: out row of bin b's position 0 (the slot base rounded down to a
    // line; positions below cur[b] belong to the slot before)
    __shared__ u64 cbase[EXACT ? kMaxFan : 1];
    // the tile's fresh buckets: ids s_nb, s_nb + 1, ... (below s_nend)
    __shared__ unsigned s_nb, s_nend;
    // the previous tile's largest bin when it held more than kTile / 8 rows,
    // else ~0.  The next tile's lanes of that bin count with one LDS atomic
    // per wave instruction: a skewed key puts most of a wave on ONE counter,
    // and the serialised same-address atomics made the workgroups holding
    // the hot segment the pass's stragglers (C4 S pass 2: 2.3 vs 1.7 ms).
    __shared__ unsigned s_hot;
    __shared__ unsigned s_hole;
    const unsigned F = 1u << a.fbits;
    const unsigned PB = 1u << a.out_pbl;
    const unsigned T_ = pass_tiles<FORM, kTile>(a);
    const unsigned t0 = (unsigned)((u64)blockIdx.x * T_ / gridDim.x);
    const unsigned t1 = (unsigned)((u64)(blockIdx.x + 1) * T_ / gridDim.x);
    T *out = (T *)a.out_rows;
    for (unsigned b = threadIdx.x; b < F; b += kPassThreads) {
        cnt[b] = 0u;
        if constexpr (EXACT) {
            const u64 sbase = a.slot_base[(u64)b * gridDim.x + blockIdx.x];
            const unsigned off0 = (unsigned)(sbase & (L - 1));
            cbase[b] = sbase - off0;
            cur[b] = off0;    // the slot's first position
            fill[b] = off0;   // (no tail rows yet)
        } else {
            cur[b] = kNoBucket;
            fill[b] = PB;   // no open bucket (and no tail: PB is a whole number of lines)
        }
    }
    // the tile's x-th fresh bucket
    auto fresh = [&](unsigned x) -> unsigned { return s_nb + x < s_nend ? s_nb + x : kNoBucket; };
    // fresh bucket ids come from the workgroup's own range (k_id_plan
    // sizes it for the worst case of its tiles): no global atomic.  (A
    // shared counter, even one returning atomic per 64 ids, cost 0.25-0.3 ms
    // per 2^28-row pass: waiting for its result also waited for the next
    // tile's loads, profiles/r01_micro_pass2.txt "no bucket atomic".)
    const unsigned id_end = EXACT ? 0u : a.wstart[blockIdx.x + 1];
    unsigned id_next = EXACT ? 0u : a.wstart[blockIdx.x];
    // row slot of position p (>= the line start of fill[b]) of bin b's run
    // in the current tile: the open bucket, then the tile's fresh buckets
    auto slot = [&](unsigned b, unsigned p) -> u64 {
        if constexpr (EXACT) {
            const u64 o = cbase[b] + p;
            return o < a.out_max_rows ? o : ~0ull;
        }
        const unsigned k = p >> a.out_pbl;
        const unsigned bk = k == 0 ? cur[b] : fresh(nbase[b] + k - 1);
        return bk < a.max_buckets ? ((u64)bk << a.out_pbl) + (p & (PB - 1)) : ~0ull;
    };
    int seg_cur = -1;
    // close this workgroup's open buckets: write each tail (the bucket's
    // last, partial line); their fill is final
    auto close_all = [&]() {
        if constexpr (EXACT) {   // the slots' last, partial lines
            for (unsigned q = threadIdx.x; q < F * (L - 1); q += kPassThreads) {
                const unsigned b = q / (L - 1), i = q - b * (L - 1);
                const unsigned f = fill[b], tl = f & (L - 1);
                const unsigned p = f - tl + i;
                if (i < tl && p >= cur[b] && cbase[b] + p < a.out_max_rows) out[cbase[b] + p] = tail[q];
            }
            return;
        }
        for (unsigned b = threadIdx.x; b < F; b += kPassThreads) {
            const unsigned f = fill[b], tl = f & (L - 1);
            if (cur[b] != kNoBucket && cur[b] < a.max_buckets) {
                for (unsigned i = 0; i < tl; ++i) out[((u64)cur[b] << a.out_pbl) + (f - tl + i)] = tail[b * (L - 1) + i];
                a.bfill[cur[b]] = f;
                if (a.rcnt) atomicAdd(&a.rcnt[((unsigned)seg_cur << a.fbits) | b], (u64)runs_of(f));
            }
            cur[b] = kNoBucket;
            fill[b] = PB;
        }
    };
    // rows of tile tl into registers (br = 0 valid, ~0 none)
    auto load_tile = [&](u64 tlo, T (&row)[IT], unsigned (&br)[IT]) {
        if constexpr ((ABL & 2) != 0) {
#pragma unroll
            for (int i = 0; i < IT; ++i) {
                const u64 v = tlo * 7 + (u64)i * kPassThreads + threadIdx.x;
                row[i] = R::make(fmix64(v), v);
                br[i] = 0u;
            }
        } else if constexpr (WIDE && FORM == kCols64) {
            // two consecutive rows per lane: one 16-B load from each column
            // (rows lo + 2 * (i * NT + t) + {0, 1}; order inside a tile is free)
            const u64 *kc = (const u64 *)a.in.key, *pc = (const u64 *)a.in.pay;
            if (a.cols_aligned && tlo + (u64)kTile <= a.n) {
                // a whole, aligned tile (a uniform branch): no per-lane guard,
                // so the loads are not EXEC-masked beside the guarded ones
                // below -- two masked paths writing the same registers made
                // the compiler wait vmcnt(0) (the previous tile's stores)
                // before issuing them
#pragma unroll
                for (int i = 0; i < IT / 2; ++i) {
                    const u64 r = tlo + 2ull * ((u64)i * kPassThreads + threadIdx.x);
                    const ulonglong2 k2 = ld_s<kNtPassLd>((const ulonglong2 *)(kc + r));
                    const ulonglong2 p2 = ld_s<kNtPassLd>((const ulonglong2 *)(pc + r));
                    row[2 * i] = R::make(k2.x, p2.x);
                    row[2 * i + 1] = R::make(k2.y, p2.y);
                    br[2 * i] = 0u;
                    br[2 * i + 1] = 0u;
                }
                return;
            }
#pragma unroll
            for (int i = 0; i < IT / 2; ++i) {
                const u64 r = tlo + 2ull * ((u64)i * kPassThreads + threadIdx.x);
                const bool v0 = r < a.n, v1 = r + 1 < a.n;
                if (a.cols_aligned && v1) {
                    const ulonglong2 k2 = ld_s<kNtPassLd>((const ulonglong2 *)(kc + r));
                    const ulonglong2 p2 = ld_s<kNtPassLd>((const ulonglong2 *)(pc + r));
                    row[2 * i] = R::make(k2.x, p2.x);
                    row[2 * i + 1] = R::make(k2.y, p2.y);
                } else {
                    row[2 * i] = v0 ? R::make(kc[r], pc[r]) : R::zero();
                    row[2 * i + 1] = v1 ? R::make(kc[r + 1], pc[r + 1]) : R::zero();
                }
                // (one assignment per element: stores in both branches made
                // the compiler keep br in scratch memory)
                br[2 * i] = v0 ? 0u : 0xFFFFFFFFu;
                br[2 * i + 1] = v1 ? 0u : 0xFFFFFFFFu;
            }
        } else if constexpr (FORM != kBucketed) {
#pragma unroll
            for (int i = 0; i < IT; ++i) {
                if (!tile_row<WIDE, FORM>(a, tlo, (unsigned)i * kPassThreads + threadIdx.x, row[i])) {
                    row[i] = R::zero();
                    br[i] = 0xFFFFFFFFu;
                } else {
                    br[i] = 0u;
                }
            }
        }
    };
    // FORM == kBucketed: row v of a tile is row v % 64 of the tile's run
    // v / 64 (a wave's 64 lanes read one run, <= 64 rows of one bucket, so a
    // partly filled bucket idles at most its last run's tail).  Tile t's rows
    // are loaded in iteration t - 1 from its run entries (lane j holds entry
    // j), loaded in iteration t - 2 from its descriptor, loaded in iteration
    // t - 3: each load waits only on data that was in flight for a whole
    // tile.  (Issued back to back, the chain descriptor -> entry -> row cost
    // several memory latencies per tile: 2.23 ms for pass 2 vs 1.89 ms for
    // pass 1, profiles/r01_micro_pass2.txt.)
    const unsigned lane = threadIdx.x & 63u;
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto get_desc = [&](unsigned t) -> ulonglong2 {
        return t < t1 ? *(const ulonglong2 *)&a.tdesc[t] : make_ulonglong2(0ull, 0ull);
    };
    auto get_ents = [&](const ulonglong2 &d) -> u64 {
        return lane < (unsigned)d.y && d.x + lane < a.in_max_runs ? a.in_runs[d.x + lane] : 0ull;
    };
    auto rows_from = [&](u64 ent, T (&row)[IT], unsigned (&br)[IT]) {
        const unsigned elo = (unsigned)ent, ehi = (unsigned)(ent >> 32);
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            const unsigned src = (unsigned)i * (kPassThreads >> kRunLog) + wave;   // run of this row slot
            // (readlane returns int: widen through unsigned, not sign-extended)
            const u64 e = ((u64)(unsigned)__builtin_amdgcn_readlane(ehi, src) << 32) |
                          (u64)(unsigned)__builtin_amdgcn_readlane(elo, src);
            if (lane < (unsigned)(e & 127u) && (e >> 7) + lane < a.in_max_rows) {
                row[i] = ld_s<kNtPassLd>((const T *)a.in_rows + (e >> 7) + lane);
                br[i] = 0u;
            } else {
                row[i] = R::zero();
                br[i] = 0xFFFFFFFFu;
            }
        }
    };
    auto seg_of = [&](const ulonglong2 &d) -> int { return (int)__builtin_amdgcn_readfirstlane((unsigned)(d.y >> 32)); };
    T row[IT];
    unsigned br[IT];   // bin << 16 | rank within the tile's bin
    u64 tlo = 0;    // first row of the current tile (row sources)
    int tseg = 0;   // segment of the current tile (row sources: 0)
    ulonglong2 dn = make_ulonglong2(0ull, 0ull), dn2 = dn;   // kBucketed: descriptors of tiles t + 1, t + 2
    u64 en = 0ull;                                            // kBucketed: run entries of tile t + 1
    if (t0 < t1) {
        if constexpr (FORM == kBucketed) {
            const ulonglong2 d0 = get_desc(t0);
            rows_from(get_ents(d0), row, br);
            tseg = seg_of(d0);
            dn = get_desc(t0 + 1);
            en = get_ents(dn);
            dn2 = get_desc(t0 + 2);
        } else {
            tlo = (u64)t0 * kTile;
            load_tile(tlo, row, br);
        }
    }
    // The first tile's rows arrive here, before the loop: otherwise the
    // compiler's wait counting merges "rows still loading" from this entry
    // into every iteration and waits vmcnt(0) -- i.e. for the NEXT tile's
    // loads, issued after the count -- before the scatter writes the rows to
    // the stage, which left those loads in flight during the scan only.
    __builtin_amdgcn_s_waitcnt(0);
    u64 ph[6] = {0, 0, 0, 0, 0, 0}, tp = 0;
    auto mark = [&](int k) {
        if constexpr ((ABL & 8) != 0) {
            const u64 now = __builtin_amdgcn_s_memtime();
            if (k >= 0) ph[k] += now - tp;
            tp = now;
        }
    };
    for (unsigned t = t0; t < t1; ++t) {
        mark(-1);
        if (tseg != seg_cur) {   // uniform: every thread sees the same tile
            __syncthreads();
            close_all();
            seg_cur = tseg;
            __syncthreads();
        }
        const unsigned hb = t == t0 ? 0xFFFFFFFFu : s_hot;
        if (hb == 0xFFFFFFFFu) {
#pragma unroll
            for (int i = 0; i < IT; ++i) {
                if (br[i] == 0xFFFFFFFFu) continue;
                const unsigned b = (unsigned)(rhash(R::key(row[i])) >> a.shift) & (F - 1);
                br[i] = (b << 16) | atomicAdd(&cnt[b], 1u);
            }
        } else {
            // all of the tile's atomics issue before the first return is
            // used; a wave's hot rows of all its row slots take their ranks
            // from ONE add (same-address LDS atomics serialise across waves:
            // one add per slot cost the hot segment's tiles ~2k cycles,
            // micro/skew_micro.hip)
            const unsigned lane = threadIdx.x & 63u;
            u64 hm[IT];
            unsigned hr[IT], hpre[IT], htot = 0u;
#pragma unroll
            for (int i = 0; i < IT; ++i) {
                const bool v = br[i] != 0xFFFFFFFFu;
                const unsigned b = v ? (unsigned)(rhash(R::key(row[i])) >> a.shift) & (F - 1) : 0u;
                const bool h = v && b == hb;
                hm[i] = __ballot(h);
                hpre[i] = htot;
                htot += (unsigned)__popcll(hm[i]);
                hr[i] = 0u;
                if (v && !h) hr[i] = atomicAdd(&cnt[b], 1u);
                br[i] = v ? (b << 16) | (h ? 0x8000u : 0u) : 0xFFFFFFFFu;
            }
            unsigned hbase = 0u;
            if (htot) {   // uniform
                unsigned r = 0u;
                if (lane == 0) r = atomicAdd(&cnt[hb], htot);
                hbase = (unsigned)__builtin_amdgcn_readlane((int)r, 0);
            }
#pragma unroll
            for (int i = 0; i < IT; ++i) {
                if (br[i] != 0xFFFFFFFFu && (br[i] & 0x8000u))
                    hr[i] = hbase + hpre[i] + __builtin_amdgcn_mbcnt_hi((unsigned)(hm[i] >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((unsigned)hm[i], 0u));
                if (br[i] != 0xFFFFFFFFu) br[i] = (br[i] & 0xFFFF0000u) | hr[i];
            }
        }
        __syncthreads();
        mark(0);
        // the next tile's loads are in flight from here on (through the
        // scan, the LDS scatter and this tile's stores)
        const int seg = tseg;
        T nrow[IT];
        unsigned nbr[IT];
        int nseg_t = tseg;
        const u64 ntlo = (u64)(t + 1) * kTile;
        if constexpr (FORM == kBucketed) {
            if (t + 1 < t1) {
                rows_from(en, nrow, nbr);
                nseg_t = seg_of(dn);
                dn = dn2;
                en = get_ents(dn);   // tile t + 2
                dn2 = get_desc(t + 3);
            }
        } else {
            if (t + 1 < t1) load_tile(ntlo, nrow, nbr);
        }
        if (threadIdx.x < 64) {
            // wave 0: exclusive scans of the bin counts (-> start) and of the
            // fresh buckets each bin needs (-> nbase, relative); the tile's
            // fresh buckets are the next ids of the workgroup's range
            const int lane = threadIdx.x;
            // (BPL bins per lane moved as 16-B LDS accesses per array: wave
            // 0 alone is on the critical path here)
            constexpr int BPL = FMAX / 64, Q = BPL / 4;
            unsigned c[BPL], k[BPL], ln[BPL], s = 0, sk = 0, sl = 0;
#pragma unroll
            for (int qd = 0; qd < Q; ++qd) {
                const uint4 c4 = ((const uint4 *)cnt)[lane * Q + qd];
                const uint4 f4 = ((const uint4 *)fill)[lane * Q + qd];
                const unsigned cv[4] = {c4.x, c4.y, c4.z, c4.w};
                const unsigned fv[4] = {f4.x, f4.y, f4.z, f4.w};
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int j = qd * 4 + jj;
                    c[j] = (unsigned)(lane * BPL + j) < F ? cv[jj] : 0u;
                    k[j] = (!EXACT && c[j]) ? (fv[jj] + c[j] - 1) >> a.out_pbl : 0u;
                    // complete lines: the old tail's and the new rows'
                    ln[j] = c[j] ? ((fv[jj] & (L - 1)) + c[j]) / L : 0u;
                    s += c[j];
                    sk += k[j];
                    sl += ln[j];
                }
            }
            {   // the largest bin (count << 16 | bin), for the next tile's count
                unsigned mx = 0u;
#pragma unroll
                for (int j = 0; j < BPL; ++j) {
                    const unsigned y = (c[j] << 16) | (unsigned)(lane * BPL + j);
                    mx = y > mx ? y : mx;
                }
                mx = wave_max_all(mx);
                if (lane == 0) s_hot = (mx >> 16) > (unsigned)(kTile / 8) ? (mx & 0xffffu) : 0xFFFFFFFFu;
            }
            const unsigned x = wave_incl_add(s), xk = wave_incl_add(sk), xl = wave_incl_add(sl);
            unsigned run = x - s, runk = xk - sk, runl = xl - sl;
            unsigned sv[BPL], nv[BPL], lv[BPL];
#pragma unroll
            for (int j = 0; j < BPL; ++j) {
                sv[j] = run;
                nv[j] = runk;
                lv[j] = runl;
                run += c[j];
                runk += k[j];
                runl += ln[j];
            }
            if ((unsigned)(lane * BPL) < F) {   // (entries of bins >= F are written but never read)
#pragma unroll
                for (int qd = 0; qd < Q; ++qd) {
                    ((uint4 *)start)[lane * Q + qd] = make_uint4(sv[qd * 4], sv[qd * 4 + 1], sv[qd * 4 + 2], sv[qd * 4 + 3]);
                    ((uint4 *)nbase)[lane * Q + qd] = make_uint4(nv[qd * 4], nv[qd * 4 + 1], nv[qd * 4 + 2], nv[qd * 4 + 3]);
                    ((uint4 *)lstart)[lane * Q + qd] = make_uint4(lv[qd * 4], lv[qd * 4 + 1], lv[qd * 4 + 2], lv[qd * 4 + 3]);
                }
            }
            if (lane == 63) {
                s_nl = xl;
                s_nb = id_next;
                s_nend = id_end;
                id_next = xk < id_end - id_next ? id_next + xk : id_end;
            }
        }
        __syncthreads();
        mark(1);
        // Bin b's rows now span positions [fill, fill + cnt) of its bucket
        // run; lines end below E = (fill + cnt) & ~(L - 1).  Rows below E go
        // to the stage (packed by bin), the rest become the bin's new tail
        // (kept in registers until the old tails have been read).
        unsigned tpos[IT];   // new tail index of row i, or ~0
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            tpos[i] = 0xFFFFFFFFu;
            if (br[i] == 0xFFFFFFFFu) continue;
            const unsigned b = br[i] >> 16, rk = br[i] & 0xffffu;
            const unsigned f = fill[b], p = f + rk, e = (f + cnt[b]) & ~(L - 1);
            if (p >= e) tpos[i] = b * (L - 1) + (p - e);
            else stage[start[b] + rk] = row[i];
        }
        // the line -> bin map (a bin owner per thread)
        // (this tile's largest bin, when it holds more than kTile / 8 rows
        // -- s_hot, set by the scan for the next tile's count -- is mapped by
        // the whole workgroup: one thread's serial loop over a skewed bin's
        // 256 lines cost ~3.5k cycles per tile of C4's hot segment,
        // micro/skew_micro.hip)
        const unsigned hot = s_hot;
        for (unsigned b = threadIdx.x; b < F; b += kPassThreads) {
            const unsigned c = cnt[b];
            if (!c || b == hot) continue;
            const unsigned nl = ((fill[b] & (L - 1)) + c) / L, l0 = lstart[b];
            for (unsigned x = 0; x < nl; ++x) lbin[l0 + x] = (unsigned short)b;
        }
        if (hot != 0xFFFFFFFFu) {   // (uniform)
            const unsigned nl = ((fill[hot] & (L - 1)) + cnt[hot]) / L, l0 = lstart[hot];
            for (unsigned x = threadIdx.x; x < nl; x += kPassThreads) lbin[l0 + x] = (unsigned short)hot;
        }
        __syncthreads();
        mark(2);
        if constexpr (!WIDE && !EXACT) {
            // 8-B rows: two rows per lane, one 16-B store (L / 2 lanes per
            // line, 128 / L lines per store instruction): REF-B's passes
            // 0.80 -> 0.74 ms each (16-B loads of two rows per lane were
            // tried with it and lost that again: profiles/r04_join_entries.txt)
            constexpr unsigned LH = L / 2, LPW2 = 64u / LH;
            const unsigned nl = s_nl, g = (threadIdx.x & 63u) / LH, r2 = (threadIdx.x & (LH - 1)) * 2u;
            for (unsigned l0 = wave * LPW2; l0 < nl; l0 += (unsigned)(kPassThreads / 64) * LPW2) {
                const unsigned x = l0 + g;
                if (x >= nl) continue;
                const unsigned b = lbin[x];
                const unsigned f = fill[b], tl0 = f & (L - 1);
                const unsigned off = (x - lstart[b]) * L + r2;
                const unsigned p = f - tl0 + off;
                const T v0 = off < tl0 ? tail[b * (L - 1) + off] : stage[start[b] + (off - tl0)];
                const T v1 = off + 1 < tl0 ? tail[b * (L - 1) + off + 1] : stage[start[b] + (off + 1 - tl0)];
                const u64 o = slot(b, p);
                if ((ABL & 4) == 0 && o != ~0ull) st_s<kNtPassSt>((ulonglong2 *)(out + o), make_ulonglong2(v0, v1));
            }
        } else {
            // complete lines: L lanes per line, 64 / L lines per store
            // instruction; a line's rows are the bin's old tail rows, then
            // its staged new rows
            constexpr unsigned LPW = 64u / L;
            const unsigned nl = s_nl, g = (threadIdx.x & 63u) / L, r = threadIdx.x & (L - 1);
            for (unsigned l0 = wave * LPW; l0 < nl; l0 += (unsigned)(kPassThreads / 64) * LPW) {
                const unsigned x = l0 + g;
                if (x >= nl) continue;
                const unsigned b = lbin[x];
                const unsigned f = fill[b], tl0 = f & (L - 1);
                const unsigned off = (x - lstart[b]) * L + r;
                const unsigned p = f - tl0 + off;
                if (EXACT && p < cur[b]) continue;   // (the slot before's rows)
                const T v = off < tl0 ? tail[b * (L - 1) + off] : stage[start[b] + (off - tl0)];
                const u64 o = slot(b, p);
                if ((ABL & 4) == 0 && o != ~0ull) st_s<kNtPassSt>(out + o, v);
            }
        }
        __syncthreads();
        mark(3);
#pragma unroll
        for (int i = 0; i < IT; ++i)
            if (tpos[i] != 0xFFFFFFFFu) tail[tpos[i]] = row[i];
        for (unsigned b = threadIdx.x; b < F; b += kPassThreads) {
            const unsigned c = cnt[b];
            cnt[b] = 0u;
            if (!c) continue;
            const unsigned f = fill[b];
            if constexpr (EXACT) {
                fill[b] = f + c;
                continue;
            }
            const unsigned k = (f + c - 1) >> a.out_pbl;
            if (k) {
                // the replaced open bucket is full (all its lines stored);
                // record the fresh ones, and the full ones' runs for the listing
                unsigned full = 0;
                if (cur[b] != kNoBucket && cur[b] < a.max_buckets) {
                    a.bfill[cur[b]] = PB;
                    ++full;
                }
                const unsigned pid = ((unsigned)seg << a.fbits) | b;
                for (unsigned i = 0; i < k; ++i) {
                    const unsigned bk = fresh(nbase[b] + i);
                    if (bk == kNoBucket) continue;
                    a.bbin[bk] = pid;
                    if (i + 1 < k) {
                        a.bfill[bk] = PB;
                        ++full;
                    }
                }
                if (a.rcnt && full) atomicAdd(&a.rcnt[pid], (u64)full << (a.out_pbl - kRunLog));
                cur[b] = fresh(nbase[b] + k - 1);
                fill[b] = f + c - (k << a.out_pbl);
            } else {
                fill[b] = f + c;
            }
        }
        __syncthreads();
        mark(4);
        tseg = nseg_t;
        tlo = ntlo;
#pragma unroll
        for (int i = 0; i < IT; ++i) {
            row[i] = nrow[i];
            br[i] = nbr[i];
        }
    }
    close_all();
    if constexpr (!EXACT) {
        // ids of the range left unused are holes for the bucket listing
        if (threadIdx.x == 63) s_hole = id_next;
        __syncthreads();
        for (unsigned i = s_hole + threadIdx.x; i < id_end; i += kPassThreads) a.bbin[i] = kNoBucket;
    }
    if constexpr ((ABL & 8) != 0) {
        if (threadIdx.x == 0 && a.prof)
            for (int k = 0; k < 6; ++k) a.prof[blockIdx.x * 8 + k] = ph[k];
    }
}

// Bucket id ranges of a pass's workgroups (block 0, G <= 1024): workgroup
// w gets ceil(rows_w / PB) + segs_w * F + 1 ids, rows_w <= its tiles * kTile
// and segs_w the segments its tiles span.  A bin's rows of one segment run
// fill ceil(r / PB) <= r / PB + 1 buckets (a bucket is only taken for rows),
// so the range never runs out.  *nb = the ids handed out (listing bound).
__global__ __launch_bounds__(1024) void k_id_plan(PassArgs a, bool bucketed, unsigned G, unsigned *wstart, u64 *zero_a,
                                                  u64 *zero_b, u64 zero_n) {
    __shared__ u64 wsum[16];
    // every block: zero the listing's run counts and cursors (P + 1 each)
    for (u64 i = (u64)blockIdx.x * 1024 + threadIdx.x; i < zero_n; i += (u64)gridDim.x * 1024) {
        zero_a[i] = 0ull;
        zero_b[i] = 0ull;
    }
    if (blockIdx.x != 0) return;
    const unsigned w = threadIdx.x;
    const unsigned T_ = bucketed ? a.tile_start[a.nseg] : (unsigned)((a.n + a.tile_rows - 1) / a.tile_rows);
    u64 q = 0;
    if (w < G) {
        const unsigned t0 = (unsigned)((u64)w * T_ / G), t1 = (unsigned)((u64)(w + 1) * T_ / G);
        if (t1 > t0) {
            const u64 segs = bucketed ? (u64)(a.tdesc[t1 - 1].seg - a.tdesc[t0].seg + 1) : 1ull;
            const u64 PB = 1ull << a.out_pbl;
            q = ((u64)(t1 - t0) * a.tile_rows + PB - 1) / PB + segs * (1ull << a.fbits) + 1;
        }
    }
    u64 tot;
    const u64 pre = block_excl_scan<1024>(q, wsum, &tot);
    if (w <= G) wstart[w] = (unsigned)(pre < a.max_buckets ? pre : a.max_buckets);
    if (w == G) *a.nb = (unsigned)(tot < a.max_buckets ? tot : a.max_buckets);
}

// A bucketed pass's plan in ONE launch (chunk_map + k_tile_desc + k_id_plan
// + the listing's zeroing: five launches before), for nseg <= kPlanSegs.
// Every block loads the input set's run starts (nseg + 1) and scans their
// tile counts (ceil(runs / 64)) in LDS; block 0 writes the tile starts and
// the workgroups' bucket id ranges (k_id_plan's rule), all blocks write the
// tile descriptors (grid-strided; a tile's segment by binary search over the
// starts in LDS) and zero the next listing's counters.
constexpr int kPlanSegs = 4096;
struct TilePlanArgs {
    PassArgs a;
    const u64 *rstart;
    unsigned G, tb;
    unsigned *tile_start;
    TileDesc *desc;
    unsigned *wstart;
    u64 *zero_a, *zero_b;
    u64 zero_n;
};

// (block bid of nblk: the body of k_tile_plan, or of k_place_plan's plan blocks)
__device__ __forceinline__ void tile_plan_body(const TilePlanArgs &p, unsigned bid, unsigned nblk) {
    const PassArgs &a = p.a;
    const u64 *rstart = p.rstart;
    const unsigned G = p.G, tb = p.tb;
    unsigned *tile_start = p.tile_start;
    TileDesc *desc = p.desc;
    unsigned *wstart = p.wstart;
    u64 *zero_a = p.zero_a, *zero_b = p.zero_b;
    const u64 zero_n = p.zero_n;
    __shared__ unsigned ts[kPlanSegs + 1];
    __shared__ u64 wsum[16];
    constexpr int PER = kPlanSegs / 1024;
    const int nseg = a.nseg;
    const unsigned rpt = a.tile_rows >> kRunLog;   // runs per tile
    unsigned c[PER], sum = 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int sg = threadIdx.x * PER + i;
        c[i] = sg < nseg ? (unsigned)((rstart[sg + 1] - rstart[sg] + rpt - 1) / rpt) : 0u;
        sum += c[i];
    }
    u64 total;
    u64 run = block_excl_scan<1024>(sum, wsum, &total);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int sg = threadIdx.x * PER + i;
        if (sg < nseg) ts[sg] = (unsigned)run;
        run += c[i];
    }
    if (threadIdx.x == 0) ts[nseg] = (unsigned)total;
    __syncthreads();
    const unsigned T = (unsigned)total;
    // segment of tile t: the last sg with ts[sg] <= t (ts[nseg] = T > t)
    auto seg_of_tile = [&](unsigned t) -> unsigned {
        unsigned lo = 0, hi = (unsigned)nseg;   // ts[lo] <= t < ts[hi]
        while (hi - lo > 1) {
            const unsigned mid = (lo + hi) >> 1;
            if (ts[mid] <= t) lo = mid;
            else hi = mid;
        }
        return lo;
    };
    for (unsigned t = bid * 1024 + threadIdx.x; t < T && t < tb; t += nblk * 1024) {
        const unsigned sg = seg_of_tile(t);
        const u64 lo = rstart[sg] + (u64)(t - ts[sg]) * rpt;
        const u64 e = rstart[sg + 1];
        TileDesc d;
        d.lo = lo;
        d.cnt = (unsigned)(e - lo < (u64)rpt ? e - lo : (u64)rpt);
        d.seg = sg;
        desc[t] = d;
    }
    for (u64 i = (u64)bid * 1024 + threadIdx.x; i < zero_n; i += (u64)nblk * 1024) {
        zero_a[i] = 0ull;
        zero_b[i] = 0ull;
    }
    if (bid != 0) return;
    for (int sg = threadIdx.x; sg <= nseg; sg += 1024) tile_start[sg] = ts[sg];
    const unsigned w = threadIdx.x;
    u64 q = 0;
    if (w < G) {
        const unsigned t0 = (unsigned)((u64)w * T / G), t1 = (unsigned)((u64)(w + 1) * T / G);
        if (t1 > t0) {
            const u64 segs = (u64)(seg_of_tile(t1 - 1) - seg_of_tile(t0) + 1);
            const u64 PB = 1ull << a.out_pbl;
            q = ((u64)(t1 - t0) * a.tile_rows + PB - 1) / PB + segs * (1ull << a.fbits) + 1;
        }
    }
    u64 tot;
    const u64 pre = block_excl_scan<1024>(q, wsum, &tot);
    if (w <= G) wstart[w] = (unsigned)(pre < a.max_buckets ? pre : a.max_buckets);
    if (w == G) *a.nb = (unsigned)(tot < a.max_buckets ? tot : a.max_buckets);
}

__global__ __launch_bounds__(1024) void k_tile_plan(TilePlanArgs p) { tile_plan_body(p, blockIdx.x, gridDim.x); }

// Runs by partition: the pass counted every bucket's runs per partition
// (PassArgs::rcnt), an exclusive scan (scan_one) gives the partitions'
// starts, then k_bplace places each bucket's runs at its partition's cursor.
// Blocks aggregate in LDS first when partitions are few (pass 1: 512).
// Buckets [0, *nb) of a pass, clamped to the set's capacity; holes (unused
// ids of a workgroup's range) are kNoBucket.
constexpr int kListPer = 4;   // (1, 2 per thread: within 10 %; 1 again in round 4: r04g)
constexpr int kListLds = 4096;


struct PlaceArgs {
    const unsigned *bbin, *bfill, *nb;
    unsigned max_buckets;
    int pbl;
    const u64 *rstart;
    u64 *rcur, *runs;
    int P;
    // raw run counts (P + 1 <= kRawCntWords) still to be scanned: k_place_plan
    // scans them itself into rstart (null: rstart is already scanned)
    const u64 *raw = nullptr;
};
static_assert(kRawCntWords == (u64)kPlanSegs + 1, "raw count words: a plan's segments + 1");

__device__ __forceinline__ void bplace_body(const PlaceArgs &pa, unsigned bid) {
    const unsigned *bbin = pa.bbin, *bfill = pa.bfill, *nb = pa.nb;
    const unsigned max_buckets = pa.max_buckets;
    const int pbl = pa.pbl;
    const u64 *rstart = pa.rstart;
    u64 *rcur = pa.rcur, *runs = pa.runs;
    const int P = pa.P;
    __shared__ unsigned cr[kListLds];
    __shared__ u64 cbr[kListLds];
    const unsigned n = *nb < max_buckets ? *nb : max_buckets;
    const u64 base = (u64)bid * 1024 * kListPer;
    if (base >= n) return;
    // bucket j's runs: rows (j << pbl) + 64 k, count min(64, fill - 64 k).
    // Called by the whole wave (every lane, `ok` = it holds a bucket): the
    // wave writes its buckets' runs cooperatively, R = 2^(pbl - 6) lanes per
    // bucket, so each store instruction fills 64 / R whole run ranges (one
    // 128-B line per full 1024-row bucket) instead of 64 scattered 8-B words
    const unsigned lane_ = threadIdx.x & 63u;
    auto put_runs = [&](bool ok, u64 j, unsigned f, u64 at) {
        const int rl = pbl > kRunLog ? (pbl - kRunLog < 6 ? pbl - kRunLog : 6) : 0;
        const unsigned R = 1u << rl, k0 = lane_ & (R - 1u);
        for (unsigned b0 = 0; b0 < 64u; b0 += 64u >> rl) {
            const int src = (int)(b0 + (lane_ >> rl));
            const bool o = __shfl((int)ok, src) != 0;
            const unsigned fs = (unsigned)__shfl((int)f, src);
            const u64 js = ((u64)(unsigned)__shfl((int)(j >> 32), src) << 32) | (unsigned)__shfl((int)j, src);
            const u64 as = ((u64)(unsigned)__shfl((int)(at >> 32), src) << 32) | (unsigned)__shfl((int)at, src);
            // (k0 + R m: the rest of a bucket past R runs -- pbl > 12 only)
            for (unsigned k = k0; o && (k << kRunLog) < fs; k += R) {
                const unsigned cnt = fs - (k << kRunLog) < (1u << kRunLog) ? fs - (k << kRunLog) : (1u << kRunLog);
                runs[as + k] = ((((u64)js << pbl) + ((u64)k << kRunLog)) << 7) | cnt;
            }
        }
    };
    if (P > kListLds) {
        // as k_bcount: the lanes of the wave's first partition take their
        // places from one cursor add (prefix of their run counts), the
        // others one add each; all adds issue before any result is used
        const unsigned lane = threadIdx.x & 63u;
        unsigned bi[kListPer], fi[kListPer], pre[kListPer], l0i[kListPer];
        u64 ri[kListPer];
#pragma unroll
        for (int i = 0; i < kListPer; ++i) {
            const u64 j = base + (u64)i * 1024 + threadIdx.x;
            bi[i] = j < n ? bbin[j] : kNoBucket;
            const bool valid = bi[i] < (unsigned)P;
            fi[i] = valid ? bfill[j] : 0u;
            const unsigned nr = runs_of(fi[i]);
            const u64 vm = __ballot(valid);
            l0i[i] = vm ? (unsigned)__ffsll((long long)vm) - 1u : 64u;   // uniform
            ri[i] = 0ull;
            pre[i] = 0u;
            if (!vm) continue;
            const unsigned b0 = (unsigned)__builtin_amdgcn_readlane((int)bi[i], (int)l0i[i]);
            const bool same = valid && bi[i] == b0;
            const unsigned v = same ? nr : 0u;
            const unsigned incl = wave_incl_add(v);
            const unsigned tot = (unsigned)__builtin_amdgcn_readlane((int)incl, 63);
            pre[i] = same ? incl - v : ~0u;   // ~0: not in the group
            if (valid && !same) ri[i] = atomicAdd(&rcur[bi[i]], (u64)nr);
            if (lane == l0i[i]) ri[i] = atomicAdd(&rcur[b0], (u64)tot);
        }
#pragma unroll
        for (int i = 0; i < kListPer; ++i) {
            if (l0i[i] == 64u) continue;   // uniform: no valid lane
            const unsigned b0 = (unsigned)__builtin_amdgcn_readlane((int)bi[i], (int)l0i[i]);
            const u64 g = ((u64)(unsigned)__builtin_amdgcn_readlane((int)(ri[i] >> 32), (int)l0i[i]) << 32) |
                          (u64)(unsigned)__builtin_amdgcn_readlane((int)ri[i], (int)l0i[i]);
            const bool ok = bi[i] < (unsigned)P;
            const u64 j = base + (u64)i * 1024 + threadIdx.x;
            const u64 at = !ok ? 0ull : (pre[i] != ~0u ? rstart[b0] + g + pre[i] : rstart[bi[i]] + ri[i]);
            put_runs(ok, j, fi[i], at);
        }
        return;
    }
    for (int i = threadIdx.x; i < P; i += 1024) cr[i] = 0u;
    __syncthreads();
    unsigned rr[kListPer], bn[kListPer], fl[kListPer];
#pragma unroll
    for (int i = 0; i < kListPer; ++i) {
        const u64 j = base + (u64)i * 1024 + threadIdx.x;
        bn[i] = j < n ? bbin[j] : kNoBucket;
        if (bn[i] >= (unsigned)P) bn[i] = kNoBucket;
        fl[i] = bn[i] != kNoBucket ? bfill[j] : 0u;
        if (bn[i] != kNoBucket) rr[i] = atomicAdd(&cr[bn[i]], runs_of(fl[i]));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += 1024)
        if (cr[i]) cbr[i] = rstart[i] + atomicAdd(&rcur[i], (u64)cr[i]);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kListPer; ++i) {
        const u64 j = base + (u64)i * 1024 + threadIdx.x;
        const bool ok = bn[i] != kNoBucket;
        put_runs(ok, j, fl[i], ok ? cbr[bn[i]] + rr[i] : 0ull);
    }
}

__global__ __launch_bounds__(1024) void k_bplace(PlaceArgs pa) { bplace_body(pa, blockIdx.x); }

// One launch for two independent steps that both only need the scanned run
// starts of pass p: pass p's run placement (blocks [0, nplace)) and pass p +
// 1's plan (the rest).  (They use separate bucket-count words and cursor
// arrays: the plan zeroes pass p + 1's while pass p's are in use.)
// pa.raw: every block scans the previous pass's raw run counts (<= kPlanSegs
// + 1 of them) into LDS and both bodies read the starts from there; block 0
// also writes them to pa.rstart for the kernels after this one.  (This is
// the scan launch the listing of a small pass had of its own.)
__global__ __launch_bounds__(1024) void k_place_plan(PlaceArgs pa, unsigned nplace, TilePlanArgs tp) {
    __shared__ u64 rs[kPlanSegs + 1];
    if (pa.raw) {
        __shared__ u64 wsum[16];
        constexpr int PER = (kPlanSegs + 1 + 1023) / 1024;
        const int n = pa.P + 1;
        u64 v[PER], sum = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x * PER + i;
            v[i] = e < n ? pa.raw[e] : 0ull;
            sum += v[i];
        }
        u64 total;
        u64 run = block_excl_scan<1024>(sum, wsum, &total);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x * PER + i;
            if (e < n) {
                rs[e] = run;
                if (blockIdx.x == 0) ((u64 *)pa.rstart)[e] = run;
            }
            run += v[i];
        }
        __syncthreads();
        pa.rstart = rs;
        tp.rstart = rs;
    }
    if (blockIdx.x < nplace) bplace_body(pa, blockIdx.x);
    else tile_plan_body(tp, blockIdx.x - nplace, gridDim.x - nplace);
}

// --------------------------------------------------------------- join
struct JoinArgs {
    const void *r, *s;               // final-pass bucket rows
    const u64 *r_runs, *s_runs;      // runs by partition (row << 7 | count)
    const u64 *r_rstart, *s_rstart;  // P + 1 each
    int P;
    const unsigned *work_start;      // P + 1: S chunks per partition (0 if no R rows)
    const struct ItemDesc *desc;     // per work item (k_item_desc)
    int tshift;                      // LDS slot = (hash >> tshift) & (slots - 1)
    void *out_r, *out_s;
    long long cap;
    u64 *counter;
    u64 *dup_flag;                   // set to 1 if any partition's build rows repeat a key
    // k_join_u appends the items it leaves (repeated / INT64_MIN build keys,
    // build side over one round) to defer[0 .. *defer_n); k_join in list
    // mode (list != nullptr) joins exactly those items
    unsigned *defer = nullptr, *defer_n = nullptr;
    const unsigned *list = nullptr, *list_n = nullptr;
    // build-time sample of the build side (k_rsample): {rows, rows whose key
    // repeated}; modes: bit m = this launch runs when sample_mode() == m
    const u64 *sample = nullptr;
    unsigned modes = 7u;
    // k_join_b (i32 rows): items past a workgroup's first two are handed out
    // by this counter (zeroed by k_item_desc) instead of w += grid, so
    // workgroups that drew heavy items (a hot key's chunks) take fewer
    unsigned *next_item = nullptr;
    // k_join (radix_detect): build only -- every item's S chunk is empty
    bool empty_s = false;
    // a LIST launch that takes EVERY item instead when the build-time sample
    // says most build keys repeat (mode 2): the kernel the fast launch
    // before it left to it (k_join for int64 rows, k_join_grp for i32 rows),
    // so that launch and the mode-2 one are one launch (no exit-only launch)
    bool all_if_mode2 = false;
    // k_join: exit at once when *skip_if_set != 0 (radix_detect's self-join)
    const u64 *skip_if_set = nullptr;
};

constexpr unsigned kModeUnique = 1u, kModeSome = 2u, kModeMostlyRepeated = 4u;
constexpr unsigned kModesAll = kModeUnique | kModeSome | kModeMostlyRepeated;
constexpr int kSampleParts = 64;   // build partitions sampled (one workgroup each)

// Scalar (s_load) reads of wave-uniform words that no kernel writes while
// the join runs: through the constant address space.  Plain pointers here
// compile to vector loads whose results the allocator spilled, and each
// spill's vmcnt(0) then waited for every row load in flight.
typedef __attribute__((address_space(4))) const u64 cu64_t;
__device__ __forceinline__ u64 sload(const u64 *p) { return *(cu64_t *)p; }

// 0: build keys (sampled) unique, 1: some repeat (>= 1/64 of the sampled
// rows: C1-ref's uniform keys, ~3 %), 2: most repeat (> 1/4: REF-A's ~100
// copies per key).  Deterministic: a function of exact counts.
__host__ __device__ __forceinline__ int sample_mode(u64 rows, u64 repeats) {
    return repeats * 4 > rows ? 2 : (repeats * 64 >= rows && repeats ? 1 : 0);
}
__device__ __forceinline__ bool join_runs(const JoinArgs &a) {
    const int m = a.sample ? sample_mode(sload(a.sample), sload(a.sample + 1)) : 0;
    return (a.modes >> m) & 1u;
}
// a LIST kernel's item source: the list, or every item (all_if_mode2 and a
// mode-2 sample)
__device__ __forceinline__ bool join_uses_list(const JoinArgs &a) {
    return !(a.all_if_mode2 && a.sample && sample_mode(sload(a.sample), sload(a.sample + 1)) == 2);
}

// Build-side sample, launched after R's partition (radix_sample): workgroup
// i takes partition i * P / nsamp, inserts up to kCap of its keys into an LDS
// set and counts the rows whose key was already there.  sample[0] += rows
// inserted, sample[1] += repeats (sample zeroed by the caller).
template <bool WIDE>
__global__ __launch_bounds__(1024) void k_rsample(const void *rows, const u64 *runs, const u64 *rstart, int P,
                                                  unsigned nsamp, u64 *sample) {
    constexpr int TS = 8192;
    constexpr unsigned kCap = TS / 2;
    constexpr u64 kE = ~0ull;   // (a wide key of all ones is skipped: not sampled)
    __shared__ u64 set[TS];
    __shared__ unsigned s_n, s_rep;
    const int p = (int)(((u64)blockIdx.x * (u64)P) / nsamp);
    for (int j = threadIdx.x; j < TS; j += 1024) set[j] = kE;
    if (threadIdx.x == 0) s_n = s_rep = 0u;
    __syncthreads();
    const u64 lo = rstart[p], hi = rstart[p + 1];
    const unsigned off = threadIdx.x & 63u;
    unsigned rep = 0;
    for (u64 li = lo + (threadIdx.x >> 6); li < hi; li += 16) {
        const u64 e = runs[li];
        if (off >= (unsigned)(e & 127u)) continue;
        const u64 row = (e >> 7) + off;
        const u64 key = WIDE ? ((const ulonglong2 *)rows)[row].x : (((const u64 *)rows)[row] >> 32);
        if (key == kE || atomicAdd(&s_n, 1u) >= kCap) continue;
        unsigned h = (unsigned)((key * 0xD6E8FEB86659FD93ull) >> 51);
        while (true) {
            const u64 old = atomicCAS(&set[h], kE, key);
            if (old == kE) break;
            if (old == key) {
                ++rep;
                break;
            }
            h = (h + 1u) & (TS - 1u);
        }
    }
    if (rep) atomicAdd(&s_rep, rep);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned n = s_n < kCap ? s_n : kCap;
        if (n) atomicAdd(sample, (u64)n);
        if (s_rep) atomicAdd(sample + 1, (u64)s_rep);
    }
}

struct ItemDesc {
    u64 s_lo, s_hi, r_lo, r_hi;      // run positions of the item's S chunk / the partition's R
};

// One descriptor per work item, so the join reads its item with one
// (scalar) load instead of the owner -> partition -> offsets chain.
// Items of partitions with >= 2 chunks (a skewed key's: heavy) come first,
// then the one-chunk items, each group in partition order (split scan of
// k_chunk_count: heavy chunks before partition p in the high half).  The
// join kernels stride items w = wg, wg + grid, ...: heavy items then spread
// evenly over the workgroups instead of landing where their partitions fall
// (C4 Zipf: join 2.89 -> 2.71 ms, profiles/r03_heavy_first.txt; int64 rows only).
__global__ __launch_bounds__(256) void k_item_desc(const unsigned *work_start, const unsigned *work_owner,
                                                   const u64 *s_rstart, const u64 *r_rstart, int P, unsigned chr,
                                                   ItemDesc *desc, unsigned *zero, unsigned *zero2, unsigned *zero3,
                                                   const u64 *split, u64 *zero_count) {
    const unsigned w = blockIdx.x * 256 + threadIdx.x;
    if (w == 0 && zero_count) *zero_count = 0ull;   // the join's output counter (no memset launch)
    if (w == 0 && zero) *zero = 0u;
    if (w == 0 && zero2) *zero2 = 0u;
    if (w == 0 && zero3) *zero3 = 0u;
    if (w >= work_start[P]) return;
    const int p = (int)work_owner[w];
    const unsigned c = w - work_start[p];
    ItemDesc d;
    d.s_lo = s_rstart[p] + (u64)c * chr;
    const u64 e = s_rstart[p + 1];
    d.s_hi = d.s_lo + chr < e ? d.s_lo + chr : e;
    d.r_lo = r_rstart[p];
    d.r_hi = r_rstart[p + 1];
    unsigned at = w;
    if (split) {
        const unsigned hp = (unsigned)(split[p] >> 32);
        at = work_start[p + 1] - work_start[p] >= 2 ? hp + c
                                                    : (unsigned)(split[P] >> 32) + (work_start[p] - hp);
    }
    desc[at] = d;
}

// A persistent workgroup of NT threads walks work items w = wg, wg + grid, ...
// Work item = (partition, chunk of up to kJoinSub * NT * SI / 64 S runs):
// build the partition's R runs into a 2^TSL-slot LDS table (rounds of
// RCAP / 64 runs for oversized partitions), then probe the chunk in
// sub-chunks of NT * SI / 64 runs.
// ABL (diagnostics only, micro/join_micro.hip; the product uses 0) switches
// phases off: 1 no cursor atomic, 2 no output writes, 4 no probe, 8 no build,
// 16 probe reads the first slot only.
// WPS: minimum waves per SIMD (4: <= 128 VGPRs, 2 workgroups of 512 per CU;
// 2: <= 256 VGPRs).  RCAPX: build rows per round (0: 5/8 of the slots).
// LIST: the items of a.list (what the fast kernels deferred) instead of all.
template <bool WIDE, bool WRITE, int TSL, int NT, int ABL = 0, int SI_ = kJoinItems, int WPS = 4, int RCAPX = 0,
          bool LIST = false>
__global__ __launch_bounds__(NT, WPS) void k_join(JoinArgs a) {
    typedef Row<WIDE> R;
    typedef typename R::T T;
    typedef typename std::conditional<WIDE, u64, unsigned>::type PT;   // output element
    constexpr int TS = 1 << TSL;
    constexpr unsigned kMask = TS - 1;
    constexpr int SI = SI_;                   // S rows per thread per sub-chunk
    constexpr int RCAP = RCAPX ? RCAPX : TS * 5 / 8;   // build rows per round (load factor <= 0.625)
    constexpr int RI = RCAP / NT;             // build rows per thread per round
    constexpr int SUBR = NT * SI;             // rows per sub-chunk
    constexpr unsigned rb = (unsigned)RCAP >> kRunLog;       // runs per build round
    constexpr unsigned subb = (unsigned)SUBR >> kRunLog;     // runs per sub-chunk
    constexpr unsigned chb = (unsigned)kJoinSub * subb;      // runs per work item
    static_assert((rb << kRunLog) == RCAP && (subb << kRunLog) == SUBR, "rounds must be whole runs");
    // A round loads RI rows per thread (runs lo + i * NW + wave) but steps
    // the run cursor by rb: rows past RI * NT in a round would never be
    // built.  Round 5's dropped int64 shape (512 threads over 2048 slots:
    // RCAP 1280, RI 2 -> 1024 rows loaded per 1280 stepped) lost one build
    // row in five in every deferred partition -- 16,986 of 20,942 pairs on a
    // 1-bit plan.
    static_assert(RI * NT == RCAP, "a build round must load exactly RCAP rows");
    // wide: EMPTY key INT64_MIN (rows with that key take the null path);
    // narrow: the all-ones word (row ids < 2^31 never produce it)
    constexpr u64 kEmpty = WIDE ? kEmptyKey64 : ~0ull;
    __shared__ u64 tkey[TS];                  // wide: keys; narrow: packed rows
    __shared__ u64 tpay[WIDE ? TS : 1];
    __shared__ u64 wsum[16];
    __shared__ u64 s_base;
    __shared__ unsigned s_dup;
    constexpr int NW = NT / 64;
    __shared__ unsigned s_cw[SI * NW];        // per (row slot, wave) match counts, then offsets

    const bool use_list = LIST && join_uses_list(a);
    const unsigned total = use_list ? *a.list_n : a.work_start[a.P];
    unsigned w = blockIdx.x;
    if (w >= total) return;
    // (radix_detect's self-join of the deferred partitions: nothing to
    // answer once a repeat is known -- and a hot key's copies would walk
    // each other's chains, ~m^2 steps)
    if (a.skip_if_set && __hip_atomic_load(a.skip_if_set, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const T *rrows = (const T *)a.r;
    const T *srows = (const T *)a.s;
    PT *orr = (PT *)a.out_r;
    PT *oss = (PT *)a.out_s;
    auto item = [&](unsigned x) {
        ItemDesc d = use_list ? a.desc[a.list[x]] : a.desc[x];
        if (a.empty_s) d.s_hi = d.s_lo;
        return d;
    };

    // Row slot i of wave v is run lo + i * NW + v, lane l its row l: the
    // run entry is wave-uniform (scalar loads into SGPRs) and can be
    // fetched one item ahead without costing VGPRs; a partly filled bucket
    // idles at most the tail of its last run.
    constexpr unsigned G = NT >> kRunLog;
    const unsigned wv0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> kRunLog);
    const unsigned off = threadIdx.x & ((1u << kRunLog) - 1u);
    // run entries (row << 7 | count; 0 = none) of positions [lo, min(lo + n*G, hi))
    auto ents = [&](const u64 *list, u64 lo, u64 hi, u64 *e, int n) {
#pragma unroll
        for (int i = 0; i < n; ++i) {
            const u64 li = lo + (u64)i * G + wv0;
            e[i] = li < hi ? list[li] : 0ull;
        }
    };
    auto rows_of = [&](const T *rows, const u64 *e, T *v, int n) {
        unsigned ok = 0;
#pragma unroll
        for (int i = 0; i < n; ++i) {
            if (off < (unsigned)(e[i] & 127u)) {
                v[i] = ld_s<kNtJoinLd>(rows + (e[i] >> 7) + off);
                ok |= 1u << i;
            } else {
                v[i] = R::zero();
            }
        }
        return ok;
    };
    T sv_[SI], rv_[RI];
    unsigned rok = 0, sok = 0;   // bit i: rv_[i] / sv_[i] holds a row
    u64 er[RI], es[SI];
    bool dup_sent = false;   // this workgroup has set a.dup_flag
    ItemDesc it = item(w);
    ents(a.r_runs, it.r_lo, it.r_lo + rb < it.r_hi ? it.r_lo + rb : it.r_hi, er, RI);
    ents(a.s_runs, it.s_lo, it.s_lo + subb < it.s_hi ? it.s_lo + subb : it.s_hi, es, SI);
    ItemDesc nx = item(w + gridDim.x < total ? w + gridDim.x : w);
    auto load_r = [&](u64 r0) {
        ents(a.r_runs, r0, r0 + rb < it.r_hi ? r0 + rb : it.r_hi, er, RI);
        return rows_of(rrows, er, rv_, RI);
    };
    auto load_s = [&](u64 s0) {
        ents(a.s_runs, s0, s0 + subb < it.s_hi ? s0 + subb : it.s_hi, es, SI);
        return rows_of(srows, es, sv_, SI);
    };
    while (true) {
        // this item's first R round and first S sub-chunk: issued before the
        // table init so their latency hides behind it.  (Prefetching the next
        // item's R rows instead costs VGPRs -> spills at 4 waves per SIMD, and
        // measured slower: profiles/r01_micro_join_buckets.txt,
        // profiles/r02_join_prefetch.txt.)
        rok = rows_of(rrows, er, rv_, RI);
        sok = rows_of(srows, es, sv_, SI);
        const bool more = w + gridDim.x < total;
        u64 ner[RI], nes[SI];
        ItemDesc nnx = nx;
        if (more) {
            ents(a.r_runs, nx.r_lo, nx.r_lo + rb < nx.r_hi ? nx.r_lo + rb : nx.r_hi, ner, RI);
            ents(a.s_runs, nx.s_lo, nx.s_lo + subb < nx.s_hi ? nx.s_lo + subb : nx.s_hi, nes, SI);
            if (w + 2 * gridDim.x < total) nnx = item(w + 2 * gridDim.x);
        }

        u64 n_null_r = 0;
        bool any_null_s = false;
        for (u64 r0 = it.r_lo; r0 < it.r_hi; r0 += rb) {
            if (r0 != it.r_lo) rok = load_r(r0);   // later rounds (oversized partitions)
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
                const u64 key = R::key(rv_[i]);
                act[i] = (rok >> i) & 1u;
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
            // once per workgroup: every table with a repeated key storing to
            // the one flag serialised those stores at the memory side (C1-ref
            // at 2^28: +3.5 ms, micro/join_micro.hip mode 1)
            if (!unique && !dup_sent) {
                if (threadIdx.x == 0) __hip_atomic_store(a.dup_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dup_sent = true;
            }

            // ---- probe the chunk, one sub-chunk of S rows at a time
            for (u64 sb = it.s_lo; sb < it.s_hi; sb += subb) {
                if (sb != it.s_lo || r0 != it.r_lo) sok = load_s(sb);
                // first slot of every row read before any is resolved (SI
                // independent LDS reads in flight); most rows end there
                unsigned m[SI], hp[SI];
                u64 e0[SI];
                bool pa[SI];
                u64 cnt = 0;
                unsigned mb = 0u;   // general path, wide rows: bit i = row slot i has a match
#pragma unroll
                for (int i = 0; i < SI; ++i) {
                    m[i] = 0xFFFFFFFFu;
                    const u64 key = R::key(sv_[i]);
                    pa[i] = (sok >> i) & 1u;
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
                if (unique) {
                    // duplicate-free build: a row's chain ends at its match
                    // or at EMPTY -- a two-exit loop with nothing else in it
                    // (the general loop below costs ~3x per step)
                    // Row slots walk in pairs: one loop advances both chains,
                    // two LDS reads in flight per step, and the wave waits
                    // for the longest chain of each pair instead of each slot
                    auto open = [&](u64 e, u64 key) { return e != kEmpty && (WIDE ? e : (e >> 32)) != key; };
#pragma unroll
                    for (int i = 0; i < SI; i += 2) {
                        const int j = i + 1 < SI ? i + 1 : i;
                        const u64 ka = R::key(sv_[i]), kb = R::key(sv_[j]);
                        unsigned ha = hp[i], hb = hp[j];
                        u64 ea = e0[i], eb = e0[j];
                        bool la = pa[i] && open(ea, ka);
                        bool lb = j != i && pa[j] && open(eb, kb);
                        while (la || lb) {
                            if constexpr ((ABL & 16) != 0) break;
                            if (la) {
                                ha = (ha + 1) & kMask;
                                ea = tkey[ha];
                            }
                            if (lb) {
                                hb = (hb + 1) & kMask;
                                eb = tkey[hb];
                            }
                            la = la && open(ea, ka);
                            lb = lb && open(eb, kb);
                        }
                        if (pa[i] && ea != kEmpty && (WIDE ? ea : (ea >> 32)) == ka) {
                            ++cnt;
                            m[i] = ha;
                        }
                        if (j != i && pa[j] && eb != kEmpty && (WIDE ? eb : (eb >> 32)) == kb) {
                            ++cnt;
                            m[j] = hb;
                        }
                    }
                } else {
                    // every chain walks to EMPTY (a key may repeat); row
                    // slots in pairs as above
                    // (narrow rows: m[i] counts row slot i's matches on this
                    // path, for the cooperative writes below; wide rows keep
                    // one bit each in mb -- five live counts spilled there)
                    auto hit = [&](u64 e, u64 key) { return (WIDE ? e : (e >> 32)) == key; };
                    if constexpr (!WIDE) {
#pragma unroll
                        for (int i = 0; i < SI; ++i) m[i] = 0u;
                    }
#pragma unroll
                    for (int i = 0; i < SI; i += 2) {
                        const int j = i + 1 < SI ? i + 1 : i;
                        const u64 ka = R::key(sv_[i]), kb = R::key(sv_[j]);
                        unsigned ha = hp[i], hb = hp[j];
                        u64 ea = e0[i], eb = e0[j];
                        bool la = pa[i] && ea != kEmpty;
                        bool lb = j != i && pa[j] && eb != kEmpty;
                        while (la || lb) {
                            if (la) {
                                if (hit(ea, ka)) {
                                    ++cnt;
                                    if constexpr (WIDE) mb |= 1u << i;
                                    else ++m[i];
                                }
                                ha = (ha + 1) & kMask;
                                ea = tkey[ha];
                            }
                            if (lb) {
                                if (hit(eb, kb)) {
                                    ++cnt;
                                    if constexpr (WIDE) mb |= 1u << j;
                                    else ++m[j];
                                }
                                hb = (hb + 1) & kMask;
                                eb = tkey[hb];
                            }
                            if constexpr ((ABL & 16) != 0) break;
                            la = la && ea != kEmpty;
                            lb = lb && eb != kEmpty;
                        }
                    }
                }
                if (WRITE && unique) {
                    // <= 1 match per row: ballot compaction in row-slot-major
                    // order, so lanes with a match store to consecutive
                    // addresses (one coalesced run per wave and slot)
                    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
                    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
                    unsigned lpre[SI];
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const u64 bal = __ballot(m[i] != 0xFFFFFFFFu);
                        lpre[i] = (unsigned)__popcll(bal & lt);
                        if (lane == 0) s_cw[i * NW + wv] = (unsigned)__popcll(bal);
                    }
                    __syncthreads();
                    if (wv == 0) {   // exclusive scan of the SI * NW run lengths
                        constexpr int K = (SI * NW + 63) / 64;
                        unsigned v[K], sum = 0;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int j = lane * K + k;
                            v[k] = j < SI * NW ? s_cw[j] : 0u;
                            sum += v[k];
                        }
                        const unsigned x = wave_incl_add(sum);
                        unsigned run = x - sum;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int j = lane * K + k;
                            if (j < SI * NW) s_cw[j] = run;
                            run += v[k];
                        }
                        if (lane == 63 && x)
                            s_base = (ABL & 1) ? (u64)w * chb << kRunLog : atomicAdd(a.counter, (u64)x);
                    }
                    __syncthreads();
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        if constexpr ((ABL & 2) != 0) break;
                        if (m[i] == 0xFFFFFFFFu) continue;
                        const u64 pos = s_base + s_cw[i * NW + wv] + lpre[i];
                        if (pos < (u64)a.cap) {
                            st_s<kNtJoinSt>(orr + pos, WIDE ? (PT)tpay[m[i]] : (PT)(tkey[m[i]] & 0xffffffffull));
                            st_s<kNtJoinSt>(oss + pos, (PT)R::pay(sv_[i]));
                        }
                    }
                    __syncthreads();   // s_cw / s_base reused by the next sub-chunk
                    continue;
                }
                u64 tot;
                const u64 pre = block_excl_scan<NT>(cnt, wsum, &tot);
                if constexpr (!WRITE) {
                    if (threadIdx.x == 0 && tot) atomicAdd(a.counter, tot);
                } else if (tot) {
                    if (threadIdx.x == 0) s_base = (ABL & 1) ? (u64)w * chb << kRunLog : atomicAdd(a.counter, tot);
                    __syncthreads();
                    u64 pos = s_base + pre;
                    // (narrow rows only: in the wide kernel the extra state cost
                    // the duplicate-free path a scratch spill)
                    if (!WIDE && !unique && tot > (u64)(2 * SUBR)) {
                        // many matches per probe row (the reference's 10M x 10M
                        // keys in [1, 100k] workload: ~100 each): a lane's own
                        // pairs would go out as one partial line per lane and
                        // store.  Instead the wave takes its rows one at a time
                        // and scans the row's chain 64 slots per step, one slot
                        // per lane; matching lanes write consecutive positions.
                        // Rows go lane by lane (a lane's rows own consecutive
                        // positions, thread-major), so the wave's stores advance
                        // through one region and every line is completed by the
                        // next row's stores while it is still in L2 (slot by
                        // slot, the wave kept 64 regions open, ~800 KB per CU,
                        // and lines left L2 half written: REF-A join 3.3 ms).
                        const unsigned lane = threadIdx.x & 63u;
                        const u64 lt = lane ? (~0ull >> (64u - lane)) : 0ull;
                        for (int l = 0; l < 64; ++l) {
                            if constexpr ((ABL & 2) != 0) break;
                            u64 p = ((u64)(unsigned)__builtin_amdgcn_readlane((int)(pos >> 32), l) << 32) |
                                    (u64)(unsigned)__builtin_amdgcn_readlane((int)pos, l);
#pragma unroll
                            for (int i = 0; i < SI; ++i) {
                                if (__builtin_amdgcn_readlane((int)m[i], l) == 0) continue;   // uniform
                                const u64 key_i = R::key(sv_[i]);
                                const u64 pay_i = (u64)R::pay(sv_[i]);
                                const u64 k = ((u64)(unsigned)__builtin_amdgcn_readlane((int)(key_i >> 32), l) << 32) |
                                              (u64)(unsigned)__builtin_amdgcn_readlane((int)key_i, l);
                                const PT sp_ = (PT)(((u64)(unsigned)__builtin_amdgcn_readlane((int)(pay_i >> 32), l) << 32) |
                                                    (u64)(unsigned)__builtin_amdgcn_readlane((int)pay_i, l));
                                unsigned h = (unsigned)(rhash(k) >> a.tshift) & kMask;
                                while (true) {
                                    const unsigned hs = (h + lane) & kMask;
                                    const u64 e = tkey[hs];
                                    const u64 emp = __ballot(e == kEmpty);
                                    const unsigned lim = emp ? (unsigned)__ffsll((long long)emp) - 1u : 64u;
                                    const bool hitm = lane < lim && (WIDE ? e : (e >> 32)) == k;
                                    const u64 mm = __ballot(hitm);
                                    if (hitm) {
                                        const u64 q = p + (u64)__popcll(mm & lt);
                                        if (q < (u64)a.cap) {
                                            orr[q] = WIDE ? (PT)tpay[hs] : (PT)(e & 0xffffffffull);
                                            oss[q] = sp_;
                                        }
                                    }
                                    p += (u64)__popcll(mm);
                                    if (emp) break;
                                    h = (h + 64u) & kMask;
                                }
                            }
                        }
                        __syncthreads();   // s_base reused by the next sub-chunk
                        continue;
                    }
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
                            const u64 key = R::key(sv_[i]);
                            // rows without a match skip the second walk (with
                            // duplicate keys most probes still miss: C1-ref)
                            if (WIDE ? !((mb >> i) & 1u) : !m[i]) continue;
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
                for (u64 sb = it.s_lo; sb < it.s_hi; sb += subb) {
                    sok = load_s(sb);
                    u64 cnt = 0;
#pragma unroll
                    for (int i = 0; i < SI; ++i)
                        if (((sok >> i) & 1u) && R::key(sv_[i]) == kEmptyKey64) cnt += nn;
                    u64 tot;
                    const u64 pre = block_excl_scan<NT>(cnt, wsum, &tot);
                    if constexpr (!WRITE) {
                        if (threadIdx.x == 0 && tot) atomicAdd(a.counter, tot);
                    } else if (tot) {
                        if (threadIdx.x == 0) s_base = atomicAdd(a.counter, tot);
                        __syncthreads();
                        u64 pos = s_base + pre;
                        for (int i = 0; i < SI; ++i) {
                            if (!(((sok >> i) & 1u) && R::key(sv_[i]) == kEmptyKey64)) continue;
                            for (u64 li = it.r_lo; li < it.r_hi; ++li) {
                                const u64 le = a.r_runs[li];
                                for (unsigned o = 0; o < (unsigned)(le & 127u); ++o) {
                                    const T rr = rrows[(le >> 7) + o];
                                    if (R::key(rr) != kEmptyKey64) continue;
                                    if (pos < (u64)a.cap) {
                                        orr[pos] = (PT)R::pay(rr);
                                        oss[pos] = (PT)R::pay(sv_[i]);
                                    }
                                    ++pos;
                                }
                            }
                        }
                        __syncthreads();
                    }
                }
            }
        }

        if (!more) break;
        w += gridDim.x;
        it = nx;
        nx = nnx;
#pragma unroll
        for (int i = 0; i < RI; ++i) er[i] = ner[i];
#pragma unroll
        for (int i = 0; i < SI; ++i) es[i] = nes[i];
    }
}

// --------------------------------------------------------------- join, fast path
// k_join_u: the join of items whose partition holds no INT64_MIN build key
// and at most rmax runs (load factor <= 0.75) -- every item of the PK-FK
// and uniform-key configs.  Against k_join it drops the null pass, the
// oversized-partition rounds that re-probe S, the paired duplicate walk
// and the wave-cooperative writes, so it needs ~80 instead of ~127 VGPRs
// and runs 768-thread workgroups at 6 waves per SIMD (k_join: 4).  An item
// it cannot take is appended to a.defer (one atomic per such item, before
// any of its pairs is written) and k_join joins the list afterwards.
// Run entries, table, duplicate-free probe walk, ballot-compacted output
// and the ONE cursor atomic per sub-chunk are as in k_join; a partition
// with a repeated build key (GEN) takes a plain per-row walk to EMPTY.
__device__ __forceinline__ ItemDesc sload(const ItemDesc *p) {
    const u64 *q = (const u64 *)p;
    return ItemDesc{sload(q), sload(q + 1), sload(q + 2), sload(q + 3)};
}

// ABL (micro/join3_micro.hip ablations only; 0 in the product): bit 0 no
// output cursor atomic (a per-item position instead), bit 1 no output
// stores, bit 2 no probe walks, bit 3 no build inserts, bit 4 no build
// collision walks, bit 5 no payload stores into the table (an interleaved
// form of the collision walks, every row's CAS in flight at once, measured
// slower: C3 join 2.75 -> 2.99 ms; so was a walk reading the aligned slot
// pair ahead and CASing only an EMPTY slot: narrow 1.85 -> 2.25 ms)
template <bool WIDE, int TSL, int NT, int SI>
struct JoinUSmem {
    u64 tkey[1 << TSL];
    u64 tpay[WIDE ? (1 << TSL) : 1];
    u64 s_base;
    unsigned s_bad, s_dup, s_rows;
    unsigned s_cw[SI * (NT / 64)];
    u64 wsum[16];
};

template <bool WIDE, bool WRITE, int TSL, int NT, int RI, int SI, int WPS, bool GEN = true, int ABL = 0>
__device__ __forceinline__ void join_u_body(JoinArgs a, JoinUSmem<WIDE, TSL, NT, SI> &sm) {
    typedef Row<WIDE> R;
    typedef typename R::T T;
    typedef typename std::conditional<WIDE, u64, unsigned>::type PT;
    constexpr int TS = 1 << TSL;
    constexpr unsigned kMask = TS - 1;
    constexpr int NW = NT / 64;
    constexpr unsigned rb = (unsigned)(NW * RI);    // runs per build round (RI per wave)
    constexpr unsigned subb = (unsigned)(NW * SI);  // runs per sub-chunk
    // A partition's runs may be partly filled (a small build side partitioned
    // by many workgroups: C2's 2^20 rows, ~32-50 runs of ~2048 rows), so the
    // table takes up to TS / 64 runs (<= TS rows: every insert walk ends) and
    // the item is deferred when the rows counted during the build exceed
    // rmax_rows (load factor 0.75).
    constexpr unsigned rmax = (unsigned)TS >> kRunLog;
    constexpr unsigned rmax_rows = (unsigned)(TS * 3 / 4);
    static_assert(NT % 64 == 0 && rb <= rmax, "one round must fit the table");
    constexpr u64 kEmpty = WIDE ? kEmptyKey64 : ~0ull;
    auto &tkey = sm.tkey;
    auto &tpay = sm.tpay;
    auto &s_base = sm.s_base;
    auto &s_bad = sm.s_bad;
    auto &s_dup = sm.s_dup;
    auto &s_rows = sm.s_rows;
    auto &s_cw = sm.s_cw;
    auto &wsum = sm.wsum;
    bool dup_sent = false;   // this workgroup has set a.dup_flag

    const unsigned total = __builtin_amdgcn_readfirstlane(a.work_start[a.P]);
    unsigned w = blockIdx.x;
    if (w >= total || !join_runs(a)) return;
    const T *rrows = (const T *)a.r;
    const T *srows = (const T *)a.s;
    PT *orr = (PT *)a.out_r;
    PT *oss = (PT *)a.out_s;
    const unsigned wv0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> kRunLog);
    const unsigned off = threadIdx.x & ((1u << kRunLog) - 1u);
    const int lane = threadIdx.x & 63;
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    auto ents = [&](const u64 *list, u64 lo, u64 hi, u64 *e, int n) {
#pragma unroll
        for (int i = 0; i < n; ++i) {
            const u64 li = lo + (u64)i * NW + wv0;
            e[i] = li < hi ? sload(list + li) : 0ull;
        }
    };
    // Every lane loads (a lane past its run's end re-reads the run's first
    // row; no run: row 0), so the loads are straight-line code and the build
    // waits for the R rows only (vmcnt(SI)), not for the S rows behind them.
    auto rows_of = [&](const T *rows, const u64 *e, T *v, int n) {
        unsigned ok = 0;
#pragma unroll
        for (int i = 0; i < n; ++i) {
            const bool in = off < (unsigned)(e[i] & 127u);
            v[i] = ld_s<kNtJoinLd>(rows + (e[i] >> 7) + (in ? off : 0u));
            ok |= (unsigned)in << i;
        }
        return ok;
    };
    T sv_[SI], rv_[RI];
    u64 er[RI], es[SI];
    ItemDesc it = sload(a.desc + w);
    ents(a.r_runs, it.r_lo, it.r_hi, er, RI);
    ents(a.s_runs, it.s_lo, it.s_lo + subb < it.s_hi ? it.s_lo + subb : it.s_hi, es, SI);
    while (true) {
        const bool fits = it.r_hi - it.r_lo <= (u64)rmax;   // uniform
        unsigned rok = 0, sok = 0;
        if (fits) {
            rok = rows_of(rrows, er, rv_, RI);
            sok = rows_of(srows, es, sv_, SI);
        }
        // the next item's descriptor and run entries (scalar loads): their
        // latency passes while this item's rows are in flight
        const bool more = w + gridDim.x < total;
        u64 ner[RI], nes[SI];
        ItemDesc nx = it;
        if (more) {
            nx = sload(a.desc + w + gridDim.x);
            ents(a.r_runs, nx.r_lo, nx.r_hi, ner, RI);
            ents(a.s_runs, nx.s_lo, nx.s_lo + subb < nx.s_hi ? nx.s_lo + subb : nx.s_hi, nes, SI);
        }
        if (!fits) {
            if (threadIdx.x == 0) a.defer[atomicAdd(a.defer_n, 1u)] = w;
        } else {
            for (int j = threadIdx.x; j < TS / 2; j += NT) ((ulonglong2 *)tkey)[j] = make_ulonglong2(kEmpty, kEmpty);
            if (threadIdx.x == 0) s_bad = s_dup = s_rows = 0u;
            __syncthreads();
            // ---- build: every row's first CAS issued before any result is
            // used; a partition of more than rb runs (up to rmax) takes more
            // rounds into the same table
            bool bad = false;
            unsigned ndup = 0;   // this thread's rows whose CAS walk met their own key
            for (u64 r0 = it.r_lo;;) {
            unsigned hb[RI];
            u64 ob[RI], vb[RI];
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                const u64 key = R::key(rv_[i]);
                bool act = ((rok >> i) & 1u) && !(ABL & 8);
                if (WIDE && act && key == kEmptyKey64) {   // the null pass lives in k_join
                    bad = true;
                    act = false;
                }
                hb[i] = (unsigned)(rhash(key) >> a.tshift) & kMask;
                if constexpr (WIDE) vb[i] = key;
                else vb[i] = rv_[i];
                ob[i] = act ? atomicCAS(&tkey[hb[i]], kEmpty, vb[i]) : kEmpty;
                if (!act) rok &= ~(1u << i);
            }
            {   // the round's inserted rows, counted per wave (ballots: no VGPRs)
                unsigned wn = 0;
#pragma unroll
                for (int i = 0; i < RI; ++i) wn += (unsigned)__popcll(__ballot((rok >> i) & 1u));
                // the wave whose rows push the table past rmax_rows defers the item
                if (lane == 0 && wn && atomicAdd(&s_rows, wn) + wn > rmax_rows) s_bad = 1u;
            }
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                if (!((rok >> i) & 1u)) continue;
                const u64 key = R::key(rv_[i]);
                unsigned h = hb[i];
                u64 old = ob[i];
                bool d = false;
                while (!(ABL & 16) && old != kEmpty) {
                    d |= WIDE ? (old == key) : ((old >> 32) == key);
                    h = (h + 1) & kMask;
                    old = atomicCAS(&tkey[h], kEmpty, vb[i]);
                }
                ndup += d ? 1u : 0u;
                if constexpr (WIDE && !(ABL & 32)) tpay[h] = R::pay(rv_[i]);
            }
            r0 += rb;
            if (r0 >= it.r_hi) break;
            ents(a.r_runs, r0, it.r_hi, er, RI);
            rok = rows_of(rrows, er, rv_, RI);
            }
            if (bad || (!GEN && ndup)) s_bad = 1u;
            if (ndup) atomicAdd(&s_dup, ndup);
            __syncthreads();
            const unsigned nd = s_dup;
            const bool unique = nd == 0u;
            // i32 rows whose keys mostly repeat (the reference's 10M x 10M keys
            // in [1, 100k]: ~100 copies each) produce many pairs per probe row:
            // k_join's wave-cooperative writes take them, before any probe
            const bool defer_it = s_bad ||
                                  (!WIDE && WRITE && (u64)nd * 4u > (it.r_hi - it.r_lo) << kRunLog);
            if (!unique && !dup_sent) {   // once per workgroup (k_join)
                if (threadIdx.x == 0) __hip_atomic_store(a.dup_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dup_sent = true;
            }
            if (defer_it) {
                if (threadIdx.x == 0) a.defer[atomicAdd(a.defer_n, 1u)] = w;
            } else {
                // ---- probe the chunk, one sub-chunk of S rows at a time
                for (u64 sb = it.s_lo; sb < it.s_hi; sb += subb) {
                    if (sb != it.s_lo) {
                        ents(a.s_runs, sb, sb + subb < it.s_hi ? sb + subb : it.s_hi, es, SI);
                        sok = rows_of(srows, es, sv_, SI);
                    }
                    // an INT64_MIN probe key matches nothing here: the
                    // partition has no null build row (else deferred)
                    unsigned pm = 0u;   // bit i: row slot i probes
#pragma unroll
                    for (int i = 0; i < SI; ++i)
                        if (((sok >> i) & 1u) && !(WIDE && R::key(sv_[i]) == kEmptyKey64) && !(ABL & 4)) pm |= 1u << i;
                    if (GEN && !unique) {
                        // a repeated build key: every row walks its chain to
                        // EMPTY, counting, then again writing at its prefix
                        unsigned cnt = 0, mb = 0u;   // mb bit i: row slot i has a match
#pragma unroll
                        for (int i = 0; i < SI; ++i) {
                            if (!((pm >> i) & 1u)) continue;
                            const u64 key = R::key(sv_[i]);
                            unsigned h = (unsigned)(rhash(key) >> a.tshift) & kMask;
                            u64 e = tkey[h];
                            const unsigned c0 = cnt;
                            while (e != kEmpty) {
                                if ((WIDE ? e : (e >> 32)) == key) ++cnt;
                                h = (h + 1) & kMask;
                                e = tkey[h];
                            }
                            if (cnt != c0) mb |= 1u << i;
                        }
                        u64 tot;
                        const u64 pre = block_excl_scan<NT>((u64)cnt, wsum, &tot);
                        if (!WIDE && WRITE && sb == it.s_lo && tot > (u64)(2 * NT * SI)) {
                            // many pairs per probe row (the reference's 10M x 10M
                            // keys in [1, 100k]): one lane per row would store
                            // one partial line per pair; k_join's wave-cooperative
                            // writes take the item (nothing of it written yet)
                            if (threadIdx.x == 0) a.defer[atomicAdd(a.defer_n, 1u)] = w;
                            break;
                        }
                        if constexpr (!WRITE) {
                            if (threadIdx.x == 0 && tot) atomicAdd(a.counter, tot);
                        } else if (tot) {
                            if (threadIdx.x == 0) s_base = atomicAdd(a.counter, tot);
                            __syncthreads();
                            u64 pos = s_base + pre;
#pragma unroll
                            for (int i = 0; i < SI; ++i) {
                                if (!((mb >> i) & 1u)) continue;
                                const u64 key = R::key(sv_[i]);
                                const PT spay = (PT)R::pay(sv_[i]);
                                unsigned h = (unsigned)(rhash(key) >> a.tshift) & kMask;
                                u64 e = tkey[h];
                                while (e != kEmpty) {
                                    if ((WIDE ? e : (e >> 32)) == key) {
                                        if (pos < (u64)a.cap) {
                                            orr[pos] = WIDE ? (PT)tpay[h] : (PT)(e & 0xffffffffull);
                                            oss[pos] = spay;
                                        }
                                        ++pos;
                                    }
                                    h = (h + 1) & kMask;
                                    e = tkey[h];
                                }
                            }
                        }
                        __syncthreads();   // s_base reused by the next sub-chunk
                        continue;
                    }
                    // first slot of every row read before any is resolved
                    unsigned m[SI], hp[SI];
                    u64 e0[SI];
                    bool pa[SI];
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        m[i] = 0xFFFFFFFFu;
                        pa[i] = (pm >> i) & 1u;
                        hp[i] = (unsigned)(rhash(R::key(sv_[i])) >> a.tshift) & kMask;
                        e0[i] = pa[i] ? tkey[hp[i]] : kEmpty;
                    }
                    auto open = [&](u64 e, u64 key) { return e != kEmpty && (WIDE ? e : (e >> 32)) != key; };
#pragma unroll
                    for (int i = 0; i < SI; i += 2) {
                        const int j = i + 1 < SI ? i + 1 : i;
                        const u64 ka = R::key(sv_[i]), kb = R::key(sv_[j]);
                        unsigned ha = hp[i], hb2 = hp[j];
                        u64 ea = e0[i], eb = e0[j];
                        bool la = pa[i] && open(ea, ka);
                        bool lb = j != i && pa[j] && open(eb, kb);
                        while (la || lb) {
                            if (la) {
                                ha = (ha + 1) & kMask;
                                ea = tkey[ha];
                            }
                            if (lb) {
                                hb2 = (hb2 + 1) & kMask;
                                eb = tkey[hb2];
                            }
                            la = la && open(ea, ka);
                            lb = lb && open(eb, kb);
                        }
                        if (pa[i] && ea != kEmpty && (WIDE ? ea : (ea >> 32)) == ka) m[i] = ha;
                        if (j != i && pa[j] && eb != kEmpty && (WIDE ? eb : (eb >> 32)) == kb) m[j] = hb2;
                    }
                    // <= 1 match per row: ballot compaction in row-slot-major
                    // order (one coalesced run per wave and slot)
                    const int wv = threadIdx.x >> 6;
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const u64 bal = __ballot(m[i] != 0xFFFFFFFFu);
                        if (lane == 0) s_cw[i * NW + wv] = (unsigned)__popcll(bal);
                    }
                    __syncthreads();
                    if (wv == 0) {   // exclusive scan of the SI * NW run lengths
                        constexpr int K = (SI * NW + 63) / 64;
                        unsigned v[K], sum = 0;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int jj = lane * K + k;
                            v[k] = jj < SI * NW ? s_cw[jj] : 0u;
                            sum += v[k];
                        }
                        const unsigned x = wave_incl_add(sum);
                        unsigned run = x - sum;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int jj = lane * K + k;
                            if (jj < SI * NW) s_cw[jj] = run;
                            run += v[k];
                        }
                        if (lane == 63 && x) {
                            if constexpr (ABL & 1) s_base = ((u64)w << 11) % (u64)(a.cap > 8192 ? a.cap - 8192 : 1);
                            else if constexpr (WRITE) s_base = atomicAdd(a.counter, (u64)x);
                            else atomicAdd(a.counter, (u64)x);
                        }
                    }
                    if constexpr (WRITE && !(ABL & 2)) {
                        __syncthreads();
#pragma unroll
                        for (int i = 0; i < SI; ++i) {
                            // the lane's rank among the wave's matches of row slot i
                            // (ballot again rather than keep SI ranks live across the barrier)
                            const u64 bal = __ballot(m[i] != 0xFFFFFFFFu);
                            if (m[i] == 0xFFFFFFFFu) continue;
                            const u64 pos = s_base + s_cw[i * NW + wv] + (unsigned)__popcll(bal & lt);
                            if (pos < (u64)a.cap) {
                                st_s<kNtJoinSt>(orr + pos, WIDE ? (PT)tpay[m[i]] : (PT)(tkey[m[i]] & 0xffffffffull));
                                st_s<kNtJoinSt>(oss + pos, (PT)R::pay(sv_[i]));
                            }
                        }
                    }
                    // s_cw / s_base reused by the next sub-chunk (after the
                    // last one, the table barrier below covers them)
                    if (sb + subb < it.s_hi) __syncthreads();
                }
            }
            __syncthreads();   // table reused by the next item
        }
        if (!more) break;
        w += gridDim.x;
        it = nx;
#pragma unroll
        for (int i = 0; i < RI; ++i) er[i] = ner[i];
#pragma unroll
        for (int i = 0; i < SI; ++i) es[i] = nes[i];
    }
}

template <bool WIDE, bool WRITE, int TSL, int NT, int RI, int SI, int WPS, bool GEN = true, int ABL = 0>
__global__ __launch_bounds__(NT, WPS) void k_join_u(JoinArgs a) {
    __shared__ JoinUSmem<WIDE, TSL, NT, SI> sm;
    join_u_body<WIDE, WRITE, TSL, NT, RI, SI, WPS, GEN, ABL>(a, sm);
}

// k_join_b: k_join_u's item loop, loads, defer rules and output compaction
// over a BUCKETED LDS table (4 slots per bucket, 1024 buckets, a count per
// bucket) instead of linear probing -- wide rows, the fast shape
// (profiles/r02_join_cost_structure.txt: k_join_u's CAS walks and probe
// chains are most of its time).
//   build  = one returning LDS add on the home bucket's count per row (rank
//            < 4: the slot; else the next bucket, and so on -- rare at load
//            0.5), then plain stores of key and payload; no EMPTY marker,
//            no table fill (the counts say which slots are live)
//            A row that finds its home bucket full ORs its key's overflow bit
//            (1 of 16, from hash bits below the bucket's) into the home
//            bucket's word before walking on.
//   probe  = the home bucket's word and its 4 keys (two 16-B reads), all
//            rows' reads in flight together: the first match and the number
//            of matching slots there.  Only a key whose overflow bit is set
//            in its home word can have copies further on; those rows walk the
//            rest of the chain (on while a bucket's count exceeds 4: a row
//            passed it), counting.  A row with more than one matching slot is
//            a multi row: its pairs go out by a chain walk.
// Repeated build keys thus cost nothing when no probe row meets one: no
// build-time repeat check (the suspect walks the kernel ran until round 3
// cost C3 0.2 ms, C1-ref 0.26 ms: the walks sat between the build barrier
// and the first ballot barrier).  The context's "build keys repeat" flag is
// set by a probe row that met a repeated key; the exact answer for build
// keys no probe row met comes from DETECT (hj_ctx_build_has_duplicates, on
// demand): the same build, with every row ORing a 1-of-32 signature of its
// key into its home bucket's signature word (returning LDS or); a row that
// finds its bit already set is a suspect and looks for another live slot
// holding its key along its chain.  Exact: of c copies of a key all but the
// first to OR its bit are suspects and each finds a twin.
// A bucket's count keeps growing as rows pass it (<= 4096 < 2^16).  The
// i32 rows keep keys and row ids apart (a bucket's keys are one 16-B read);
// an item whose probe rows would write many pairs per row (the reference's
// keys in [1, 100k]) goes to k_join_grp before anything of it is written.
// the int64 rows' fast join shape (see "join shapes" below)
constexpr int kFastNTc = 768, kFastRIc = 3, kFastSIc = 3, kFastWPSc = 6;
#ifndef HJ_WIDE_DYN
#define HJ_WIDE_DYN 1   // int64 rows claim items from a counter (0: static w += grid, for A/B)
#endif

template <bool WIDE, int NT, int SI, bool DETECT, int TSL>
struct JoinBSmem {
    static constexpr int TS = 1 << TSL, NB = TS / 4, NW = NT / 64;
    static constexpr unsigned kSusCap = 512;
    // int64 rows: bucket words and control words double-buffered (an item
    // clears the next item's set: no clear barrier); i32 rows' 64-KiB table
    // leaves no room for a second set at two workgroups per CU
    static constexpr bool DBL = WIDE && !DETECT;
    alignas(16) u64 tkey[TS];
    alignas(16) u64 tpay[WIDE ? TS : 2];
    alignas(16) unsigned bcnt[NB];
    alignas(16) unsigned bcnt2[DBL ? NB : 4];
    alignas(16) unsigned s_ctl2[4];
    alignas(16) unsigned bsig[DETECT ? NB : 4];
    unsigned sus[DETECT ? kSusCap : 1];
    u64 s_base;
    alignas(16) unsigned s_ctl[4];
    unsigned s_cw[SI * NW + NW];
    unsigned s_skip;
    unsigned s_mpre[NT];
    unsigned s_next;
};

template <bool WIDE, bool WRITE, int NT, int RI, int SI, int WPS, bool DETECT = false, int TSL = 12>
__device__ __forceinline__ void join_b_body(JoinArgs a, JoinBSmem<WIDE, NT, SI, DETECT, TSL> &sm) {
    typedef Row<WIDE> R;
    typedef typename R::T T;
    typedef typename std::conditional<WIDE, u64, unsigned>::type PT;
    constexpr int TS = 1 << TSL;   // table slots (a.tshift is set for TSL hash bits)
    constexpr int BW = 4;
    constexpr int NB = TS / BW;
    constexpr unsigned kBMask = NB - 1;
    constexpr int NW = NT / 64;
    constexpr unsigned rb = (unsigned)(NW * RI);
    constexpr unsigned subb = (unsigned)(NW * SI);
    constexpr unsigned rmax = (unsigned)TS >> kRunLog;
    constexpr unsigned rmax_rows = (unsigned)(TS * 3 / 4);
    static_assert(NT % 64 == 0 && rb <= rmax, "one round must fit the table");
    constexpr unsigned kNone = 0xFFFFFFFFu, kMulti = 0xFFFFFFFEu;
    // a bucket's word: its count (rows stored in it or passed it, <= 4096) in
    // the low half, the overflow bits of the keys stored past it in the high
    constexpr unsigned kCntMask = 0xFFFFu;
    auto &tkey = sm.tkey;
    auto &tpay = sm.tpay;
    unsigned *bcnt = sm.bcnt;   // this item's bucket words (DBL: flips per table built)
    // (DETECT) per home bucket the OR of its rows' 1-of-32 key signatures,
    // and the suspect slots: slot | home bucket << 16
    constexpr unsigned kSusCap = JoinBSmem<WIDE, NT, SI, DETECT, TSL>::kSusCap;
    auto &bsig = sm.bsig;
    auto &sus = sm.sus;
    auto &s_base = sm.s_base;
    // [0] bad (defer the item), [1] dup (a repeated build key met), [2] rows
    // in the table, [3] suspects (DETECT): one 16-B clear; DBL: flips with bcnt
    unsigned *s_ctl = sm.s_ctl;
    constexpr bool DBL = JoinBSmem<WIDE, NT, SI, DETECT, TSL>::DBL;
    // per (row slot, wave) ballot counts, then per wave the multi rows' pairs
    auto &s_cw = sm.s_cw;
    auto &s_skip = sm.s_skip;   // i32 rows: the item goes to k_join_grp (many pairs per probe row)
    auto &s_mpre = sm.s_mpre;   // a thread's multi pairs before it in its wave (kept out of registers)
    // a.next_item (DETECT walks w += grid): iteration k claims the item of
    // iteration k + 2 at its top and stores it into s_next after its build
    // barrier, and the top of iteration k + 1 reads it (a workgroup's first two items are static: blockIdx.x,
    // blockIdx.x + grid).  int64 rows claim since round 5: the double-buffered
    // words took the clear barrier and 4 VGPRs off the kernel, and the claim
    // no longer spills (round 3: 20 B, C3 -6 %); C3 join 2.46 -> 2.30 ms, C4
    // 2.82 -> 2.45 (profiles/r05/r05y_wdyn_alt.jsonl: skewed items no longer
    // pile up on the workgroups a static stride gave them to)
    auto &s_next = sm.s_next;
    bool dup_sent = false;

    const unsigned total = __builtin_amdgcn_readfirstlane(a.work_start[a.P]);
    unsigned w = blockIdx.x;
    if (w >= total || !join_runs(a)) return;
    const T *rrows = (const T *)a.r;
    const T *srows = (const T *)a.s;
    PT *orr = (PT *)a.out_r;
    PT *oss = (PT *)a.out_s;
    // the 10 hash bits above the LDS slot's low 2 (a.tshift is set for 12 bits)
    const unsigned bsh = a.tshift + 2u;
    const unsigned fsh = a.tshift - 5u;   // (a.tshift >= 28: 64 - <= 24 partition bits - 12)
    auto bucket = [&](u64 key) { return (unsigned)(rhash(key) >> bsh) & kBMask; };
    // i32 rows: the table's 32 KiB hold the keys (tkn) and, apart, the row
    // ids (tidn): a bucket's 4 keys are one 16-B read
    unsigned *const tkn = (unsigned *)tkey;
    unsigned *const tidn = tkn + TS;
    auto key_at = [&](unsigned slot) -> u64 { return WIDE ? tkey[slot] : (u64)tkn[slot]; };
    auto pay_at = [&](unsigned slot) -> PT { return WIDE ? (PT)tpay[slot] : (PT)tidn[slot]; };
    const unsigned wv0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> kRunLog);
    const unsigned off = threadIdx.x & ((1u << kRunLog) - 1u);
    const int lane = threadIdx.x & 63;
    const u64 lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    // i32 rows: the wave's n consecutive entries [lo + wv0 * n, + n) as they
    // are (adjacent scalar loads, merged into one: strided conditional ones
    // each waited for the one before; a list has kRunPad readable entries
    // past any hi); returns how many are the list's -- rows_of drops the
    // others, so no instruction uses a loaded word before the rows are wanted
    auto ents = [&](const u64 *list, u64 lo, u64 hi, u64 *e, int n) -> unsigned {
        if constexpr (WIDE) {
            // entries lo + i * NW + wv0 (the wide shape measured 1-3 % slower
            // with the narrow one's contiguous entries: profiles/r04_join_entries.txt)
#pragma unroll
            for (int i = 0; i < n; ++i) {
                const u64 li = lo + (u64)i * NW + wv0;
                e[i] = li < hi ? sload(list + li) : 0ull;
            }
            return (unsigned)n;
        }
        const u64 b0 = lo + (u64)wv0 * n;
        const u64 bl = b0 < hi ? b0 : 0ull;
#pragma unroll
        for (int i = 0; i < n; ++i) e[i] = sload(list + bl + i);
        return b0 < hi ? (hi - b0 < (u64)n ? (unsigned)(hi - b0) : (unsigned)n) : 0u;
    };
    auto rows_of = [&](const T *rows, const u64 *e0, unsigned nv, T *v, int n) {
        unsigned ok = 0;
        u64 e[RI > SI ? RI : SI];
#pragma unroll
        for (int i = 0; i < n; ++i) e[i] = (unsigned)i < nv ? e0[i] : 0ull;
#pragma unroll
        for (int i = 0; i < n; ++i) {
            const bool in = off < (unsigned)(e[i] & 127u);
            v[i] = ld_s<kNtJoinLd>(rows + (e[i] >> 7) + (in ? off : 0u));
            ok |= (unsigned)in << i;
        }
        return ok;
    };
    // (a key's overflow bit: 1 of the 16 high bits of its home bucket's word)
    auto ovf_bit = [&](u64 key) { return 1u << (16u + ((unsigned)(rhash(key) >> fsh) & 15u)); };
    // live keys of bucket b: its count (capped at BW) and its 4 slots; returns
    // the bucket's word (its overflow bits)
    auto read_bucket = [&](unsigned b, unsigned &c, u64 *k4) {
        const unsigned raw = bcnt[b];
        c = raw & kCntMask;
        if constexpr (WIDE) {
            const ulonglong2 q0 = ((const ulonglong2 *)tkey)[b * 2], q1 = ((const ulonglong2 *)tkey)[b * 2 + 1];
            k4[0] = q0.x;
            k4[1] = q0.y;
            k4[2] = q1.x;
            k4[3] = q1.y;
        } else {
            const uint4 q = ((const uint4 *)tkn)[b];
            k4[0] = q.x;
            k4[1] = q.y;
            k4[2] = q.z;
            k4[3] = q.w;
        }
        return raw;
    };
    T sv_[SI], rv_[RI];
    u64 er[RI], es[SI];
    ItemDesc it = sload(a.desc + w);
    unsigned nvr = ents(a.r_runs, it.r_lo, it.r_hi, er, RI), nvs = 0;
    // (DETECT reads no probe rows)
    if (!DETECT) nvs = ents(a.s_runs, it.s_lo, it.s_lo + subb < it.s_hi ? it.s_lo + subb : it.s_hi, es, SI);
    constexpr bool dyn = !DETECT && (!WIDE || HJ_WIDE_DYN);
    if (dyn) {
        if (threadIdx.x == 0) s_next = w + gridDim.x;
        __syncthreads();
    }
    if constexpr (DBL) {
        // the first table's words (each later table's are cleared by the item
        // before it)
        for (unsigned j = threadIdx.x; j < (unsigned)NB; j += NT) bcnt[j] = 0u;
        if (threadIdx.x < 4) s_ctl[threadIdx.x] = 0u;
        __syncthreads();
    }
    while (true) {
        const bool fits = it.r_hi - it.r_lo <= (u64)rmax;
        unsigned rok = 0, sok = 0;
        if (fits) {
            rok = rows_of(rrows, er, nvr, rv_, RI);
            if (!DETECT) sok = rows_of(srows, es, nvs, sv_, SI);
        }
        const unsigned wn = dyn ? __builtin_amdgcn_readfirstlane(s_next) : w + gridDim.x;
        const bool more = wn < total;
        // the claim of the item after next, issued now and stored into s_next
        // after the build barrier (every thread has read s_next by then): its
        // return is waited for only there, once the build has covered its
        // latency (stored right after the claim, wave 0 waited for it -- and,
        // vector memory counts retiring in order, for the S rows just
        // issued -- before it could start its share of the build)
        unsigned claim = 0u;
        if (dyn && threadIdx.x == 0) claim = atomicAdd(a.next_item, 1u);
        u64 ner[RI], nes[SI];
        unsigned nnvr = 0, nnvs = 0;
        ItemDesc nx = it;
        if (more) {
            nx = sload(a.desc + wn);
            nnvr = ents(a.r_runs, nx.r_lo, nx.r_hi, ner, RI);
            if (!DETECT) nnvs = ents(a.s_runs, nx.s_lo, nx.s_lo + subb < nx.s_hi ? nx.s_lo + subb : nx.s_hi, nes, SI);
        }
        if (!fits) {
            // (DETECT: to k_join's list-mode build, which flags repeats)
            if (threadIdx.x == 0) a.defer[atomicAdd(a.defer_n, 1u)] = w;
            if (dyn) {   // (every thread has read s_next above; the claim is read next iteration)
                __syncthreads();
                if (threadIdx.x == 0) s_next = 2u * gridDim.x + claim;
                __syncthreads();
            }
        } else {
            // (zeros from the item's descriptor -- r_lo < 2^63 -- or the
            // compiler keeps a constant zero quad live across the loop and
            // spills it)
            const unsigned z = (unsigned)(it.r_lo >> 63);
            const uint4 z4 = make_uint4(z, z, z, z);
            // (thread 0 clears the control words: it is also the one that
            // reads the previous item's dup word after the item's last barrier)
            static_assert(NB / 4 <= NT, "one 16-B clear per thread: bucket words");
            // (the index carries z too: a loop-invariant clear address was
            // hoisted out of the item loop and spilled)
            const unsigned ci = threadIdx.x + z;
            if constexpr (DBL) {
                // the NEXT table's words (this one's were cleared by the item
                // before, or before the loop): no barrier here
                unsigned *const nb_ = bcnt == sm.bcnt ? sm.bcnt2 : sm.bcnt;
                if (ci < NB / 4) ((uint4 *)nb_)[ci] = z4;
                if (threadIdx.x == 0) *(uint4 *)(s_ctl == sm.s_ctl ? sm.s_ctl2 : sm.s_ctl) = z4;
            } else {
                if (ci < NB / 4) ((uint4 *)bcnt)[ci] = z4;
                if (DETECT)
                    for (unsigned j = ci; j < NB / 4; j += NT) ((uint4 *)bsig)[j] = z4;
                if (threadIdx.x == 0) *(uint4 *)s_ctl = z4;
                __syncthreads();
            }
            // ---- build: every row's rank add issued before any is used
            bool bad = false;
            for (u64 r0 = it.r_lo;;) {
                unsigned bb[RI], rk[RI], susm = 0u;   // (DETECT) susm bit i: row i's signature bit was set
#pragma unroll
                for (int i = 0; i < RI; ++i) {
                    const u64 key = R::key(rv_[i]);
                    bool act = (rok >> i) & 1u;
                    if (WIDE && act && key == kEmptyKey64) {   // the null pass lives in k_join
                        bad = true;
                        act = false;
                    }
                    const u64 hh = rhash(key);
                    bb[i] = (unsigned)(hh >> bsh) & kBMask;
                    rk[i] = act ? atomicAdd(&bcnt[bb[i]], 1u) & kCntMask : 0u;
                    if constexpr (DETECT) {
                        const unsigned fp = 1u << ((unsigned)(hh >> fsh) & 31u);
                        if (act && (atomicOr(&bsig[bb[i]], fp) & fp)) susm |= 1u << i;
                    }
                    if (!act) rok &= ~(1u << i);
                }
                {
                    unsigned wn = 0;
#pragma unroll
                    for (int i = 0; i < RI; ++i) wn += (unsigned)__popcll(__ballot((rok >> i) & 1u));
                    if (lane == 0 && wn && atomicAdd(&s_ctl[2], wn) + wn > rmax_rows) s_ctl[0] = 1u;
                }
#pragma unroll
                for (int i = 0; i < RI; ++i) {
                    if (!((rok >> i) & 1u)) continue;
                    const unsigned home = bb[i];
                    // a row stored past its home bucket leaves its key's
                    // overflow bit there: the probe walks on past a home bucket
                    // only for a key whose bit is set
                    if (!DETECT && rk[i] >= (unsigned)BW) atomicOr(&bcnt[home], ovf_bit(R::key(rv_[i])));
                    // a full bucket: the next one (the table never fills:
                    // <= rmax_rows rows, else the item is deferred and a
                    // full table's walk is cut at NB buckets)
                    for (unsigned g = 0; rk[i] >= (unsigned)BW && g < (unsigned)NB; ++g) {
                        bb[i] = (bb[i] + 1u) & kBMask;
                        rk[i] = atomicAdd(&bcnt[bb[i]], 1u) & kCntMask;
                    }
                    if (rk[i] >= (unsigned)BW) {   // (only past rmax_rows: deferred)
                        s_ctl[0] = 1u;
                        continue;
                    }
                    const unsigned slot = bb[i] * BW + rk[i];
                    if constexpr (WIDE) {
                        tkey[slot] = R::key(rv_[i]);
                        tpay[slot] = R::pay(rv_[i]);
                    } else {
                        tkn[slot] = (unsigned)R::key(rv_[i]);
                        tidn[slot] = (unsigned)R::pay(rv_[i]);
                    }
                    if (DETECT && ((susm >> i) & 1u)) {
                        const unsigned q = atomicAdd(&s_ctl[3], 1u);
                        if (q < kSusCap) sus[q] = slot | home << 16;
                    }
                }
                r0 += rb;
                if (r0 >= it.r_hi) break;
                nvr = ents(a.r_runs, r0, it.r_hi, er, RI);
                rok = rows_of(rrows, er, nvr, rv_, RI);
            }
            if (bad) s_ctl[0] = 1u;
            __syncthreads();
            if (dyn && threadIdx.x == 0) s_next = 2u * gridDim.x + claim;
            if (s_ctl[0]) {
                // (DETECT: as well -- to k_join's list-mode build)
                if (threadIdx.x == 0) a.defer[atomicAdd(a.defer_n, 1u)] = w;
            } else if constexpr (DETECT) {
                // ---- the exact "build keys repeat" answer: each suspect walks
                // its chain (home bucket, then on while a bucket's count says a
                // row passed it) for another live slot holding its key.  Of c
                // copies of a key all but the first to OR its signature bit are
                // suspects and each finds a twin; a suspect without a twin is a
                // signature collision.
                // (more suspects than sus[] holds: every live slot checks)
                bool twin = false;
                const unsigned nsus = s_ctl[3];
                const bool all = nsus > kSusCap;
                for (unsigned q = threadIdx.x; q < (all ? (unsigned)TS : nsus) && !twin; q += NT) {
                    unsigned slot, h;
                    u64 key;
                    if (all) {
                        const unsigned lc = bcnt[q / BW] & kCntMask;
                        if (q % BW >= (lc < (unsigned)BW ? lc : (unsigned)BW)) continue;
                        slot = q;
                        key = key_at(slot);
                        h = bucket(key);
                    } else {
                        const unsigned e = sus[q];
                        slot = e & 0xFFFFu;
                        key = key_at(slot);
                        h = e >> 16;
                    }
                    for (unsigned g = 0; g < (unsigned)NB; ++g) {
                        unsigned c;
                        u64 k4[BW];
                        read_bucket(h, c, k4);
#pragma unroll
                        for (int j = 0; j < BW; ++j)
                            twin |= (unsigned)j < c && h * BW + (unsigned)j != slot && k4[j] == key;
                        if (c <= (unsigned)BW) break;
                        h = (h + 1u) & kBMask;
                    }
                }
                if (twin) s_ctl[1] = 1u;
                __syncthreads();
                if (threadIdx.x == 0 && s_ctl[1] && !dup_sent) {
                    __hip_atomic_store(a.dup_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    dup_sent = true;
                }
            } else {
            // the matches of `key` along its chain: counted, or written from pos
            auto chain = [&](u64 key, bool wr, u64 pos, PT spay) {
                unsigned h = bucket(key), cnt = 0;
                for (unsigned g = 0; g < (unsigned)NB; ++g) {
                    unsigned c;
                    u64 k4[BW];
                    read_bucket(h, c, k4);
#pragma unroll
                    for (int j = 0; j < BW; ++j) {
                        if ((unsigned)j < c && k4[j] == key) {
                            if (WRITE && wr && pos + cnt < (u64)a.cap) {
                                orr[pos + cnt] = pay_at(h * BW + j);
                                oss[pos + cnt] = spay;
                            }
                            ++cnt;
                        }
                    }
                    if (c <= (unsigned)BW) break;
                    h = (h + 1u) & kBMask;
                }
                return cnt;
            };
                for (u64 sb = it.s_lo; sb < it.s_hi; sb += subb) {
                    if (sb != it.s_lo) {
                        nvs = ents(a.s_runs, sb, sb + subb < it.s_hi ? sb + subb : it.s_hi, es, SI);
                        sok = rows_of(srows, es, nvs, sv_, SI);
                    }
                    unsigned pm = 0u;
#pragma unroll
                    for (int i = 0; i < SI; ++i)
                        if (((sok >> i) & 1u) && !(WIDE && R::key(sv_[i]) == kEmptyKey64)) pm |= 1u << i;
                    // every row's home bucket, all rows' reads in flight
                    // together: its first match there and how many slots match
                    // (cb: the bucket's count | matching slots << 16)
                    unsigned m[SI], hb[SI], cb[SI];
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        m[i] = kNone;
                        hb[i] = bucket(R::key(sv_[i]));
                        cb[i] = 0u;
                        if ((pm >> i) & 1u) {
                            u64 k4[BW];
                            const u64 key = R::key(sv_[i]);
                            unsigned c, nm = 0u;
                            const unsigned ov = read_bucket(hb[i], c, k4);
#pragma unroll
                            for (int j = BW - 1; j >= 0; --j) {
                                if ((unsigned)j < c && k4[j] == key) {
                                    m[i] = hb[i] * BW + j;
                                    ++nm;
                                }
                            }
                            // no copy of the key went past its home bucket:
                            // the home bucket held all of them
                            cb[i] = (ov & ovf_bit(key) ? c : 0u) | nm << 16;
                        }
                    }
                    // keys with a copy past the home bucket (or a collision of
                    // overflow bits): the rest of the chain -- on while a
                    // bucket's count says a row passed it
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const u64 key = R::key(sv_[i]);
                        unsigned h = hb[i], c = cb[i] & kCntMask;
                        for (unsigned g = 0; c > (unsigned)BW && g < (unsigned)NB; ++g) {
                            h = (h + 1u) & kBMask;
                            u64 k4[BW];
                            read_bucket(h, c, k4);
                            unsigned f = kNone;
#pragma unroll
                            for (int j = BW - 1; j >= 0; --j) {
                                if ((unsigned)j < c && k4[j] == key) {
                                    f = h * BW + j;
                                    cb[i] += 1u << 16;
                                }
                            }
                            if (m[i] == kNone) m[i] = f;
                        }
                    }
                    const int wv = threadIdx.x >> 6;
                    // multi rows (m = kMulti: more than one slot holds the key):
                    // all their pairs go out by a chain walk from a wave-prefix
                    // position; the others by ballot compaction
                    unsigned cntm = 0u;
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        if ((cb[i] >> 16) > 1u) {
                            m[i] = kMulti;
                            cntm += cb[i] >> 16;
                        }
                    }
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const u64 bal = __ballot(m[i] < kMulti);
                        if (lane == 0) s_cw[i * NW + wv] = (unsigned)__popcll(bal);
                    }
                    {
                        const unsigned xm = wave_incl_add(cntm);
                        if (cntm) {
                            s_mpre[threadIdx.x] = xm - cntm;
                            s_ctl[1] = 1u;
                        }
                        if (lane == 63) s_cw[SI * NW + wv] = xm;
                    }
                    __syncthreads();
                    if (wv == 0) {
                        constexpr int NE = SI * NW + NW;
                        constexpr int K = (NE + 63) / 64;
                        unsigned v[K], sum = 0, msum = 0;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int jj = lane * K + k;
                            v[k] = jj < NE ? s_cw[jj] : 0u;
                            sum += v[k];
                            msum += jj >= SI * NW ? v[k] : 0u;
                        }
                        const unsigned x = wave_incl_add(sum);
                        const unsigned mt = wave_incl_add(msum);
                        unsigned run = x - sum;
#pragma unroll
                        for (int k = 0; k < K; ++k) {
                            const int jj = lane * K + k;
                            if (jj < NE) s_cw[jj] = run;
                            run += v[k];
                        }
                        if (lane == 63) {
                            // i32 rows with many pairs per probe row (the
                            // reference's keys in [1, 100k]): the item goes to
                            // k_join_grp before anything of it is written
                            const bool skip = !WIDE && WRITE && sb == it.s_lo && mt > (unsigned)(2 * NT * SI);
                            s_skip = skip ? 1u : 0u;
                            if (skip) a.defer[atomicAdd(a.defer_n, 1u)] = w;
                            else if (x) {
                                if constexpr (WRITE) s_base = atomicAdd(a.counter, (u64)x);
                                else atomicAdd(a.counter, (u64)x);
                            }
                            // a probe row met a repeated build key: the
                            // context's repeat flag, once per workgroup (k_join)
                            if (s_ctl[1] && !dup_sent) {
                                __hip_atomic_store(a.dup_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                dup_sent = true;
                            }
                        }
                    }
                    if constexpr (WRITE) {
                        __syncthreads();
                        if (s_skip) break;
#pragma unroll
                        for (int i = 0; i < SI; ++i) {
                            const u64 bal = __ballot(m[i] < kMulti);
                            if (m[i] >= kMulti) continue;
                            const u64 pos = s_base + s_cw[i * NW + wv] + (unsigned)__popcll(bal & lt);
                            if (pos < (u64)a.cap) {
                                st_s<kNtJoinSt>(orr + pos, pay_at(m[i]));
                                st_s<kNtJoinSt>(oss + pos, (PT)R::pay(sv_[i]));
                            }
                        }
                        if (cntm) {
                            u64 pos = s_base + s_cw[SI * NW + wv] + s_mpre[threadIdx.x];
#pragma unroll
                            for (int i = 0; i < SI; ++i)
                                if (m[i] == kMulti) pos += chain(R::key(sv_[i]), true, pos, (PT)R::pay(sv_[i]));
                        }
                    }
                    if (sb + subb < it.s_hi) __syncthreads();
                }
            }
            __syncthreads();   // table reused by the next item
            if constexpr (DBL) {
                bcnt = bcnt == sm.bcnt ? sm.bcnt2 : sm.bcnt;
                s_ctl = s_ctl == sm.s_ctl ? sm.s_ctl2 : sm.s_ctl;
            }
        }
        if (!more) break;
        w = wn;
        it = nx;
        // (plain loops: with DETECT's unused S entries the unroll pragma
        // could not be honoured for its instantiation and warned)
        for (int i = 0; i < RI; ++i) er[i] = ner[i];
        nvr = nnvr;
        if constexpr (!DETECT) {
            for (int i = 0; i < SI; ++i) es[i] = nes[i];
            nvs = nnvs;
        }
    }
}

template <bool WIDE, bool WRITE, int NT, int RI, int SI, int WPS, bool DETECT = false, int TSL = 12>
__global__ __launch_bounds__(NT, WPS) void k_join_b(JoinArgs a) {
    __shared__ JoinBSmem<WIDE, NT, SI, DETECT, TSL> sm;
    join_b_body<WIDE, WRITE, NT, RI, SI, WPS, DETECT, TSL>(a, sm);
}


// --------------------------------------------------------------- grouped join
// k_join_grp: narrow rows (the reference's i32 keys / row ids) whose build
// keys repeat many times -- join-performances.md:3-6's 10M x 10M keys in
// [1, 100k], ~100 copies of every key on both sides, ~1e9 pairs.  The
// partition's build rows are GROUPED BY KEY in LDS instead of inserted into
// a linear-probing table:
//
//   gkey[TS]   key << 32 | count, one slot per distinct key (open
//              addressing, EMPTY = all ones: a count never reaches 2^32 - 1)
//   gend[TS]   the key's group start, and after the placement its end
//   grow[TS]   the build row ids, grouped by key
//
// build = one slot claim + one count add per row, a block scan of the
// counts, one placement add per row; probe = one short walk per S row to its
// key's (start, count); output = copies of the group, written lane-major
// (each wave's stores advance through one output region).  The linear-
// probing build walked every row past all earlier copies of its key (REF-A:
// 0.65 ms of CAS walks) and the probe scanned the mixed cluster 64 slots per
// step (profiles/r02_refa_join_ablation.txt).  Items of more than 63 runs
// (> TS - 64 build rows) go to a.defer (k_join's rounds take them).  LIST: the items of a.list
// (k_join_u's deferrals) instead of all.
// WIDE (int64 key / int64 payload rows, round 5): the same grouping over
// 2048 slots -- gkey holds the key (EMPTY = INT64_MIN: an item with that
// build key goes to a.defer), gcnt the counts, grow the payloads -- at two
// workgroups per CU (48 KiB of LDS each; at three the writing kernel spilled
// at 80 VGPRs); REF-A's keys as int64 rows (REF-A64) took k_join's
// linear-probing rounds 10.8 ms.
template <bool WIDE, bool WRITE, int NT, int RI, int SI, bool LIST>
__global__ __launch_bounds__(NT, 4) void k_join_grp(JoinArgs a) {
    typedef Row<WIDE> R;
    typedef typename R::T T;
    typedef typename std::conditional<WIDE, u64, unsigned>::type PT;   // payload (wide) / row id
    constexpr int TSL = WIDE ? 11 : 12, TS = 1 << TSL;
    constexpr unsigned kMask = TS - 1;
    constexpr int NW = NT / 64;
    constexpr unsigned rb = (unsigned)(NW * RI), subb = (unsigned)(NW * SI);
    // runs: <= TS - 64 rows, so >= 64 slots stay EMPTY and every walk ends
    // (64 full runs of distinct keys would fill the table, and a probe for a
    // missing key would never meet EMPTY)
    constexpr unsigned rmax = ((unsigned)TS >> kRunLog) - 1u;
    constexpr int PER = TS / NT;                         // table slots per thread in the scan
    static_assert(TS % NT == 0 && PER <= 16, "slots per thread");
    // narrow: key << 32 | count, EMPTY all ones; wide: the key, EMPTY INT64_MIN
    constexpr u64 kE = WIDE ? (u64)kEmptyKey64 : ~0ull;
    __shared__ u64 gkey[TS];
    __shared__ unsigned gend[TS];
    __shared__ unsigned gcnt[WIDE ? TS : 1];
    __shared__ PT grow[TS];
    __shared__ u64 wsum[16];
    __shared__ u64 s_base;
    __shared__ unsigned s_rep, s_bad;
    const bool use_list = LIST && join_uses_list(a);
    const unsigned total = use_list ? *a.list_n : a.work_start[a.P];
    if (!join_runs(a)) return;
    const T *rrows = (const T *)a.r;
    const T *srows = (const T *)a.s;
    PT *orr = (PT *)a.out_r;
    PT *oss = (PT *)a.out_s;
    const unsigned wv0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> kRunLog);
    const unsigned lane = threadIdx.x & 63u;
    bool dup_sent = false;
    auto ents = [&](const u64 *list, u64 lo, u64 hi, u64 *e, int n) {
#pragma unroll
        for (int i = 0; i < n; ++i) {
            const u64 li = lo + (u64)i * NW + wv0;
            e[i] = li < hi ? sload(list + li) : 0ull;
        }
    };
    auto rows_of = [&](const T *rows, const u64 *e, T *v, int n) {
        unsigned ok = 0;
#pragma unroll
        for (int i = 0; i < n; ++i) {
            const bool in = lane < (unsigned)(e[i] & 127u);
            v[i] = ld_s<kNtJoinLd>(rows + (e[i] >> 7) + (in ? lane : 0u));
            ok |= (unsigned)in << i;
        }
        return ok;
    };
    // a slot's key / count
    auto key_is = [&](u64 e, u64 key) { return WIDE ? e == key : (e >> 32) == key; };
    auto count_at = [&](unsigned h, u64 e) -> unsigned { return WIDE ? gcnt[h] : (unsigned)e; };
    // slot of `key` (claimed when absent); the walk ends: <= TS keys per item
    auto slot_of = [&](u64 key) -> unsigned {
        unsigned h = (unsigned)(rhash(key) >> a.tshift) & kMask;
        while (true) {
            u64 e = gkey[h];
            if (e == kE) {
                e = atomicCAS(&gkey[h], kE, WIDE ? key : key << 32);
                if (e == kE) return h;
            }
            if (key_is(e, key)) return h;
            h = (h + 1) & kMask;
        }
    };
    for (unsigned w = blockIdx.x; w < total; w += gridDim.x) {
        const unsigned wi = use_list ? a.list[w] : w;
        const ItemDesc it = sload(a.desc + wi);
        if (it.r_hi - it.r_lo > (u64)rmax) {   // uniform
            if (threadIdx.x == 0) a.defer[atomicAdd(a.defer_n, 1u)] = wi;
            continue;
        }
        for (int j = threadIdx.x; j < TS / 2; j += NT) ((ulonglong2 *)gkey)[j] = make_ulonglong2(kE, kE);
        if constexpr (WIDE)
            for (int j = threadIdx.x; j < TS; j += NT) gcnt[j] = 0u;
        if (threadIdx.x == 0) s_rep = s_bad = 0u;
        __syncthreads();
        // ---- count: every row claims / finds its key's slot and adds 1
        const bool one_round = it.r_hi - it.r_lo <= (u64)rb;   // uniform: rows stay in registers
        T rv[RI];
        u64 er[RI];
        unsigned rok = 0, rh[RI];
        for (u64 r0 = it.r_lo; r0 < it.r_hi; r0 += rb) {
            ents(a.r_runs, r0, r0 + rb < it.r_hi ? r0 + rb : it.r_hi, er, RI);
            rok = rows_of(rrows, er, rv, RI);
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                rh[i] = 0u;
                if (!((rok >> i) & 1u)) continue;
                if (WIDE && R::key(rv[i]) == kE) {   // the EMPTY key: k_join's null handling takes the item
                    s_bad = 1u;
                    rok &= ~(1u << i);
                    continue;
                }
                rh[i] = slot_of(R::key(rv[i]));
                if constexpr (WIDE) atomicAdd(&gcnt[rh[i]], 1u);
                else atomicAdd(&gkey[rh[i]], 1ull);
            }
        }
        __syncthreads();
        if (WIDE && s_bad) {   // uniform
            if (threadIdx.x == 0) a.defer[atomicAdd(a.defer_n, 1u)] = wi;
            __syncthreads();   // (tables reused by the next item)
            continue;
        }
        // ---- group starts: exclusive scan of the counts in slot order
        {
            unsigned c[PER], sum = 0, rep = 0;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const unsigned h = threadIdx.x * PER + j;
                const u64 e = gkey[h];
                c[j] = e == kE ? 0u : count_at(h, e);
                rep |= c[j] > 1u ? 1u : 0u;
                sum += c[j];
            }
            u64 tot;
            unsigned run = (unsigned)block_excl_scan<NT>((u64)sum, wsum, &tot);
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                gend[threadIdx.x * PER + j] = run;
                run += c[j];
            }
            if (rep) s_rep = 1u;
        }
        __syncthreads();
        if (s_rep && !dup_sent) {   // once per workgroup (k_join)
            if (threadIdx.x == 0) __hip_atomic_store(a.dup_flag, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            dup_sent = true;
        }
        // ---- placement: payloads (row ids) into their key's group
        for (u64 r0 = it.r_lo; r0 < it.r_hi; r0 += rb) {
            if (!one_round) {
                ents(a.r_runs, r0, r0 + rb < it.r_hi ? r0 + rb : it.r_hi, er, RI);
                rok = rows_of(rrows, er, rv, RI);
            }
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                if (!((rok >> i) & 1u)) continue;
                const unsigned h = one_round ? rh[i] : slot_of(R::key(rv[i]));
                grow[atomicAdd(&gend[h], 1u)] = (PT)R::pay(rv[i]);
            }
        }
        __syncthreads();
        // ---- probe, one sub-chunk of S rows at a time
        for (u64 sb = it.s_lo; sb < it.s_hi; sb += subb) {
            u64 es[SI];
            T sv[SI];
            ents(a.s_runs, sb, sb + subb < it.s_hi ? sb + subb : it.s_hi, es, SI);
            const unsigned sok = rows_of(srows, es, sv, SI);
            unsigned cnt[SI], st[SI];
            u64 mine = 0;
#pragma unroll
            for (int i = 0; i < SI; ++i) {
                cnt[i] = st[i] = 0u;
                if (!((sok >> i) & 1u)) continue;
                const u64 key = R::key(sv[i]);
                // (wide: an S key equal to EMPTY ends at the first empty slot:
                // no build row holds it, items with one were deferred above)
                unsigned h = (unsigned)(rhash(key) >> a.tshift) & kMask;
                u64 e = gkey[h];
                while (e != kE && !key_is(e, key)) {
                    h = (h + 1) & kMask;
                    e = gkey[h];
                }
                if (e != kE) {
                    cnt[i] = count_at(h, e);
                    st[i] = gend[h] - cnt[i];
                }
                mine += cnt[i];
            }
            u64 tot;
            const u64 pre = block_excl_scan<NT>(mine, wsum, &tot);
            if constexpr (!WRITE) {
                if (threadIdx.x == 0 && tot) atomicAdd(a.counter, tot);
                continue;
            }
            if (!tot) continue;   // uniform
            if (threadIdx.x == 0) s_base = atomicAdd(a.counter, tot);
            __syncthreads();
            const u64 pos = s_base + pre;
            if (tot > 2ull * (subb << kRunLog)) {
                // many pairs per probe row: the wave copies one row's group at
                // a time, 64 pairs per step, lane by lane (a lane's rows own
                // consecutive positions, so the wave's stores stay in one region)
                for (int l = 0; l < 64; ++l) {
                    u64 p = ((u64)(unsigned)__builtin_amdgcn_readlane((int)(pos >> 32), l) << 32) |
                            (u64)(unsigned)__builtin_amdgcn_readlane((int)pos, l);
#pragma unroll
                    for (int i = 0; i < SI; ++i) {
                        const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)cnt[i], l);
                        if (!c) continue;   // uniform
                        const unsigned s0 = (unsigned)__builtin_amdgcn_readlane((int)st[i], l);
                        const u64 spay = R::pay(sv[i]);
                        PT sp = (PT)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)spay, l);
                        if constexpr (WIDE)
                            sp |= (PT)((u64)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(spay >> 32), l) << 32);
                        // (plain stores: a group's run starts and ends inside
                        // lines, and non-temporal stores skip the L2 that
                        // assembles them with the neighbouring rows' pairs)
                        for (unsigned j = lane; j < c; j += 64u) {
                            const u64 q = p + j;
                            if (q < (u64)a.cap) {
                                orr[q] = grow[s0 + j];
                                oss[q] = sp;
                            }
                        }
                        p += c;
                    }
                }
            } else {
                u64 q = pos;
#pragma unroll
                for (int i = 0; i < SI; ++i) {
                    for (unsigned j = 0; j < cnt[i]; ++j, ++q) {
                        if (q < (u64)a.cap) {
                            orr[q] = grow[st[i] + j];
                            oss[q] = (PT)R::pay(sv[i]);
                        }
                    }
                }
            }
            __syncthreads();   // s_base reused by the next sub-chunk
        }
        __syncthreads();   // tables reused by the next item
    }
}

// --------------------------------------------------------------- join shapes
// One product kernel per (row width, shape), chosen from facts known when
// the join is launched -- never from an earlier join's statistics:
//   int64 rows, fast shape: k_join_b (bucketed table) -- or k_join_u when the
//     build-time sample found repeated build keys (its counting walks lose to
//     k_join_u's per-row walks there: C1-ref);
//   int64 rows, probe side >= 8x the build side: k_join_u's stream shape;
//   i32 rows: k_join_b (narrow shape), its deferrals to k_join_grp, or
//     k_join_grp over every item when the sample says most build keys repeat
//     (the reference's 10M x 10M keys in [1, 100k]);
//   whatever those defer: k_join (list mode).
// The sample (k_rsample, at build time) lives on the device; every kernel of
// the join reads it and the ones not chosen exit at once, so the choice is a
// pure function of the data and needs no host round trip.
// Fast shape: 768 threads, 3 build + 3 probe rows per thread, 6 waves per
// SIMD (profiles/r02_join_fast.txt: C3 k_join 3.50 -> 2.81 ms, C2 12.34 ->
// 9.45 ms, C1-ref 1.31 -> 0.96 ms; k_join_b: C3 2.77 -> 2.55 ms).
constexpr int kFastNT = kFastNTc, kFastRI = kFastRIc, kFastSI = kFastSIc, kFastWPS = kFastWPSc;
// probe sides much larger than the build side (C2: 2^30 x 2^20, ~1000 S rows
// per R row): many sub-chunks per item, so bigger sub-chunks and more waves
// (1024 threads x 4 S rows, 8 waves per SIMD): C2 join 9.45 -> 8.77 ms, C3
// 2.79 -> 3.32 ms (profiles/r02_join_shapes.txt).  3 S rows per thread since
// round 3: the 4-row shape carried a 12-B scratch spill at the 64-VGPR cap;
// without it C2's join 6.49 -> 6.16 ms on one box (768 x 3+4: 6.25, 768 x
// 2+5: 6.30, 1024 x 1+4: 6.47; profiles/r03_narrow_shapes.txt 8)
constexpr int kStreamNT = 1024, kStreamRI = 2, kStreamSI = 3, kStreamWPS = 8;
// grouped join (narrow rows with repeated keys): 512 threads, 2 workgroups per CU (64 KiB of LDS),
// 3 build + 8 probe rows per thread (round 5; 4 + 4 before): a REF-A item's
// probe rows in one sub-chunk, REF-A join 1.85 -> 1.79 ms (profiles/r05/r05zu_grouped_rows_ab.jsonl;
// 4 + 8 1.80, 4 + 10 1.80, 3 + 5 / 4 + 5 unchanged; 110 VGPRs of the 128 two workgroups allow)
constexpr int kGrpNT = 512, kGrpRI = 3, kGrpSI = 8;
// int64 rows: 512 threads x 3 + 3 rows over 2048 slots, two workgroups per CU (at three, 80 VGPRs spilled)
constexpr int kGrpWideRI = 3, kGrpWideSI = 3, kGrpWidePerCU = 2;
constexpr int kTableLog = 12;   // LDS table slots of the int64-row joins (2^12 x 16 B)
// i32 rows: k_join_b over 8192 slots (keys and row ids apart: 64 KiB), 768
// threads x 4 build + 5 probe rows, 6 waves per SIMD, 2 workgroups per CU;
// plan partitions of ~4096 rows (log2 of twice the average build rows).
// Round 5: 3 + 5 instead of 4 + 4 -- a REF-B partition (~3050 rows, ~48
// runs) takes two build rounds instead of one or two, but its probe rows
// one sub-chunk instead of two, and a sub-chunk (scan, output atomic, three
// barriers) costs more than a build round: REF-B join 0.766 -> 0.695 ms
// (profiles/r05/r05zq_narrow_3p5_ab.jsonl; 5 + 3 0.87, 2 + 6 / 3 + 6 spill).
// Round 6: 4 + 5 (80 VGPRs, no spill): most REF-B partitions now take one
// build round as well -- join 0.695-0.697 -> 0.687 ms, step -0.5 % in three
// alternating pairs (profiles/r06/r06o_narrow_4p5_ab.jsonl); 4 + 6, 5 + 5
// and 4 + 7 spill 24 / 12 / 60 B.
// REF-B's join (profiles/r03_narrow_shapes.txt; the other shapes live on in
// micro/ only): k_join_u over 8192 slots 1.16 ms; k_join_b over 4096 slots
// 768 x 3+3 0.92, 512 x 5+4 at 3 per CU 0.96, 512 x 5+3 at 4 per CU 1.35 and
// 1024 x 3+3 1.12 (both spill at the 64-VGPR cap); over 8192 slots 768 x 3+3
// 0.886, 768 x 4+4 0.779 (this shape); 4+6 and 5+5 spill.  Round 4: 72 %
// of REF-B's partitions hold more than this shape's 48 runs per build round
// (micro/runs_micro.hip), so shapes with larger rounds were tried
// (profiles/r04_narrow_rounds.txt): 640 x 5+5 at 5 waves per SIMD 1.31 ms,
// 640 x 6+6 1.24, 896 x 4+4 at 7 per SIMD 1.08, against 0.82 for this one.
constexpr int kNarrowNT = 768, kNarrowRI = 4, kNarrowSI = 5, kNarrowWPS = 6, kNarrowPerCU = 2, kTableLogNarrow = 13,
              kPlanLogNarrow = 13;

int cu_count() {
    static int n = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return cus > 0 ? cus : 256;
    }();
    return n;
}

inline unsigned blocks_for(u64 n, u64 per) { return (unsigned)((n + per - 1) / per); }

// Workgroups of a partition pass over n rows: one per CU, fewer for small
// inputs (each open bucket per workgroup and bin is potential slack).
unsigned pass_grid(u64 n) {
    const u64 tiles = (n + kTile - 1) / kTile;
    const u64 g = tiles / 8 > 0 ? tiles / 8 : 1;   // >= 8 tiles per workgroup
    const u64 cus = (u64)cu_count();
    return (unsigned)(g < cus ? g : cus);
}

// The k_pass variant of a pass of fb bits: passes of <= 8 bits run the
// half-size workgroups, two per CU (kSmallPassThreads).
inline bool small_pass(int fb) { return fb <= 8; }
// (i32 rows: 8 rows per thread in the half-size workgroups -- 4096-row tiles
// of 8-B rows -- so a tile's fixed LDS work and barriers serve as many bytes
// as an int64 tile's; the 1024-thread variant keeps 4: registers)
constexpr int kSmallNarrowRows = 8;
inline unsigned pass_tile_rows(int fb, bool wide = true) {
    if (!small_pass(fb)) return (unsigned)kTile;
    return (unsigned)(kSmallPassThreads * (wide ? kPassRows : kSmallNarrowRows));
}
unsigned pass_grid(u64 n, int fb, bool wide = true) {
    if (!small_pass(fb)) return pass_grid(n);
    const u64 tiles = (n + pass_tile_rows(fb, wide) - 1) / pass_tile_rows(fb, wide);
    const u64 g = tiles / 8 > 0 ? tiles / 8 : 1;
    const u64 w = 2ull * (u64)cu_count();
    return (unsigned)(g < w ? g : w);
}

// Exclusive scan of a u64 array of len elements in place (k_scan_*).
void scan_u64(u64 *v, u64 len, u64 *sums, hipStream_t st) {
    const unsigned nb = blocks_for(len, kScanBlock);
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(1024), 0, st, v, len, sums);
    if (nb > 1) hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(1024), 0, st, v, len, (const u64 *)sums);
}

// Exclusive scan of len u64 in place in one launch: one block, or the
// look-back scan over ws.scan_state.
void scan_one(u64 *v, u64 len, const RadixWork &ws, hipStream_t st) {
    if (len <= (u64)kScanBlock) {
        hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, st, v, len, ws.scan_sums);
        return;
    }
    hipLaunchKernelGGL((k_scan_lb<false>), dim3(blocks_for(len, kLbTile)), dim3(kLbThreads), 0, st, v, len,
                       ws.scan_state, ChunkMapArgs{});
}

// chunk_map in one launch (k_scan_lb's MAP mode): start[0..nseg], owner[],
// and the count scan (split order) in ws.pcur.
void chunk_map_one(const u64 *off_a, const u64 *off_b, int nseg, unsigned chunk, unsigned *start, unsigned *owner,
                   const RadixWork &ws, hipStream_t st, bool split = false) {
    ChunkMapArgs m{off_a, off_b, chunk, split, start, owner};
    const u64 n = (u64)nseg + 1;
    hipLaunchKernelGGL((k_scan_lb<true>), dim3(blocks_for(n, kLbTile)), dim3(kLbThreads), 0, st, ws.pcur, n,
                       ws.scan_state, m);
}

// per_seg: about how many chunks a segment has (sizes the owner fill's
// threads per segment)
void chunk_map(const u64 *off_a, const u64 *off_b, int nseg, unsigned chunk, unsigned *start, unsigned *owner,
               u64 *scratch, u64 *sums, hipStream_t st, u64 per_seg = 1, bool split = false) {
    const unsigned g = blocks_for((u64)nseg + 1, 256);
    hipLaunchKernelGGL(k_chunk_count, dim3(g), dim3(256), 0, st, off_a, off_b, nseg, chunk, scratch, split);
    scan_u64(scratch, (u64)nseg + 1, sums, st);
    int tl = 0;
    while (tl < 6 && (2ull << tl) <= per_seg) ++tl;
    hipLaunchKernelGGL(k_chunk_finish, dim3(blocks_for(((u64)nseg + 1) << tl, 256)), dim3(256), 0, st,
                       (const u64 *)scratch, nseg, start, owner, tl);
}

}  // namespace

// ----------------------------------------------------------------- planning
RadixPlan radix_plan(long long n_build, int force_bits, bool wide) {
    // average build rows per partition <= half the join kernel's LDS slots
    const int tsl = wide ? kTableLog : kPlanLogNarrow;
    RadixPlan pl;
    int bits = 1;
    while (bits < 24 && ((unsigned long long)n_build >> bits) > (1ull << (tsl - 1))) ++bits;
    if (force_bits > 0) bits = force_bits < 24 ? force_bits : 24;
    pl.total_bits = bits;
    pl.passes = (bits + 8) / 9;   // <= 9 bits (512-way fan-out) per pass
    int left = bits;
    for (int i = 0; i < pl.passes; ++i) {
        pl.bits[i] = (left + (pl.passes - i) - 1) / (pl.passes - i);   // (the larger fan-out first: r04g)
        left -= pl.bits[i];
        pl.pbl[i] = i == pl.passes - 1 ? kFinalPbl : kPassPbl;
    }
    for (int i = pl.passes; i < 3; ++i) pl.bits[i] = pl.pbl[i] = 0;
    return pl;
}

// Pass i writes the final set when (passes - 1 - i) is even, else the ping
// set.  It allocates at most n / PB full buckets plus one open bucket per
// (workgroup segment run, bin): runs <= G + nseg_in; and a bucket is only
// allocated to take rows.
RadixNeed radix_need(long long n, const RadixPlan &pl, bool final_set) {
    RadixNeed need{1, 1};
    const u64 rows = n > 0 ? (u64)n : 1;
    u64 nseg = 1, prev_b = 0;
    for (int i = 0; i < pl.passes; ++i) {
        const bool to_final = ((pl.passes - 1 - i) % 2) == 0;
        const u64 F = 1ull << pl.bits[i];
        // k_id_plan's ranges: sum over workgroups of ceil(tiles_w * kTile /
        // PB) + segs_w * F + 1, with sum segs_w <= nseg + G; tiles of a
        // bucketed pass <= runs / 64 + nseg, runs <= rows / 64 + buckets_in
        const u64 G = pass_grid(rows, pl.bits[i]);
        const u64 tr = pass_tile_rows(pl.bits[i]), rpt = tr >> kRunLog;
        const u64 tiles = i == 0 ? (rows + tr - 1) / tr : (rows / 64 + prev_b) / rpt + nseg + 1;
        const u64 b = (tiles * tr >> pl.pbl[i]) + G + (nseg + G) * F + G + 1;
        prev_b = b;
        if (to_final == final_set) {
            if (b > need.buckets) need.buckets = b;
            if ((b << pl.pbl[i]) > need.rows) need.rows = b << pl.pbl[i];
        }
        nseg *= F;
    }
    return need;
}

unsigned long long radix_tiles(long long n, int max_nseg) {
    // bucketed tiles: >= kSmallPassThreads * kPassRows / 64 runs each (the
    // smaller variant), <= one partial tile per segment; every run holds >= 1
    // row, so runs <= n (the bound is loose but small)
    return (u64)(n > 0 ? n : 1) / ((kSmallPassThreads * kPassRows) >> kRunLog) + (u64)max_nseg + 2;
}

size_t radix_item_desc_bytes() { return sizeof(ItemDesc); }

unsigned long long radix_work_words(const RadixPlan &pl, unsigned long long s_runs) {
    return (1ull << pl.total_bits) + 4ull + 3ull * radix_join_items(pl, s_runs);
}

hipError_t exclusive_scan_u64(unsigned long long *v, unsigned long long len, unsigned long long *sums,
                              hipStream_t st) {
    if (len == 0) return hipSuccess;
    scan_u64(v, len, sums, st);
    return hipGetLastError();
}

size_t exclusive_scan_sums(unsigned long long len) { return (size_t)(len / kScanBlock + 2); }

unsigned long long radix_join_items(const RadixPlan &pl, unsigned long long s_runs) {
    // the smallest item of any shape (radix_join sizes items by its kernel's sub-chunk)
    const u64 sub = (u64)kFastNT * kFastSI < (u64)kNarrowNT * kNarrowSI ? (u64)kFastNT * kFastSI
                                                                         : (u64)kNarrowNT * kNarrowSI;
    const u64 chr = (u64)kJoinSub * (sub >> kRunLog);
    return s_runs / chr + (1ull << pl.total_bits) + 2;
}

namespace {
// Bin sizes of every (bin, workgroup) pair of an EXACT pass over the same
// tiles: hist[b * G + w] (k_pass's tile ranges, bin = the top fbits of the
// hash), zeroed by the kernel itself.
template <bool WIDE, int FORM>
__global__ __launch_bounds__(1024) void k_slot_hist(PassArgs a, u64 *hist) {
    typedef Row<WIDE> R;
    __shared__ unsigned c[kMaxFan];
    const unsigned F = 1u << a.fbits;
    for (unsigned b = threadIdx.x; b < F; b += 1024) c[b] = 0u;
    __syncthreads();
    const unsigned T_ = (unsigned)((a.n + kTile - 1) / kTile);
    const unsigned t0 = (unsigned)((u64)blockIdx.x * T_ / gridDim.x);
    const unsigned t1 = (unsigned)((u64)(blockIdx.x + 1) * T_ / gridDim.x);
    const u64 r0 = (u64)t0 * kTile, r1 = (u64)t1 * kTile < a.n ? (u64)t1 * kTile : a.n;
    // 8 keys per thread in flight per step (a tile = 4096 rows = 1024 x 4:
    // two tiles per step); key columns as 16-B pairs when aligned
    constexpr int U = 8;
    auto key_at = [&](u64 r) -> u64 {
        if constexpr (FORM == kCols64) return ((const u64 *)a.in.key)[r];
        else return R::key(((const typename R::T *)a.in.key)[r]);
    };
    for (u64 rb = r0; rb < r1; rb += (u64)U * 1024) {
        u64 k[U];
        bool v[U];
        if (FORM == kCols64 && (((uintptr_t)a.in.key) & 15) == 0 && rb + (u64)U * 1024 <= r1) {
#pragma unroll
            for (int i = 0; i < U / 2; ++i) {
                const ulonglong2 k2 = ((const ulonglong2 *)((const u64 *)a.in.key + rb))[(u64)i * 1024 + threadIdx.x];
                k[2 * i] = k2.x;
                k[2 * i + 1] = k2.y;
                v[2 * i] = v[2 * i + 1] = true;
            }
        } else {
#pragma unroll
            for (int i = 0; i < U; ++i) {
                const u64 r = rb + (u64)i * 1024 + threadIdx.x;
                v[i] = r < r1;
                k[i] = v[i] ? key_at(r) : 0ull;
            }
        }
#pragma unroll
        for (int i = 0; i < U; ++i)
            if (v[i]) atomicAdd(&c[(unsigned)(rhash(k[i]) >> a.shift) & (F - 1)], 1u);
    }
    __syncthreads();
    for (unsigned b = threadIdx.x; b < F; b += 1024) hist[(u64)b * gridDim.x + blockIdx.x] = c[b];
}

// Bin sizes from the scanned slot bases.
__global__ __launch_bounds__(256) void k_slot_counts(const u64 *base, unsigned F, unsigned G, u64 n, u64 *counts) {
    const unsigned b = blockIdx.x * 256 + threadIdx.x;
    if (b < F) counts[b] = (b + 1 < F ? base[(u64)(b + 1) * G] : n) - base[(u64)b * G];
}
}  // namespace

size_t radix_route_scratch(long long n, int rbits) {
    const u64 G = pass_grid((u64)(n > 0 ? n : 1));
    return (size_t)(((u64)1 << rbits) * G + 1);
}

hipError_t radix_route(const SrcDev &src, int rbits, void *out_tuples, unsigned long long *counts,
                       unsigned long long *hist, unsigned long long *scan_sums, hipStream_t st) {
    if (rbits < 1 || rbits > 9 || (src.form != kCols64 && src.form != kPacked64)) return hipErrorInvalidValue;
    const u64 n = (u64)(src.n > 0 ? src.n : 0);
    const unsigned F = 1u << rbits;
    if (n == 0) return hipMemsetAsync(counts, 0, F * sizeof(u64), st);
    const unsigned G = pass_grid(n);
    PassArgs a;
    a.in = src;
    a.n = n;
    a.cols_aligned = ((((uintptr_t)src.key) | ((uintptr_t)src.pay)) & 15) == 0;
    a.in_rows = nullptr;
    a.in_runs = nullptr;
    a.in_rstart = nullptr;
    a.in_max_rows = a.in_max_runs = 0;
    a.tile_start = nullptr;
    a.tdesc = nullptr;
    a.nseg = 1;
    a.out_rows = out_tuples;
    a.bbin = a.bfill = a.nb = nullptr;
    a.wstart = nullptr;
    a.max_buckets = 0;
    a.out_pbl = 0;
    a.shift = 64 - rbits;
    a.fbits = rbits;
    a.rcnt = nullptr;
    a.slot_base = (const u64 *)hist;
    a.out_max_rows = n;
    if (src.form == kCols64) hipLaunchKernelGGL((k_slot_hist<true, kCols64>), dim3(G), dim3(1024), 0, st, a, (u64 *)hist);
    else hipLaunchKernelGGL((k_slot_hist<true, kPackedRow>), dim3(G), dim3(1024), 0, st, a, (u64 *)hist);
    scan_u64((u64 *)hist, (u64)F * G, (u64 *)scan_sums, st);
    hipLaunchKernelGGL(k_slot_counts, dim3(blocks_for(F, 256)), dim3(256), 0, st, (const u64 *)hist, F, G, n,
                       (u64 *)counts);
    if (src.form == kCols64) hipLaunchKernelGGL((k_pass<true, kCols64, 0, true>), dim3(G), dim3(kPassThreads), 0, st, a);
    else hipLaunchKernelGGL((k_pass<true, kPackedRow, 0, true>), dim3(G), dim3(kPassThreads), 0, st, a);
    return hipGetLastError();
}

namespace {
// Passes first .. pl.passes - 1 of plan pl; the first of them reads `prev`
// (a bucket set over nseg segments) or, when prev is null, the source rows.
hipError_t radix_passes(const SrcDev &src, u64 n, bool wide, const RadixPlan &pl, int first, const BucketSet *prev,
                        int nseg, const RadixWork &ws, const BucketSet &out, hipStream_t st) {
    int shift = 64 - pl.skip;
    for (int pass = 0; pass < first; ++pass) shift -= pl.bits[pass];
    // a pass's run placement waits for the next pass's plan and shares its
    // launch (k_place_plan): both only need the pass's scanned run starts
    bool pending = false;
    PlaceArgs pa_prev{};
    unsigned np_prev = 0;
    auto place_alone = [&]() {
        if (pending) hipLaunchKernelGGL(k_bplace, dim3(np_prev), dim3(1024), 0, st, pa_prev);
        pending = false;
    };
    for (int pass = first; pass < pl.passes; ++pass) {
        const int fb = pl.bits[pass];
        const unsigned grid = pass_grid(n > 0 ? n : 1, fb, wide);
        const bool small = small_pass(fb);
        shift -= fb;
        const BucketSet &dst = ((pl.passes - 1 - pass) % 2) == 0 ? out : ws.tmp;
        // bucket-count word and placement cursors by pass parity (the plan of
        // pass + 1 zeroes its own while pass's placement still uses these)
        unsigned *nbw = ws.nb + (pass & 1);
        u64 *rcur = (pass & 1) ? ws.pcur : ws.rcur;
        PassArgs a;
        a.in = src;
        a.n = n;
        a.cols_aligned = ((((uintptr_t)src.key) | ((uintptr_t)src.pay)) & 15) == 0;
        a.in_rows = prev ? prev->rows : nullptr;
        a.in_runs = prev ? prev->runs : nullptr;
        a.in_rstart = prev ? prev->rstart : nullptr;
        a.in_max_rows = prev ? prev->max_rows : 0;
        a.in_max_runs = prev ? prev->max_runs : 0;
        a.tile_start = ws.tile_start;
        a.tdesc = nullptr;
        a.nseg = nseg;
        a.out_rows = dst.rows;
        a.bbin = dst.bbin;
        a.bfill = dst.bfill;
        a.nb = nbw;
        {
            // a write past either array is impossible by the capacity bound
            // (radix_need); the kernel still clamps to this
            const u64 by_rows = dst.max_rows >> pl.pbl[pass];
            a.max_buckets = (unsigned)(by_rows < dst.max_buckets ? by_rows : dst.max_buckets);
        }
        a.out_pbl = pl.pbl[pass];
        a.shift = shift;
        a.fbits = fb;
        a.tile_rows = pass_tile_rows(fb, wide);
        a.wstart = ws.wstart;
        // the pass counts its buckets' runs per partition into dst.rstart;
        // the plan kernel zeroes them and the placement cursors first.  A
        // small pass followed by another counts into ws.raw_cnt instead, and
        // the next pass's plan launch (k_place_plan) scans them itself.
        const u64 P = (u64)nseg << fb;
        const bool fuse = ws.raw_cnt && pass + 1 < pl.passes && P <= (u64)kPlanSegs;
        u64 *cnt = fuse ? ws.raw_cnt + (u64)(pass & 1) * kRawCntWords : dst.rstart;
        a.rcnt = n > 0 ? cnt : nullptr;
        if (grid > 1023) return hipErrorInvalidValue;   // plans: one thread per workgroup + 1
        const unsigned zgrid = blocks_for(P + 1, 1024);
        if (prev && nseg <= kPlanSegs) {
            // tile map, descriptors, id ranges and zeroing in one launch,
            // with the previous pass's placement when one is pending
            const u64 tb = radix_tiles((long long)n, nseg);
            a.tdesc = (const TileDesc *)ws.tdesc;
            unsigned pg = blocks_for(tb, 1024);
            if (pg < zgrid) pg = zgrid;
            if (pg > 1024) pg = 1024;
            TilePlanArgs tp{a, (const u64 *)prev->rstart, grid, (unsigned)tb, ws.tile_start, (TileDesc *)ws.tdesc,
                            ws.wstart, cnt, rcur, P + 1};
            if (pending) hipLaunchKernelGGL(k_place_plan, dim3(np_prev + pg), dim3(1024), 0, st, pa_prev, np_prev, tp);
            else hipLaunchKernelGGL(k_tile_plan, dim3(pg), dim3(1024), 0, st, tp);
            pending = false;
        } else {
            place_alone();
            if (prev) {
                // tiles of kTile / 64 runs per segment, tile -> segment, and one
                // descriptor per tile
                const unsigned rpt = a.tile_rows >> kRunLog;
                chunk_map(prev->rstart, nullptr, nseg, rpt, ws.tile_start, ws.tile_owner, ws.pcur, ws.scan_sums, st,
                          (u64)n / (u64)(nseg > 0 ? nseg : 1) / (u64)a.tile_rows);
                const u64 tb = radix_tiles((long long)n, nseg);
                hipLaunchKernelGGL(k_tile_desc, dim3(blocks_for(tb, 256)), dim3(256), 0, st,
                                   (const unsigned *)ws.tile_start, (const unsigned *)ws.tile_owner,
                                   (const u64 *)prev->rstart, nseg, (unsigned)tb, (TileDesc *)ws.tdesc, rpt);
                a.tdesc = (const TileDesc *)ws.tdesc;
            }
            hipLaunchKernelGGL(k_id_plan, dim3(zgrid < 1024 ? zgrid : 1024), dim3(1024), 0, st, a, prev != nullptr, grid,
                               ws.wstart, cnt, rcur, P + 1);
        }
        if (n > 0) {
#define HJ_PASS(W, FORM)                                                                                    \
    do {                                                                                                    \
        if (small)                                                                                          \
            hipLaunchKernelGGL((k_pass<W, FORM, 0, false, kSmallPassThreads, kSmallFan,                     \
                                       W ? kPassRows : kSmallNarrowRows>),                                  \
                               dim3(grid), dim3(kSmallPassThreads), 0, st, a);                              \
        else hipLaunchKernelGGL((k_pass<W, FORM>), dim3(grid), dim3(kPassThreads), 0, st, a);               \
    } while (0)
            if (prev) {
                if (wide) HJ_PASS(true, kBucketed);
                else HJ_PASS(false, kBucketed);
            } else if (wide) {
                if (src.form == kCols64) HJ_PASS(true, kCols64);
                else HJ_PASS(true, kPackedRow);   // kPacked64 input == packed row layout
            } else {
                if (src.form == kCol32) HJ_PASS(false, kCol32);
                else HJ_PASS(false, kPackedRow);
            }
#undef HJ_PASS
        }
        // runs fit by construction (max_runs >= max_rows / 64 + max_buckets)
        if (dst.max_runs < (dst.max_rows >> kRunLog) + dst.max_buckets) return hipErrorInvalidValue;
        if (!fuse) scan_one(dst.rstart, P + 1, ws, st);
        pa_prev = PlaceArgs{(const unsigned *)dst.bbin, (const unsigned *)dst.bfill, (const unsigned *)nbw, a.max_buckets,
                            pl.pbl[pass], (const u64 *)dst.rstart, rcur, dst.runs, (int)P,
                            fuse ? (const u64 *)cnt : nullptr};
        np_prev = blocks_for(dst.max_buckets, 1024 * kListPer);
        pending = true;
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        prev = &dst;
        nseg = (int)P;
    }
    place_alone();
    return hipGetLastError();
}

// Routed rows as a first-pass bucket set: tuples hold, for each source in
// order, that source's rows of segments 0 .. nseg-1 in segment order,
// cnt[s * nseg + b] of them; segment b lists its rows as runs (<= 64 rows,
// row << 7 | count), source by source.  One block per segment.
__global__ __launch_bounds__(256) void k_routed_list(const u64 *cnt, int nsrc, int nseg, u64 *runs, u64 *rstart,
                                                     u64 max_runs) {
    __shared__ u64 tot[kMaxRouteSources], before[kMaxRouteSources];
    __shared__ u64 runs_before, runs_all;
    const int b = blockIdx.x;
    for (int i = threadIdx.x; i < nsrc; i += 256) tot[i] = before[i] = 0ull;
    if (threadIdx.x == 0) runs_before = runs_all = 0ull;
    __syncthreads();
    u64 rb = 0, ra = 0;
    for (int i = threadIdx.x; i < nsrc * nseg; i += 256) {
        const int s = i / nseg, bb = i - s * nseg;
        const u64 c = cnt[i], r = (c + 63) >> kRunLog;
        atomicAdd(&tot[s], c);
        ra += r;
        if (bb < b) {
            atomicAdd(&before[s], c);
            rb += r;
        }
    }
    if (rb) atomicAdd(&runs_before, rb);
    if (b == 0 && ra) atomicAdd(&runs_all, ra);
    __syncthreads();
    if (threadIdx.x == 0) {
        rstart[b] = runs_before;
        if (b == 0) rstart[nseg] = runs_all;
    }
    // source s's rows of segment b: row base = the rows of sources < s, then
    // s's rows of segments < b; its runs follow those of sources < s
    u64 row0 = 0, run0 = runs_before;
    for (int s = 0; s < nsrc; ++s) {
        const u64 c = cnt[(u64)s * nseg + b], base = row0 + before[s];
        const u64 r = (c + 63) >> kRunLog;
        for (u64 j = threadIdx.x; j < r; j += 256) {
            const u64 len = c - (j << kRunLog) < 64 ? c - (j << kRunLog) : 64;
            if (run0 + j < max_runs) runs[run0 + j] = ((base + (j << kRunLog)) << 7) | len;
        }
        row0 += tot[s];
        run0 += r;
    }
}
}  // namespace

// Partition one relation into the plan's 2^total_bits partitions: bucket
// rows in `out` (with runs / rstart by partition).  ws.tmp is the ping set
// of multi-pass plans.  Asynchronous; no allocation.
hipError_t radix_partition(const SrcDev &src, bool wide, const RadixPlan &pl, const RadixWork &ws,
                           const BucketSet &out, hipStream_t st) {
    const u64 n = (u64)(src.n > 0 ? src.n : 0);
    return radix_passes(src, n, wide, pl, 0, nullptr, 1, ws, out, st);
}

hipError_t radix_partition_routed(const void *tuples, long long n, const unsigned long long *cnt, int nsrc, int nseg,
                                  const RadixPlan &pl, const RadixWork &ws, const BucketSet &out, hipStream_t st) {
    if (pl.passes != 2 || nsrc < 1 || nsrc > kMaxRouteSources || nseg < 1) return hipErrorInvalidValue;
    // the routed listing borrows the ping set's run arrays (a 2-pass plan's
    // second pass writes `out`, not ws.tmp)
    hipLaunchKernelGGL(k_routed_list, dim3(nseg), dim3(256), 0, st, (const u64 *)cnt, nsrc, nseg, ws.tmp.runs,
                       ws.tmp.rstart, (u64)ws.tmp.max_runs);
    BucketSet in = ws.tmp;
    in.rows = const_cast<void *>(tuples);
    in.max_rows = (u64)(n > 0 ? n : 0);
    SrcDev src{};
    src.key = tuples;
    src.pay = nullptr;
    src.n = n;
    src.form = kPacked64;
    return radix_passes(src, (u64)(n > 0 ? n : 0), true, pl, 1, &in, nseg, ws, out, st);
}

hipError_t radix_join(bool wide, const RadixPlan &pl, const RadixWork &ws, const BucketSet &r, const BucketSet &s,
                      unsigned long long s_runs, unsigned *work_start, void *desc, void *out_r, void *out_s, long long cap,
                      unsigned long long *counter, unsigned long long *dup_flag, bool count_only, hipStream_t st,
                      const unsigned long long *sample, bool stream, int nparts) {
    const int P = nparts >= 0 ? nparts : 1 << pl.total_bits;
    unsigned *work_owner = work_start + P + 1;
    if (pl.pbl[pl.passes - 1] != kFinalPbl) return hipErrorInvalidValue;
    // persistent grids: two workgroups per CU (LDS-limited); i32 rows' fast
    // kernel kNarrowPerCU
    const unsigned pg = (unsigned)(2 * cu_count());
    const unsigned pgn = (unsigned)(kNarrowPerCU * cu_count());
    // the probe-heavy stream shape: int64 rows only (i32 rows keep the fast shape)
    const bool stream_shape = stream && wide;
    // S runs per work item: at least kJoinSub sub-chunks, more when S is
    // large against the partition count (each item rebuilds its R table), as
    // long as ~16 items per workgroup remain for balance
    const unsigned subb = stream_shape ? (unsigned)((kStreamNT * kStreamSI) >> kRunLog)
                                       : (wide ? (unsigned)((kFastNT * kFastSI) >> kRunLog)
                                               : (unsigned)((kNarrowNT * kNarrowSI) >> kRunLog));
    u64 chb = (u64)kJoinSub * subb;
    const u64 want = (u64)s_runs / (16ull * (wide ? pg : pgn));
    if (want > chb) chb = (want + subb - 1) / subb * subb;
    // heavy-first item order for int64 rows (longest items claimed first);
    // i32 rows keep partition order (k_join_grp lost 0.2 ms on REF-A with it)
    const bool heavy_first = kHeavyFirst && wide;
    chunk_map_one(s.rstart, r.rstart, P, (unsigned)chb, work_start, work_owner, ws, st, heavy_first);
    const unsigned items = (unsigned)((u64)s_runs / chb + (u64)P + 1);
    // the deferred-item lists live after the work map: the fast kernels'
    // (for k_join, or for k_join_grp with i32 rows), then k_join_grp's
    unsigned *defer_n = work_owner + radix_join_items(pl, s_runs);
    unsigned *defer2_n = defer_n + 1 + radix_join_items(pl, s_runs);
    unsigned *next_item = defer2_n + 1 + radix_join_items(pl, s_runs);
    hipLaunchKernelGGL(k_item_desc, dim3(blocks_for(items, 256)), dim3(256), 0, st, (const unsigned *)work_start,
                       (const unsigned *)work_owner, (const u64 *)s.rstart, (const u64 *)r.rstart, P, (unsigned)chb,
                       (ItemDesc *)desc, defer_n, defer2_n, next_item,
                       heavy_first ? (const u64 *)ws.pcur : nullptr, counter);
    JoinArgs a;
    a.r = r.rows;
    a.s = s.rows;
    a.r_runs = r.runs;
    a.s_runs = s.runs;
    a.r_rstart = r.rstart;
    a.s_rstart = s.rstart;
    a.P = P;
    a.work_start = work_start;
    a.desc = (const ItemDesc *)desc;
    // the hash bits right below the partition bits: LDS slot / bucket
    a.tshift = 64 - pl.skip - pl.total_bits - (wide ? kTableLog : kTableLogNarrow);
    a.out_r = out_r;
    a.out_s = out_s;
    a.cap = cap;
    a.counter = counter;
    a.dup_flag = dup_flag;
    a.sample = sample;
    a.defer = defer_n + 1;
    a.defer_n = defer_n;
    const unsigned grid = items < pg ? items : pg;
#define HJ_LAUNCH(K, NT) hipLaunchKernelGGL(K, dim3(grid), dim3(NT), 0, st, a)
#define HJ_WR(K_T, K_F, NT)      \
    do {                         \
        if (count_only) HJ_LAUNCH(K_F, NT); \
        else HJ_LAUNCH(K_T, NT); \
    } while (0)
    if (wide) {
        if (stream_shape) {
            a.modes = kModesAll;
            HJ_WR((k_join_u<true, true, kTableLog, kStreamNT, kStreamRI, kStreamSI, kStreamWPS>),
                  (k_join_u<true, false, kTableLog, kStreamNT, kStreamRI, kStreamSI, kStreamWPS>), kStreamNT);
        } else {
            // k_join_b unless most build keys repeat; then k_join takes every
            // item (below, the same launch that takes k_join_b's deferrals:
            // no exit-only launch of a kernel the sample did not choose).
            // (k_join_u served mode 2 before round 5 in a launch of its own;
            // both bodies in one kernel spilled 20 B at the 80-VGPR cap.)
            a.modes = kModeUnique | kModeSome;
            if (HJ_WIDE_DYN) a.next_item = next_item;
            HJ_WR((k_join_b<true, true, kFastNT, kFastRI, kFastSI, kFastWPS>),
                  (k_join_b<true, false, kFastNT, kFastRI, kFastSI, kFastWPS>), kFastNT);
            a.next_item = nullptr;
            // k_join_grp (int64 rows, 2048 slots, two workgroups per CU):
            // k_join_b's deferrals, or every item when most build keys
            // repeat; what it defers (INT64_MIN build keys, > 31 runs) goes
            // to k_join below
            a.modes = kModesAll;
            a.list = defer_n + 1;
            a.list_n = defer_n;
            a.all_if_mode2 = true;
            a.defer = defer2_n + 1;
            a.defer_n = defer2_n;
            {
                const unsigned g3 = items < (unsigned)(kGrpWidePerCU * cu_count()) ? items
                                                                                   : (unsigned)(kGrpWidePerCU * cu_count());
                if (count_only)
                    hipLaunchKernelGGL((k_join_grp<true, false, kGrpNT, kGrpWideRI, kGrpWideSI, true>), dim3(g3),
                                       dim3(kGrpNT), 0, st, a);
                else
                    hipLaunchKernelGGL((k_join_grp<true, true, kGrpNT, kGrpWideRI, kGrpWideSI, true>), dim3(g3),
                                       dim3(kGrpNT), 0, st, a);
            }
            a.all_if_mode2 = false;
        }
    } else {
        // i32 rows: k_join_b (keys and row ids apart in LDS: a bucket's 4
        // keys are one 16-B read) unless most build keys repeat; k_join_grp
        // takes its deferrals (list mode) or, for mostly repeated keys, every
        // item
        a.modes = kModeUnique | kModeSome;
        {
            const unsigned gn = items < pgn ? items : pgn;
            a.next_item = next_item;
            if (count_only)
                hipLaunchKernelGGL((k_join_b<false, false, kNarrowNT, kNarrowRI, kNarrowSI, kNarrowWPS, false,
                                             kTableLogNarrow>),
                                   dim3(gn), dim3(kNarrowNT), 0, st, a);
            else
                hipLaunchKernelGGL((k_join_b<false, true, kNarrowNT, kNarrowRI, kNarrowSI, kNarrowWPS, false,
                                             kTableLogNarrow>),
                                   dim3(gn), dim3(kNarrowNT), 0, st, a);
            a.next_item = nullptr;
        }
        // k_join_grp: k_join_b's deferrals, or every item when most build
        // keys repeat (one launch either way)
        a.modes = kModesAll;
        a.list = defer_n + 1;
        a.list_n = defer_n;
        a.all_if_mode2 = true;
        a.defer = defer2_n + 1;
        a.defer_n = defer2_n;
        HJ_WR((k_join_grp<false, true, kGrpNT, kGrpRI, kGrpSI, true>), (k_join_grp<false, false, kGrpNT, kGrpRI, kGrpSI, true>), kGrpNT);
        a.all_if_mode2 = false;
    }
    // what the kernels above deferred (INT64_MIN build keys, oversized
    // partitions, full tables): k_join over that list, a persistent grid that
    // exits at once when it is empty
    a.modes = kModesAll;
    a.list = wide && stream_shape ? defer_n + 1 : defer2_n + 1;
    a.list_n = wide && stream_shape ? defer_n : defer2_n;
    a.all_if_mode2 = false;
    if (wide) HJ_WR((k_join<true, true, kTableLog, 512, 0, kJoinItems, 4, 0, true>),
                    (k_join<true, false, kTableLog, 512, 0, kJoinItems, 4, 0, true>), 512);
    else HJ_WR((k_join<false, true, kTableLog, 512, 0, kJoinItems, 4, 0, true>),
               (k_join<false, false, kTableLog, 512, 0, kJoinItems, 4, 0, true>), 512);
#undef HJ_WR
#undef HJ_LAUNCH
    return hipGetLastError();
}

// radix_detect's deferred partitions: rows[1] += the rows of every listed
// item (sum of its R run counts); the last workgroup to finish sets
// *dup_flag when the self-join's pair count rows[0] exceeds them.
__global__ __launch_bounds__(256) void k_defer_rows(const unsigned *list, const unsigned *list_n, const ItemDesc *desc,
                                                    const u64 *runs, u64 *rows, u64 *dup_flag) {
    __shared__ u64 wsum[16];
    const unsigned n = *list_n;
    u64 s = 0;
    for (unsigned x = blockIdx.x; x < n; x += gridDim.x) {
        const ItemDesc d = desc[list[x]];
        for (u64 i = d.r_lo + threadIdx.x; i < d.r_hi; i += 256) s += runs[i] & 127u;
    }
    u64 tot;
    (void)block_excl_scan<256>(s, wsum, &tot);
    if (threadIdx.x == 0) {
        if (tot) atomicAdd(&rows[1], tot);
        __threadfence();
        if (atomicAdd(&rows[2], 1ull) == (u64)gridDim.x - 1ull) {
            __threadfence();
            const u64 pairs = atomicAdd(&rows[0], 0ull), have = atomicAdd(&rows[1], 0ull);
            if (pairs > have) atomicExch(dup_flag, 1ull);
        }
    }
}

hipError_t radix_detect(bool wide, const RadixPlan &pl, const RadixWork &ws, const BucketSet &r, unsigned *work_start,
                        void *desc, unsigned long long *dup_flag, const unsigned long long *sample, hipStream_t st) {
    // one item per non-empty partition of the WHOLE build side (a work map
    // from r.rstart alone: partitions no probe row reached are checked too)
    const int P = 1 << pl.total_bits;
    unsigned *work_owner = work_start + P + 1;
    const unsigned whole = 0x7FFFFFFFu;   // runs per item: a partition is one item
    chunk_map_one(r.rstart, r.rstart, P, whole, work_start, work_owner, ws, st);
    unsigned *defer_n = work_owner + radix_join_items(pl, 0);
    hipLaunchKernelGGL(k_item_desc, dim3(blocks_for((u64)P + 1, 256)), dim3(256), 0, st, (const unsigned *)work_start,
                       (const unsigned *)work_owner, (const u64 *)r.rstart, (const u64 *)r.rstart, P, whole,
                       (ItemDesc *)desc, defer_n, nullptr, nullptr, nullptr, nullptr);
    JoinArgs a{};
    a.r = r.rows;
    a.s = r.rows;
    a.r_runs = r.runs;
    a.s_runs = r.runs;
    a.r_rstart = r.rstart;
    a.s_rstart = r.rstart;
    a.P = P;
    a.work_start = work_start;
    a.desc = (const ItemDesc *)desc;
    a.tshift = 64 - pl.skip - pl.total_bits - (wide ? kTableLog : kTableLogNarrow);
    a.dup_flag = dup_flag;
    a.sample = sample;
    a.modes = kModesAll;
    // partitions the bucketed table cannot take (oversized) are deferred to
    // k_join's list-mode build below, which flags repeats inside each of its
    // build rounds
    a.defer = defer_n + 1;
    a.defer_n = defer_n;
    if (wide)
        hipLaunchKernelGGL((k_join_b<true, false, kFastNT, kFastRI, kFastSI, kFastWPS, true>), dim3(2 * cu_count()),
                           dim3(kFastNT), 0, st, a);
    else
        // (its signature words and suspect list on top of the table: one
        // workgroup per CU at 8192 slots: 3 waves per SIMD, register budget as for 4)
        hipLaunchKernelGGL((k_join_b<false, false, kNarrowNT, kNarrowRI, kNarrowSI, (kTableLogNarrow > 12 ? 3 : kNarrowWPS),
                                     true, kTableLogNarrow>),
                           dim3(kNarrowPerCU * cu_count()), dim3(kNarrowNT), 0, st, a);
    // the deferred partitions: k_join builds them (its probe sees an empty S
    // chunk: an item's S runs are [s_lo, s_lo) below)
    a.list = defer_n + 1;
    a.list_n = defer_n;
    a.empty_s = true;
    a.counter = ws.pcur;   // (no probe rows: nothing is counted; a valid word all the same)
    if (wide)
        hipLaunchKernelGGL((k_join<true, false, kTableLog, 512, 0, kJoinItems, 4, 0, true>), dim3(2 * cu_count()),
                           dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((k_join<false, false, kTableLog, 512, 0, kJoinItems, 4, 0, true>), dim3(2 * cu_count()),
                           dim3(512), 0, st, a);
    // That build flags a key repeated inside one of its rounds only.  The
    // exact answer for a deferred (oversized) partition: the count-only
    // self-join of its rows across every round (S = the partition itself)
    // has more pairs than the partition has rows iff some key repeats
    // (ADVICE r04).  pcur[0] = pairs, pcur[1] = rows of the deferred items,
    // pcur[2] = k_defer_rows's done count.
    hipError_t e = hipMemsetAsync(ws.pcur, 0, 3 * sizeof(u64), st);
    if (e != hipSuccess) return e;
    a.empty_s = false;
    a.counter = ws.pcur;
    // (skipped when the launches above already found a repeat: a key that
    // repeats m times inside one partition has >= 2 copies in some build
    // round once m exceeds the rounds, so the self-join only ever runs over
    // partitions whose keys repeat at most once per round)
    a.skip_if_set = dup_flag;
    if (wide)
        hipLaunchKernelGGL((k_join<true, false, kTableLog, 512, 0, kJoinItems, 4, 0, true>), dim3(2 * cu_count()),
                           dim3(512), 0, st, a);
    else
        hipLaunchKernelGGL((k_join<false, false, kTableLog, 512, 0, kJoinItems, 4, 0, true>), dim3(2 * cu_count()),
                           dim3(512), 0, st, a);
    hipLaunchKernelGGL(k_defer_rows, dim3(2 * cu_count()), dim3(256), 0, st, (const unsigned *)(defer_n + 1),
                       (const unsigned *)defer_n, (const ItemDesc *)desc, (const u64 *)r.runs, ws.pcur, dup_flag);
    return hipGetLastError();
}

hipError_t radix_sample(bool wide, const RadixPlan &pl, const BucketSet &r, unsigned long long *sample,
                        hipStream_t st) {
    const int P = 1 << pl.total_bits;
    const unsigned nsamp = (unsigned)(P < kSampleParts ? P : kSampleParts);
    if (wide) hipLaunchKernelGGL((k_rsample<true>), dim3(nsamp), dim3(1024), 0, st, (const void *)r.rows,
                                 (const u64 *)r.runs, (const u64 *)r.rstart, P, nsamp, sample);
    else hipLaunchKernelGGL((k_rsample<false>), dim3(nsamp), dim3(1024), 0, st, (const void *)r.rows,
                            (const u64 *)r.runs, (const u64 *)r.rstart, P, nsamp, sample);
    return hipGetLastError();
}

int join_kernel_choice(bool wide, bool stream, unsigned long long rows, unsigned long long repeats) {
    const int m = sample_mode(rows, repeats);
    if (wide) {
        if (stream) return HJ_JOIN_KERNEL_STREAM;
        return m == 2 ? HJ_JOIN_KERNEL_GROUPED : HJ_JOIN_KERNEL_BUCKETED;
    }
    return m == 2 ? HJ_JOIN_KERNEL_GROUPED : HJ_JOIN_KERNEL_BUCKETED;
}

}  // namespace hj
