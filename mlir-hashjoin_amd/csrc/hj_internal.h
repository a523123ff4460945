// hj_internal.h -- device data layout and kernel launchers of the MI355X
// hash join.  Not part of the public ABI (that is include/hj.h).
//
// Hash table = open addressing with linear probing (north_star), replacing the
// reference's bucket-chained heads + SoA linked list (join_v1.mlir:25-39,
// :213-249).  Two slot layouts:
//
//   wide   : 16-B slot {u64 key, u64 payload}; EMPTY key = INT64_MIN.
//            R rows whose key IS INT64_MIN go to a side list (payload only)
//            and are matched by a side loop whose cost is proportional to
//            the output it produces.
//   narrow : 8-B slot (u32 key << 32 | u32 row id), the reference's i32 key /
//            i32 row-id types (join_v1.mlir:546-549, :604-605).  Row ids are
//            < 2^31, so the all-ones word can never be a real slot: EMPTY.
//
// Both: power-of-two capacity >= 2 * |R| (load factor <= 0.5), slot index =
// top bits of a Fibonacci multiplicative hash, one 64-bit atomicCAS claims a
// slot; duplicate build keys each take their own slot (the reference visits
// every chain node, join_v2.mlir:363-384, so duplicates must all match).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hj_gen.h"

namespace hj {

constexpr unsigned long long kEmptyKey64 = 0x8000000000000000ull;
constexpr unsigned long long kEmptySlot32 = ~0ull;

// Wave64 scans by DPP: row shifts 1, 2, 4, 8 inside each row of 16 lanes,
// then row broadcasts of lane 15 (into rows 1, 3) and lane 31 (into rows 2,
// 3).  A handful of VALU cycles per step, where __shfl_up / __shfl_xor are a
// ds_bpermute (an LDS round trip) each; a wave scanning alone on a
// workgroup's critical path (the partition pass's bin scan, the join's
// output claim) waits for six of them in a row (micro/dpp_micro.hip).
// A lane a DPP step reads from outside the row / mask contributes 0.
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned dpp_or0(unsigned x) {
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ unsigned long long dpp_or0(unsigned long long x) {
    const unsigned lo = dpp_or0<CTRL, ROWS>((unsigned)x), hi = dpp_or0<CTRL, ROWS>((unsigned)(x >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
// inclusive prefix sum over the wave's 64 lanes (all lanes active)
template <typename T>
__device__ __forceinline__ T wave_incl_add_t(T x) {
    x += dpp_or0<0x111, 0xf>(x);   // row_shr:1
    x += dpp_or0<0x112, 0xf>(x);   // row_shr:2
    x += dpp_or0<0x114, 0xf>(x);   // row_shr:4
    x += dpp_or0<0x118, 0xf>(x);   // row_shr:8
    x += dpp_or0<0x142, 0xa>(x);   // row_bcast:15
    x += dpp_or0<0x143, 0xc>(x);   // row_bcast:31
    return x;
}
__device__ __forceinline__ unsigned wave_incl_add(unsigned x) { return wave_incl_add_t(x); }
__device__ __forceinline__ unsigned long long wave_incl_add64(unsigned long long x) { return wave_incl_add_t(x); }
// maximum over the wave's 64 lanes, in every lane (all lanes active)
__device__ __forceinline__ unsigned wave_max_all(unsigned x) {
    auto mx = [](unsigned a, unsigned b) { return a > b ? a : b; };
    x = mx(x, dpp_or0<0x111, 0xf>(x));
    x = mx(x, dpp_or0<0x112, 0xf>(x));
    x = mx(x, dpp_or0<0x114, 0xf>(x));
    x = mx(x, dpp_or0<0x118, 0xf>(x));
    x = mx(x, dpp_or0<0x142, 0xa>(x));
    x = mx(x, dpp_or0<0x143, 0xc>(x));
    return (unsigned)__builtin_amdgcn_readlane((int)x, 63);
}

struct alignas(16) Slot64 {
    unsigned long long key;
    unsigned long long pay;
};

// Device-side table descriptor, passed by value to kernels.
struct TableDev {
    void *slots;                     // Slot64[cap] or u64[cap]
    unsigned long long mask;         // cap - 1
    int shift;                       // 64 - log2(cap)
    unsigned long long *side;        // wide: payloads of INT64_MIN-key rows
    unsigned long long *meta;        // [0] side count, [1] dup-seen flag, [3] slow-tile count, [8..] cursors
};

enum Layout : int { kWide = 0, kNarrow = 1 };

// Source forms of a relation on the device.
enum SrcForm : int { kCols64 = 0, kPacked64 = 1, kCol32 = 2 };

struct SrcDev {
    const void *key;    // int64 column, packed {key,pay} tuples or int32 column
    const void *pay;    // int64 column (kCols64 only)
    long long n;
    long long row_base; // kCol32: row id = row_base + row
    int form;
};

struct OutDev {
    void *r;            // int64 or int32 column (R payload / row id)
    void *s;            // int64 or int32 column (S payload / row id)
    long long cap;      // rows the caller allocated
    unsigned long long *counter;  // device u64: total match count (all rows, even past cap)
};

// launchers (hipError_t of the launch; all asynchronous on `st`)
hipError_t launch_init(const TableDev &t, int layout, unsigned long long cap, hipStream_t st);
hipError_t launch_build(const TableDev &t, int layout, const SrcDev &src, hipStream_t st);
// slow: >= probe_tiles(src.n) words (tiles handed to the general path; the
// count lives in meta[3])
size_t probe_tiles(long long n);
// slow_cap: entries of `slow` (tiles beyond it are never written; the
// callers size it from probe_tiles so that cannot happen)
hipError_t launch_probe(const TableDev &t, int layout, const SrcDev &src, const OutDev &out,
                        bool count_only, unsigned *slow, size_t slow_cap, hipStream_t st);

// ---------------------------------------------------------------- radix join
// (hj_radix.hip) partitions both relations by the top bits of the key hash
// until a partition's build rows fit one workgroup's LDS table, then joins
// partition pairs in LDS.  A pass writes rows into fixed-size buckets (one
// partition per bucket, bucket chaining): no histogram pass, no global scan.
// The radix join's key hash: partitions, passes' bins and LDS slots are its
// bit fields from the top down (odd multiplier: a bijection of the key).
__host__ __device__ __forceinline__ unsigned long long radix_hash(unsigned long long k) {
    return k * 0x9E3779B97F4A7C15ull;
}

struct RadixPlan {
    int passes;       // 1..3 partition passes
    int bits[3];      // fan-out bits per pass (<= 9 each)
    int pbl[3];       // log2 rows per bucket written by each pass
    int total_bits;   // P = 2^total_bits partitions
    int skip = 0;     // top hash bits above the partition bits (the owning GPU of a folded routing)
};

// One pass's output: packed rows in buckets of 2^pbl rows; bucket j holds
// bfill[j] rows of partition bbin[j].  After the pass the rows are listed
// as RUNS of <= 64 consecutive rows of one bucket (row << 7 | count; a
// bucket of f rows gives ceil(f / 64) runs), grouped by partition: p owns
// runs[rstart[p] .. rstart[p+1]).  Consumers map one wave to one run, so a
// partly filled bucket idles at most one wave's tail.
constexpr int kRunLog = 6;
// readable entries past max_runs in a run list: the joins load a wave's
// entries in one scalar load of up to 4, past the list's end included
constexpr int kRunPad = 8;
constexpr int kPassPbl = 10;   // 1024-row buckets for intermediate passes (9: 1 % slower C3 step)
constexpr int kFinalPbl = 9;   // 512-row buckets for the join's input (8 / 9 / 10+9 measured: profiles/r01_bucket_sizes.txt)
struct BucketSet {
    void *rows;                    // >= max_buckets << pbl rows
    unsigned *bbin, *bfill;        // >= max_buckets
    unsigned long long *runs;      // >= max_runs + kRunPad (readable)
    unsigned long long *rstart;    // >= P + 1 (P of the pass writing the set)
    unsigned max_buckets;          // bbin / bfill entries
    unsigned long long max_rows;   // rows entries
    unsigned long long max_runs;   // runs entries (max_rows / 64 + max_buckets covers any fill)
};

struct RadixWork {                 // scratch shared by the partition passes
    BucketSet tmp;                 // ping set of multi-pass plans
    unsigned *nb;                  // device bucket counter
    unsigned long long *pcur;      // >= P + 1: chunk-map scratch
    unsigned long long *rcur;      // >= P + 1: run placement cursors
    unsigned *tile_start;          // >= P + 1
    unsigned *tile_owner;          // >= radix_tiles(n, P)
    void *tdesc;                   // >= radix_tiles(n, P) * 16 B: bucketed-pass tile descriptors
    unsigned *wstart;              // >= 1025: per-workgroup bucket id ranges of a pass
    unsigned long long *scan_sums; // >= P / 8192 + 2
    unsigned long long *scan_state;// >= P / 1024 + 4, zero between calls (the one-launch scan's tile words)
    // 2 x (kRawCntWords): a small pass's raw run counts by pass parity, when
    // the next pass's plan launch scans them itself (null: a scan launch)
    unsigned long long *raw_cnt = nullptr;
};
constexpr unsigned long long kRawCntWords = 4097;   // kPlanSegs + 1 (hj_radix.hip)

struct RadixNeed {                 // sizes of one bucket set
    unsigned long long buckets, rows;
};

// force_bits > 0: fixed 2^bits partitions; wide: int64 rows (else i32 rows, twice the rows per partition)
RadixPlan radix_plan(long long n_build, int force_bits = 0, bool wide = true);
// Bucket capacity of the final set (`final_set`) or the ping set of plan pl for n rows.
RadixNeed radix_need(long long n, const RadixPlan &pl, bool final_set);
unsigned long long radix_tiles(long long n, int max_nseg);
unsigned long long radix_join_items(const RadixPlan &pl, unsigned long long s_runs);
// words of radix_join's work_start buffer: work map (P + 1 + items), then two
// deferred-item lists (count + items each: the fast join's, the grouped join's)
unsigned long long radix_work_words(const RadixPlan &pl, unsigned long long s_runs);
// Partitioned rows are packed: 16 B {key, pay} (wide) or 8 B key << 32 | row id (narrow).
hipError_t radix_partition(const SrcDev &src, bool wide, const RadixPlan &pl, const RadixWork &ws,
                           const BucketSet &out, hipStream_t st);
size_t radix_item_desc_bytes();
// work_start: >= radix_work_words words; desc: >= radix_join_items * radix_item_desc_bytes()
// sample: the build side's {rows, repeats} from radix_sample (device memory,
// may be null = "unique"); stream = the probe side is many times the build
// side (C2): int64 rows take the larger-sub-chunk shape.  The kernel that
// joins follows from (wide, stream, sample) alone: join_kernel_choice.
// nparts >= 0: join that many partitions (r.rstart / s.rstart views of a
// sub-range) instead of the plan's 2^total_bits.
hipError_t radix_join(bool wide, const RadixPlan &pl, const RadixWork &ws, const BucketSet &r, const BucketSet &s,
                      unsigned long long s_runs, unsigned *work_start, void *desc, void *out_r, void *out_s, long long cap,
                      unsigned long long *counter, unsigned long long *dup_flag, bool count_only, hipStream_t st,
                      const unsigned long long *sample, bool stream, int nparts = -1);
// Folded routing's send side: rows (int64 columns or packed tuples) grouped
// by the top rbits (<= 9) of radix_hash into out_tuples, exact and contiguous
// per bin, bins in order; counts[2^rbits] their sizes.  One EXACT partition
// pass (k_pass's tiles, line tails and loads) behind a key histogram; hist
// and scan_sums: radix_route_scratch(n, rbits) and exclusive_scan_sums(that)
// u64 each.
size_t radix_route_scratch(long long n, int rbits);
hipError_t radix_route(const SrcDev &src, int rbits, void *out_tuples, unsigned long long *counts,
                       unsigned long long *hist, unsigned long long *scan_sums, hipStream_t st);
// Folded multi-GPU routing: `tuples` (packed int64 {key, payload}) were
// routed by the top pl.skip + pl.bits[0] bits of radix_hash, so they arrive
// already split into the plan's first-pass segments: for each of nsrc sources
// in order, that source's rows of segments 0 .. nseg-1 (cnt[s * nseg + b]
// rows each).  Runs the plan's second pass only (pl.passes == 2) into `out`.
hipError_t radix_partition_routed(const void *tuples, long long n, const unsigned long long *cnt, int nsrc, int nseg,
                                  const RadixPlan &pl, const RadixWork &ws, const BucketSet &out, hipStream_t st);
// After R's partition: sample up to 64 build partitions for repeated keys,
// adding {rows sampled, rows whose key repeated} into sample[0..1] (zeroed by
// the caller).  Deterministic for given data.
hipError_t radix_sample(bool wide, const RadixPlan &pl, const BucketSet &r, unsigned long long *sample,
                        hipStream_t st);
// The exact "build keys repeat" answer for the whole build side r (the
// plan's 2^total_bits partitions): k_join_b's DETECT build over one item per
// non-empty partition (a work map rebuilt from r.rstart alone, in work_start /
// desc), the partitions it cannot take by k_join's list-mode build (repeats
// inside each of its build rounds); sets *dup_flag.  The joins themselves only
// flag repeats of partitions they built (k_join_b: that a probe row met).
hipError_t radix_detect(bool wide, const RadixPlan &pl, const RadixWork &ws, const BucketSet &r, unsigned *work_start,
                        void *desc, unsigned long long *dup_flag, const unsigned long long *sample, hipStream_t st);
// HJ_JOIN_KERNEL_* of the radix join for this shape and sample (host mirror
// of the device-side choice)
int join_kernel_choice(bool wide, bool stream, unsigned long long rows, unsigned long long repeats);

// Routing fan-out limit: k_part_scatter (> 512 parts) keeps 12 B of LDS
// counters per part, k_part_hist 4 B (<= 96 KiB of the 160 KiB).
constexpr int kMaxRouteParts = 8192;
constexpr int kMaxRouteSources = 64;   // ranks a folded routing's receiver takes rows from
// rbits > 0: parts = the top rbits of radix_hash (nparts = 2^rbits), else an
// fmix64 multiply-shift onto [0, nparts) independent of the radix bits.
hipError_t launch_partition(const SrcDev &src, int nparts, void *out_tuples,
                            unsigned long long *counts, unsigned long long *cursors,
                            hipStream_t st, int rbits = 0);

// exclusive scan of a u64 array in place (hj_radix.hip); sums >= exclusive_scan_sums(len)
hipError_t exclusive_scan_u64(unsigned long long *v, unsigned long long len, unsigned long long *sums,
                              hipStream_t st);
size_t exclusive_scan_sums(unsigned long long len);

// selection (hj_kernels.hip): tiles >= select_tiles(n) + 1 words, sums >= exclusive_scan_sums(tiles)
size_t select_tiles(long long n);
hipError_t launch_select_f32(const float *in, long long n, int op, float c, float *out, long long *out_row,
                             long long cap, unsigned long long *count, unsigned long long *tiles,
                             unsigned long long *sums, hipStream_t st);
hipError_t launch_select_i64(const long long *in, long long n, int op, long long c, long long *out,
                             long long *out_row, long long cap, unsigned long long *count, unsigned long long *tiles,
                             unsigned long long *sums, hipStream_t st);
// copy floors (hj_dev_stream_copy): shape 0 persistent (cus workgroups), 1 flat
hipError_t launch_stream_copy(const void *in, void *out, long long rows, int shape, int cus, hipStream_t st);
// the partition pass's write pattern (buckets of bucket_bytes: 4-16 KiB) vs a
// flat write of the same bytes into a fresh buffer (>= cus x 256 buckets):
// *ratio = pattern time / flat time, ~1.0 at a good physical placement,
// 1.25-1.35 at a bad one (hj_kernels.hip)
hipError_t placement_probe(void *buf, size_t bytes, size_t bucket_bytes, int cus, float *ratio);

// nested-loop.mlir result rows (hj_kernels.hip)
hipError_t launch_key_col_i32(const int *t, long long rows, long long ld, int *out, hipStream_t st);
hipError_t launch_gather_rows_i32(const int *x, long long ldx, int cx, const int *y, long long ldy, int cy,
                                  const int *px, const int *py, const unsigned long long *count, long long cap,
                                  int *out, long long ldo, hipStream_t st);

hipError_t launch_gen_pkfk(unsigned long long seed, long long NR, unsigned long long hit_thr,
                           long long r0, long long nr, long long *rkey, long long *rpay,
                           long long s0, long long ns, long long *skey, long long *spay,
                           hipStream_t st);
hipError_t launch_gen_zipf(unsigned long long seed, const ZipfParams &z, long long s0, long long ns, long long *skey,
                           long long *spay, hipStream_t st);
hipError_t launch_gen_uniform_i64(unsigned long long seed, unsigned long long stream_id,
                                  long long lo, long long hi, long long i0, long long n,
                                  long long *key, long long *pay, hipStream_t st);
hipError_t launch_gen_uniform_i32(unsigned long long seed, unsigned long long stream_id,
                                  int lo, int hi, long long i0, long long n, int *key,
                                  hipStream_t st);

}  // namespace hj
