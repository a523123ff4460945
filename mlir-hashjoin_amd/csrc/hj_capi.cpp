// hj_capi.cpp -- the C ABI of libhj.so (declared in include/hj.h).
//
// Host side of the join, C++ over HIP.  It replaces the reference's host
// functions inside join_v1.mlir / join_v2.mlir (@allocateHashTable,
// @initializeHashTable, @buildTable, @countRows, @probeRelation: join_v2.mlir:
// 25-199) and the @main data path (:607-730).  The reference lowers every
// gpu.launch_func to stream create -> module load -> launch -> unload ->
// synchronize -> destroy (join_v2.ll:133-172); here one context keeps its
// workspace and every device phase is an asynchronous launch on the caller's
// stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <functional>
#include <thread>
#include <type_traits>
#include <vector>

#include "hj.h"
#include "hj_internal.h"

using hj::kNarrow;
using hj::kWide;

namespace {

thread_local std::string g_err;

int fail(int code, const char *file, int line, const std::string &msg) {
    g_err = std::string(file) + ":" + std::to_string(line) + ": " + msg;
    if (code == HJ_ERR_HIP || code == HJ_ERR_NOMEM) std::fprintf(stderr, "hj: %s\n", g_err.c_str());
    return code;
}

#define HJ_FAIL(code, msg) return fail((code), __FILE__, __LINE__, (msg))
#define HJ_HIP(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(HJ_ERR_HIP, __FILE__, __LINE__, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
// A radix call that fails may leave the one-launch scan's tile words set
// (they are zeroed only on allocation, and every completed scan clears
// them): reset them on the stream before reporting the failure.
#define HJ_RADIX(ctx, st, expr)                                                                    \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            if ((ctx)->scan_state.p) (void)hipMemsetAsync((ctx)->scan_state.p, 0, (ctx)->scan_state.bytes, (st)); \
            return fail(HJ_ERR_HIP, __FILE__, __LINE__, std::string(#expr) + ": " + hipGetErrorString(e_)); \
        }                                                                                          \
    } while (0)
#define HJ_TRY(expr)              \
    do {                          \
        int r_ = (expr);          \
        if (r_ != HJ_OK) return r_; \
    } while (0)

int ceil_log2(unsigned long long x) {
    int b = 0;
    while ((1ull << b) < x) ++b;
    return b;
}

// Table capacity for n build rows: power of two >= 2n (load factor <= 0.5),
// at least 16 slots.
int table_bits(int64_t n) {
    const unsigned long long want = 2ull * (unsigned long long)(n > 0 ? n : 1);
    int b = ceil_log2(want);
    return b < 4 ? 4 : b;
}

// HJ_TRACE=1: synchronise and log every phase to stderr (diagnostics).
bool trace_on() {
    static const bool on = getenv("HJ_TRACE") != nullptr;
    return on;
}
void trace(const char *what, hipStream_t st, long long n = -1) {
    if (!trace_on()) return;
    const hipError_t e = hipStreamSynchronize(st);
    std::fprintf(stderr, "hj trace: %s n=%lld -> %s\n", what, n, hipGetErrorString(e));
}

enum Ev { kEvInit0, kEvInit1, kEvBuild1, kEvProbe0, kEvProbeMid, kEvProbe1, kEvPart0, kEvPart1, kEvCount };

// Build sides at least this large use the radix-partitioned join (LDS
// tables); smaller ones a global linear-probing table (HJ_STRATEGY_AUTO).
constexpr int64_t kRadixMinRows = 1ll << 21;
// AUTO with a smaller build side whose global table outgrows one XCD's L2
// (>= 2^18 rows = 8 MiB of slots) also radix-partitions R at build time
// (~20 us); a probe side of >= 2^24 rows then takes the radix join: the
// global probe of a MALL-resident table is latency-bound (~40 G rows/s,
// C2 26.4 ms) while partition + LDS join streams (C2 19.7 ms).
constexpr int64_t kDualMinBuildRows = 1ll << 18;
constexpr int64_t kRadixProbeMinRows = 1ll << 24;
// A probe side KNOWN before the build (hj_ctx_probe_hint) takes the radix
// join alone from these many rows on: 2^22 for build sides of >= 2^20 rows,
// else 2^24 (round 6, profiles/r06/r06sc_strategy_cross.txt: 2^20 x 2^22
// radix 0.204 ms, global 0.233; 2^19 x 2^21 global 0.134, radix 0.166).
// Without a hint the dual build keeps kRadixProbeMinRows: its global table
// is already paid for, and its global probe beats partitioning S below 2^24.
inline int64_t radix_probe_min_rows(int64_t n_build) { return n_build >= (1ll << 20) ? 1ll << 22 : kRadixProbeMinRows; }

struct Buf {
    void *p = nullptr;
    size_t bytes = 0;
};

// Device buffers of one radix bucket set (hj::BucketSet).
struct SetBufs {
    Buf rows, bbin, bfill, runs, rstart;
    unsigned max_buckets = 0;
    unsigned long long max_rows = 0;
    unsigned long long max_runs = 0;
};

}  // namespace

struct hj_ctx {
    int device = 0;
    void *table = nullptr;
    size_t table_bytes = 0;
    unsigned long long *side = nullptr;   // wide-layout side list (INT64_MIN keys)
    size_t side_rows = 0;
    unsigned long long *meta = nullptr;   // [0] side count, [1] dup flag, [8..] partition cursors
    size_t meta_words = 0;
    // current table
    int layout = -1;
    int bits = 0;
    int64_t n_build = 0;
    int strategy = HJ_STRATEGY_AUTO;   // requested
    int radix_bits = 0;                // 0: planner chooses
    int used = 0;                      // HJ_STRATEGY_GLOBAL / _RADIX of the current build
    bool dual = false;                 // global build whose R is ALSO radix-partitioned (probe-time choice)
    int64_t probe_hint = -1;           // expected probe rows (hj_ctx_probe_hint; < 0 unknown)
    int probe_used = -1;               // strategy of the last probe (-1: none since the build)
    // radix-join workspace (hj_radix.hip)
    hj::RadixPlan plan;
    SetBufs rset, sset, tset;   // R and S final partitions, ping set of multi-pass plans
    Buf nb, pcur, rcur, tile_start, tile_owner, tdesc, wstart, work_start, work_desc, scan_sums, scan_state, raw_cnt;
    Buf slow;   // global-table probe: tiles for the general path
    Buf rows_kx, rows_ky, rows_px, rows_py;   // row materialisation: key columns, pair row ids
    Buf sel_tiles, sel_sums;                  // selection: per-tile counts (then offsets), scan sums
    Buf route_hist, route_sums;               // folded routing: (bin, workgroup) slot bases, scan sums
    // timing: the records go to event set `cur`.  Accumulating mode
    // (hj_ctx_timing_accumulate) moves to the next set of a ring at every
    // build and reads a set back only when the ring comes round to it again
    // or the totals are asked for, so back-to-back build + probe steps need
    // no host synchronisation between them.
    static constexpr int kEvSets = 64;
    struct EvSet {
        hipEvent_t ev[kEvCount];
        bool rec[4] = {false, false, false, false};
        bool rec_mid = false;
    };
    bool timing = false;
    bool ev_ready = false;   // set 0 created
    int ev_made = 0;         // sets created (1, or all of them once accumulating was asked for)
    bool acc = false;        // accumulating
    int cur = 0;
    EvSet sets[kEvSets];
    double tot[6] = {0, 0, 0, 0, 0, 0};
    long long tot_sets = 0;
    EvSet &evs() { return sets[cur]; }
    // host memref path.  One host thread at a time per context: every host
    // entry point holds host_mu (they share the staging buffers, dcount and
    // host_stream).
    std::mutex host_mu;
    hipStream_t host_stream = nullptr;
    static constexpr int kDbufs = 10;
    void *dbuf[kDbufs] = {};
    size_t dbuf_bytes[kDbufs] = {};
    unsigned long long *dcount = nullptr;
    // count -> probe reuse (join_v1.mlir:110-176: @countRows leaves its table
    // for @probeRelation).  hj_count_* uploads both relations into dbuf[6],
    // dbuf[7], builds, and COUNTS (no pairs); it keeps the built table, the
    // staged probe side and a content digest of each input memref.  The next
    // hj_probe_* digests its memrefs on the host (no upload) and, when both
    // digests match, only probes into M-row buffers and downloads.  Any other
    // build on the context invalidates it.
    struct Digest {
        unsigned long long a = 0, b = 0;
        bool operator==(const Digest &o) const { return a == o.a && b == o.b; }
    };
    struct Memo {
        bool valid = false;
        int layout = -1;
        int64_t nr = 0, ns = 0;
        Digest dr, ds;   // R (keys, payloads), S (keys, payloads)
        int64_t m = 0;
        int reuse = 0;   // HJ_REUSE_* the count ran under
        // HJ_REUSE_EXACT: the count's inputs, compacted (keys, then payloads)
        std::vector<unsigned char> cr, cs;
        // drop the memo; the EXACT-mode copies (GBs at 2^28 rows) give
        // their memory back unless `keep` (a count about to refill them)
        void invalidate(bool keep = false) {
            valid = false;
            if (keep) {
                cr.clear();
                cs.clear();
            } else {
                std::vector<unsigned char>().swap(cr);
                std::vector<unsigned char>().swap(cs);
            }
        }
    } memo;
    long long memo_hits = 0;
    // the last radix probe's shape, for hj_ctx_join_kernel (the kernel itself
    // follows from these and the build-time sample in meta[2..3])
    bool join_ran = false, join_wide = false, join_stream = false;
    bool routed = false;   // the current build came from hj_dev_build_routed_i64 (plan.skip owner bits)
    bool dup_checked = false;   // hj_ctx_build_has_duplicates ran its DETECT build for this build
    bool host_building = false;  // host_join's build is running (do_build keeps the memo's input copies)
};

namespace {

int set_device(hj_ctx *c) {
    HJ_HIP(hipSetDevice(c->device));
    return HJ_OK;
}

int ensure_meta(hj_ctx *c, size_t words) {
    if (c->meta_words >= words) return HJ_OK;
    if (c->meta) HJ_HIP(hipFree(c->meta));
    c->meta = nullptr;
    size_t w = words < 64 ? 64 : words;
    if (hipMalloc(&c->meta, w * sizeof(unsigned long long)) != hipSuccess) HJ_FAIL(HJ_ERR_NOMEM, "hipMalloc meta");
    HJ_HIP(hipMemset(c->meta, 0, w * sizeof(unsigned long long)));
    c->meta_words = w;
    return HJ_OK;
}

int ensure_table(hj_ctx *c, int64_t n, int layout) {
    const int bits = table_bits(n);
    const size_t need = (size_t(1) << bits) * (layout == kWide ? 16 : 8);
    if (c->table_bytes < need) {
        if (c->table) HJ_HIP(hipFree(c->table));
        c->table = nullptr;
        c->table_bytes = 0;
        if (hipMalloc(&c->table, need) != hipSuccess) HJ_FAIL(HJ_ERR_NOMEM, "hipMalloc table " + std::to_string(need));
        c->table_bytes = need;
    }
    if (layout == kWide && c->side_rows < (size_t)(n > 0 ? n : 1)) {
        if (c->side) HJ_HIP(hipFree(c->side));
        c->side = nullptr;
        const size_t rows = (size_t)(n > 0 ? n : 1);
        if (hipMalloc(&c->side, rows * 8) != hipSuccess) HJ_FAIL(HJ_ERR_NOMEM, "hipMalloc side list");
        c->side_rows = rows;
    }
    return ensure_meta(c, 64);
}

hj::TableDev table_dev(const hj_ctx *c) {
    hj::TableDev t;
    t.slots = c->table;
    t.mask = (1ull << c->bits) - 1ull;
    t.shift = 64 - c->bits;
    t.side = c->side;
    t.meta = c->meta;
    return t;
}

void record(hj_ctx *c, int ev, hipStream_t st) {
    if (c->timing && c->ev_ready) (void)hipEventRecord(c->evs().ev[ev], st);
}

// ms of one event set's phases: init, build, probe, routing partition,
// probe-side partitioning, join (-1: not recorded)
int set_ms(hj_ctx::EvSet &s, float ms[8]) {
    for (int i = 0; i < 8; ++i) ms[i] = -1.0f;
    auto el = [&](int a, int b, float *out) -> int {
        HJ_HIP(hipEventSynchronize(s.ev[b]));
        HJ_HIP(hipEventElapsedTime(out, s.ev[a], s.ev[b]));
        return HJ_OK;
    };
    if (s.rec[0]) HJ_TRY(el(kEvInit0, kEvInit1, &ms[0]));
    if (s.rec[1]) HJ_TRY(el(kEvInit1, kEvBuild1, &ms[1]));
    if (s.rec[2]) HJ_TRY(el(kEvProbe0, kEvProbe1, &ms[2]));
    if (s.rec[3]) HJ_TRY(el(kEvPart0, kEvPart1, &ms[3]));
    if (s.rec[2]) {
        if (s.rec_mid) {
            HJ_TRY(el(kEvProbe0, kEvProbeMid, &ms[4]));
            HJ_TRY(el(kEvProbeMid, kEvProbe1, &ms[5]));
        } else {
            ms[4] = 0.0f;
            ms[5] = ms[2];
        }
    }
    return HJ_OK;
}

// accumulating mode: add set k's phases to the totals and forget them
int fold_set(hj_ctx *c, int k) {
    hj_ctx::EvSet &s = c->sets[k];
    if (!(s.rec[0] || s.rec[1] || s.rec[2] || s.rec[3])) return HJ_OK;
    float ms[8];
    HJ_TRY(set_ms(s, ms));
    for (int i = 0; i < 6; ++i)
        if (ms[i] > 0.0f) c->tot[i] += ms[i];
    ++c->tot_sets;
    s.rec[0] = s.rec[1] = s.rec[2] = s.rec[3] = s.rec_mid = false;
    return HJ_OK;
}

// a build starts a step: accumulating, it records into the ring's next set
// (summing what that set held first: a ring's length of steps ago)
int timing_advance(hj_ctx *c) {
    if (!c->acc || !c->timing) return HJ_OK;
    c->cur = (c->cur + 1) % hj_ctx::kEvSets;
    return fold_set(c, c->cur);
}

int ensure_buf(Buf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return HJ_OK;
    if (b.p) HJ_HIP(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    if (hipMalloc(&b.p, bytes) != hipSuccess) HJ_FAIL(HJ_ERR_NOMEM, "hipMalloc radix workspace " + std::to_string(bytes));
    b.bytes = bytes;
    return HJ_OK;
}

void free_buf(Buf &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

// Placement of the bucket sets' row buffers (the partition passes' only
// destinations).  The passes write each tile's rows as one line into each of
// ~512 open buckets per workgroup, and into some physical placements of a
// buffer that pattern runs 25-35 % slower than a flat write (a property of
// the allocation, bimodal: 4-10 of 12 fresh 6 GiB buffers on one box,
// profiles/r05/r05t_place_micro.txt; the same pass into two such buffers: 1.46
// vs 1.76 ms).  A large row buffer is therefore probed when it is allocated
// (hj::placement_probe: the pass's pattern against a flat write, ~2 ms) and
// redrawn while it is slow: up to kPlaceDraws allocations.  Rejected draws
// are held (so the allocator cannot hand the same memory back), at most
// kPlaceHeld of them at once -- a further reject frees the oldest held one --
// and another draw is taken only while free memory is at least kPlaceSpare
// times the buffer (the same rule as hashjoin.join.placed_rows); the best draw
// is kept and the rest freed.  A buffer whose draws stopped before a good one
// is a give-up, counted (and why) in hj_placement_stats_ex and in every bench
// line.  HJ_PLACEMENT_PROBE=0 turns it off.
// (smaller buffers, and 4-KiB buckets (i32 rows' final sets), probe too short
// a pattern to judge: REF-B's sets were rejected 9 draws in 10 at unchanged
// pass times, profiles/r05/r05y_*)
constexpr size_t kPlaceMinBytes = size_t(1) << 30;
constexpr size_t kPlaceMinBucket = size_t(8) << 10;
constexpr int kPlaceDraws = 24;   // (a box where 86 % of draws were slow: r05_final)
constexpr int kPlaceHeld = 2;     // rejected draws held at once
constexpr size_t kPlaceSpare = 3; // another draw while free memory >= 3 x the buffer
std::atomic<float> g_place_good{1.12f};   // pattern / flat at a good placement: 0.98-1.05
struct PlaceStats {
    long long probes = 0, rejected = 0, gave_up = 0, gave_up_low_mem = 0, held_max = 0;
    double worst_kept = 0.0, last_kept = 0.0;
};
PlaceStats g_place;
std::mutex g_place_mu;

bool placement_probe_on() {
    static const bool on = [] {
        const char *e = getenv("HJ_PLACEMENT_PROBE");
        return !(e && e[0] == '0');
    }();
    return on;
}

int ensure_rows(Buf &b, size_t bytes, size_t bucket_bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return HJ_OK;
    if (bytes < kPlaceMinBytes || bucket_bytes < kPlaceMinBucket || !placement_probe_on()) return ensure_buf(b, bytes);
    free_buf(b);
    int dev = 0, cus = 0;
    HJ_HIP(hipGetDevice(&dev));
    HJ_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const float good = g_place_good.load();
    std::vector<Buf> held;   // rejected draws still held (oldest first)
    Buf best;
    float best_r = 1e30f;
    int draws = 0;
    long long rejected = 0, held_max = 0;
    bool low_mem = false;
    for (; draws < kPlaceDraws; ++draws) {
        if (draws > 0) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < kPlaceSpare * bytes) {
                (void)hipGetLastError();
                low_mem = true;
                break;
            }
        }
        Buf cand;
        if (hipMalloc(&cand.p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            low_mem = true;
            break;
        }
        cand.bytes = bytes;
        float r = 0.0f;
        if (hj::placement_probe(cand.p, bytes, bucket_bytes, cus, &r) != hipSuccess) {
            (void)hipGetLastError();
            r = 0.0f;   // no verdict: take it
        }
        Buf rej;
        if (r < best_r) {
            rej = best;
            best = cand;
            best_r = r;
        } else {
            rej = cand;
        }
        if (rej.p) {
            ++rejected;
            held.push_back(rej);
            if ((int)held.size() > kPlaceHeld) {
                free_buf(held.front());
                held.erase(held.begin());
            }
            if ((long long)held.size() > held_max) held_max = (long long)held.size();
        }
        if (best_r <= good) {
            ++draws;
            break;
        }
    }
    for (Buf &x : held) free_buf(x);
    if (!best.p) HJ_FAIL(HJ_ERR_NOMEM, "hipMalloc radix rows " + std::to_string(bytes));
    b = best;
    const bool gave_up = best_r > good;
    {
        std::lock_guard<std::mutex> lk(g_place_mu);
        g_place.probes += draws;
        g_place.rejected += rejected;
        if (gave_up) {
            ++g_place.gave_up;
            if (low_mem) ++g_place.gave_up_low_mem;
        }
        if (held_max > g_place.held_max) g_place.held_max = held_max;
        g_place.last_kept = best_r;
        if (best_r > g_place.worst_kept) g_place.worst_kept = best_r;
    }
    if (trace_on() || (gave_up && low_mem))
        std::fprintf(stderr, "hj %s: rows placement %zu B: %d draw(s), kept pattern/flat %.3f%s\n",
                     trace_on() ? "trace" : "note", bytes, draws, (double)best_r,
                     gave_up ? (low_mem ? " (gave up: free memory below 3x the buffer)" : " (gave up: draws spent)") : "");
    return HJ_OK;
}

int ensure_set(SetBufs &sb, const hj::RadixNeed &need, size_t esz, size_t P, int pbl) {
    if (need.buckets > 0xFFFFFFF0ull) HJ_FAIL(HJ_ERR_CAPACITY, "radix partition: too many buckets");
    HJ_TRY(ensure_rows(sb.rows, (size_t)need.rows * esz, esz << pbl));
    HJ_TRY(ensure_buf(sb.bbin, (size_t)need.buckets * 4));
    HJ_TRY(ensure_buf(sb.bfill, (size_t)need.buckets * 4));
    HJ_TRY(ensure_buf(sb.rstart, (P + 1) * 8));
    // capacity actually held (buffers may be larger than this need)
    size_t cap = sb.bbin.bytes / 4;
    if (sb.bfill.bytes / 4 < cap) cap = sb.bfill.bytes / 4;
    sb.max_buckets = (unsigned)(cap < 0xFFFFFFF0ull ? cap : 0xFFFFFFF0ull);
    sb.max_rows = sb.rows.bytes / esz;
    // a bucket of f rows lists ceil(f / 64) runs: <= rows / 64 + buckets
    HJ_TRY(ensure_buf(sb.runs, (size_t)((sb.max_rows >> hj::kRunLog) + sb.max_buckets + hj::kRunPad) * 8));
    sb.max_runs = sb.runs.bytes / 8 - hj::kRunPad;
    return HJ_OK;
}

hj::BucketSet bucket_set(SetBufs &sb) {
    hj::BucketSet b;
    b.rows = sb.rows.p;
    b.bbin = (unsigned *)sb.bbin.p;
    b.bfill = (unsigned *)sb.bfill.p;
    b.runs = (unsigned long long *)sb.runs.p;
    b.rstart = (unsigned long long *)sb.rstart.p;
    b.max_buckets = sb.max_buckets;
    b.max_rows = sb.max_rows;
    b.max_runs = sb.max_runs;
    return b;
}

// Partition scratch for n rows under plan pl (shared by R and S), plus the
// relation's own final set.
int ensure_radix_scratch(hj_ctx *c, SetBufs &fin, int64_t n, size_t esz, const hj::RadixPlan &pl) {
    const size_t P = size_t(1) << pl.total_bits;
    HJ_TRY(ensure_set(fin, hj::radix_need(n, pl, true), esz, P, hj::kFinalPbl));
    if (pl.passes > 1) HJ_TRY(ensure_set(c->tset, hj::radix_need(n, pl, false), esz, P, hj::kPassPbl));
    HJ_TRY(ensure_buf(c->nb, 16));
    HJ_TRY(ensure_buf(c->pcur, (P + 1) * 8));
    HJ_TRY(ensure_buf(c->rcur, (P + 1) * 8));
    HJ_TRY(ensure_buf(c->tile_start, (P + 1) * 4));
    HJ_TRY(ensure_buf(c->tile_owner, (size_t)hj::radix_tiles(n, (int)P) * 4));
    HJ_TRY(ensure_buf(c->tdesc, (size_t)hj::radix_tiles(n, (int)P) * 16));
    HJ_TRY(ensure_buf(c->wstart, 1025 * 4));
    // work map: P + 1 chunk starts, then the item -> partition owner list
    const size_t items = (size_t)hj::radix_join_items(pl, fin.max_runs);
    // work_start (P + 1) + work_owner (items) + two deferred-item lists (1 + items each)
    HJ_TRY(ensure_buf(c->work_start, (size_t)hj::radix_work_words(pl, fin.max_runs) * 4));
    HJ_TRY(ensure_buf(c->work_desc, items * hj::radix_item_desc_bytes()));
    HJ_TRY(ensure_buf(c->scan_sums, ((P + 1) / 8192 + 2) * 8));
    HJ_TRY(ensure_buf(c->raw_cnt, 2 * hj::kRawCntWords * 8));
    {
        // the one-launch scan's tile words: zero on allocation, and every
        // scan leaves them zero
        const size_t had = c->scan_state.bytes;
        HJ_TRY(ensure_buf(c->scan_state, ((P + 1) / 1024 + 4) * 8));
        if (c->scan_state.bytes != had) HJ_HIP(hipMemset(c->scan_state.p, 0, c->scan_state.bytes));
    }
    return HJ_OK;
}

hj::RadixWork radix_work(hj_ctx *c) {
    hj::RadixWork w;
    w.tmp = bucket_set(c->tset);
    w.nb = (unsigned *)c->nb.p;
    w.pcur = (unsigned long long *)c->pcur.p;
    w.rcur = (unsigned long long *)c->rcur.p;
    w.tile_start = (unsigned *)c->tile_start.p;
    w.tile_owner = (unsigned *)c->tile_owner.p;
    w.tdesc = c->tdesc.p;
    w.wstart = (unsigned *)c->wstart.p;
    w.scan_sums = (unsigned long long *)c->scan_sums.p;
    w.scan_state = (unsigned long long *)c->scan_state.p;
    w.raw_cnt = (unsigned long long *)c->raw_cnt.p;
    return w;
}

int choose_strategy(const hj_ctx *c, int64_t n_build) {
    if (c->strategy == HJ_STRATEGY_GLOBAL || c->strategy == HJ_STRATEGY_RADIX) return c->strategy;
    if (n_build >= kRadixMinRows) return HJ_STRATEGY_RADIX;
    if (n_build >= kDualMinBuildRows && c->probe_hint >= radix_probe_min_rows(n_build)) return HJ_STRATEGY_RADIX;
    return HJ_STRATEGY_GLOBAL;
}

int do_build(hj_ctx *c, int layout, const hj::SrcDev &src, hipStream_t st) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (src.n < 0 || (src.n > 0 && !src.key) || (src.form == hj::kCols64 && src.n > 0 && !src.pay))
        HJ_FAIL(HJ_ERR_ARG, "bad build relation");
    if (layout == kNarrow && src.n > 0x7fffffffll) HJ_FAIL(HJ_ERR_ARG, "i32 row ids: build side must have < 2^31 rows");
    HJ_TRY(set_device(c));
    HJ_TRY(ensure_meta(c, 64));
    HJ_TRY(timing_advance(c));
    c->layout = layout;
    c->n_build = src.n;
    c->used = choose_strategy(c, src.n);
    c->probe_used = -1;
    c->join_ran = false;
    c->dup_checked = false;
    c->routed = false;
    // (hj_count_*'s kept table is gone; a host join's own build keeps the
    // EXACT copies it has just taken of its inputs)
    if (c->host_building) c->memo.valid = false;
    else c->memo.invalidate();
    // (a known probe side settled the strategy in choose_strategy: no dual)
    c->dual = c->used == HJ_STRATEGY_GLOBAL && c->strategy == HJ_STRATEGY_AUTO && src.n >= kDualMinBuildRows &&
              c->probe_hint < 0;
    if (c->used == HJ_STRATEGY_RADIX || c->dual) {
        // build = radix-partition R by the top key-hash bits (tables are built
        // per partition in LDS at probe time)
        const bool wide = layout == kWide;
        const size_t esz = wide ? 16 : 8;   // packed partitioned rows
        c->plan = hj::radix_plan(src.n, c->radix_bits, wide);
        HJ_TRY(ensure_radix_scratch(c, c->rset, src.n, esz, c->plan));
        record(c, kEvInit0, st);
        // meta[0] side count, [1] dup flag, [2..3] the build-side sample
        HJ_HIP(hipMemsetAsync(c->meta, 0, 4 * sizeof(unsigned long long), st));
        record(c, kEvInit1, st);
        trace("build: workspace", st, src.n);
        HJ_RADIX(c, st, hj::radix_partition(src, wide, c->plan, radix_work(c), bucket_set(c->rset), st));
        // repeated build keys, sampled: decides the join kernel (radix_join)
        HJ_HIP(hj::radix_sample(wide, c->plan, bucket_set(c->rset), c->meta + 2, st));
        trace("build: R partitioned", st, (long long)c->plan.total_bits);
        if (!c->dual) {
            record(c, kEvBuild1, st);
            c->evs().rec[0] = c->evs().rec[1] = c->timing;
            return HJ_OK;
        }
    }
    HJ_TRY(ensure_table(c, src.n, layout));
    c->bits = table_bits(src.n);
    const hj::TableDev t = table_dev(c);
    if (!c->dual) record(c, kEvInit0, st);   // (dual: the build phase starts at R's partition)
    HJ_HIP(hj::launch_init(t, layout, 1ull << c->bits, st));
    if (!c->dual) record(c, kEvInit1, st);
    HJ_HIP(hj::launch_build(t, layout, src, st));
    record(c, kEvBuild1, st);
    c->evs().rec[0] = c->evs().rec[1] = c->timing;
    return HJ_OK;
}

int do_probe(hj_ctx *c, int layout, const hj::SrcDev &src, void *out_r, void *out_s, int64_t cap,
             uint64_t *d_count, bool count_only, hipStream_t st) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (c->layout != layout) HJ_FAIL(HJ_ERR_STATE, "probe without a matching build");
    if (!d_count) HJ_FAIL(HJ_ERR_ARG, "null count pointer");
    if (src.n < 0 || (src.n > 0 && !src.key)) HJ_FAIL(HJ_ERR_ARG, "bad probe relation");
    if (!count_only && (cap < 0 || (cap > 0 && (!out_r || !out_s)))) HJ_FAIL(HJ_ERR_ARG, "bad output");
    HJ_TRY(set_device(c));
    // (the radix join zeroes the counter in its work-map kernel: no memset launch)
    const bool radix = c->used == HJ_STRATEGY_RADIX || (c->dual && src.n >= kRadixProbeMinRows);
    c->probe_used = radix ? HJ_STRATEGY_RADIX : HJ_STRATEGY_GLOBAL;
    c->join_ran = false;
    if (radix) {
        const bool wide = layout == kWide;
        const size_t esz = wide ? 16 : 8;
        trace("probe: enter", st, src.n);
        HJ_TRY(ensure_radix_scratch(c, c->sset, src.n, esz, c->plan));
        trace("probe: workspace", st, (long long)c->sset.max_buckets);
        record(c, kEvProbe0, st);
        HJ_RADIX(c, st, hj::radix_partition(src, wide, c->plan, radix_work(c), bucket_set(c->sset), st));
        trace("probe: S partitioned", st, src.n);
        record(c, kEvProbeMid, st);
        // the kernel: a function of (row width, size ratio, build-time sample)
        const bool stream = src.n >= 8 * c->n_build;
        HJ_RADIX(c, st, hj::radix_join(wide, c->plan, radix_work(c), bucket_set(c->rset), bucket_set(c->sset), c->sset.max_runs,
                              (unsigned *)c->work_start.p, c->work_desc.p, out_r, out_s, count_only ? 0 : cap,
                              (unsigned long long *)d_count, c->meta + 1, count_only, st, c->meta + 2, stream));
        c->join_ran = true;
        c->join_wide = wide;
        c->join_stream = stream;
        trace("probe: joined", st, cap);
        record(c, kEvProbe1, st);
        c->evs().rec[2] = c->timing;
        c->evs().rec_mid = c->timing;
        return HJ_OK;
    }
    HJ_HIP(hipMemsetAsync(d_count, 0, sizeof(uint64_t), st));
    hj::OutDev out;
    out.r = out_r;
    out.s = out_s;
    out.cap = count_only ? 0 : cap;
    out.counter = (unsigned long long *)d_count;
    record(c, kEvProbe0, st);
    size_t slow_cap = hj::probe_tiles(src.n);
    HJ_TRY(ensure_buf(c->slow, slow_cap * sizeof(unsigned)));
    HJ_HIP(hj::launch_probe(table_dev(c), layout, src, out, count_only, (unsigned *)c->slow.p, slow_cap, st));
    record(c, kEvProbe1, st);
    c->evs().rec[2] = c->timing;
    c->evs().rec_mid = false;
    return HJ_OK;
}

int do_partition(hj_ctx *c, const hj::SrcDev &src, int nparts, int64_t *out, uint64_t *d_counts, hipStream_t st) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (nparts < 1 || nparts > hj::kMaxRouteParts) HJ_FAIL(HJ_ERR_ARG, "nparts must be in [1, 8192]");
    if (src.n < 0 || (src.n > 0 && (!src.key || !out))) HJ_FAIL(HJ_ERR_ARG, "bad partition input");
    if (!d_counts) HJ_FAIL(HJ_ERR_ARG, "null counts");
    HJ_TRY(set_device(c));
    HJ_TRY(ensure_meta(c, 8 + (size_t)nparts));
    record(c, kEvPart0, st);
    HJ_HIP(hj::launch_partition(src, nparts, out, (unsigned long long *)d_counts, c->meta + 8, st));
    record(c, kEvPart1, st);
    c->evs().rec[3] = c->timing;
    return HJ_OK;
}

hj::SrcDev src_cols64(const int64_t *k, const int64_t *p, int64_t n) {
    hj::SrcDev s;
    s.key = k;
    s.pay = p;
    s.n = n;
    s.row_base = 0;
    s.form = hj::kCols64;
    return s;
}
hj::SrcDev src_packed(const int64_t *t, int64_t n) {
    hj::SrcDev s;
    s.key = t;
    s.pay = nullptr;
    s.n = n;
    s.row_base = 0;
    s.form = hj::kPacked64;
    return s;
}
hj::SrcDev src_col32(const int32_t *k, int64_t n, int64_t row_base) {
    hj::SrcDev s;
    s.key = k;
    s.pay = nullptr;
    s.n = n;
    s.row_base = row_base;
    s.form = hj::kCol32;
    return s;
}

// ---------------------------------------------------------------- host path
std::mutex g_default_mu;
std::atomic<int> g_reuse{HJ_REUSE_DIGEST};   // hj_host_set_reuse
std::map<int, hj_ctx *> g_default;

hj_ctx *default_ctx() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(g_default_mu);
    auto it = g_default.find(dev);
    if (it != g_default.end()) return it->second;
    hj_ctx *c = hj_ctx_create(dev);
    if (c) g_default[dev] = c;
    return c;
}

// nested-loop.mlir (:29-192, @main :195-289) as a hash join plus a row
// gather.  Roles as %table_1_or_2_as_inner (:247): the larger table is the
// outer X (ties: t1), the smaller the inner Y; every pair X[i][0] == Y[j][0]
// yields the row [X[i][0 .. cx), Y[j][1 .. cy)].  Y is the build side (i32
// keys, payload = row id), X probes; pair row ids are staged in ctx buffers
// and k_gather_rows_i32 writes the rows (<= cap of them; *d_count = M).
struct RowTables {
    const int32_t *t1;
    int64_t r1, c1, ld1;
    const int32_t *t2;
    int64_t r2, c2, ld2;
};

int do_join_rows(hj_ctx *c, const RowTables &a, int32_t *out, int64_t ldo, int64_t cap, uint64_t *d_count,
                 bool count_only, hipStream_t st) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (!d_count) HJ_FAIL(HJ_ERR_ARG, "null count pointer");
    if (a.r1 < 0 || a.r2 < 0 || a.c1 < 1 || a.c2 < 1 || a.ld1 < a.c1 || a.ld2 < a.c2)
        HJ_FAIL(HJ_ERR_ARG, "bad table shape");
    if ((a.r1 > 0 && !a.t1) || (a.r2 > 0 && !a.t2)) HJ_FAIL(HJ_ERR_ARG, "null table");
    if (a.r1 > 0x7fffffffll || a.r2 > 0x7fffffffll) HJ_FAIL(HJ_ERR_ARG, "i32 row ids: tables must have < 2^31 rows");
    const bool t2_outer = a.r1 < a.r2;   // nested-loop.mlir:247
    const int32_t *x = t2_outer ? a.t2 : a.t1, *y = t2_outer ? a.t1 : a.t2;
    const int64_t rx = t2_outer ? a.r2 : a.r1, cx = t2_outer ? a.c2 : a.c1, ldx = t2_outer ? a.ld2 : a.ld1;
    const int64_t ry = t2_outer ? a.r1 : a.r2, cy = t2_outer ? a.c1 : a.c2, ldy = t2_outer ? a.ld1 : a.ld2;
    const int64_t oc = cx + cy - 1;
    if (!count_only && (cap < 0 || (cap > 0 && (!out || ldo < oc)))) HJ_FAIL(HJ_ERR_ARG, "bad row output");
    HJ_TRY(set_device(c));
    HJ_TRY(ensure_buf(c->rows_kx, (size_t)(rx > 0 ? rx : 1) * 4));
    HJ_TRY(ensure_buf(c->rows_ky, (size_t)(ry > 0 ? ry : 1) * 4));
    int32_t *kx = (int32_t *)c->rows_kx.p, *ky = (int32_t *)c->rows_ky.p;
    HJ_HIP(hj::launch_key_col_i32(x, rx, ldx, kx, st));
    HJ_HIP(hj::launch_key_col_i32(y, ry, ldy, ky, st));
    HJ_TRY(do_build(c, kNarrow, src_col32(ky, ry, 0), st));
    if (count_only) return do_probe(c, kNarrow, src_col32(kx, rx, 0), nullptr, nullptr, 0, d_count, true, st);
    HJ_TRY(ensure_buf(c->rows_px, (size_t)(cap > 0 ? cap : 1) * 4));
    HJ_TRY(ensure_buf(c->rows_py, (size_t)(cap > 0 ? cap : 1) * 4));
    int32_t *px = (int32_t *)c->rows_px.p, *py = (int32_t *)c->rows_py.p;
    // R payload = Y row, S payload = X row
    HJ_TRY(do_probe(c, kNarrow, src_col32(kx, rx, 0), py, px, cap, d_count, false, st));
    HJ_HIP(hj::launch_gather_rows_i32(x, ldx, (int)cx, y, ldy, (int)cy, px, py, (const unsigned long long *)d_count,
                                      cap, out, ldo, st));
    return HJ_OK;
}

// Experiments/selection.mlir (:34-155) generalised: survivors of v <op> c,
// order-preserving, optional source row ids.
template <class V>
int do_select(hj_ctx *c, const V *in, int64_t n, int op, V value, V *out, int64_t *out_row, int64_t cap,
              uint64_t *d_count, hipStream_t st) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (!d_count) HJ_FAIL(HJ_ERR_ARG, "null count pointer");
    if (n < 0 || (n > 0 && !in)) HJ_FAIL(HJ_ERR_ARG, "bad selection input");
    if (op < HJ_CMP_LT || op > HJ_CMP_NE) HJ_FAIL(HJ_ERR_ARG, "unknown comparison");
    if (cap < 0 || (cap > 0 && !out)) HJ_FAIL(HJ_ERR_ARG, "bad selection output");
    HJ_TRY(set_device(c));
    const size_t nt = hj::select_tiles(n) + 1;
    HJ_TRY(ensure_buf(c->sel_tiles, nt * 8));
    HJ_TRY(ensure_buf(c->sel_sums, hj::exclusive_scan_sums(nt) * 8));
    hipError_t e;
    if constexpr (std::is_same<V, float>::value)
        e = hj::launch_select_f32(in, n, op, value, out, (long long *)out_row, cap, (unsigned long long *)d_count,
                                  (unsigned long long *)c->sel_tiles.p, (unsigned long long *)c->sel_sums.p, st);
    else
        e = hj::launch_select_i64((const long long *)in, n, op, (long long)value, (long long *)out,
                                  (long long *)out_row, cap, (unsigned long long *)d_count,
                                  (unsigned long long *)c->sel_tiles.p, (unsigned long long *)c->sel_sums.p, st);
    HJ_HIP(e);
    return HJ_OK;
}

int dbuf(hj_ctx *c, int i, size_t bytes, void **p) {
    if (bytes == 0) bytes = 16;
    if (c->dbuf_bytes[i] < bytes) {
        if (c->dbuf[i]) HJ_HIP(hipFree(c->dbuf[i]));
        c->dbuf[i] = nullptr;
        c->dbuf_bytes[i] = 0;
        if (hipMalloc(&c->dbuf[i], bytes) != hipSuccess) HJ_FAIL(HJ_ERR_NOMEM, "hipMalloc staging");
        c->dbuf_bytes[i] = bytes;
    }
    *p = c->dbuf[i];
    return HJ_OK;
}

// Copy a strided host memref (aligned + offset, size, stride) into device
// buffer `dst` (contiguous).  shared.cpp reads through the aligned pointer
// (shared.cpp:40, :67, :148); we additionally honour offset and stride.
// (a plain pageable copy: a page-locked staging mirror of d2h below ran the
// count's 537-MB upload slower, 20-21 -> 25-26 ms, profiles/r05/r05zi_*)
template <class T>
int upload(void *dst, const T *aligned, int64_t off, int64_t size, int64_t stride, hipStream_t st) {
    if (size <= 0) return HJ_OK;
    if (!aligned) HJ_FAIL(HJ_ERR_ARG, "null memref");
    const T *base = aligned + off;
    if (stride == 1) {
        HJ_HIP(hipMemcpyAsync(dst, base, sizeof(T) * (size_t)size, hipMemcpyHostToDevice, st));
        HJ_HIP(hipStreamSynchronize(st));
        return HJ_OK;
    }
    std::vector<T> tmp((size_t)size);
    for (int64_t i = 0; i < size; ++i) tmp[(size_t)i] = base[i * stride];
    HJ_HIP(hipMemcpyAsync(dst, tmp.data(), sizeof(T) * (size_t)size, hipMemcpyHostToDevice, st));
    HJ_HIP(hipStreamSynchronize(st));
    return HJ_OK;
}

int host_stream(hj_ctx *c) {
    if (!c->host_stream) HJ_HIP(hipStreamCreateWithFlags(&c->host_stream, hipStreamNonBlocking));
    if (!c->dcount) {
        if (hipMalloc(&c->dcount, 64) != hipSuccess) HJ_FAIL(HJ_ERR_NOMEM, "hipMalloc counter");
    }
    return HJ_OK;
}

// ---- content digests of host memrefs (count -> probe reuse)
// 128 bits from four multiply-rotate lanes over the elements' bytes (lane j
// takes every 4th 8-B word), cut into up to 8 chunks hashed on host threads;
// a changed element changes its lane's state, which no later word undoes
// except by a crafted value.  Memory-bound: ~2^29 B (two 2^24-row int64
// relations) in ~10 ms, overlapped with the upload in hj_count_*.
typedef hj_ctx::Digest Digest;
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t dstep(uint64_t h, uint64_t w) { return rotl64((h ^ w) * 0x9E3779B97F4A7C15ull, 31); }
inline uint64_t fmix(uint64_t k) {
    k ^= k >> 33;
    k *= 0xFF51AFD7ED558CCDull;
    k ^= k >> 33;
    k *= 0xC4CEB9FE1A85EC53ull;
    return k ^ (k >> 33);
}

Digest digest_mem(const void *aligned, int64_t off, int64_t size, int64_t stride, int esz) {
    Digest d;
    d.a = fmix((uint64_t)size * 16 + (uint64_t)esz);
    d.b = fmix(d.a ^ 0x5EEDull);
    if (size <= 0 || !aligned) return d;
    const char *base = (const char *)aligned + off * esz;
    const int64_t bytes = size * esz;
    const unsigned hw = std::thread::hardware_concurrency();
    unsigned T = (unsigned)(bytes >> 22) + 1;   // >= 4 MiB per thread
    if (T > 8) T = 8;
    if (hw && T > hw) T = hw;
    std::vector<Digest> part(T);
    auto work = [&](unsigned t) {
        const int64_t e0 = size * t / T, e1 = size * (t + 1) / T;
        uint64_t h[4] = {0x243F6A8885A308D3ull, 0x13198A2E03707344ull, 0xA4093822299F31D0ull, 0x082EFA98EC4E6C89ull};
        if (stride == 1) {
            const char *p = base + e0 * esz;
            const size_t n = (size_t)(e1 - e0) * (size_t)esz;
            size_t i = 0;
            for (; i + 32 <= n; i += 32) {
                uint64_t w[4];
                std::memcpy(w, p + i, 32);
                for (int j = 0; j < 4; ++j) h[j] = dstep(h[j], w[j]);
            }
            uint64_t w[4] = {0, 0, 0, 0};
            std::memcpy(w, p + i, n - i);
            for (int j = 0; j < 4; ++j) h[j] = dstep(h[j], w[j] ^ (uint64_t)(n - i));
        } else {
            for (int64_t e = e0; e < e1; ++e) {
                uint64_t w = 0;
                std::memcpy(&w, base + e * stride * esz, (size_t)esz);
                h[e & 3] = dstep(h[e & 3], w);
            }
        }
        part[t].a = fmix(h[0]) ^ fmix(h[1] + 0x9E3779B97F4A7C15ull);
        part[t].b = fmix(h[2]) ^ fmix(h[3] + 0x9E3779B97F4A7C15ull);
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    for (unsigned t = 0; t < T; ++t) {
        d.a = fmix(d.a ^ part[t].a) + t;
        d.b = fmix(d.b ^ part[t].b) + t;
    }
    return d;
}

// ---- exact copies (HJ_REUSE_EXACT): the count keeps the inputs' bytes,
// compacted; the probe compares its memrefs with them (same threading as
// digest_mem: up to 8 host threads, >= 4 MiB each).
template <class F>
void chunked(int64_t size, int esz, F &&work) {
    const unsigned hw = std::thread::hardware_concurrency();
    unsigned T = (unsigned)((size * esz) >> 22) + 1;
    if (T > 8) T = 8;
    if (hw && T > hw) T = hw;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; ++t) th.emplace_back(work, size * t / T, size * (t + 1) / T);
    work((int64_t)0, size / T);
    for (auto &x : th) x.join();
}

void gather_mem(const void *aligned, int64_t off, int64_t size, int64_t stride, int esz, unsigned char *dst) {
    if (size <= 0 || !aligned) return;
    const char *base = (const char *)aligned + off * esz;
    chunked(size, esz, [&](int64_t e0, int64_t e1) {
        if (stride == 1) std::memcpy(dst + e0 * esz, base + e0 * esz, (size_t)(e1 - e0) * (size_t)esz);
        else
            for (int64_t e = e0; e < e1; ++e) std::memcpy(dst + e * esz, base + e * stride * esz, (size_t)esz);
    });
}

bool same_mem(const void *aligned, int64_t off, int64_t size, int64_t stride, int esz, const unsigned char *ref) {
    if (size <= 0) return true;
    if (!aligned) return false;
    const char *base = (const char *)aligned + off * esz;
    std::atomic<bool> diff{false};
    chunked(size, esz, [&](int64_t e0, int64_t e1) {
        bool d = false;
        if (stride == 1) d = std::memcmp(ref + e0 * esz, base + e0 * esz, (size_t)(e1 - e0) * (size_t)esz) != 0;
        else
            for (int64_t e = e0; e < e1 && !d; ++e) d = std::memcmp(ref + e * esz, base + e * stride * esz, (size_t)esz) != 0;
        if (d) diff = true;
    });
    return !diff;
}

// One host relation of the memref ABI: a key column and (int64 rows) an
// optional payload column (null: payload = row id, the reference's rowId,
// join_v1.mlir:255).
struct HostRel {
    const void *k;
    int64_t k_off, k_stride;
    const void *p;
    int64_t p_off, p_stride;
    int64_t n;
};

void copy_rel(const HostRel &r, int esz, std::vector<unsigned char> &out) {
    const size_t col = (size_t)(r.n > 0 ? r.n : 0) * (size_t)esz;
    out.resize(col * (r.p ? 2 : 1));
    gather_mem(r.k, r.k_off, r.n, r.k_stride, esz, out.data());
    if (r.p) gather_mem(r.p, r.p_off, r.n, r.p_stride, esz, out.data() + col);
}

bool same_rel(const HostRel &r, int esz, const std::vector<unsigned char> &ref) {
    const size_t col = (size_t)(r.n > 0 ? r.n : 0) * (size_t)esz;
    if (ref.size() != col * (r.p ? 2 : 1)) return false;
    return same_mem(r.k, r.k_off, r.n, r.k_stride, esz, ref.data()) &&
           (!r.p || same_mem(r.p, r.p_off, r.n, r.p_stride, esz, ref.data() + col));
}

Digest digest_rel(const HostRel &r, int esz) {
    Digest d = digest_mem(r.k, r.k_off, r.n, r.k_stride, esz);
    if (r.p) {
        const Digest e = digest_mem(r.p, r.p_off, r.n, r.p_stride, esz);
        d.a = fmix(d.a ^ e.a);
        d.b = fmix(d.b ^ e.b) + 1;
    }
    return d;
}

// Relation r into device buffer dst (keys, then int64 payloads: given or
// row ids); the device source of the join.
int upload_rel(hj_ctx *c, int layout, const HostRel &r, void *dst, hj::SrcDev *src) {
    hipStream_t st = c->host_stream;
    if (layout == kNarrow) {
        HJ_TRY(upload<int32_t>(dst, (const int32_t *)r.k, r.k_off, r.n, r.k_stride, st));
        *src = src_col32((const int32_t *)dst, r.n, 0);
        return HJ_OK;
    }
    void *dp = (char *)dst + 8 * (size_t)r.n;
    HJ_TRY(upload<int64_t>(dst, (const int64_t *)r.k, r.k_off, r.n, r.k_stride, st));
    if (r.p) {
        HJ_TRY(upload<int64_t>(dp, (const int64_t *)r.p, r.p_off, r.n, r.p_stride, st));
    } else if (r.n > 0) {
        std::vector<int64_t> iota((size_t)r.n);
        for (int64_t i = 0; i < r.n; ++i) iota[(size_t)i] = i;
        HJ_TRY(upload<int64_t>(dp, iota.data(), 0, r.n, 1, st));
    }
    *src = src_cols64((const int64_t *)dst, (const int64_t *)dp, r.n);
    return HJ_OK;
}

// Probe into dbuf[2] / dbuf[3] sized optimistically (|S| rows, or the known
// M), once more at the exact M when that was too small; *m = M.
int host_probe_all(hj_ctx *c, int layout, const hj::SrcDev &probe, size_t esz, int64_t guess, int64_t *m) {
    hipStream_t st = c->host_stream;
    int64_t cap = guess > 0 ? guess : 1;
    uint64_t cnt = 0;
    for (int pass = 0; pass < 2; ++pass) {
        void *o_r, *o_s;
        HJ_TRY(dbuf(c, 2, esz * (size_t)cap, &o_r));
        HJ_TRY(dbuf(c, 3, esz * (size_t)cap, &o_s));
        HJ_TRY(do_probe(c, layout, probe, o_r, o_s, cap, (uint64_t *)c->dcount, false, st));
        HJ_HIP(hipMemcpyAsync(&cnt, c->dcount, 8, hipMemcpyDeviceToHost, st));
        HJ_HIP(hipStreamSynchronize(st));
        if (cnt >> 63) HJ_FAIL(HJ_ERR_CAPACITY, "probe: internal work list overflow (count flagged)");
        if ((int64_t)cnt <= cap) break;
        cap = (int64_t)cnt;   // exact M known: second pass fits
    }
    *m = (int64_t)cnt;
    return HJ_OK;
}

// Joins a std::thread on every exit path.
struct Joiner {
    std::thread t;
    ~Joiner() {
        if (t.joinable()) t.join();
    }
};

// Host-memref join (the reference's @main data path, join_v2.mlir:627-696).
//   kHostCount: upload, build, COUNT (no pairs); remember the inputs'
//               digests (computed while uploading) -- @countRows.
//   kHostProbe: if both memrefs digest as the last count's, probe the kept
//               table with the staged probe side into M-row buffers (no
//               upload, no build) -- @probeRelation; else the whole join.
//               The digests run on host threads WHILE the kept table is
//               probed and, through `deliver`, the pairs are downloaded into
//               the caller's outputs (speculatively: changed inputs then get
//               the whole join, whose pairs are delivered again).
//   kHostJoin:  the whole join (one-memref-out C interface), no memo.
// Pairs land in dbuf[2], dbuf[3] (not for kHostCount); *m = M.
enum HostMode { kHostCount, kHostProbe, kHostJoin };
typedef std::function<int(const void *, const void *, int64_t)> Deliver;
int host_join(hj_ctx *c, int layout, const HostRel &r, const HostRel &s, HostMode mode, int64_t *m, void **d_or,
              void **d_os, const Deliver *deliver = nullptr, bool *delivered = nullptr) {
    if (r.n < 0 || s.n < 0) HJ_FAIL(HJ_ERR_ARG, "negative memref size");
    HJ_TRY(set_device(c));
    HJ_TRY(host_stream(c));
    hipStream_t st = c->host_stream;
    const int esz = layout == kWide ? 8 : 4;
    hj_ctx::Memo &mm = c->memo;
    const int reuse = g_reuse.load();
    // a memo an EXACT count left on this context after the mode moved on:
    // its input copies (GBs at 2^28 rows) go now (hj_host_set_reuse frees
    // those of the default contexts at once; user contexts' here)
    if (mm.reuse == HJ_REUSE_EXACT && reuse != HJ_REUSE_EXACT && (!mm.cr.empty() || !mm.cs.empty())) mm.invalidate();
    Digest dr, ds;
    bool same_r = false, same_s = false;   // HJ_REUSE_EXACT: byte-equal to the count's inputs
    if (delivered) *delivered = false;
    if (mode == kHostProbe && mm.valid && mm.reuse == reuse && reuse != HJ_REUSE_OFF && mm.layout == layout &&
        mm.nr == r.n && mm.ns == s.n) {
        int rc = HJ_OK;
        int64_t mp = 0;
        bool sent = false;
        {
            Joiner dig_r, dig_s;
            if (reuse == HJ_REUSE_EXACT) {
                dig_r.t = std::thread([&] { same_r = same_rel(r, esz, mm.cr); });
                dig_s.t = std::thread([&] { same_s = same_rel(s, esz, mm.cs); });
            } else {
                dig_r.t = std::thread([&] { dr = digest_rel(r, esz); });
                dig_s.t = std::thread([&] { ds = digest_rel(s, esz); });
            }
            const hj::SrcDev src = layout == kWide
                                       ? src_cols64((const int64_t *)c->dbuf[7], (const int64_t *)c->dbuf[7] + s.n, s.n)
                                       : src_col32((const int32_t *)c->dbuf[7], s.n, 0);
            rc = host_probe_all(c, layout, src, (size_t)esz, mm.m, &mp);
            if (rc == HJ_OK && deliver && mp == mm.m) {
                const int d = (*deliver)(c->dbuf[2], c->dbuf[3], mp);   // (1: outputs of another size, not sent)
                sent = d == HJ_OK;
                if (d < 0) rc = d;
            }
        }
        if (rc != HJ_OK) return rc;
        if (reuse == HJ_REUSE_EXACT ? (same_r && same_s) : (dr == mm.dr && ds == mm.ds)) {
            ++c->memo_hits;
            *m = mp;
            *d_or = c->dbuf[2];
            *d_os = c->dbuf[3];
            if (delivered) *delivered = sent;
            return HJ_OK;
        }
    }
    mm.invalidate(mode == kHostCount && reuse == HJ_REUSE_EXACT);
    const size_t rb = (size_t)(layout == kWide ? 16 : 4) * (size_t)r.n;
    const size_t sb = (size_t)(layout == kWide ? 16 : 4) * (size_t)s.n;
    void *dr_buf, *ds_buf;
    HJ_TRY(dbuf(c, 6, rb, &dr_buf));
    HJ_TRY(dbuf(c, 7, sb, &ds_buf));
    hj::SrcDev rsrc, ssrc;
    {
        Joiner dig;
        if (mode == kHostCount && reuse == HJ_REUSE_DIGEST) dig.t = std::thread([&] {   // overlapped with the upload
            dr = digest_rel(r, esz);
            ds = digest_rel(s, esz);
        });
        else if (mode == kHostCount && reuse == HJ_REUSE_EXACT) dig.t = std::thread([&] {
            copy_rel(r, esz, mm.cr);
            copy_rel(s, esz, mm.cs);
        });
        HJ_TRY(upload_rel(c, layout, r, dr_buf, &rsrc));
        HJ_TRY(upload_rel(c, layout, s, ds_buf, &ssrc));
    }
    c->host_building = true;
    const int64_t hint = c->probe_hint;
    c->probe_hint = s.n;
    const int brc = do_build(c, layout, rsrc, st);
    c->probe_hint = hint;
    c->host_building = false;
    HJ_TRY(brc);
    if (mode != kHostCount) {
        HJ_TRY(host_probe_all(c, layout, ssrc, (size_t)esz, s.n, m));
        *d_or = c->dbuf[2];
        *d_os = c->dbuf[3];
        return HJ_OK;
    }
    uint64_t cnt = 0;
    HJ_TRY(do_probe(c, layout, ssrc, nullptr, nullptr, 0, (uint64_t *)c->dcount, true, st));
    HJ_HIP(hipMemcpyAsync(&cnt, c->dcount, 8, hipMemcpyDeviceToHost, st));
    HJ_HIP(hipStreamSynchronize(st));
    // (a flagged count is an error, never a row count -- and never memoised)
    if (cnt >> 63) HJ_FAIL(HJ_ERR_CAPACITY, "count: internal work list overflow (count flagged)");
    mm.layout = layout;
    mm.nr = r.n;
    mm.ns = s.n;
    mm.dr = dr;
    mm.ds = ds;
    mm.m = (int64_t)cnt;
    mm.reuse = reuse;
    mm.valid = reuse != HJ_REUSE_OFF;
    *m = (int64_t)cnt;
    *d_or = *d_os = nullptr;
    return HJ_OK;
}

HostRel rel32(const int32_t *k, int64_t off, int64_t n, int64_t stride) { return HostRel{k, off, stride, nullptr, 0, 1, n}; }
HostRel rel64(const int64_t *k, int64_t k_off, int64_t k_stride, const int64_t *p, int64_t p_off, int64_t p_stride,
              int64_t n) {
    return HostRel{k, k_off, k_stride, p, p_off, p_stride, n};
}

// ---- device -> pageable host memory through page-locked staging.  A plain
// hipMemcpy into a pageable buffer (the caller's memref) ran at ~17 GB/s
// (bench host_memref: 2 x 134 MB in 16 ms); here 32-MiB chunks are DMA'd into
// one of two page-locked buffers while the host copies the previous chunk out
// with up to 8 threads (chunked).  The staging pairs are process-wide, taken
// from a free list (concurrent host joins each take their own pair); a pair's
// events belong to the device that was current when it was made, so a pair
// is only handed out again on that device (an event recorded on
// another device's stream is an invalid handle).
constexpr size_t kStageChunk = size_t(32) << 20;
constexpr size_t kStageMin = size_t(16) << 20;   // below this: one plain copy
struct Staging {
    void *p[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    int dev = -1;
};
std::mutex g_stage_mu;
std::vector<Staging *> g_stage_free;

Staging *stage_take() {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    {
        std::lock_guard<std::mutex> lk(g_stage_mu);
        for (size_t i = 0; i < g_stage_free.size(); ++i) {
            if (g_stage_free[i]->dev != dev) continue;
            Staging *s = g_stage_free[i];
            g_stage_free.erase(g_stage_free.begin() + (std::ptrdiff_t)i);
            return s;
        }
    }
    Staging *s = new Staging;
    s->dev = dev;
    bool ok = true;
    for (int i = 0; i < 2 && ok; ++i) {
        ok = hipHostMalloc(&s->p[i], kStageChunk, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&s->ev[i], hipEventDisableTiming) == hipSuccess;
    }
    if (!ok) {
        (void)hipGetLastError();
        for (int i = 0; i < 2; ++i) {
            if (s->p[i]) (void)hipHostFree(s->p[i]);
            if (s->ev[i]) (void)hipEventDestroy(s->ev[i]);
        }
        delete s;
        return nullptr;
    }
    return s;
}

void stage_give(Staging *s) {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    g_stage_free.push_back(s);
}

int d2h(void *dst, const void *src, size_t bytes, hipStream_t st) {
    if (bytes == 0) return HJ_OK;
    Staging *sg = bytes >= kStageMin ? stage_take() : nullptr;
    if (!sg) {
        HJ_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
        HJ_HIP(hipStreamSynchronize(st));
        return HJ_OK;
    }
    const size_t nch = (bytes + kStageChunk - 1) / kStageChunk;
    auto len_of = [&](size_t i) { return i + 1 < nch ? kStageChunk : bytes - i * kStageChunk; };
    auto issue = [&](size_t i) -> hipError_t {
        hipError_t e = hipMemcpyAsync(sg->p[i & 1], (const char *)src + i * kStageChunk, len_of(i),
                                      hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(sg->ev[i & 1], st);
        return e;
    };
    hipError_t e = issue(0);
    for (size_t i = 0; i < nch && e == hipSuccess; ++i) {
        // chunk i + 1 lands in the buffer chunk i - 1 was copied out of
        if (i + 1 < nch) e = issue(i + 1);
        if (e == hipSuccess) e = hipEventSynchronize(sg->ev[i & 1]);
        if (e != hipSuccess) break;
        char *out = (char *)dst + i * kStageChunk;
        const char *in = (const char *)sg->p[i & 1];
        chunked((int64_t)len_of(i), 1, [&](int64_t a, int64_t b) { std::memcpy(out + a, in + a, (size_t)(b - a)); });
    }
    if (e != hipSuccess) (void)hipStreamSynchronize(st);   // (nothing left in flight into the staging)
    stage_give(sg);
    HJ_HIP(e);
    return HJ_OK;
}

// Device column -> strided host memref.
template <class T>
int download(T *aligned, int64_t off, int64_t size, int64_t stride, const void *src, hipStream_t st) {
    if (size <= 0) return HJ_OK;
    if (!aligned) HJ_FAIL(HJ_ERR_ARG, "null output memref");
    T *base = aligned + off;
    if (stride == 1) return d2h(base, src, sizeof(T) * (size_t)size, st);
    std::vector<T> tmp((size_t)size);
    HJ_TRY(d2h(tmp.data(), src, sizeof(T) * (size_t)size, st));
    for (int64_t i = 0; i < size; ++i) base[i * stride] = tmp[(size_t)i];
    return HJ_OK;
}

// Interleave two device columns into a malloc'ed memref<?x2xT> descriptor.
template <class T, class D>
int fill_result(D *res, const void *d_r, const void *d_s, int64_t m, hipStream_t st) {
    std::memset(res, 0, sizeof(D));
    T *buf = (T *)std::malloc(sizeof(T) * 2 * (size_t)(m > 0 ? m : 1));
    if (!buf) HJ_FAIL(HJ_ERR_NOMEM, "malloc result");
    if (m > 0) {
        std::vector<T> a((size_t)m), b((size_t)m);
        int rc = d2h(a.data(), d_r, sizeof(T) * (size_t)m, st);
        if (rc == HJ_OK) rc = d2h(b.data(), d_s, sizeof(T) * (size_t)m, st);
        if (rc != HJ_OK) {
            std::free(buf);   // (the descriptor stays empty: allocated == NULL)
            return rc;
        }
        for (int64_t i = 0; i < m; ++i) {
            buf[2 * i] = a[(size_t)i];
            buf[2 * i + 1] = b[(size_t)i];
        }
    }
    res->allocated = buf;
    res->aligned = buf;
    res->offset = 0;
    res->sizes[0] = m;
    res->sizes[1] = 2;
    res->strides[0] = 2;
    res->strides[1] = 1;
    return HJ_OK;
}

}  // namespace

namespace {

// Upload a strided 2-D host memref (aligned + offset, sizes, strides) as a
// contiguous row-major rows x cols block.
int upload2(void *dst, const int32_t *aligned, int64_t off, int64_t rows, int64_t cols, int64_t s0, int64_t s1,
            hipStream_t st) {
    if (rows <= 0 || cols <= 0) return HJ_OK;
    if (!aligned) HJ_FAIL(HJ_ERR_ARG, "null memref");
    const int32_t *base = aligned + off;
    if (s1 == 1 && s0 == cols) {
        HJ_HIP(hipMemcpyAsync(dst, base, sizeof(int32_t) * (size_t)(rows * cols), hipMemcpyHostToDevice, st));
    } else {
        std::vector<int32_t> tmp((size_t)(rows * cols));
        for (int64_t i = 0; i < rows; ++i)
            for (int64_t j = 0; j < cols; ++j) tmp[(size_t)(i * cols + j)] = base[i * s0 + j * s1];
        HJ_HIP(hipMemcpyAsync(dst, tmp.data(), sizeof(int32_t) * tmp.size(), hipMemcpyHostToDevice, st));
        HJ_HIP(hipStreamSynchronize(st));
        return HJ_OK;
    }
    HJ_HIP(hipStreamSynchronize(st));
    return HJ_OK;
}

// Host-memref row join: tables copied in, rows materialised on the device
// into staging buffer dbuf[4] (M x oc, contiguous); *m = M, *oc_out = columns.
int host_join_rows(hj_ctx *c, const int32_t *a1, int64_t o1, int64_t r1, int64_t c1, int64_t s10, int64_t s11,
                   const int32_t *a2, int64_t o2, int64_t r2, int64_t c2, int64_t s20, int64_t s21, bool count_only,
                   int64_t *m, int64_t *oc_out, void **d_out) {
    if (r1 < 0 || r2 < 0 || c1 < 1 || c2 < 1) HJ_FAIL(HJ_ERR_ARG, "bad memref shape");
    HJ_TRY(set_device(c));
    HJ_TRY(host_stream(c));
    hipStream_t st = c->host_stream;
    void *d1, *d2;
    HJ_TRY(dbuf(c, 0, sizeof(int32_t) * (size_t)(r1 * c1), &d1));
    HJ_TRY(dbuf(c, 1, sizeof(int32_t) * (size_t)(r2 * c2), &d2));
    HJ_TRY(upload2(d1, a1, o1, r1, c1, s10, s11, st));
    HJ_TRY(upload2(d2, a2, o2, r2, c2, s20, s21, st));
    const RowTables t{(const int32_t *)d1, r1, c1, c1, (const int32_t *)d2, r2, c2, c2};
    *oc_out = c1 + c2 - 1;
    uint64_t cnt = 0;
    HJ_TRY(do_join_rows(c, t, nullptr, 0, 0, (uint64_t *)c->dcount, true, st));
    HJ_HIP(hipMemcpyAsync(&cnt, c->dcount, 8, hipMemcpyDeviceToHost, st));
    HJ_HIP(hipStreamSynchronize(st));
    *m = (int64_t)cnt;
    if (count_only) return HJ_OK;
    HJ_TRY(dbuf(c, 4, sizeof(int32_t) * (size_t)(*m > 0 ? *m * *oc_out : 1), d_out));
    HJ_TRY(do_join_rows(c, t, (int32_t *)*d_out, *oc_out, *m, (uint64_t *)c->dcount, false, st));
    HJ_HIP(hipStreamSynchronize(st));
    return HJ_OK;
}

}  // namespace

extern "C" {

int hj_abi_version(void) { return HJ_ABI_VERSION; }

int hj_device_info(int device, int64_t out[8]) {
    if (!out) HJ_FAIL(HJ_ERR_ARG, "null output");
    hipDeviceProp_t p;
    HJ_HIP(hipGetDeviceProperties(&p, device));
    out[0] = p.multiProcessorCount;
    out[1] = p.memoryClockRate;   // kHz
    out[2] = p.memoryBusWidth;    // bits
    out[3] = p.l2CacheSize;
    out[4] = (int64_t)p.totalGlobalMem;
    out[5] = p.clockRate;         // kHz
    out[6] = (int64_t)p.maxSharedMemoryPerMultiProcessor;
    // HBM3E: 4 transfers per reported memory clock (MI355X reports 2.0 GHz
    // and 8192 bits: 8 Gb/s per pin, 8.19 TB/s -- the 8.0 TB/s spec)
    out[7] = (int64_t)(4.0 * (double)p.memoryClockRate * 1e3 * (double)p.memoryBusWidth / 8.0 / 1e6);   // MB/s
    return HJ_OK;
}

int hj_host_set_reuse(int mode) {
    if (mode != HJ_REUSE_DIGEST && mode != HJ_REUSE_EXACT && mode != HJ_REUSE_OFF) HJ_FAIL(HJ_ERR_ARG, "bad reuse mode");
    const int prev = g_reuse.exchange(mode);
    if (prev == HJ_REUSE_EXACT && mode != HJ_REUSE_EXACT) {
        // the EXACT copies can no longer be used: give their memory back
        // (the default contexts' now -- g_default_mu held throughout, so
        // hj_ctx_destroy, which takes a context out of g_default before it
        // frees anything, cannot free one under us; user contexts drop
        // theirs at their next host join)
        std::lock_guard<std::mutex> lk(g_default_mu);
        for (auto &kv : g_default) {
            std::lock_guard<std::mutex> host_lk(kv.second->host_mu);
            kv.second->memo.invalidate();
        }
    }
    return prev;
}

int64_t hj_host_memo_hits(void) {
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    return c->memo_hits;
}
const char *hj_last_error(void) { return g_err.c_str(); }

hj_ctx *hj_ctx_create(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        fail(HJ_ERR_HIP, __FILE__, __LINE__, "no HIP device visible");
        return nullptr;
    }
    if (device < 0 || device >= n) {
        fail(HJ_ERR_ARG, __FILE__, __LINE__, "device index out of range");
        return nullptr;
    }
    hj_ctx *c = new hj_ctx();
    c->device = device;
    if (set_device(c) != HJ_OK || ensure_meta(c, 64) != HJ_OK) {
        delete c;
        return nullptr;
    }
    return c;
}

void hj_ctx_destroy(hj_ctx *c) {
    if (!c) return;
    {   // out of the default registry first (hj_host_set_reuse walks it)
        std::lock_guard<std::mutex> lk(g_default_mu);
        for (auto it = g_default.begin(); it != g_default.end(); ++it)
            if (it->second == c) {
                g_default.erase(it);
                break;
            }
    }
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    if (c->table) (void)hipFree(c->table);
    if (c->side) (void)hipFree(c->side);
    if (c->meta) (void)hipFree(c->meta);
    if (c->dcount) (void)hipFree(c->dcount);
    for (int i = 0; i < hj_ctx::kDbufs; ++i)
        if (c->dbuf[i]) (void)hipFree(c->dbuf[i]);
    if (c->host_stream) (void)hipStreamDestroy(c->host_stream);
    for (SetBufs *sb : {&c->rset, &c->sset, &c->tset})
        for (Buf *b : {&sb->rows, &sb->bbin, &sb->bfill, &sb->runs, &sb->rstart}) free_buf(*b);
    for (Buf *b : {&c->nb, &c->pcur, &c->rcur, &c->tile_start, &c->tile_owner, &c->tdesc, &c->wstart, &c->work_start, &c->work_desc, &c->scan_sums, &c->scan_state, &c->raw_cnt,
                   &c->slow, &c->rows_kx, &c->rows_ky, &c->rows_px, &c->rows_py, &c->sel_tiles, &c->sel_sums,
                   &c->route_hist, &c->route_sums})
        free_buf(*b);
    for (int k = 0; k < c->ev_made; ++k)
        for (int i = 0; i < kEvCount; ++i) (void)hipEventDestroy(c->sets[k].ev[i]);
    delete c;
}

int hj_ctx_reserve(hj_ctx *c, int64_t max_build_rows, int key_bits) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (max_build_rows < 0 || (key_bits != 32 && key_bits != 64)) HJ_FAIL(HJ_ERR_ARG, "bad reserve arguments");
    HJ_TRY(set_device(c));
    HJ_TRY(ensure_meta(c, 64));
    const size_t esz = key_bits == 64 ? 16 : 8;
    if (choose_strategy(c, max_build_rows) == HJ_STRATEGY_GLOBAL) {
        HJ_TRY(ensure_table(c, max_build_rows, key_bits == 64 ? kWide : kNarrow));
        if (c->strategy != HJ_STRATEGY_AUTO || max_build_rows < kDualMinBuildRows) return HJ_OK;
    }
    const hj::RadixPlan pl = hj::radix_plan(max_build_rows, c->radix_bits, key_bits == 64);
    return ensure_radix_scratch(c, c->rset, max_build_rows, esz, pl);
}

int64_t hj_ctx_table_capacity(const hj_ctx *c) {
    if (!c || c->layout < 0) return 0;
    if (c->used == HJ_STRATEGY_RADIX) return (int64_t)(1ll << c->plan.total_bits);   // partitions
    return (int64_t)(1ll << c->bits);
}

int hj_ctx_radix_plan(const hj_ctx *c, int *passes, int bits[3]) {
    if (!c || !passes || !bits) HJ_FAIL(HJ_ERR_ARG, "null argument");
    const bool radix = c->layout >= 0 && (c->used == HJ_STRATEGY_RADIX || c->dual);
    *passes = radix ? c->plan.passes : 0;
    for (int i = 0; i < 3; ++i) bits[i] = radix ? c->plan.bits[i] : 0;
    return HJ_OK;
}

int hj_ctx_build_has_duplicates(hj_ctx *c) {
    if (!c || c->layout < 0) HJ_FAIL(HJ_ERR_STATE, "no table built");
    HJ_TRY(set_device(c));
    unsigned long long v = 0;
    HJ_HIP(hipDeviceSynchronize());
    HJ_HIP(hipMemcpy(&v, c->meta + 1, 8, hipMemcpyDeviceToHost));
    if (!v && c->used == HJ_STRATEGY_RADIX && !c->dup_checked) {
        // the joins flag only the repeats of partitions they built (k_join_b:
        // only those a probe row met): the exact answer, once per build, is a
        // DETECT build over every partition of R (the work map is rebuilt from
        // R alone; the last join's map is not needed again)
        HJ_RADIX(c, nullptr, hj::radix_detect(c->layout == kWide, c->plan, radix_work(c), bucket_set(c->rset),
                                               (unsigned *)c->work_start.p, c->work_desc.p, c->meta + 1,
                                               c->meta + 2, nullptr));
        HJ_HIP(hipDeviceSynchronize());
        HJ_HIP(hipMemcpy(&v, c->meta + 1, 8, hipMemcpyDeviceToHost));
        c->dup_checked = true;
    }
    return v ? 1 : 0;
}

int hj_ctx_join_kernel(hj_ctx *c) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (!c->join_ran || c->layout < 0) return 0;
    HJ_TRY(set_device(c));
    unsigned long long v[2] = {0, 0};
    HJ_HIP(hipDeviceSynchronize());
    HJ_HIP(hipMemcpy(v, c->meta + 2, sizeof(v), hipMemcpyDeviceToHost));
    return hj::join_kernel_choice(c->join_wide, c->join_stream, v[0], v[1]);
}

int hj_ctx_set_timing(hj_ctx *c, int enable) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    HJ_TRY(set_device(c));
    if (enable && !c->ev_ready) {
        for (int i = 0; i < kEvCount; ++i) HJ_HIP(hipEventCreate(&c->sets[0].ev[i]));
        c->ev_ready = true;
        c->ev_made = 1;
    }
    c->timing = enable != 0;
    return HJ_OK;
}

int hj_ctx_timing_accumulate(hj_ctx *c, int enable) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (enable) HJ_TRY(hj_ctx_set_timing(c, 1));
    if (enable && c->ev_made < hj_ctx::kEvSets) {
        for (int k = c->ev_made; k < hj_ctx::kEvSets; ++k) {
            for (int i = 0; i < kEvCount; ++i) HJ_HIP(hipEventCreate(&c->sets[k].ev[i]));
            c->ev_made = k + 1;
        }
    }
    if (enable) c->acc = true;
    if (!c->acc) return HJ_OK;
    // a fresh start: nothing recorded so far counts
    for (auto &s : c->sets) s.rec[0] = s.rec[1] = s.rec[2] = s.rec[3] = s.rec_mid = false;
    for (double &t : c->tot) t = 0.0;
    c->tot_sets = 0;
    if (!enable) {
        // (the sets stay created; set `cur` keeps taking the records)
        c->acc = false;
    }
    return HJ_OK;
}

int hj_ctx_timing_totals(hj_ctx *c, float ms[8], long long *sets) {
    if (!c || !ms || !sets) HJ_FAIL(HJ_ERR_ARG, "null argument");
    if (!c->acc) HJ_FAIL(HJ_ERR_STATE, "timing totals need hj_ctx_timing_accumulate(c, 1)");
    HJ_TRY(set_device(c));
    for (int k = 1; k <= hj_ctx::kEvSets; ++k) HJ_TRY(fold_set(c, (c->cur + k) % hj_ctx::kEvSets));
    for (int i = 0; i < 8; ++i) ms[i] = i < 6 ? (float)c->tot[i] : -1.0f;
    *sets = c->tot_sets;
    for (double &t : c->tot) t = 0.0;
    c->tot_sets = 0;
    return HJ_OK;
}

int hj_ctx_last_timing_ex(hj_ctx *c, float ms[8]) {
    if (!c || !ms) HJ_FAIL(HJ_ERR_ARG, "null argument");
    for (int i = 0; i < 8; ++i) ms[i] = -1.0f;
    if (!c->ev_ready) return HJ_OK;
    HJ_TRY(set_device(c));
    return set_ms(c->evs(), ms);
}

int hj_ctx_last_timing(hj_ctx *c, float ms[4]) {
    float ex[8];
    HJ_TRY(hj_ctx_last_timing_ex(c, ex));
    for (int i = 0; i < 4; ++i) ms[i] = ex[i];
    return HJ_OK;
}

int hj_ctx_set_strategy(hj_ctx *c, int strategy) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (strategy != HJ_STRATEGY_AUTO && strategy != HJ_STRATEGY_GLOBAL && strategy != HJ_STRATEGY_RADIX)
        HJ_FAIL(HJ_ERR_ARG, "unknown strategy");
    c->strategy = strategy;
    return HJ_OK;
}

int hj_ctx_set_radix_bits(hj_ctx *c, int bits) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (bits < 0 || bits > 24) HJ_FAIL(HJ_ERR_ARG, "radix bits must be in [0, 24]");
    c->radix_bits = bits;
    return HJ_OK;
}


int hj_ctx_strategy_used(const hj_ctx *c) {
    if (!c || c->layout < 0) return 0;
    return c->probe_used >= 0 ? c->probe_used : c->used;
}

int hj_ctx_probe_hint(hj_ctx *c, int64_t probe_rows) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    c->probe_hint = probe_rows < 0 ? -1 : probe_rows;
    return HJ_OK;
}

int hj_ctx_reserve_probe(hj_ctx *c, int64_t max_probe_rows, int key_bits) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (max_probe_rows < 0 || (key_bits != 32 && key_bits != 64)) HJ_FAIL(HJ_ERR_ARG, "bad reserve arguments");
    if (c->layout < 0 || (c->used != HJ_STRATEGY_RADIX && !c->dual)) return HJ_OK;   // the global table needs none
    HJ_TRY(set_device(c));
    const size_t esz = key_bits == 64 ? 16 : 8;
    return ensure_radix_scratch(c, c->sset, max_probe_rows, esz, c->plan);
}

// ------------------------------------------------------------ device phases
int hj_dev_build_i64(hj_ctx *c, const int64_t *rkey, const int64_t *rpay, int64_t n, void *stream) {
    return do_build(c, kWide, src_cols64(rkey, rpay, n), (hipStream_t)stream);
}
int hj_dev_count_i64(hj_ctx *c, const int64_t *skey, int64_t n, uint64_t *d_count, void *stream) {
    hj::SrcDev s = src_cols64(skey, skey, n);   // payload unused when counting
    return do_probe(c, kWide, s, nullptr, nullptr, 0, d_count, true, (hipStream_t)stream);
}
int hj_dev_probe_i64(hj_ctx *c, const int64_t *skey, const int64_t *spay, int64_t n, int64_t *out_r,
                     int64_t *out_s, int64_t out_cap, uint64_t *d_count, void *stream) {
    if (n > 0 && !spay) HJ_FAIL(HJ_ERR_ARG, "null probe payload");
    return do_probe(c, kWide, src_cols64(skey, spay, n), out_r, out_s, out_cap, d_count, false,
                    (hipStream_t)stream);
}
int hj_dev_build_tuples_i64(hj_ctx *c, const int64_t *tuples, int64_t n, void *stream) {
    return do_build(c, kWide, src_packed(tuples, n), (hipStream_t)stream);
}
int hj_dev_probe_tuples_i64(hj_ctx *c, const int64_t *tuples, int64_t n, int64_t *out_r, int64_t *out_s,
                            int64_t out_cap, uint64_t *d_count, void *stream) {
    return do_probe(c, kWide, src_packed(tuples, n), out_r, out_s, out_cap, d_count, false, (hipStream_t)stream);
}
int hj_dev_build_i32(hj_ctx *c, const int32_t *rkey, int64_t n, int64_t row_base, void *stream) {
    if (row_base < 0 || row_base + n > 0x7fffffffll) HJ_FAIL(HJ_ERR_ARG, "i32 row ids out of range");
    return do_build(c, kNarrow, src_col32(rkey, n, row_base), (hipStream_t)stream);
}
int hj_dev_count_i32(hj_ctx *c, const int32_t *skey, int64_t n, uint64_t *d_count, void *stream) {
    return do_probe(c, kNarrow, src_col32(skey, n, 0), nullptr, nullptr, 0, d_count, true, (hipStream_t)stream);
}
int hj_dev_probe_i32(hj_ctx *c, const int32_t *skey, int64_t n, int64_t row_base, int32_t *out_r, int32_t *out_s,
                     int64_t out_cap, uint64_t *d_count, void *stream) {
    if (row_base < 0 || row_base + n > 0x7fffffffll) HJ_FAIL(HJ_ERR_ARG, "i32 row ids out of range");
    return do_probe(c, kNarrow, src_col32(skey, n, row_base), out_r, out_s, out_cap, d_count, false,
                    (hipStream_t)stream);
}

int hj_dev_partition_i64(hj_ctx *c, const int64_t *key, const int64_t *pay, int64_t n, int nparts,
                         int64_t *out_tuples, uint64_t *d_counts, void *stream) {
    if (n > 0 && !pay) HJ_FAIL(HJ_ERR_ARG, "null payload");
    return do_partition(c, src_cols64(key, pay, n), nparts, out_tuples, d_counts, (hipStream_t)stream);
}
int hj_dev_partition_tuples_i64(hj_ctx *c, const int64_t *tuples, int64_t n, int nparts, int64_t *out_tuples,
                                uint64_t *d_counts, void *stream) {
    return do_partition(c, src_packed(tuples, n), nparts, out_tuples, d_counts, (hipStream_t)stream);
}

int hj_route_plan(int64_t n_build_global, int nranks, int *sub_bits) {
    if (!sub_bits) HJ_FAIL(HJ_ERR_ARG, "null argument");
    *sub_bits = 0;
    if (nranks < 1 || nranks > hj::kMaxRouteSources || (nranks & (nranks - 1)) || n_build_global < 0)
        return HJ_OK;
    const int g = ceil_log2((unsigned long long)nranks);
    const int64_t local = (n_build_global + nranks - 1) / nranks;
    if (local < kRadixMinRows || g >= 9) return HJ_OK;
    const int t = hj::radix_plan(local, 0, true).total_bits;
    const int b1 = 9 - g < t - 1 ? 9 - g : t - 1;
    if (b1 >= 1 && t - b1 <= 9) *sub_bits = b1;
    return HJ_OK;
}

int hj_dev_route_i64(hj_ctx *c, const int64_t *key, const int64_t *pay, int64_t n, int nranks, int sub_bits,
                     int64_t *out_tuples, uint64_t *d_counts, void *stream) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (n > 0 && (!key || !pay || !out_tuples)) HJ_FAIL(HJ_ERR_ARG, "bad route input");
    if (!d_counts) HJ_FAIL(HJ_ERR_ARG, "null counts");
    if (nranks < 1 || (nranks & (nranks - 1)) || sub_bits < 1) HJ_FAIL(HJ_ERR_ARG, "nranks: a power of two; sub_bits >= 1");
    const int rbits = ceil_log2((unsigned long long)nranks) + sub_bits;
    if (rbits > 9) HJ_FAIL(HJ_ERR_ARG, "nranks << sub_bits must be <= 512");
    hipStream_t st = (hipStream_t)stream;
    HJ_TRY(set_device(c));
    const size_t hw = hj::radix_route_scratch(n, rbits);
    HJ_TRY(ensure_buf(c->route_hist, hw * 8));
    HJ_TRY(ensure_buf(c->route_sums, hj::exclusive_scan_sums(hw) * 8));
    record(c, kEvPart0, st);
    HJ_HIP(hj::radix_route(src_cols64(key, pay, n), rbits, out_tuples, (unsigned long long *)d_counts,
                           (unsigned long long *)c->route_hist.p, (unsigned long long *)c->route_sums.p, st));
    record(c, kEvPart1, st);
    c->evs().rec[3] = c->timing;
    return HJ_OK;
}

int hj_dev_build_routed_i64(hj_ctx *c, const int64_t *tuples, int64_t n, const uint64_t *d_counts, int nsrc,
                            int nranks, int sub_bits, void *stream) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (n < 0 || (n > 0 && !tuples) || !d_counts) HJ_FAIL(HJ_ERR_ARG, "bad routed build relation");
    if (nsrc < 1 || nsrc > hj::kMaxRouteSources || nranks < 1 || (nranks & (nranks - 1)) || sub_bits < 1 ||
        sub_bits > 9)
        HJ_FAIL(HJ_ERR_ARG, "bad routed layout");
    hipStream_t st = (hipStream_t)stream;
    HJ_TRY(set_device(c));
    HJ_TRY(ensure_meta(c, 64));
    HJ_TRY(timing_advance(c));
    // this rank's plan: the routing's bins are its first pass (skip = the
    // owner bits above them), one local pass of <= 9 bits below them
    hj::RadixPlan pl = hj::radix_plan(n, 0, true);
    int t = pl.total_bits;
    if (t < sub_bits + 1) t = sub_bits + 1;
    if (t > sub_bits + 9) t = sub_bits + 9;
    pl.passes = 2;
    pl.bits[0] = sub_bits;
    pl.bits[1] = t - sub_bits;
    pl.bits[2] = 0;
    pl.pbl[0] = 10;   // (sizes the ping set, whose run arrays list the routed rows)
    pl.pbl[1] = hj::kFinalPbl;
    pl.pbl[2] = 0;
    pl.total_bits = t;
    pl.skip = ceil_log2((unsigned long long)nranks);
    c->layout = kWide;
    c->n_build = n;
    c->used = HJ_STRATEGY_RADIX;
    c->dual = false;
    c->probe_used = -1;
    c->join_ran = false;
    c->memo.invalidate();
    c->plan = pl;
    c->routed = true;
    c->dup_checked = false;
    HJ_TRY(ensure_radix_scratch(c, c->rset, n, 16, pl));
    record(c, kEvInit0, st);
    HJ_HIP(hipMemsetAsync(c->meta, 0, 4 * sizeof(unsigned long long), st));
    record(c, kEvInit1, st);
    HJ_RADIX(c, st, hj::radix_partition_routed(tuples, n, (const unsigned long long *)d_counts, nsrc, 1 << sub_bits, pl,
                                      radix_work(c), bucket_set(c->rset), st));
    HJ_HIP(hj::radix_sample(true, pl, bucket_set(c->rset), c->meta + 2, st));
    record(c, kEvBuild1, st);
    c->evs().rec[0] = c->evs().rec[1] = c->timing;
    return HJ_OK;
}

int hj_dev_probe_routed_i64(hj_ctx *c, const int64_t *tuples, int64_t n, const uint64_t *d_counts, int nsrc,
                            int bin0, int nbins, int64_t *out_r, int64_t *out_s, int64_t out_cap, uint64_t *d_count,
                            void *stream) {
    if (!c) HJ_FAIL(HJ_ERR_ARG, "null context");
    if (!d_count) HJ_FAIL(HJ_ERR_ARG, "null count pointer");
    if (c->layout != kWide || c->used != HJ_STRATEGY_RADIX || !c->routed)
        HJ_FAIL(HJ_ERR_STATE, "probe_routed needs a routed build");
    if (n < 0 || (n > 0 && !tuples) || !d_counts) HJ_FAIL(HJ_ERR_ARG, "bad routed probe relation");
    if (out_cap < 0 || (out_cap > 0 && (!out_r || !out_s))) HJ_FAIL(HJ_ERR_ARG, "bad output");
    const int F = 1 << c->plan.bits[0];
    if (nsrc < 1 || nsrc > hj::kMaxRouteSources || bin0 < 0 || nbins < 1 || bin0 + nbins > F)
        HJ_FAIL(HJ_ERR_ARG, "bad routed layout");
    hipStream_t st = (hipStream_t)stream;
    HJ_TRY(set_device(c));
    c->probe_used = HJ_STRATEGY_RADIX;   // (radix_join zeroes d_count)
    HJ_TRY(ensure_radix_scratch(c, c->sset, n, 16, c->plan));
    record(c, kEvProbe0, st);
    HJ_RADIX(c, st, hj::radix_partition_routed(tuples, n, (const unsigned long long *)d_counts, nsrc, nbins, c->plan,
                                      radix_work(c), bucket_set(c->sset), st));
    record(c, kEvProbeMid, st);
    // bins [bin0, bin0 + nbins): partitions [bin0, bin0 + nbins) << bits[1] of R
    hj::BucketSet r = bucket_set(c->rset);
    r.rstart += (size_t)bin0 << c->plan.bits[1];
    const bool stream_shape = n >= 8 * c->n_build;
    HJ_RADIX(c, st, hj::radix_join(true, c->plan, radix_work(c), r, bucket_set(c->sset), c->sset.max_runs,
                          (unsigned *)c->work_start.p, c->work_desc.p, out_r, out_s, out_cap,
                          (unsigned long long *)d_count, c->meta + 1, false, st, c->meta + 2, stream_shape,
                          nbins << c->plan.bits[1]));
    c->join_ran = true;
    c->join_wide = true;
    c->join_stream = stream_shape;
    record(c, kEvProbe1, st);
    c->evs().rec[2] = c->timing;
    c->evs().rec_mid = c->timing;
    return HJ_OK;
}

int hj_partition_of(int64_t key, int nparts) {
    if (nparts < 1) return -1;
    unsigned long long k = (unsigned long long)key;
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return (int)(((k >> 32) * (unsigned long long)(unsigned)nparts) >> 32);
}

int hj_dev_gen_pkfk_i64(uint64_t seed, int64_t NR, uint64_t hit_threshold, int64_t r0, int64_t nr, int64_t *rkey,
                        int64_t *rpay, int64_t s0, int64_t ns, int64_t *skey, int64_t *spay, void *stream) {
    if (NR <= 0 || nr < 0 || ns < 0) HJ_FAIL(HJ_ERR_ARG, "bad generator sizes");
    HJ_HIP(hj::launch_gen_pkfk(seed, NR, hit_threshold, r0, nr, (long long *)rkey, (long long *)rpay, s0, ns,
                               (long long *)skey, (long long *)spay, (hipStream_t)stream));
    return HJ_OK;
}
int hj_zipf_params(int64_t NR, double theta, double out[4]) {
    if (NR < 1 || !(theta > 0.0 && theta < 1.0) || !out) HJ_FAIL(HJ_ERR_ARG, "zipf: NR >= 1 and 0 < theta < 1");
    // zeta(n, theta) = sum_{k=1..n} k^-theta: exact below 2^20 terms, then
    // Euler-Maclaurin for the tail (relative error < 1e-12 at n = 2^28)
    const int64_t m = NR < (1ll << 20) ? NR : (1ll << 20);
    double z = 0.0;
    for (int64_t k = m; k >= 1; --k) z += std::pow((double)k, -theta);
    if (NR > m) {
        const double a = (double)m, b = (double)NR, e = 1.0 - theta;
        z += (std::pow(b, e) - std::pow(a, e)) / e + 0.5 * (std::pow(b, -theta) - std::pow(a, -theta)) -
             theta / 12.0 * (std::pow(b, -theta - 1.0) - std::pow(a, -theta - 1.0));
    }
    double z2 = 1.0 + std::pow(2.0, -theta);
    out[0] = z;
    out[1] = (1.0 - std::pow(2.0 / (double)NR, 1.0 - theta)) / (1.0 - z2 / z);
    out[2] = 1.0 / (1.0 - theta);
    out[3] = std::pow(0.5, theta);
    return HJ_OK;
}

int hj_dev_gen_zipf_i64(uint64_t seed, int64_t NR, double theta, int64_t s0, int64_t ns, int64_t *skey,
                        int64_t *spay, void *stream) {
    double p[4];
    HJ_TRY(hj_zipf_params(NR, theta, p));
    if (ns < 0) HJ_FAIL(HJ_ERR_ARG, "bad generator sizes");
    hj::ZipfParams z;
    z.zetan = p[0];
    z.eta = p[1];
    z.alpha = p[2];
    z.half_pow_theta = p[3];
    z.n = (unsigned long long)NR;
    HJ_HIP(hj::launch_gen_zipf(seed, z, s0, ns, (long long *)skey, (long long *)spay, (hipStream_t)stream));
    return HJ_OK;
}

int hj_dev_gen_uniform_i64(uint64_t seed, uint64_t stream_id, int64_t lo, int64_t hi, int64_t i0, int64_t n,
                           int64_t *key, int64_t *pay, void *stream) {
    if (hi < lo || n < 0) HJ_FAIL(HJ_ERR_ARG, "bad generator range");
    HJ_HIP(hj::launch_gen_uniform_i64(seed, stream_id, lo, hi, i0, n, (long long *)key, (long long *)pay,
                                      (hipStream_t)stream));
    return HJ_OK;
}
int hj_dev_gen_uniform_i32(uint64_t seed, uint64_t stream_id, int32_t lo, int32_t hi, int64_t i0, int64_t n,
                           int32_t *key, void *stream) {
    if (hi < lo || n < 0) HJ_FAIL(HJ_ERR_ARG, "bad generator range");
    HJ_HIP(hj::launch_gen_uniform_i32(seed, stream_id, lo, hi, i0, n, key, (hipStream_t)stream));
    return HJ_OK;
}

// ------------------------------------------------------- host memref ABI
int64_t hj_count_i32(int32_t *, int32_t *r_align, int64_t r_off, int64_t r_size, int64_t r_stride, int32_t *,
                     int32_t *s_align, int64_t s_off, int64_t s_size, int64_t s_stride) {
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0;
    void *a, *b;
    int rc = host_join(c, kNarrow, rel32(r_align, r_off, r_size, r_stride), rel32(s_align, s_off, s_size, s_stride),
                       kHostCount, &m, &a, &b);
    return rc == HJ_OK ? m : rc;
}

int32_t hj_probe_i32(int32_t *, int32_t *r_align, int64_t r_off, int64_t r_size, int64_t r_stride, int32_t *,
                     int32_t *s_align, int64_t s_off, int64_t s_size, int64_t s_stride, int32_t *,
                     int32_t *or_align, int64_t or_off, int64_t or_size, int64_t or_stride, int32_t *,
                     int32_t *os_align, int64_t os_off, int64_t os_size, int64_t os_stride) {
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0;
    void *d_or = nullptr, *d_os = nullptr;
    const Deliver put = [&](const void *a, const void *b, int64_t mm) -> int {
        if (or_size != mm || os_size != mm) return 1;
        HJ_TRY(download<int32_t>(or_align, or_off, mm, or_stride, a, c->host_stream));
        return download<int32_t>(os_align, os_off, mm, os_stride, b, c->host_stream);
    };
    bool sent = false;
    HJ_TRY(host_join(c, kNarrow, rel32(r_align, r_off, r_size, r_stride), rel32(s_align, s_off, s_size, s_stride),
                     kHostProbe, &m, &d_or, &d_os, or_size == os_size ? &put : nullptr, &sent));
    if (sent) return HJ_OK;
    if (or_size != m || os_size != m) HJ_FAIL(HJ_ERR_CAPACITY, "output memrefs must have exactly M rows");
    HJ_TRY(download<int32_t>(or_align, or_off, m, or_stride, d_or, c->host_stream));
    HJ_TRY(download<int32_t>(os_align, os_off, m, os_stride, d_os, c->host_stream));
    return HJ_OK;
}

int64_t hj_count_i64(int64_t *, int64_t *rk, int64_t rk_off, int64_t rk_size, int64_t rk_stride, int64_t *,
                     int64_t *rp, int64_t rp_off, int64_t rp_size, int64_t rp_stride, int64_t *, int64_t *sk,
                     int64_t sk_off, int64_t sk_size, int64_t sk_stride, int64_t *, int64_t *sp, int64_t sp_off,
                     int64_t sp_size, int64_t sp_stride) {
    if (rk_size != rp_size || sk_size != sp_size) HJ_FAIL(HJ_ERR_ARG, "key/payload sizes differ");
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0;
    void *a, *b;
    int rc = host_join(c, kWide, rel64(rk, rk_off, rk_stride, rp, rp_off, rp_stride, rk_size),
                       rel64(sk, sk_off, sk_stride, sp, sp_off, sp_stride, sk_size), kHostCount, &m, &a, &b);
    return rc == HJ_OK ? m : rc;
}

int32_t hj_probe_i64(int64_t *, int64_t *rk, int64_t rk_off, int64_t rk_size, int64_t rk_stride, int64_t *,
                     int64_t *rp, int64_t rp_off, int64_t rp_size, int64_t rp_stride, int64_t *, int64_t *sk,
                     int64_t sk_off, int64_t sk_size, int64_t sk_stride, int64_t *, int64_t *sp, int64_t sp_off,
                     int64_t sp_size, int64_t sp_stride, int64_t *, int64_t *or_align, int64_t or_off,
                     int64_t or_size, int64_t or_stride, int64_t *, int64_t *os_align, int64_t os_off,
                     int64_t os_size, int64_t os_stride) {
    if (rk_size != rp_size || sk_size != sp_size) HJ_FAIL(HJ_ERR_ARG, "key/payload sizes differ");
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0;
    void *d_or = nullptr, *d_os = nullptr;
    const Deliver put = [&](const void *a, const void *b, int64_t mm) -> int {
        if (or_size != mm || os_size != mm) return 1;
        HJ_TRY(download<int64_t>(or_align, or_off, mm, or_stride, a, c->host_stream));
        return download<int64_t>(os_align, os_off, mm, os_stride, b, c->host_stream);
    };
    bool sent = false;
    HJ_TRY(host_join(c, kWide, rel64(rk, rk_off, rk_stride, rp, rp_off, rp_stride, rk_size),
                     rel64(sk, sk_off, sk_stride, sp, sp_off, sp_stride, sk_size), kHostProbe, &m, &d_or, &d_os,
                     or_size == os_size ? &put : nullptr, &sent));
    if (sent) return HJ_OK;
    if (or_size != m || os_size != m) HJ_FAIL(HJ_ERR_CAPACITY, "output memrefs must have exactly M rows");
    HJ_TRY(download<int64_t>(or_align, or_off, m, or_stride, d_or, c->host_stream));
    HJ_TRY(download<int64_t>(os_align, os_off, m, os_stride, d_os, c->host_stream));
    return HJ_OK;
}

// ------------------------------------------------------ MLIR C-interface
void _mlir_ciface_hj_join_i32(hj_memref2_i32 *res, hj_memref1_i32 *r, hj_memref1_i32 *s) {
    if (!res) return;
    std::memset(res, 0, sizeof(*res));
    if (!r || !s) {
        fail(HJ_ERR_ARG, __FILE__, __LINE__, "null memref descriptor");
        return;
    }
    hj_ctx *c = default_ctx();
    if (!c) return;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0;
    void *d_or = nullptr, *d_os = nullptr;
    if (host_join(c, kNarrow, rel32(r->aligned, r->offset, r->sizes[0], r->strides[0]),
                  rel32(s->aligned, s->offset, s->sizes[0], s->strides[0]), kHostJoin, &m, &d_or, &d_os) != HJ_OK)
        return;
    fill_result<int32_t>(res, d_or, d_os, m, c->host_stream);
}

void _mlir_ciface_hj_join_i64(hj_memref2_i64 *res, hj_memref1_i64 *r, hj_memref1_i64 *s) {
    if (!res) return;
    std::memset(res, 0, sizeof(*res));
    if (!r || !s) {
        fail(HJ_ERR_ARG, __FILE__, __LINE__, "null memref descriptor");
        return;
    }
    hj_ctx *c = default_ctx();
    if (!c) return;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0;
    void *d_or = nullptr, *d_os = nullptr;
    if (host_join(c, kWide, rel64(r->aligned, r->offset, r->strides[0], nullptr, 0, 1, r->sizes[0]),
                  rel64(s->aligned, s->offset, s->strides[0], nullptr, 0, 1, s->sizes[0]), kHostJoin, &m, &d_or,
                  &d_os) != HJ_OK)
        return;
    fill_result<int64_t>(res, d_or, d_os, m, c->host_stream);
}

void _mlir_ciface_hj_join_kp_i64(hj_memref2_i64 *res, hj_memref1_i64 *rk, hj_memref1_i64 *rp, hj_memref1_i64 *sk,
                                 hj_memref1_i64 *sp) {
    if (!res) return;
    std::memset(res, 0, sizeof(*res));
    if (!rk || !rp || !sk || !sp || rk->sizes[0] != rp->sizes[0] || sk->sizes[0] != sp->sizes[0]) {
        fail(HJ_ERR_ARG, __FILE__, __LINE__, "bad key/payload memrefs");
        return;
    }
    hj_ctx *c = default_ctx();
    if (!c) return;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0;
    void *d_or = nullptr, *d_os = nullptr;
    if (host_join(c, kWide, rel64(rk->aligned, rk->offset, rk->strides[0], rp->aligned, rp->offset, rp->strides[0],
                                  rk->sizes[0]),
                  rel64(sk->aligned, sk->offset, sk->strides[0], sp->aligned, sp->offset, sp->strides[0], sk->sizes[0]),
                  kHostJoin, &m, &d_or, &d_os) != HJ_OK)
        return;
    fill_result<int64_t>(res, d_or, d_os, m, c->host_stream);
}

// ------------------------------------------------- nested-loop.mlir rows
int hj_dev_count_rows_i32(hj_ctx *c, const int32_t *t1, int64_t r1, int64_t c1, int64_t ld1, const int32_t *t2,
                          int64_t r2, int64_t c2, int64_t ld2, uint64_t *d_count, void *stream) {
    HJ_HIP(hipMemsetAsync(d_count, 0, sizeof(uint64_t), (hipStream_t)stream));
    return do_join_rows(c, RowTables{t1, r1, c1, ld1, t2, r2, c2, ld2}, nullptr, 0, 0, d_count, true,
                        (hipStream_t)stream);
}

int hj_dev_join_rows_i32(hj_ctx *c, const int32_t *t1, int64_t r1, int64_t c1, int64_t ld1, const int32_t *t2,
                         int64_t r2, int64_t c2, int64_t ld2, int32_t *out, int64_t ldo, int64_t out_cap,
                         uint64_t *d_count, void *stream) {
    return do_join_rows(c, RowTables{t1, r1, c1, ld1, t2, r2, c2, ld2}, out, ldo, out_cap, d_count, false,
                        (hipStream_t)stream);
}

int64_t hj_count_rows_i32(int32_t *, int32_t *a1, int64_t o1, int64_t r1, int64_t c1, int64_t s10, int64_t s11,
                          int32_t *, int32_t *a2, int64_t o2, int64_t r2, int64_t c2, int64_t s20, int64_t s21) {
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0, oc = 0;
    void *d = nullptr;
    const int rc = host_join_rows(c, a1, o1, r1, c1, s10, s11, a2, o2, r2, c2, s20, s21, true, &m, &oc, &d);
    return rc == HJ_OK ? m : rc;
}

int64_t hj_join_rows_i32(int32_t *, int32_t *a1, int64_t o1, int64_t r1, int64_t c1, int64_t s10, int64_t s11,
                         int32_t *, int32_t *a2, int64_t o2, int64_t r2, int64_t c2, int64_t s20, int64_t s21,
                         int32_t *, int32_t *ao, int64_t oo, int64_t ro, int64_t co, int64_t so0, int64_t so1) {
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0, oc = 0;
    void *d = nullptr;
    HJ_TRY(host_join_rows(c, a1, o1, r1, c1, s10, s11, a2, o2, r2, c2, s20, s21, false, &m, &oc, &d));
    if (co != oc) HJ_FAIL(HJ_ERR_ARG, "result memref must have c1 + c2 - 1 columns");
    if (ro < m) HJ_FAIL(HJ_ERR_CAPACITY, "result memref has fewer rows than the join");
    if (m > 0) {
        if (!ao) HJ_FAIL(HJ_ERR_ARG, "null result memref");
        std::vector<int32_t> tmp((size_t)(m * oc));
        HJ_HIP(hipMemcpyAsync(tmp.data(), d, sizeof(int32_t) * tmp.size(), hipMemcpyDeviceToHost, c->host_stream));
        HJ_HIP(hipStreamSynchronize(c->host_stream));
        int32_t *base = ao + oo;
        for (int64_t i = 0; i < m; ++i)
            for (int64_t j = 0; j < oc; ++j) base[i * so0 + j * so1] = tmp[(size_t)(i * oc + j)];
    }
    return m;
}

void _mlir_ciface_hj_join_rows_i32(hj_memref2_i32 *res, hj_memref2_i32 *t1, hj_memref2_i32 *t2) {
    if (!res) return;
    std::memset(res, 0, sizeof(*res));
    if (!t1 || !t2) {
        fail(HJ_ERR_ARG, __FILE__, __LINE__, "null memref descriptor");
        return;
    }
    hj_ctx *c = default_ctx();
    if (!c) return;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    int64_t m = 0, oc = 0;
    void *d = nullptr;
    if (host_join_rows(c, t1->aligned, t1->offset, t1->sizes[0], t1->sizes[1], t1->strides[0], t1->strides[1],
                       t2->aligned, t2->offset, t2->sizes[0], t2->sizes[1], t2->strides[0], t2->strides[1], false,
                       &m, &oc, &d) != HJ_OK)
        return;
    int32_t *h = (int32_t *)std::malloc(sizeof(int32_t) * (size_t)(m > 0 ? m * oc : 1));
    if (!h) {
        fail(HJ_ERR_NOMEM, __FILE__, __LINE__, "malloc result");
        return;
    }
    if (m > 0) {
        if (hipMemcpyAsync(h, d, sizeof(int32_t) * (size_t)(m * oc), hipMemcpyDeviceToHost, c->host_stream) !=
                hipSuccess ||
            hipStreamSynchronize(c->host_stream) != hipSuccess) {
            std::free(h);
            fail(HJ_ERR_HIP, __FILE__, __LINE__, "copy result");
            return;
        }
    }
    res->allocated = res->aligned = h;
    res->offset = 0;
    res->sizes[0] = m;
    res->sizes[1] = oc;
    res->strides[0] = oc;
    res->strides[1] = 1;
}

// ------------------------------------------------------------- selection
int hj_dev_select_f32(hj_ctx *c, const float *in, int64_t n, int cmp, float value, float *out, int64_t *out_row,
                      int64_t out_cap, uint64_t *d_count, void *stream) {
    return do_select<float>(c, in, n, cmp, value, out, out_row, out_cap, d_count, (hipStream_t)stream);
}

int hj_dev_select_i64(hj_ctx *c, const int64_t *in, int64_t n, int cmp, int64_t value, int64_t *out,
                      int64_t *out_row, int64_t out_cap, uint64_t *d_count, void *stream) {
    return do_select<int64_t>(c, in, n, cmp, value, out, out_row, out_cap, d_count, (hipStream_t)stream);
}

int hj_dev_stream_copy(const void *in, void *out, int64_t rows, int shape, void *stream) {
    if (shape != HJ_COPY_PERSISTENT && shape != HJ_COPY_FLAT) HJ_FAIL(HJ_ERR_ARG, "bad copy shape");
    if (rows < 0) HJ_FAIL(HJ_ERR_ARG, "negative row count");
    if (rows > 0 && (!in || !out || (((uintptr_t)in | (uintptr_t)out) & 15)))
        HJ_FAIL(HJ_ERR_ARG, "copy buffers must be non-null and 16-B aligned");
    int dev = 0, cus = 0;
    HJ_HIP(hipGetDevice(&dev));
    HJ_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HJ_HIP(hj::launch_stream_copy(in, out, rows, shape, cus, (hipStream_t)stream));
    return HJ_OK;
}

int64_t hj_select_f32(float *, float *in, int64_t in_off, int64_t in_size, int64_t in_stride, float value, float *,
                      float *out, int64_t out_off, int64_t out_size, int64_t out_stride) {
    hj_ctx *c = default_ctx();
    if (!c) return HJ_ERR_HIP;
    std::lock_guard<std::mutex> host_lk(c->host_mu);
    if (in_size < 0 || out_size < 0) HJ_FAIL(HJ_ERR_ARG, "negative memref size");
    HJ_TRY(set_device(c));
    HJ_TRY(host_stream(c));
    hipStream_t st = c->host_stream;
    void *din, *dout;
    HJ_TRY(dbuf(c, 0, sizeof(float) * (size_t)in_size, &din));
    HJ_TRY(dbuf(c, 1, sizeof(float) * (size_t)(in_size > 0 ? in_size : 1), &dout));
    HJ_TRY(upload<float>(din, in, in_off, in_size, in_stride, st));
    HJ_TRY(do_select<float>(c, (const float *)din, in_size, HJ_CMP_LT, value, (float *)dout, nullptr, in_size,
                            (uint64_t *)c->dcount, st));
    uint64_t m = 0;
    HJ_HIP(hipMemcpyAsync(&m, c->dcount, 8, hipMemcpyDeviceToHost, st));
    HJ_HIP(hipStreamSynchronize(st));
    if ((int64_t)m > out_size) HJ_FAIL(HJ_ERR_CAPACITY, "result memref smaller than the selection");
    HJ_TRY(download<float>(out, out_off, (int64_t)m, out_stride, dout, st));
    return (int64_t)m;
}

void hj_free_result(void *allocated) { std::free(allocated); }

}  // extern "C"

void hj_placement_stats(long long *probes, long long *rejected, double *last_kept, double *worst_kept) {
    std::lock_guard<std::mutex> lk(g_place_mu);
    if (probes) *probes = g_place.probes;
    if (rejected) *rejected = g_place.rejected;
    if (last_kept) *last_kept = g_place.last_kept;
    if (worst_kept) *worst_kept = g_place.worst_kept;
}

void hj_placement_stats_ex(long long out[5], double *last_kept, double *worst_kept) {
    std::lock_guard<std::mutex> lk(g_place_mu);
    if (out) {
        out[0] = g_place.probes;
        out[1] = g_place.rejected;
        out[2] = g_place.gave_up;
        out[3] = g_place.gave_up_low_mem;
        out[4] = g_place.held_max;
    }
    if (last_kept) *last_kept = g_place.last_kept;
    if (worst_kept) *worst_kept = g_place.worst_kept;
}

double hj_placement_set_good(double ratio) {
    const float prev = g_place_good.load();
    if (ratio > 0.0) g_place_good.store((float)ratio);
    return (double)prev;
}

int hj_placement_check(const void *buf, int64_t bytes, double *ratio) {
    if (!buf || bytes <= 0 || !ratio) HJ_FAIL(HJ_ERR_ARG, "placement check: null buffer / ratio or no bytes");
    *ratio = 0.0;
    int dev = 0, cus = 0;
    HJ_HIP(hipGetDevice(&dev));
    HJ_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    float r = 0.0f;
    const hipError_t e = hj::placement_probe(const_cast<void *>(buf), (size_t)bytes, size_t(16) << hj::kPassPbl, cus, &r);
    if (e == hipErrorInvalidValue) HJ_FAIL(HJ_ERR_ARG, "placement check: buffer below 4 MiB per CU");
    HJ_HIP(e);
    *ratio = r;
    return HJ_OK;
}
