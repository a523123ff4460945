/*
 * hj.h -- C ABI of the MI355X-native hash-join operator (libhj.so).
 *
 * Drop-in boundary for the reference's join program (deveshv-99/mlir-HashJoin,
 * SURVEY 8(b)).  Three layers, all plain C (pointers + sizes, no torch types):
 *
 *  1. Host memref ABI.  The reference's host functions take ranked 1-D
 *     memrefs, which MLIR's -finalize-memref-to-llvm / -convert-func-to-llvm
 *     expand into five scalars (allocated, aligned, offset, size, stride);
 *     see join_v1.ll:1262-1265 and shared_stuff/shared.cpp:35,59,83,129-132.
 *     hj_count_* / hj_probe_* use exactly that expansion, so a .mlir module
 *     declares them `func.func private` and links libhj.so through
 *     mlir-cpu-runner --shared-libs (run_test.sh:33), the way it links
 *     shared.so today (join_v1.mlir:651-658).
 *
 *  2. MLIR C-interface (`llvm.emit_c_interface`) one-memref-out joins:
 *     _mlir_ciface_hj_join_*(result*, R*, S*) -- the "two-memref-in /
 *     one-memref-out" entry point of north_star.  The result buffer is
 *     malloc'ed (allocated == aligned) so MLIR's memref.dealloc (free) or
 *     hj_free_result() releases it.
 *
 *  3. Device-resident phases (hj_dev_*): the hot path.  Inputs and outputs
 *     are device pointers, every call is asynchronous on the given HIP stream
 *     (NULL = default stream) and launches kernels only (no allocation, no
 *     synchronisation) once hj_ctx_reserve() has sized the workspace, so the
 *     sequence can be captured into a hipGraph.
 *
 * Semantics (all layers): an equi-join of R and S on the key column; the
 * output is the multiset {(R.pay[i], S.pay[j]) : R.key[i] == S.key[j]} --
 * every pair, duplicates on either side included, exactly the nested-loop
 * definition of shared_stuff/shared.cpp:154-165 (payload = row id in the
 * reference types).  Row order is unspecified (the reference's is decided by
 * atomics too); compare after sorting, as shared.cpp:168-171 does.
 *
 * Errors: functions returning int return HJ_OK (0) or a negative HJ_ERR_*;
 * hj_last_error() gives "file:line: message" of the last failure on this
 * thread.  The reference has no error channel besides check()'s 1/0/-1
 * (shared.cpp:158-171).
 */
#ifndef HJ_H_
#define HJ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HJ_ABI_VERSION 1

#define HJ_OK 0
#define HJ_ERR_ARG (-1)      /* bad argument / size mismatch */
#define HJ_ERR_HIP (-2)      /* HIP runtime error (see hj_last_error) */
#define HJ_ERR_NOMEM (-3)    /* device or host allocation failed */
#define HJ_ERR_STATE (-4)    /* call order: probe before build, wrong layout */
#define HJ_ERR_CAPACITY (-5) /* output memref smaller than the join result */

typedef struct hj_ctx hj_ctx;

int hj_abi_version(void);
const char *hj_last_error(void);
/* Device facts for the roofline: [0] CUs, [1] memory clock (kHz), [2] memory
 * bus width (bits), [3] L2 bytes (one XCD), [4] HBM bytes, [5] shader clock
 * (kHz), [6] LDS bytes per CU, [7] peak HBM MB/s = 4 x memory clock x bus
 * bytes (HBM3E: 4 transfers per reported clock). */
int hj_device_info(int device, int64_t out[8]);

/* ------------------------------------------------------------------ context
 * One context = one device + its hash-table workspace.  Replaces the
 * reference's @allocateHashTable (join_v2.mlir:25-39: gpu.alloc of heads and
 * linked list) -- allocation is hoisted out of the per-join path. */
hj_ctx *hj_ctx_create(int device);
void hj_ctx_destroy(hj_ctx *ctx);
/* Size the workspace for builds of up to max_build_rows rows with 32- or
 * 64-bit keys (key_bits = 32 | 64). */
int hj_ctx_reserve(hj_ctx *ctx, int64_t max_build_rows, int key_bits);
/* Probe-side workspace of the radix strategy (no-op for the global table). */
int hj_ctx_reserve_probe(hj_ctx *ctx, int64_t max_probe_rows, int key_bits);
/* Join strategy.  GLOBAL: one linear-probing table in HBM (build = 64-bit CAS
 * per row, probe = random slot reads).  RADIX: both relations radix-
 * partitioned by the key hash until a partition's build rows fit an LDS
 * table; partitions are joined in LDS.  AUTO picks RADIX for large build
 * sides.  The result multiset is identical. */
#define HJ_STRATEGY_AUTO 0
#define HJ_STRATEGY_GLOBAL 1
#define HJ_STRATEGY_RADIX 2
int hj_ctx_set_strategy(hj_ctx *ctx, int strategy);
/* RADIX: partition into exactly 2^bits partitions (1..24; 0 = planner's
 * choice, ~4096 build rows per partition).  For tests and tuning. */
int hj_ctx_set_radix_bits(hj_ctx *ctx, int bits);
/* Strategy of the last probe since the current build (else of the build):
 * HJ_STRATEGY_GLOBAL / _RADIX, 0 if none.  Under HJ_STRATEGY_AUTO a build side
 * of [2^18, 2^21) rows gets the global table AND a radix partition; a probe
 * side of >= 2^24 rows then takes the radix join. */
int hj_ctx_strategy_used(const hj_ctx *ctx);
/* The probe side's expected rows, given before the build (< 0: unknown, the
 * default).  AUTO with a [2^18, 2^21)-row build side then builds ONE
 * strategy instead of both: radix from 2^24 hinted probe rows on (2^22 for
 * build sides of >= 2^20 rows), else the global table (2^20 x 2^20: 0.21 ->
 * 0.15 ms per join; 2^20 x 2^22: 0.24 -> 0.20).  A later, larger probe still joins correctly, through
 * the global table.  HashJoin.join and the host memref entry points set it. */
int hj_ctx_probe_hint(hj_ctx *ctx, int64_t probe_rows);
/* GLOBAL: slot capacity of the table (power of two, >= 2 x build rows);
 * RADIX: number of partitions. */
int64_t hj_ctx_table_capacity(const hj_ctx *ctx);
/* RADIX: partition passes of the current build (1..3) and their fan-out bits
 * (bits[0..passes-1]); returns 0 passes for GLOBAL / no build. */
int hj_ctx_radix_plan(const hj_ctx *ctx, int *passes, int bits[3]);
/* 1 if the build side repeats a key, 0 if not (synchronises).  Known after
 * the build (GLOBAL) or after the first probe (RADIX: a repeat that a probe
 * row met is flagged by the join; the first call after a join whose kernel
 * was k_join_b checks every partition of the build side on the device,
 * including those no probe row reached and, after routed probes in several
 * bin ranges, every range). */
int hj_ctx_build_has_duplicates(hj_ctx *ctx);
/* Per-phase kernel timing with HIP events on the caller's stream. */
int hj_ctx_set_timing(hj_ctx *ctx, int enable);
/* ms of the last init, build, probe/count and partition launches (synchronises). */
int hj_ctx_last_timing(hj_ctx *ctx, float ms[4]);
/* Same plus the probe's split: [4] probe-side partitioning (RADIX, else 0),
 * [5] probe/join kernel; [6], [7] reserved (-1). */
int hj_ctx_last_timing_ex(hj_ctx *ctx, float ms[8]);
/* Accumulating timing (enable = 1; turns timing on): every build starts a
 * new event set of a 64-set ring and a set is read back only when the ring
 * comes round to it, so back-to-back build + probe steps run with no host
 * synchronisation between them (a probe repeated without a build replaces
 * that set's probe times).  Enabling again, or 0, drops what was recorded.
 * hj_ctx_timing_totals sums every recorded set (synchronises on them) into
 * ms[0..5] as hj_ctx_last_timing_ex orders them, *sets = how many, and
 * starts the totals again; HJ_ERR_STATE unless accumulating. */
int hj_ctx_timing_accumulate(hj_ctx *ctx, int enable);
int hj_ctx_timing_totals(hj_ctx *ctx, float ms[8], long long *sets);
/* RADIX: the join kernel of the last probe.  A pure function of the row
 * width, the probe / build size ratio (>= 8: the probe-heavy shape) and the
 * build side's repeated keys, sampled at build time over up to 64 partitions
 * -- never of an earlier join's statistics: HJ_JOIN_KERNEL_BUCKETED
 * (k_join_b), _STREAM (k_join_u, probe-heavy shape), _GROUPED (k_join_grp
 * over every item: most build keys repeated; i32 and, since round 5, int64
 * rows); 0 if the last probe was no radix join.  Items those kernels defer
 * (INT64_MIN build keys, oversized partitions) run k_join afterwards.
 * (_LINEAR, k_join_u outside the stream shape, and _GENERAL, k_join over
 * every int64 item, are no longer chosen since round 5.)  Synchronises. */
#define HJ_JOIN_KERNEL_BUCKETED 1
#define HJ_JOIN_KERNEL_LINEAR 2
#define HJ_JOIN_KERNEL_STREAM 3
#define HJ_JOIN_KERNEL_GROUPED 4
#define HJ_JOIN_KERNEL_GENERAL 5
int hj_ctx_join_kernel(hj_ctx *ctx);

/* ------------------------------------------------------------ device phases
 * build:  @initializeHashTable + @buildTable   (join_v2.mlir:54-108)
 * count:  @countRows                           (join_v2.mlir:110-147)
 * probe:  @probeRelation                       (join_v2.mlir:149-199)
 * d_count (device uint64): set to M, the exact number of result rows, even
 * when M > out_cap (rows past out_cap are dropped; re-run with a larger
 * output).  The counter is zeroed by the call.  Bit 63 set means an internal
 * work list overflowed (a sizing bug, never expected): the result is invalid
 * and the host entry points return HJ_ERR_CAPACITY for it. */

/* 64-bit key / 64-bit payload column pairs (north_star types). */
int hj_dev_build_i64(hj_ctx *ctx, const int64_t *rkey, const int64_t *rpay, int64_t n, void *stream);
int hj_dev_count_i64(hj_ctx *ctx, const int64_t *skey, int64_t n, uint64_t *d_count, void *stream);
int hj_dev_probe_i64(hj_ctx *ctx, const int64_t *skey, const int64_t *spay, int64_t n,
                     int64_t *out_r, int64_t *out_s, int64_t out_cap, uint64_t *d_count, void *stream);
/* Same with rows as packed 16-B {key, payload} tuples (the exchange format). */
int hj_dev_build_tuples_i64(hj_ctx *ctx, const int64_t *tuples, int64_t n, void *stream);
int hj_dev_probe_tuples_i64(hj_ctx *ctx, const int64_t *tuples, int64_t n,
                            int64_t *out_r, int64_t *out_s, int64_t out_cap, uint64_t *d_count, void *stream);

/* Reference types: i32 keys, payload = row id (global thread index in
 * join_v1.mlir:255), (rowR, rowS) i32 output (join_v1.mlir:604-605).
 * row_base is added to row ids (0 for the reference). */
int hj_dev_build_i32(hj_ctx *ctx, const int32_t *rkey, int64_t n, int64_t row_base, void *stream);
int hj_dev_count_i32(hj_ctx *ctx, const int32_t *skey, int64_t n, uint64_t *d_count, void *stream);
int hj_dev_probe_i32(hj_ctx *ctx, const int32_t *skey, int64_t n, int64_t row_base,
                     int32_t *out_r, int32_t *out_s, int64_t out_cap, uint64_t *d_count, void *stream);

/* Radix partition of rows into nparts (1..8192) groups by a key hash independent of
 * the table's slot hash: out_tuples (2*n int64) receives packed {key, pay}
 * tuples grouped by partition in order 0..nparts-1, d_counts (nparts uint64)
 * the group sizes.  Multi-GPU routing step (north_star: "build-side
 * partitioning ... probe tuples routed by the same radix"). */
int hj_dev_partition_i64(hj_ctx *ctx, const int64_t *key, const int64_t *pay, int64_t n, int nparts,
                         int64_t *out_tuples, uint64_t *d_counts, void *stream);
int hj_dev_partition_tuples_i64(hj_ctx *ctx, const int64_t *tuples, int64_t n, int nparts,
                                int64_t *out_tuples, uint64_t *d_counts, void *stream);
/* Owning partition of one key (host-side, same function as the kernels). */
int hj_partition_of(int64_t key, int nparts);

/* Folded routing (north_star: "probe tuples routed by the same radix"): a
 * row's owner AND its receiver's first radix-pass bin are the top
 * log2(nranks) + sub_bits bits of the radix join's own key hash, so the
 * received tuples are already first-pass partitioned and the receiver runs
 * one local pass fewer per relation (R and S).
 * hj_route_plan: sub_bits for a join of n_build_global build rows over nranks
 * ranks (a power of two, <= 64); *sub_bits = 0 when the fold does not apply
 * (small or non-radix local build sides, other rank counts): route with
 * hj_dev_partition_* then.  The same value on every rank. */
int hj_route_plan(int64_t n_build_global, int nranks, int *sub_bits);
/* out_tuples (2n int64): packed {key, pay} grouped by part = owner << sub_bits
 * | bin (<= 512 parts), parts in order; d_counts (nranks << sub_bits uint64):
 * part sizes.  One exact partition pass (line-tailed, like a radix pass) after
 * a key histogram. */
int hj_dev_route_i64(hj_ctx *ctx, const int64_t *key, const int64_t *pay, int64_t n, int nranks, int sub_bits,
                     int64_t *out_tuples, uint64_t *d_counts, void *stream);
/* Build from routed tuples: nsrc sources' rows one after another, each
 * source's grouped by bin 0 .. 2^sub_bits - 1; d_counts (device, nsrc x
 * 2^sub_bits uint64, row s = source s's bin sizes).  nranks, sub_bits as
 * routed. */
int hj_dev_build_routed_i64(hj_ctx *ctx, const int64_t *tuples, int64_t n, const uint64_t *d_counts, int nsrc,
                            int nranks, int sub_bits, void *stream);
/* Probe routed tuples of bins [bin0, bin0 + nbins) only (the part of the probe
 * side that has arrived), laid out as for the build; d_counts nsrc x nbins.
 * Output as hj_dev_probe_i64. */
int hj_dev_probe_routed_i64(hj_ctx *ctx, const int64_t *tuples, int64_t n, const uint64_t *d_counts, int nsrc,
                            int bin0, int nbins, int64_t *out_r, int64_t *out_s, int64_t out_cap, uint64_t *d_count,
                            void *stream);

/* Deterministic synthetic relations (counter-based, so any slice of a
 * global relation can be generated independently on any GPU). */
int hj_dev_gen_pkfk_i64(uint64_t seed, int64_t NR, uint64_t hit_threshold,
                        int64_t r0, int64_t nr, int64_t *rkey, int64_t *rpay,
                        int64_t s0, int64_t ns, int64_t *skey, int64_t *spay, void *stream);
/* Zipf(theta) probe keys over the PK-FK build side of the same seed: S.key =
 * R.key[row(rank)], rank ~ Zipf(theta) over [0, NR) (Gray et al. inverse
 * CDF), S.pay = global row.  hj_zipf_params returns
 * {zeta(NR, theta), eta, alpha, 0.5^theta} (host, for the oracle). */
int hj_zipf_params(int64_t NR, double theta, double out[4]);
int hj_dev_gen_zipf_i64(uint64_t seed, int64_t NR, double theta, int64_t s0, int64_t ns, int64_t *skey,
                        int64_t *spay, void *stream);
int hj_dev_gen_uniform_i64(uint64_t seed, uint64_t stream_id, int64_t lo, int64_t hi,
                           int64_t i0, int64_t n, int64_t *key, int64_t *pay, void *stream);
int hj_dev_gen_uniform_i32(uint64_t seed, uint64_t stream_id, int32_t lo, int32_t hi,
                           int64_t i0, int64_t n, int32_t *key, void *stream);

/* nested-loop.mlir result rows (:29-192, @main :195-289).  Row-major int32
 * tables with the key in column 0 and row strides ld1 / ld2 (elements).
 * Roles as %table_1_or_2_as_inner (:247): the larger table is the outer X
 * (ties: t1), the smaller the inner Y; every pair X[i][0] == Y[j][0] yields
 * the row [X[i][0 .. cx), Y[j][1 .. cy)] (cx + cy - 1 columns).  Executed as
 * a hash join (build Y, probe X) plus a row gather.  d_count = M; rows past
 * out_cap are dropped.  Rows are in no particular order (as the reference's
 * atomic block offsets). */
int hj_dev_count_rows_i32(hj_ctx *ctx, const int32_t *t1, int64_t r1, int64_t c1, int64_t ld1, const int32_t *t2,
                          int64_t r2, int64_t c2, int64_t ld2, uint64_t *d_count, void *stream);
int hj_dev_join_rows_i32(hj_ctx *ctx, const int32_t *t1, int64_t r1, int64_t c1, int64_t ld1, const int32_t *t2,
                         int64_t r2, int64_t c2, int64_t ld2, int32_t *out, int64_t ldo, int64_t out_cap,
                         uint64_t *d_count, void *stream);

/* Selection (Experiments/selection.mlir:34-155): the elements v of `in`
 * with `v <cmp> value`, compacted in input order into out[0 .. min(M,
 * out_cap)), their source indices into out_row (optional, may be NULL);
 * d_count = M.  Float compares are ordered: NaN never passes (the reference
 * uses `cmpf olt`). */
#define HJ_CMP_LT 0
#define HJ_CMP_LE 1
#define HJ_CMP_GT 2
#define HJ_CMP_GE 3
#define HJ_CMP_EQ 4
#define HJ_CMP_NE 5
int hj_dev_select_f32(hj_ctx *ctx, const float *in, int64_t n, int cmp, float value, float *out, int64_t *out_row,
                      int64_t out_cap, uint64_t *d_count, void *stream);
int hj_dev_select_i64(hj_ctx *ctx, const int64_t *in, int64_t n, int cmp, int64_t value, int64_t *out,
                      int64_t *out_row, int64_t out_cap, uint64_t *d_count, void *stream);

/* Copy floor (measurement helper, no reference counterpart: SURVEY 8(d)
 * asks every figure to be set against the box's own HBM rate).  Copies
 * `rows` 16-B rows from `in` to `out` (device pointers, 16-B aligned) with
 * non-temporal loads and stores, in one of two shapes:
 *   HJ_COPY_PERSISTENT: one 1024-thread workgroup per CU over a contiguous
 *     range of 4096-row tiles, next tile's loads in flight (the radix
 *     partition passes' loop shape);
 *   HJ_COPY_FLAT: one row per thread over a grid of 256-thread workgroups
 *     (the fastest streamed copy this chip runs).
 * Asynchronous on `stream`; HJ_ERR_ARG for a bad shape or misaligned
 * pointer. */
#define HJ_COPY_PERSISTENT 0
#define HJ_COPY_FLAT 1
int hj_dev_stream_copy(const void *in, void *out, int64_t rows, int shape, void *stream);

/* Placement of the radix bucket sets' row buffers (diagnostics, no reference
 * counterpart).  A row buffer of >= 1 GiB (buckets >= 8 KiB) is probed when allocated: the
 * partition pass's write pattern against a flat write of the same bytes
 * (some physical placements run the pattern 25-35 % slower), redrawn up to 24
 * times while slow, best draw kept; HJ_PLACEMENT_PROBE=0 in the environment
 * turns the probe off.  Process-wide counts since load: draws probed, draws
 * rejected, and the pattern/flat ratio of the last and of the worst kept
 * buffer (0 when none was probed).  Any pointer may be null. */
void hj_placement_stats(long long *probes, long long *rejected, double *last_kept, double *worst_kept);
/* Since round 6 a probe holds at most 2 rejected draws at once (a further
 * reject frees the oldest) and draws again only while free memory is >= 3x
 * the buffer.  out[0] draws probed, [1] rejected, [2] buffers that kept a
 * slow draw (gave up), [3] of those, gave up because free memory ran short,
 * [4] most rejected draws held at once; ratios as hj_placement_stats. */
void hj_placement_stats_ex(long long out[5], double *last_kept, double *worst_kept);
/* The pattern/flat ratio a draw must reach to be kept at once (default
 * 1.12); returns the previous value, ratio <= 0 only reads it.  A knob for
 * tests (a low ratio makes every draw a reject). */
double hj_placement_set_good(double ratio);
/* The same probe on a caller's device buffer of >= 4 MiB per CU (its
 * contents are overwritten): *ratio = pass-pattern time / flat-write time
 * (~1.0 good placement, 1.25-1.35 slow).  Synchronous on the default stream.
 * The Python host side draws the routed-tuple buffers of hj_dev_route_i64
 * with it (hashjoin.HashJoin.route). */
int hj_placement_check(const void *buf, int64_t bytes, double *ratio);

/* Out-of-core join of HOST-resident int64 key/payload columns (relations
 * larger than HBM; the reference leaves the partitioned join out,
 * projectDescription.md:23-24).  When R does not fit device_budget bytes
 * (0 = 80 % of free HBM), R and S are routed by hj_partition_of into groups
 * that do, through the GPU in chunks; each group is built on the GPU and its
 * S side streamed through the probe with copies overlapping the probe.
 * Pairs (R.pay, S.pay) go to out_r/out_s (host); returns M (rows past
 * out_cap dropped) or < 0. */
int64_t hj_host_join_ooc_i64(hj_ctx *ctx, const int64_t *rkey, const int64_t *rpay, int64_t nr, const int64_t *skey,
                             const int64_t *spay, int64_t ns, int64_t *out_r, int64_t *out_s, int64_t out_cap,
                             uint64_t device_budget);

/* ------------------------------------------------------- host memref ABI
 * Two-phase, reference-shaped (mirrors @countRows -> alloc -> @probeRelation,
 * join_v2.mlir:672-688).  Each memref is the 5-scalar expansion; offset and
 * stride of every memref are honoured.  hj_probe_* returns HJ_OK, or
 * HJ_ERR_CAPACITY when the output memrefs' size differs from the join's row
 * count.
 *
 * Count -> probe reuse: the reference's @countRows leaves its table for
 * @probeRelation (join_v1.mlir:110-176).  hj_count_* uploads both relations,
 * BUILDS and COUNTS (no pairs are materialised) and keeps the built table and
 * the staged probe side.  A following hj_probe_* with inputs of the same
 * sizes probes that kept table (no upload, no build) when the inputs are
 * judged unchanged since the count, under the process-wide reuse mode:
 *   HJ_REUSE_DIGEST (default): a 128-bit content digest of every input
 *     memref, taken by the count and again by the probe on host threads
 *     (four multiply-rotate lanes, hj_capi.cpp digest_mem), matches.  The
 *     digest is NOT cryptographic: inputs crafted to collide with the counted
 *     ones would be joined as the counted ones.
 *   HJ_REUSE_EXACT: every input byte equals the count's (the count keeps a
 *     compacted host copy of its inputs -- host memory of the inputs' size --
 *     and the probe compares with memcmp on host threads).
 *   HJ_REUSE_OFF: nothing is kept; every hj_probe_* runs the whole join.
 * Anything else (changed inputs, another mode, another build in between)
 * runs the whole join.  Reused or not, the result is the join of the inputs
 * passed to hj_probe_*.
 * Output delivery is speculative: while the verdict is computed the kept
 * table's pairs are already written into the caller's output memrefs (when
 * their size equals the count's M); if the inputs turn out changed, the fresh
 * join's pairs are written over them.  On any error return the contents of
 * the output memrefs are undefined.  hj_host_memo_hits() counts the reuses.
 *
 * Threading: these host-memref entry points (and the ciface / rows /
 * selection ones below) use one default context per device; each call holds
 * that context's lock, so concurrent callers are serialised, never mixed. */
#define HJ_REUSE_DIGEST 0
#define HJ_REUSE_EXACT 1
#define HJ_REUSE_OFF 2
/* Set the reuse mode; returns the previous one, or HJ_ERR_ARG. */
int hj_host_set_reuse(int mode);
int64_t hj_host_memo_hits(void);
int64_t hj_count_i32(int32_t *r_alloc, int32_t *r_align, int64_t r_off, int64_t r_size, int64_t r_stride,
                     int32_t *s_alloc, int32_t *s_align, int64_t s_off, int64_t s_size, int64_t s_stride);
int32_t hj_probe_i32(int32_t *r_alloc, int32_t *r_align, int64_t r_off, int64_t r_size, int64_t r_stride,
                     int32_t *s_alloc, int32_t *s_align, int64_t s_off, int64_t s_size, int64_t s_stride,
                     int32_t *or_alloc, int32_t *or_align, int64_t or_off, int64_t or_size, int64_t or_stride,
                     int32_t *os_alloc, int32_t *os_align, int64_t os_off, int64_t os_size, int64_t os_stride);
/* int64 key/payload column pairs (Rkey, Rpay, Skey, Spay). */
int64_t hj_count_i64(int64_t *rk_alloc, int64_t *rk_align, int64_t rk_off, int64_t rk_size, int64_t rk_stride,
                     int64_t *rp_alloc, int64_t *rp_align, int64_t rp_off, int64_t rp_size, int64_t rp_stride,
                     int64_t *sk_alloc, int64_t *sk_align, int64_t sk_off, int64_t sk_size, int64_t sk_stride,
                     int64_t *sp_alloc, int64_t *sp_align, int64_t sp_off, int64_t sp_size, int64_t sp_stride);
int32_t hj_probe_i64(int64_t *rk_alloc, int64_t *rk_align, int64_t rk_off, int64_t rk_size, int64_t rk_stride,
                     int64_t *rp_alloc, int64_t *rp_align, int64_t rp_off, int64_t rp_size, int64_t rp_stride,
                     int64_t *sk_alloc, int64_t *sk_align, int64_t sk_off, int64_t sk_size, int64_t sk_stride,
                     int64_t *sp_alloc, int64_t *sp_align, int64_t sp_off, int64_t sp_size, int64_t sp_stride,
                     int64_t *or_alloc, int64_t *or_align, int64_t or_off, int64_t or_size, int64_t or_stride,
                     int64_t *os_alloc, int64_t *os_align, int64_t os_off, int64_t os_size, int64_t os_stride);

/* nested-loop.mlir rows over host 2-D memrefs (7 scalars each: allocated,
 * aligned, offset, sizes[2], strides[2]).  hj_join_rows_i32 writes the M rows
 * into the result memref (>= M rows, c1 + c2 - 1 columns) and returns M, or
 * < 0 (HJ_ERR_CAPACITY when the result has fewer than M rows). */
int64_t hj_count_rows_i32(int32_t *t1_alloc, int32_t *t1_align, int64_t t1_off, int64_t t1_rows, int64_t t1_cols,
                          int64_t t1_s0, int64_t t1_s1, int32_t *t2_alloc, int32_t *t2_align, int64_t t2_off,
                          int64_t t2_rows, int64_t t2_cols, int64_t t2_s0, int64_t t2_s1);
int64_t hj_join_rows_i32(int32_t *t1_alloc, int32_t *t1_align, int64_t t1_off, int64_t t1_rows, int64_t t1_cols,
                         int64_t t1_s0, int64_t t1_s1, int32_t *t2_alloc, int32_t *t2_align, int64_t t2_off,
                         int64_t t2_rows, int64_t t2_cols, int64_t t2_s0, int64_t t2_s1, int32_t *o_alloc,
                         int32_t *o_align, int64_t o_off, int64_t o_rows, int64_t o_cols, int64_t o_s0,
                         int64_t o_s1);

/* selection.mlir's query over host memrefs: in[i] < value (olt) compacted
 * into the result memref; returns M, or < 0 (HJ_ERR_CAPACITY if the result
 * memref is shorter than M). */
int64_t hj_select_f32(float *in_alloc, float *in_align, int64_t in_off, int64_t in_size, int64_t in_stride,
                      float value, float *out_alloc, float *out_align, int64_t out_off, int64_t out_size,
                      int64_t out_stride);

/* ------------------------------------------------------ MLIR C-interface
 * Descriptor structs of memref<?xT> / memref<?x2xT> (MLIR's StridedMemRefType
 * layout: allocated, aligned, offset, sizes[rank], strides[rank]). */
typedef struct { int32_t *allocated; int32_t *aligned; int64_t offset; int64_t sizes[1]; int64_t strides[1]; } hj_memref1_i32;
typedef struct { int64_t *allocated; int64_t *aligned; int64_t offset; int64_t sizes[1]; int64_t strides[1]; } hj_memref1_i64;
typedef struct { int32_t *allocated; int32_t *aligned; int64_t offset; int64_t sizes[2]; int64_t strides[2]; } hj_memref2_i32;
typedef struct { int64_t *allocated; int64_t *aligned; int64_t offset; int64_t sizes[2]; int64_t strides[2]; } hj_memref2_i64;

/* memref<?xi32> R, S -> memref<?x2xi32> rows (rowR, rowS): the reference's
 * whole @main join (join_v2.mlir:607-730) as one call. */
void _mlir_ciface_hj_join_i32(hj_memref2_i32 *result, hj_memref1_i32 *r, hj_memref1_i32 *s);
/* memref<?xi64> R, S keys (payload = row id) -> memref<?x2xi64> (rowR, rowS). */
void _mlir_ciface_hj_join_i64(hj_memref2_i64 *result, hj_memref1_i64 *r, hj_memref1_i64 *s);
/* key/payload column pairs -> memref<?x2xi64> (R.pay, S.pay). */
void _mlir_ciface_hj_join_kp_i64(hj_memref2_i64 *result, hj_memref1_i64 *rkey, hj_memref1_i64 *rpay,
                                 hj_memref1_i64 *skey, hj_memref1_i64 *spay);
/* memref<?x?xi32> tables -> memref<?x?xi32> rows of nested-loop.mlir
 * (exactly M rows, malloc'ed). */
void _mlir_ciface_hj_join_rows_i32(hj_memref2_i32 *result, hj_memref2_i32 *t1, hj_memref2_i32 *t2);
/* Release a result buffer of the ciface joins (== free(allocated)). */
void hj_free_result(void *allocated);

#ifdef __cplusplus
}
#endif

#endif /* HJ_H_ */
