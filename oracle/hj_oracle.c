/*
 * hj_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hash join (deveshv-99/mlir-HashJoin,
 * /root/reference) used as the parity checker for the MI355X HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline -- the product
 * path (mlir-hashjoin_amd/) never links or calls it.
 *
 * Pinning: the restatement is checked against the reference's own result
 * definition, shared_stuff/shared.cpp:check() (nested-loop join, sort,
 * compare; shared.cpp:129-172), compiled from the reference sources into
 * oracle/_ref/ by oracle/Makefile, and against the golden fixtures in
 * tests/golden/ that tests/golden/make_golden.py generated and
 * cross-checked with that compiled check().
 *
 * Every function cites the reference file:line it restates.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* Deterministic synthetic inputs.  The reference seeds rand() from the     */
/* clock (shared.cpp:62, :86-87), so its inputs cannot be reproduced; we    */
/* use a counter-based generator whose definition is shared   */
/* bit-for-bit with the HIP generator in mlir-hashjoin_amd/csrc/hj_gen.h.   */
/* ------------------------------------------------------------------------ */

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t oracle_fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

uint64_t oracle_rand(uint64_t seed, uint64_t stream, uint64_t idx) {
    return mix64(seed + 0x9E3779B97F4A7C15ull * (idx + 1) + stream * 0xD1B54A32D192ED03ull);
}

/* PK-FK relation pair: R keys unique, R.pay = global row,
 * S keys drawn from R (hit) or from a disjoint miss domain, S.pay = global row.
 * Rows [r0, r0+nr) of R and [s0, s0+ns) of S are produced, so a shard
 * generates exactly its slice of the global relations. */
void oracle_gen_pkfk_i64(uint64_t seed, int64_t NR, uint64_t hit_thr,
                         int64_t r0, int64_t nr, int64_t *rkey, int64_t *rpay,
                         int64_t s0, int64_t ns, int64_t *skey, int64_t *spay) {
    const uint64_t salt = mix64(seed ^ 0x5EEDull);
    for (int64_t i = 0; i < nr; ++i) {
        uint64_t g = (uint64_t)(r0 + i);
        rkey[i] = (int64_t)oracle_fmix64(g ^ salt);
        rpay[i] = (int64_t)g;
    }
    for (int64_t j = 0; j < ns; ++j) {
        uint64_t g = (uint64_t)(s0 + j);
        uint64_t u = oracle_rand(seed, 1, g) % (uint64_t)NR;
        int hit = (hit_thr == UINT64_MAX) || (oracle_rand(seed, 2, g) < hit_thr);
        uint64_t src = hit ? u : ((uint64_t)NR + g);
        skey[j] = (int64_t)oracle_fmix64(src ^ salt);
        spay[j] = (int64_t)g;
    }
}

/* Zipf(theta) probe keys over the PK-FK build side of the same seed (the HIP
 * generator's definition, mlir-hashjoin_amd/csrc/hj_gen.h; params from
 * hj_zipf_params): rank by the Gray et al. inverse CDF, rank -> build row by an
 * odd-multiplier map, S.key = R.key[row].  libm pow() may differ from the
 * device's in the last ulp, so a rare rank can differ (tests allow it). */
void oracle_gen_zipf_i64(uint64_t seed, int64_t NR, double zetan, double eta, double alpha, double half_pow_theta,
                         int64_t s0, int64_t ns, int64_t *skey, int64_t *spay) {
    const uint64_t salt = mix64(seed ^ 0x5EEDull);
    for (int64_t j = 0; j < ns; ++j) {
        const uint64_t g = (uint64_t)(s0 + j);
        const double u = (double)(oracle_rand(seed, 3, g) >> 11) * (1.0 / 9007199254740992.0);
        const double uz = u * zetan;
        uint64_t r;
        if (uz < 1.0) r = 0;
        else if (uz < 1.0 + half_pow_theta) r = 1;
        else {
            const double v = (double)NR * pow(eta * u - eta + 1.0, alpha);
            r = (uint64_t)v;
            if (r >= (uint64_t)NR) r = (uint64_t)NR - 1;
        }
        const uint64_t x = r * 0x9E3779B97F4A7C15ull + mix64(seed ^ 0x2197ull);
        const uint64_t row = ((NR & (NR - 1)) == 0) ? (x & (uint64_t)(NR - 1)) : (x % (uint64_t)NR);
        skey[j] = (int64_t)oracle_fmix64(row ^ salt);
        spay[j] = (int64_t)g;
    }
}

/* Reference-style uniform keys in [lo, hi] (shared.cpp:59-80 draws
 * rand() % (U-L+1) + L); pay = global row index (shared.cpp has no payload;
 * the row id is the implicit payload, join_v1.mlir:255). */
void oracle_gen_uniform_i64(uint64_t seed, uint64_t stream, int64_t lo, int64_t hi,
                            int64_t i0, int64_t n, int64_t *key, int64_t *pay) {
    uint64_t range = (uint64_t)(hi - lo) + 1ull;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t g = (uint64_t)(i0 + i);
        uint64_t r = oracle_rand(seed, stream, g);
        key[i] = lo + (int64_t)(range ? r % range : r);
        if (pay) pay[i] = (int64_t)g;
    }
}

void oracle_gen_uniform_i32(uint64_t seed, uint64_t stream, int32_t lo, int32_t hi,
                            int64_t i0, int64_t n, int32_t *key) {
    uint64_t range = (uint64_t)((int64_t)hi - (int64_t)lo) + 1ull;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t r = oracle_rand(seed, stream, (uint64_t)(i0 + i));
        key[i] = (int32_t)((int64_t)lo + (int64_t)(r % range));
    }
}

/* ------------------------------------------------------------------------ */
/* Restatement of join_v1.mlir / join_v2.mlir, serialised.                   */
/*                                                                           */
/* The GPU grid is executed thread by thread, block by block.  Every atomic  */
/* of the reference (freeIndex add, head exchange, block-offset add, LDS     */
/* buffer/global cursors) is therefore applied in one legal serial order;    */
/* the OUTPUT MULTISET does not depend on the order (only row positions do), */
/* which is what parity compares (shared.cpp:168-171 sorts before ==).       */
/* ------------------------------------------------------------------------ */

#define REF_BLOCK 256   /* @numberOfThreadsPerBlock, join_v2.mlir:10 */
#define REF_LDS_BUF 2048 /* tempResultBuffer size, join_v2.mlir:454-458 */

typedef struct {
    int32_t *heads;    /* hashTablePointers i32[H]   (join_v2.mlir:34) */
    int64_t *ll_key;   /* linkedListKey                (:29) - widened */
    int64_t *ll_row;   /* linkedListRowId index[]      (:30) */
    int64_t *ll_next;  /* linkedListnextIndex index[]  (:31) */
} chain_table;

/* hash = key urem H (join_v2.mlir:229-233, arith.remui i32).  For the i64
 * generalisation the remainder is taken on the unsigned 64-bit key. */
static inline uint64_t ref_hash_i32(int32_t k, uint64_t H) { return (uint64_t)((uint32_t)k % (uint32_t)H); }
static inline uint64_t ref_hash_i64(int64_t k, uint64_t H) { return (uint64_t)k % H; }

static int chain_alloc(chain_table *t, int64_t n, uint64_t H) {
    t->heads = (int32_t *)malloc(sizeof(int32_t) * (H ? H : 1));
    t->ll_key = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    t->ll_row = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    t->ll_next = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    if (!t->heads || !t->ll_key || !t->ll_row || !t->ll_next) return -1;
    /* kernel initializeHT: heads[i] = -1  (join_v2.mlir:203-225) */
    for (uint64_t i = 0; i < H; ++i) t->heads[i] = -1;
    return 0;
}

static void chain_free(chain_table *t) {
    free(t->heads); free(t->ll_key); free(t->ll_row); free(t->ll_next);
}

/* kernel build + @insertNodeInHashTable (join_v2.mlir:236-300): idx =
 * atomicAdd(freeIndex, 1); node = (key, rowId); old = atomicExch(head[h], idx);
 * next[idx] = old.  Serial thread order makes idx == tid. */
static void chain_build(chain_table *t, const int64_t *key, const int64_t *row, int64_t n,
                        uint64_t H, int key_is_i32) {
    int32_t free_index = 0;
    for (int64_t tid = 0; tid < n; ++tid) {
        int32_t idx = free_index++;
        t->ll_key[idx] = key[tid];
        t->ll_row[idx] = row ? row[tid] : tid;
        uint64_t h = key_is_i32 ? ref_hash_i32((int32_t)key[tid], H) : ref_hash_i64(key[tid], H);
        int32_t old = t->heads[h];
        t->heads[h] = idx;
        t->ll_next[idx] = (int64_t)old; /* index_cast of i32 -1 -> index -1 (:268) */
    }
}

/* chain walk of kernel count (join_v2.mlir:363-384): number of equal keys */
static int64_t chain_count_one(const chain_table *t, int64_t k, uint64_t H, int key_is_i32) {
    uint64_t h = key_is_i32 ? ref_hash_i32((int32_t)k, H) : ref_hash_i64(k, H);
    int64_t cur = t->heads[h], c = 0;
    while (cur != -1) {
        if (t->ll_key[cur] == k) ++c;
        cur = t->ll_next[cur];
    }
    return c;
}

/* kernel count (join_v2.mlir:311-439): per-thread count, thread-0 serial
 * exclusive scan over the block (:393-417), block offset via atomic add on
 * globalBlockOffset (:420), prefix[g] = blockBase + threadPrefix (:429-436).
 * Returns M (the final globalBlockOffset, read back at :139-146). */
static int64_t chain_count(const chain_table *t, const int64_t *skey, int64_t ns, uint64_t H,
                           int key_is_i32, int64_t *prefix) {
    int64_t global_block_offset = 0;
    for (int64_t b0 = 0; b0 < ns; b0 += REF_BLOCK) {
        int64_t bn = (ns - b0 < REF_BLOCK) ? ns - b0 : REF_BLOCK;
        int64_t off = 0;
        for (int64_t i = 0; i < bn; ++i) {
            int64_t c = chain_count_one(t, skey[b0 + i], H, key_is_i32);
            if (prefix) prefix[b0 + i] = off;
            off += c;
        }
        if (prefix)
            for (int64_t i = 0; i < bn; ++i) prefix[b0 + i] += global_block_offset;
        global_block_offset += off;
    }
    return global_block_offset;
}

/* kernel probe v1 (join_v1.mlir:436-521): private cursor seeded from
 * prefix[g], every match written at cursor++ as (rowR, rowS). */
static void chain_probe_v1(const chain_table *t, const int64_t *skey, const int64_t *spay, int64_t ns,
                           uint64_t H, int key_is_i32, const int64_t *prefix,
                           int64_t *out_r, int64_t *out_s, int64_t cap) {
    for (int64_t g = 0; g < ns; ++g) {
        int64_t k = skey[g];
        uint64_t h = key_is_i32 ? ref_hash_i32((int32_t)k, H) : ref_hash_i64(k, H);
        int64_t cur = t->heads[h];
        int64_t w = prefix[g];
        while (cur != -1) {
            if (t->ll_key[cur] == k) {
                if (w < cap) { out_r[w] = t->ll_row[cur]; out_s[w] = spay ? spay[g] : g; }
                ++w;
            }
            cur = t->ll_next[cur];
        }
    }
}

/* kernel probe v2 (join_v2.mlir:450-604): per block, matches go to a 2048-
 * entry LDS staging buffer via an LDS atomic cursor (:525-538); when full they
 * go straight to global memory at globalWriteIndex++ (:539-549); after the
 * barrier the buffer [0, min(bufIdx, 2048)) is flushed to globalWriteIndex+i
 * (:564-602).  globalWriteIndex starts at prefix[blockStart] (:481-490). */
static void chain_probe_v2(const chain_table *t, const int64_t *skey, const int64_t *spay, int64_t ns,
                           uint64_t H, int key_is_i32, const int64_t *prefix,
                           int64_t *out_r, int64_t *out_s, int64_t cap) {
    int64_t *buf_r = (int64_t *)malloc(sizeof(int64_t) * REF_LDS_BUF);
    int64_t *buf_s = (int64_t *)malloc(sizeof(int64_t) * REF_LDS_BUF);
    for (int64_t b0 = 0; b0 < ns; b0 += REF_BLOCK) {
        int64_t bn = (ns - b0 < REF_BLOCK) ? ns - b0 : REF_BLOCK;
        uint32_t buffer_index = 0;
        int64_t gwi = prefix[b0];
        for (int64_t i = 0; i < bn; ++i) {
            int64_t g = b0 + i, k = skey[g];
            uint64_t h = key_is_i32 ? ref_hash_i32((int32_t)k, H) : ref_hash_i64(k, H);
            int64_t cur = t->heads[h];
            while (cur != -1) {
                if (t->ll_key[cur] == k) {
                    uint32_t si = buffer_index++;
                    int64_t sv = spay ? spay[g] : g;
                    if (si < REF_LDS_BUF) { buf_r[si] = t->ll_row[cur]; buf_s[si] = sv; }
                    else {
                        int64_t w = gwi++;
                        if (w < cap) { out_r[w] = t->ll_row[cur]; out_s[w] = sv; }
                    }
                }
                cur = t->ll_next[cur];
            }
        }
        uint32_t upper = buffer_index > REF_LDS_BUF ? REF_LDS_BUF : buffer_index; /* :577-584 */
        for (uint32_t i = 0; i < upper; ++i) {
            int64_t w = gwi + i;
            if (w < cap) { out_r[w] = buf_r[i]; out_s[w] = buf_s[i]; }
        }
    }
    free(buf_r); free(buf_s);
}

/* @main sequence (join_v2.mlir:607-730) minus data generation and check:
 * initializeHT -> build -> count -> probe.  variant 1 = join_v1 probe,
 * 2 = join_v2 probe.  Writes min(M, cap) pairs, returns M (or -1 on OOM). */
static int64_t chained_join(const int64_t *rkey, const int64_t *rpay, int64_t nr,
                            const int64_t *skey, const int64_t *spay, int64_t ns,
                            uint64_t H, int variant, int key_is_i32,
                            int64_t *out_r, int64_t *out_s, int64_t cap) {
    if (H == 0) return -1;
    chain_table t;
    if (chain_alloc(&t, nr, H)) { chain_free(&t); return -1; }
    chain_build(&t, rkey, rpay, nr, H, key_is_i32);
    int64_t *prefix = (int64_t *)malloc(sizeof(int64_t) * (ns ? ns : 1));
    int64_t m = chain_count(&t, skey, ns, H, key_is_i32, prefix);
    if (m > 0 && out_r && out_s) {
        if (variant == 1) chain_probe_v1(&t, skey, spay, ns, H, key_is_i32, prefix, out_r, out_s, cap);
        else chain_probe_v2(&t, skey, spay, ns, H, key_is_i32, prefix, out_r, out_s, cap);
    }
    free(prefix);
    chain_free(&t);
    return m;
}

int64_t oracle_chained_join_i64(const int64_t *rkey, const int64_t *rpay, int64_t nr,
                                const int64_t *skey, const int64_t *spay, int64_t ns,
                                uint64_t H, int variant,
                                int64_t *out_r, int64_t *out_s, int64_t cap) {
    return chained_join(rkey, rpay, nr, skey, spay, ns, H, variant, 0, out_r, out_s, cap);
}

/* Reference-typed form: i32 keys, (rowR, rowS) i32 output (join_v2.mlir:
 * 450-452: memref<?xi32> relations and resultIndicesR/S). */
int64_t oracle_chained_join_i32(const int32_t *r, int64_t nr, const int32_t *s, int64_t ns,
                                uint32_t H, int variant,
                                int32_t *out_r, int32_t *out_s, int64_t cap) {
    int64_t *rk = (int64_t *)malloc(sizeof(int64_t) * (nr ? nr : 1));
    int64_t *sk = (int64_t *)malloc(sizeof(int64_t) * (ns ? ns : 1));
    for (int64_t i = 0; i < nr; ++i) rk[i] = r[i];
    for (int64_t i = 0; i < ns; ++i) sk[i] = s[i];
    int64_t *o_r = NULL, *o_s = NULL;
    if (cap > 0 && out_r && out_s) {
        o_r = (int64_t *)malloc(sizeof(int64_t) * cap);
        o_s = (int64_t *)malloc(sizeof(int64_t) * cap);
    }
    int64_t m = chained_join(rk, NULL, nr, sk, NULL, ns, H, variant, 1, o_r, o_s, o_r ? cap : 0);
    if (o_r) {
        int64_t w = m < cap ? m : cap;
        for (int64_t i = 0; i < w; ++i) { out_r[i] = (int32_t)o_r[i]; out_s[i] = (int32_t)o_s[i]; }
    }
    free(rk); free(sk); free(o_r); free(o_s);
    return m;
}

/* ------------------------------------------------------------------------ */
/* The same grid on host threads (OpenMP): the CPU baseline ("port" of the  */
/* reference's join_v2 lowered for CPU, SURVEY F7 / BASELINE.md 2).  The    */
/* reference atomics become host atomics; blocks become loop iterations.    */
/* phase_s[4] receives init/build/count/probe seconds.                      */
/* ------------------------------------------------------------------------ */
int64_t oracle_chained_join_i64_omp(const int64_t *rkey, const int64_t *rpay, int64_t nr,
                                    const int64_t *skey, const int64_t *spay, int64_t ns,
                                    uint64_t H, int threads,
                                    int64_t *out_r, int64_t *out_s, int64_t cap,
                                    double *phase_s) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
    double t0 = omp_get_wtime();
#endif
    if (H == 0) return -1;
    int32_t *heads = (int32_t *)malloc(sizeof(int32_t) * H);
    int64_t *ll_key = (int64_t *)malloc(sizeof(int64_t) * (nr ? nr : 1));
    int64_t *ll_row = (int64_t *)malloc(sizeof(int64_t) * (nr ? nr : 1));
    int64_t *ll_next = (int64_t *)malloc(sizeof(int64_t) * (nr ? nr : 1));
    int64_t *prefix = (int64_t *)malloc(sizeof(int64_t) * (ns ? ns : 1));
    int64_t nblocks = (ns + REF_BLOCK - 1) / REF_BLOCK;
    int64_t *block_base = (int64_t *)malloc(sizeof(int64_t) * (nblocks ? nblocks : 1));
    if (!heads || !ll_key || !ll_row || !ll_next || !prefix || !block_base) return -1;

    /* initializeHT */
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)H; ++i) heads[i] = -1;
#ifdef _OPENMP
    double t1 = omp_get_wtime();
#endif
    /* build: freeIndex fetch-add + head exchange (join_v2.mlir:247, :266) */
    int32_t free_index = 0;
    #pragma omp parallel for schedule(static)
    for (int64_t tid = 0; tid < nr; ++tid) {
        int32_t idx = __atomic_fetch_add(&free_index, 1, __ATOMIC_RELAXED);
        ll_key[idx] = rkey[tid];
        ll_row[idx] = rpay ? rpay[tid] : tid;
        uint64_t h = ref_hash_i64(rkey[tid], H);
        int32_t old = __atomic_exchange_n(&heads[h], idx, __ATOMIC_RELAXED);
        ll_next[idx] = (int64_t)old;
    }
#ifdef _OPENMP
    double t2 = omp_get_wtime();
#endif
    /* count: per block serial scan + atomic block offset (join_v2.mlir:389-436) */
    int64_t gbo = 0;
    #pragma omp parallel for schedule(dynamic, 64)
    for (int64_t b = 0; b < nblocks; ++b) {
        int64_t b0 = b * REF_BLOCK, bn = (ns - b0 < REF_BLOCK) ? ns - b0 : REF_BLOCK, off = 0;
        for (int64_t i = 0; i < bn; ++i) {
            int64_t k = skey[b0 + i], cur = heads[ref_hash_i64(k, H)], c = 0;
            while (cur != -1) { if (ll_key[cur] == k) ++c; cur = ll_next[cur]; }
            prefix[b0 + i] = off;
            off += c;
        }
        int64_t base = __atomic_fetch_add(&gbo, off, __ATOMIC_RELAXED);
        for (int64_t i = 0; i < bn; ++i) prefix[b0 + i] += base;
        block_base[b] = base;
    }
#ifdef _OPENMP
    double t3 = omp_get_wtime();
#endif
    /* probe v2 semantics per block (LDS staging == per-block local buffer) */
    if (out_r && out_s) {
        #pragma omp parallel
        {
            int64_t *buf_r = (int64_t *)malloc(sizeof(int64_t) * REF_LDS_BUF);
            int64_t *buf_s = (int64_t *)malloc(sizeof(int64_t) * REF_LDS_BUF);
            #pragma omp for schedule(dynamic, 64)
            for (int64_t b = 0; b < nblocks; ++b) {
                int64_t b0 = b * REF_BLOCK, bn = (ns - b0 < REF_BLOCK) ? ns - b0 : REF_BLOCK;
                uint32_t bi = 0;
                int64_t gwi = block_base[b];
                for (int64_t i = 0; i < bn; ++i) {
                    int64_t g = b0 + i, k = skey[g], cur = heads[ref_hash_i64(k, H)];
                    int64_t sv = spay ? spay[g] : g;
                    while (cur != -1) {
                        if (ll_key[cur] == k) {
                            uint32_t si = bi++;
                            if (si < REF_LDS_BUF) { buf_r[si] = ll_row[cur]; buf_s[si] = sv; }
                            else { int64_t w = gwi++; if (w < cap) { out_r[w] = ll_row[cur]; out_s[w] = sv; } }
                        }
                        cur = ll_next[cur];
                    }
                }
                uint32_t upper = bi > REF_LDS_BUF ? REF_LDS_BUF : bi;
                for (uint32_t i = 0; i < upper; ++i) {
                    int64_t w = gwi + i;
                    if (w < cap) { out_r[w] = buf_r[i]; out_s[w] = buf_s[i]; }
                }
            }
            free(buf_r); free(buf_s);
        }
    }
#ifdef _OPENMP
    double t4 = omp_get_wtime();
    if (phase_s) { phase_s[0] = t1 - t0; phase_s[1] = t2 - t1; phase_s[2] = t3 - t2; phase_s[3] = t4 - t3; }
#else
    if (phase_s) memset(phase_s, 0, 4 * sizeof(double));
#endif
    free(heads); free(ll_key); free(ll_row); free(ll_next); free(prefix); free(block_base);
    return gbo;
}

/* ------------------------------------------------------------------------ */
/* Nested-loop join = the reference's result definition                    */
/* (shared.cpp:154-165: i over R outer, j over S inner, pair (i, j)).        */
/* ------------------------------------------------------------------------ */
int64_t oracle_nested_loop_i64(const int64_t *rkey, const int64_t *rpay, int64_t nr,
                               const int64_t *skey, const int64_t *spay, int64_t ns,
                               int64_t *out_r, int64_t *out_s, int64_t cap) {
    int64_t m = 0;
    for (int64_t i = 0; i < nr; ++i)
        for (int64_t j = 0; j < ns; ++j)
            if (rkey[i] == skey[j]) {
                if (m < cap && out_r && out_s) { out_r[m] = rpay ? rpay[i] : i; out_s[m] = spay ? spay[j] : j; }
                ++m;
            }
    return m;
}

int64_t oracle_nested_loop_i32(const int32_t *r, int64_t nr, const int32_t *s, int64_t ns,
                               int32_t *out_r, int32_t *out_s, int64_t cap) {
    int64_t m = 0;
    for (int64_t i = 0; i < nr; ++i)
        for (int64_t j = 0; j < ns; ++j)
            if (r[i] == s[j]) {
                if (m < cap && out_r && out_s) { out_r[m] = (int32_t)i; out_s[m] = (int32_t)j; }
                ++m;
            }
    return m;
}

/* Count-only nested loop on host threads: the nested-loop.mlir CPU baseline
 * (its per-thread count pass, nested-loop.mlir:78-88, on OpenMP threads). */
int64_t oracle_nested_loop_count_i64_omp(const int64_t *rkey, int64_t nr,
                                         const int64_t *skey, int64_t ns, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    int64_t m = 0;
    #pragma omp parallel for schedule(static) reduction(+:m)
    for (int64_t i = 0; i < nr; ++i) {
        int64_t k = rkey[i], c = 0;
        for (int64_t j = 0; j < ns; ++j) c += (skey[j] == k);
        m += c;
    }
    return m;
}

/* ------------------------------------------------------------------------ */
/* nested-loop.mlir @nested_join (nested-loop.mlir:29-192) with its @main   */
/* table choice (:247-263): the larger table is the outer x (ties: table 1),*/
/* rows are written per x row in ascending j, each output row is            */
/* x[g][0..xc) ++ y[j][1..yc) (:160-188).  Block offsets are taken in block */
/* order with gblock_offset starting at 0.  Row-major i32 tables.           */
/* Returns the number of result rows (min(rows, cap_rows) written).         */
/* ------------------------------------------------------------------------ */
int64_t oracle_nested_join_rows_i32(const int32_t *t1, int64_t r1, int64_t c1,
                                    const int32_t *t2, int64_t r2, int64_t c2,
                                    int32_t *out, int64_t cap_rows) {
    int t2_outer = r1 < r2; /* %table_1_or_2_as_inner (:247) */
    const int32_t *x = t2_outer ? t2 : t1, *y = t2_outer ? t1 : t2;
    int64_t xr = t2_outer ? r2 : r1, xc = t2_outer ? c2 : c1;
    int64_t yr = t2_outer ? r1 : r2, yc = t2_outer ? c1 : c2;
    int64_t oc = xc + yc - 1, w = 0;
    for (int64_t g = 0; g < xr; ++g) {
        int32_t k = x[g * xc];
        for (int64_t j = 0; j < yr; ++j) {
            if (y[j * yc] != k) continue;
            if (w < cap_rows && out) {
                for (int64_t a = 0; a < xc; ++a) out[w * oc + a] = x[g * xc + a];
                for (int64_t b = 1; b < yc; ++b) out[w * oc + xc - 1 + b] = y[j * yc + b];
            }
            ++w;
        }
    }
    return w;
}

/* Experiments/selection.mlir @run_selection (:34-155), serialised: keep
 * d_arrayA[i] when the predicate holds (`cmpf olt` against %compare_val,
 * :69-70; generalised to op 0..5 = lt le gt ge eq ne, float compares
 * ordered), written in element order (one legal order of the reference's
 * per-block atomic offsets, :120-124).  Returns the count; writes at most
 * cap values (and their indices into rows, if non-NULL). */
int64_t oracle_select_f32(const float *a, int64_t n, int op, float c, float *out, int64_t *rows, int64_t cap) {
    int64_t w = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float v = a[i];
        int keep;
        switch (op) {
            case 0: keep = v < c; break;
            case 1: keep = v <= c; break;
            case 2: keep = v > c; break;
            case 3: keep = v >= c; break;
            case 4: keep = v == c; break;
            default: keep = v < c || v > c; break;
        }
        if (!keep) continue;
        if (w < cap) {
            if (out) out[w] = v;
            if (rows) rows[w] = i;
        }
        ++w;
    }
    return w;
}

int64_t oracle_select_i64(const int64_t *a, int64_t n, int op, int64_t c, int64_t *out, int64_t *rows, int64_t cap) {
    int64_t w = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t v = a[i];
        int keep;
        switch (op) {
            case 0: keep = v < c; break;
            case 1: keep = v <= c; break;
            case 2: keep = v > c; break;
            case 3: keep = v >= c; break;
            case 4: keep = v == c; break;
            default: keep = v != c; break;
        }
        if (!keep) continue;
        if (w < cap) {
            if (out) out[w] = v;
            if (rows) rows[w] = i;
        }
        ++w;
    }
    return w;
}

/* selection.mlir @init (:20-29): arr[i] = (float)i */
void oracle_selection_init_f32(float *a, int64_t n) {
    for (int64_t i = 0; i < n; ++i) a[i] = (float)(int32_t)i;
}

/* nested-loop.mlir @init (:7-24): t[i][j] = i + j */
void oracle_nested_init_i32(int32_t *t, int64_t rows, int64_t cols) {
    for (int64_t i = 0; i < rows; ++i)
        for (int64_t j = 0; j < cols; ++j) t[i * cols + j] = (int32_t)(i + j);
}

/* Order-independent digest of a pair multiset: sum and xor of a mixed hash of
 * each (r, s) pair.  Used for full-size (2^26..2^28) parity on the GPU box. */
void oracle_pair_digest_i64(const int64_t *r, const int64_t *s, int64_t m, uint64_t *sum, uint64_t *xr) {
    uint64_t a = 0, b = 0;
    for (int64_t i = 0; i < m; ++i) {
        uint64_t h = mix64((uint64_t)r[i] * 0x9E3779B97F4A7C15ull ^ mix64((uint64_t)s[i]));
        a += h; b ^= h;
    }
    *sum = a; *xr = b;
}
