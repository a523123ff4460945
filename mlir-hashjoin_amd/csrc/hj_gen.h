// hj_gen.h -- counter-based synthetic input generators shared by the HIP
// datagen kernels.  The definition is bit-identical to oracle/hj_oracle.c
// (oracle_rand / oracle_fmix64 / oracle_gen_*), which tests cross-check; the
// reference itself seeds rand() from the clock (shared_stuff/shared.cpp:62,
// :86-87), so there is no reproducible reference generator to follow.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define HJ_HD __host__ __device__ __forceinline__
#else
#define HJ_HD inline
#endif

namespace hj {

HJ_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

HJ_HD uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

HJ_HD uint64_t rand64(uint64_t seed, uint64_t stream, uint64_t idx) {
    return mix64(seed + 0x9E3779B97F4A7C15ull * (idx + 1) + stream * 0xD1B54A32D192ED03ull);
}

HJ_HD uint64_t pkfk_salt(uint64_t seed) { return mix64(seed ^ 0x5EEDull); }

// PK-FK: R.key[g] = fmix64(g ^ salt) (unique: fmix64 is a bijection);
// S.key[g] = R.key[u] for a hit, fmix64((NR + g) ^ salt) for a miss.
HJ_HD int64_t pkfk_rkey(uint64_t salt, uint64_t g) { return (int64_t)fmix64(g ^ salt); }

HJ_HD int64_t pkfk_skey(uint64_t seed, uint64_t salt, int64_t NR, uint64_t hit_thr, uint64_t g) {
    uint64_t u = rand64(seed, 1, g) % (uint64_t)NR;
    bool hit = (hit_thr == ~0ull) || (rand64(seed, 2, g) < hit_thr);
    uint64_t src = hit ? u : ((uint64_t)NR + g);
    return (int64_t)fmix64(src ^ salt);
}

// Zipf(theta) foreign keys over a unique build side: rank r
// in [0, NR) is drawn by the inverse-CDF approximation of Gray et al.
// ("Quickly generating billion-record synthetic databases", SIGMOD'94, the
// YCSB generator); r -> build row via an odd-multiplier map so hot ranks land
// on unrelated rows (and hash partitions).  S.key = R.key[row(r)].
struct ZipfParams {
    double zetan, eta, alpha, half_pow_theta;
    unsigned long long n;
};

HJ_HD unsigned long long zipf_rank(const ZipfParams &z, double u) {
    const double uz = u * z.zetan;
    if (uz < 1.0) return 0ull;
    if (uz < 1.0 + z.half_pow_theta) return 1ull;
    double v = (double)z.n * pow(z.eta * u - z.eta + 1.0, z.alpha);
    unsigned long long r = (unsigned long long)v;
    return r >= z.n ? z.n - 1 : r;
}

HJ_HD uint64_t zipf_row(uint64_t seed, uint64_t rank, uint64_t NR) {
    const uint64_t x = rank * 0x9E3779B97F4A7C15ull + mix64(seed ^ 0x2197ull);
    return (NR & (NR - 1)) == 0 ? (x & (NR - 1)) : (x % NR);
}

HJ_HD int64_t zipf_skey(uint64_t seed, const ZipfParams &z, uint64_t g) {
    const double u = (double)(rand64(seed, 3, g) >> 11) * (1.0 / 9007199254740992.0);   // [0, 1)
    return pkfk_rkey(pkfk_salt(seed), zipf_row(seed, zipf_rank(z, u), z.n));
}

}  // namespace hj
