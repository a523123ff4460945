// hj_ooc.cpp -- out-of-core join of host-resident relations (SURVEY 8(f)
// rank 3; the reference leaves "Partitioned Hash-Join" out,
// projectDescription.md:23-24).
//
// Grace-style over the device phases of include/hj.h:
//   1. when R does not fit the device budget: stream R and S through the GPU
//      in chunks, route every row to one of K groups with
//      hj_dev_partition_i64 (fmix64 routing hash, independent of the table
//      and radix bits) and copy each routed chunk back into one page-locked
//      host buffer per relation; a group is the list of its slices of those
//      chunks (no host-side copying);
//   2. per group (or once, when R fits): copy R_g in and build it; stream S_g
//      through hj_dev_probe_* in chunks of <= 2^25 rows with two chunks in
//      flight: chunk i+1 is copied in on one stream and chunk i-1's pairs
//      copied out on another while chunk i is probed.
// The user's arrays are page-locked for the duration of the call when the
// runtime allows (hipHostRegister), so copies run at PCIe DMA rate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>

#include "hj.h"
#include "hj_internal.h"

namespace {

struct Pin {   // page-lock a host range for the call (best effort)
    void *p = nullptr;
    explicit Pin(const void *ptr, size_t bytes) {
        if (ptr && bytes && hipHostRegister(const_cast<void *>(ptr), bytes, hipHostRegisterDefault) == hipSuccess)
            p = const_cast<void *>(ptr);
        else
            (void)hipGetLastError();
    }
    ~Pin() {
        if (p) (void)hipHostUnregister(p);
    }
    Pin(const Pin &) = delete;
    Pin &operator=(const Pin &) = delete;
};

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    bool ensure(size_t b) {
        if (b == 0) b = 16;
        if (bytes >= b) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, b) != hipSuccess) return false;
        bytes = b;
        return true;
    }
};

// Page-locked host staging of routed tuples, kept across calls (pinning
// gigabytes costs far more than the copies it speeds up).
struct HostPool {
    std::mutex mu;
    void *p[2] = {nullptr, nullptr};
    size_t bytes[2] = {0, 0};
    ~HostPool() {
        for (void *x : p)
            if (x) (void)hipHostFree(x);
    }
    int64_t *get(int i, size_t b) {
        if (b == 0) b = 16;
        if (bytes[i] < b) {
            if (p[i]) (void)hipHostFree(p[i]);
            p[i] = nullptr;
            bytes[i] = 0;
            if (hipHostMalloc(&p[i], b, hipHostMallocDefault) != hipSuccess) return nullptr;
            bytes[i] = b;
        }
        return (int64_t *)p[i];
    }
};
HostPool g_pool;

struct Streams {
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    ~Streams() {
        for (hipStream_t s : {h2d, comp, d2h})
            if (s) (void)hipStreamDestroy(s);
    }
};

struct Events {
    hipEvent_t e[8] = {};
    ~Events() {
        for (hipEvent_t x : e)
            if (x) (void)hipEventDestroy(x);
    }
};

#define OOC_HIP(x)                                  \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) return HJ_ERR_HIP;    \
    } while (0)
#define OOC_TRY(x)                    \
    do {                              \
        int rc_ = (x);                \
        if (rc_ != HJ_OK) return rc_; \
    } while (0)

// Device bytes per row (conservative): a build row as input plus the radix
// bucket sets; a probe row as input, bucket sets and one output pair.
constexpr uint64_t kBuildRowBytes = 64;
constexpr uint64_t kProbeRowBytes = 96;
constexpr int64_t kMaxChunk = 1ll << 25;   // rows per streamed chunk (pipelining granularity)

// A probe side on the host: key/payload columns, or spans of packed tuples.
struct Span {
    const int64_t *tup;
    int64_t n;
};
struct ProbeSide {
    const int64_t *key = nullptr, *pay = nullptr;
    int64_t n = 0;
    std::vector<Span> spans;   // tuples form when non-empty
};

// Stream `s` through the current build; pairs go to (out_r, out_s) from *m
// on (rows past out_cap dropped, *m counts them all).
int probe_stream(hj_ctx *c, const ProbeSide &s, int64_t chunk, int64_t *out_r, int64_t *out_s, int64_t out_cap,
                 int64_t *m, Streams &st) {
    // chunk list: (span index, first row, rows)
    struct Piece {
        const int64_t *tup;
        int64_t i0, n;
    };
    std::vector<Piece> pieces;
    if (s.spans.empty()) {
        for (int64_t i0 = 0; i0 < s.n; i0 += chunk) pieces.push_back({nullptr, i0, std::min(chunk, s.n - i0)});
    } else {
        for (const Span &sp : s.spans)
            for (int64_t i0 = 0; i0 < sp.n; i0 += chunk) pieces.push_back({sp.tup, i0, std::min(chunk, sp.n - i0)});
    }
    if (pieces.empty()) return HJ_OK;
    DevBuf in[2], o_r[2], o_s[2], cnt;
    int64_t ocap[2] = {chunk, chunk};   // pairs per chunk before a resize (>= chunk for a key join)
    for (int b = 0; b < 2; ++b)
        if (!in[b].ensure((size_t)chunk * 16) || !o_r[b].ensure((size_t)chunk * 8) || !o_s[b].ensure((size_t)chunk * 8))
            return HJ_ERR_NOMEM;
    if (!cnt.ensure(64)) return HJ_ERR_NOMEM;
    Events ev;   // 0,1 loaded; 2,3 input free; 4,5 output free
    for (int i = 0; i < 6; ++i) OOC_HIP(hipEventCreateWithFlags(&ev.e[i], hipEventDisableTiming));
    for (int b = 0; b < 2; ++b) {
        OOC_HIP(hipEventRecord(ev.e[2 + b], st.comp));
        OOC_HIP(hipEventRecord(ev.e[4 + b], st.d2h));
    }
    auto upload = [&](size_t k, int b) -> int {
        const Piece &pc = pieces[k];
        OOC_HIP(hipStreamWaitEvent(st.h2d, ev.e[2 + b], 0));
        if (pc.tup) {
            OOC_HIP(hipMemcpyAsync(in[b].p, pc.tup + 2 * pc.i0, (size_t)pc.n * 16, hipMemcpyHostToDevice, st.h2d));
        } else {
            OOC_HIP(hipMemcpyAsync(in[b].p, s.key + pc.i0, (size_t)pc.n * 8, hipMemcpyHostToDevice, st.h2d));
            OOC_HIP(hipMemcpyAsync((char *)in[b].p + (size_t)chunk * 8, s.pay + pc.i0, (size_t)pc.n * 8,
                                   hipMemcpyHostToDevice, st.h2d));
        }
        OOC_HIP(hipEventRecord(ev.e[b], st.h2d));
        return HJ_OK;
    };
    OOC_TRY(upload(0, 0));
    for (size_t k = 0; k < pieces.size(); ++k) {
        const int b = (int)(k & 1);
        const Piece &pc = pieces[k];
        if (k + 1 < pieces.size()) OOC_TRY(upload(k + 1, b ^ 1));   // next chunk's copy overlaps this probe
        OOC_HIP(hipStreamWaitEvent(st.comp, ev.e[b], 0));
        OOC_HIP(hipStreamWaitEvent(st.comp, ev.e[4 + b], 0));   // this output buffer's last copy-out is done
        uint64_t got = 0;
        for (int pass = 0; pass < 2; ++pass) {
            const int64_t *dk = (const int64_t *)in[b].p;
            int rc = pc.tup ? hj_dev_probe_tuples_i64(c, dk, pc.n, (int64_t *)o_r[b].p, (int64_t *)o_s[b].p, ocap[b],
                                                      (uint64_t *)cnt.p, st.comp)
                            : hj_dev_probe_i64(c, dk, (const int64_t *)((const char *)in[b].p + (size_t)chunk * 8),
                                               pc.n, (int64_t *)o_r[b].p, (int64_t *)o_s[b].p, ocap[b],
                                               (uint64_t *)cnt.p, st.comp);
            if (rc != HJ_OK) return rc;
            OOC_HIP(hipMemcpyAsync(&got, cnt.p, 8, hipMemcpyDeviceToHost, st.comp));
            OOC_HIP(hipStreamSynchronize(st.comp));
            if ((int64_t)got <= ocap[b]) break;
            ocap[b] = (int64_t)got;   // duplicates: exact M known, probe again with room for it
            if (!o_r[b].ensure((size_t)ocap[b] * 8) || !o_s[b].ensure((size_t)ocap[b] * 8)) return HJ_ERR_NOMEM;
        }
        OOC_HIP(hipEventRecord(ev.e[2 + b], st.comp));   // input buffer reusable
        const int64_t put = std::max<int64_t>(0, std::min<int64_t>((int64_t)got, out_cap - *m));
        if (put > 0) {   // copy-out overlaps the next chunk's probe
            OOC_HIP(hipMemcpyAsync(out_r + *m, o_r[b].p, (size_t)put * 8, hipMemcpyDeviceToHost, st.d2h));
            OOC_HIP(hipMemcpyAsync(out_s + *m, o_s[b].p, (size_t)put * 8, hipMemcpyDeviceToHost, st.d2h));
        }
        OOC_HIP(hipEventRecord(ev.e[4 + b], st.d2h));
        *m += (int64_t)got;
    }
    OOC_HIP(hipStreamSynchronize(st.d2h));
    return HJ_OK;
}

// Route (key, pay) columns into K groups: each chunk is routed on the GPU and
// copied back whole into `staged` (16 B per row, chunk order); group g's rows
// are the slices spans[g].
int route(hj_ctx *c, const int64_t *key, const int64_t *pay, int64_t n, int K, int64_t chunk, int64_t *staged,
          std::vector<std::vector<Span>> &spans, Streams &st) {
    DevBuf dk, dp, dt, dc;
    const int64_t ch = std::min<int64_t>(chunk, std::max<int64_t>(n, 1));
    if (!dk.ensure((size_t)ch * 8) || !dp.ensure((size_t)ch * 8) || !dt.ensure((size_t)ch * 16) ||
        !dc.ensure((size_t)K * 8))
        return HJ_ERR_NOMEM;
    std::vector<uint64_t> cnt((size_t)K);
    for (int64_t i0 = 0; i0 < n; i0 += ch) {
        const int64_t m = std::min<int64_t>(ch, n - i0);
        OOC_HIP(hipMemcpyAsync(dk.p, key + i0, (size_t)m * 8, hipMemcpyHostToDevice, st.comp));
        OOC_HIP(hipMemcpyAsync(dp.p, pay + i0, (size_t)m * 8, hipMemcpyHostToDevice, st.comp));
        OOC_TRY(hj_dev_partition_i64(c, (const int64_t *)dk.p, (const int64_t *)dp.p, m, K, (int64_t *)dt.p,
                                     (uint64_t *)dc.p, st.comp));
        OOC_HIP(hipMemcpyAsync(cnt.data(), dc.p, (size_t)K * 8, hipMemcpyDeviceToHost, st.comp));
        OOC_HIP(hipMemcpyAsync(staged + 2 * i0, dt.p, (size_t)m * 16, hipMemcpyDeviceToHost, st.comp));
        OOC_HIP(hipStreamSynchronize(st.comp));
        int64_t off = i0;
        for (int g = 0; g < K; ++g) {
            if (cnt[(size_t)g]) spans[(size_t)g].push_back({staged + 2 * off, (int64_t)cnt[(size_t)g]});
            off += (int64_t)cnt[(size_t)g];
        }
    }
    return HJ_OK;
}

}  // namespace

extern "C" int64_t hj_host_join_ooc_i64(hj_ctx *c, const int64_t *rk, const int64_t *rp, int64_t nr, const int64_t *sk,
                                        const int64_t *sp, int64_t ns, int64_t *out_r, int64_t *out_s,
                                        int64_t out_cap, uint64_t device_budget) {
    if (!c || nr < 0 || ns < 0 || out_cap < 0) return HJ_ERR_ARG;
    if ((nr > 0 && (!rk || !rp)) || (ns > 0 && (!sk || !sp)) || (out_cap > 0 && (!out_r || !out_s)))
        return HJ_ERR_ARG;
    OOC_TRY(hj_ctx_reserve(c, 0, 64));   // selects the context's device
    if (device_budget == 0) {
        size_t fr = 0, tot = 0;
        OOC_HIP(hipMemGetInfo(&fr, &tot));
        device_budget = (uint64_t)(fr / 10 * 8);
    }
    Streams st;
    for (hipStream_t *s : {&st.h2d, &st.comp, &st.d2h}) OOC_HIP(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
    Pin p1(rk, (size_t)nr * 8), p2(rp, (size_t)nr * 8), p3(sk, (size_t)ns * 8), p4(sp, (size_t)ns * 8);
    Pin p5(out_r, (size_t)out_cap * 8), p6(out_s, (size_t)out_cap * 8);
    // half the budget for the resident build side, a quarter for each of the
    // two probe chunks in flight
    const int64_t r_fit = (int64_t)std::max<uint64_t>(1, device_budget / 2 / kBuildRowBytes);
    const int64_t chunk = std::min<int64_t>(kMaxChunk, (int64_t)std::max<uint64_t>(1024, device_budget / 4 / kProbeRowBytes));
    int64_t m = 0;
    if (nr <= r_fit) {   // in-core build, streamed probe
        OOC_TRY(hj_ctx_reserve(c, nr, 64));
        DevBuf dk, dp;
        if (!dk.ensure((size_t)nr * 8) || !dp.ensure((size_t)nr * 8)) return HJ_ERR_NOMEM;
        OOC_HIP(hipMemcpyAsync(dk.p, rk, (size_t)nr * 8, hipMemcpyHostToDevice, st.comp));
        OOC_HIP(hipMemcpyAsync(dp.p, rp, (size_t)nr * 8, hipMemcpyHostToDevice, st.comp));
        OOC_TRY(hj_dev_build_i64(c, (const int64_t *)dk.p, (const int64_t *)dp.p, nr, st.comp));
        ProbeSide s;
        s.key = sk;
        s.pay = sp;
        s.n = ns;
        OOC_TRY(probe_stream(c, s, chunk, out_r, out_s, out_cap, &m, st));
        OOC_HIP(hipStreamSynchronize(st.comp));
        return m;
    }
    // grace: K groups of R that fit the budget (x1.5 headroom for skew)
    int K = 2;
    while ((int64_t)K * r_fit < nr + nr / 2 && K < hj::kMaxRouteParts) K *= 2;   // (groups may then exceed the budget)
    std::lock_guard<std::mutex> lk(g_pool.mu);   // one grace join at a time uses the staging
    int64_t *hr = g_pool.get(0, (size_t)nr * 16), *hs = g_pool.get(1, (size_t)ns * 16);
    if (!hr || !hs) return HJ_ERR_NOMEM;
    std::vector<std::vector<Span>> gr((size_t)K), gs((size_t)K);
    OOC_TRY(route(c, rk, rp, nr, K, chunk, hr, gr, st));
    OOC_TRY(route(c, sk, sp, ns, K, chunk, hs, gs, st));
    DevBuf dt;
    for (int g = 0; g < K; ++g) {
        int64_t n_r = 0;
        for (const Span &x : gr[(size_t)g]) n_r += x.n;
        ProbeSide s;
        s.spans = gs[(size_t)g];
        for (const Span &x : s.spans) s.n += x.n;
        if (n_r == 0 || s.n == 0) continue;
        OOC_TRY(hj_ctx_reserve(c, n_r, 64));
        if (!dt.ensure((size_t)n_r * 16)) return HJ_ERR_NOMEM;
        int64_t off = 0;
        for (const Span &x : gr[(size_t)g]) {
            OOC_HIP(hipMemcpyAsync((int64_t *)dt.p + 2 * off, x.tup, (size_t)x.n * 16, hipMemcpyHostToDevice, st.comp));
            off += x.n;
        }
        OOC_TRY(hj_dev_build_tuples_i64(c, (const int64_t *)dt.p, n_r, st.comp));
        OOC_TRY(probe_stream(c, s, chunk, out_r, out_s, out_cap, &m, st));
        OOC_HIP(hipStreamSynchronize(st.comp));
    }
    return m;
}
