/*
 * hj_driver.c -- what lowered join_hj.mlir does, written in C: a non-Python
 * host drives libhj.so through the expanded memref ABI exactly as
 * mlir-cpu-runner would (join_v1.ll:1262-1265), with the reference's own
 * shared.so supplying inputs and the verdict (shared.cpp:59-172).
 *
 *   hj_driver <nR> <nS> <upperRange> <path/to/shared.so>
 *
 * Prints one JSON line: {"m": M, "probe_rc": 0, "check": 1, "ciface_rows": M,
 * "ciface_check": 1}.  upperRange overrides shared.cpp's key range global
 * (shared.cpp:14), as the reference's 100k-range runs edited it by hand.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "hj.h"

typedef void (*init_fn)(int32_t *, int32_t *, int64_t, int64_t, int64_t);
typedef int32_t (*check_fn)(int32_t *, int32_t *, int64_t, int64_t, int64_t, int32_t *, int32_t *, int64_t, int64_t,
                            int64_t, int32_t *, int32_t *, int64_t, int64_t, int64_t, int32_t *, int32_t *, int64_t,
                            int64_t, int64_t);

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s nR nS upperRange shared.so\n", argv[0]);
        return 2;
    }
    const int64_t nR = atoll(argv[1]), nS = atoll(argv[2]);
    void *ref = dlopen(argv[4], RTLD_NOW);
    if (!ref) {
        fprintf(stderr, "dlopen %s: %s\n", argv[4], dlerror());
        return 2;
    }
    init_fn initR = (init_fn)dlsym(ref, "initRelationR"), initS = (init_fn)dlsym(ref, "initRelationS");
    check_fn check = (check_fn)dlsym(ref, "check");
    int32_t *upper = (int32_t *)dlsym(ref, "upperRange");
    if (!initR || !initS || !check || !upper) return 2;
    *upper = atoi(argv[3]);

    int32_t *R = malloc(sizeof(int32_t) * (nR ? nR : 1)), *S = malloc(sizeof(int32_t) * (nS ? nS : 1));
    initR(R, R, 0, nR, 1);   /* join_v2.mlir:627-630 */
    initS(S, S, 0, nS, 1);

    /* @countRows -> alloc -> @probeRelation (join_v2.mlir:672-696) */
    const int64_t m = hj_count_i32(R, R, 0, nR, 1, S, S, 0, nS, 1);
    if (m < 0) {
        fprintf(stderr, "hj_count_i32: %s\n", hj_last_error());
        return 1;
    }
    int32_t *oR = malloc(sizeof(int32_t) * (m ? m : 1)), *oS = malloc(sizeof(int32_t) * (m ? m : 1));
    const int32_t rc = hj_probe_i32(R, R, 0, nR, 1, S, S, 0, nS, 1, oR, oR, 0, m, 1, oS, oS, 0, m, 1);
    const int32_t ok = check(R, R, 0, nR, 1, S, S, 0, nS, 1, oR, oR, 0, m, 1, oS, oS, 0, m, 1);

    /* two-memref-in / one-memref-out C interface */
    hj_memref1_i32 dr = {R, R, 0, {nR}, {1}}, ds = {S, S, 0, {nS}, {1}};
    hj_memref2_i32 res;
    _mlir_ciface_hj_join_i32(&res, &dr, &ds);
    const int64_t rows = res.sizes[0];
    int32_t *cR = malloc(sizeof(int32_t) * (rows ? rows : 1)), *cS = malloc(sizeof(int32_t) * (rows ? rows : 1));
    for (int64_t i = 0; i < rows; ++i) {
        cR[i] = res.aligned[res.offset + i * res.strides[0]];
        cS[i] = res.aligned[res.offset + i * res.strides[0] + res.strides[1]];
    }
    const int32_t ok2 = check(R, R, 0, nR, 1, S, S, 0, nS, 1, cR, cR, 0, rows, 1, cS, cS, 0, rows, 1);
    hj_free_result(res.allocated);
    printf("{\"m\": %lld, \"probe_rc\": %d, \"check\": %d, \"ciface_rows\": %lld, \"ciface_check\": %d}\n",
           (long long)m, rc, ok, (long long)rows, ok2);
    free(R); free(S); free(oR); free(oS); free(cR); free(cS);
    return (rc == 0 && ok == 1 && ok2 == 1 && rows == m) ? 0 : 1;
}
