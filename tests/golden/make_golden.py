"""Generate the golden join fixtures in tests/golden/*.npz.

The reference ships no fixtures and seeds its inputs from the clock
(SURVEY F6), so the vectors are made here, deterministically, and pinned
twice before they are written:

  * expected pairs = the CPU restatement of join_v2's build/count/probe
    (oracle/hj_oracle.c), which must equal the restated nested-loop join;
  * for every case whose keys fit in i32, the reference's OWN check()
    (shared_stuff/shared.cpp:129-172, compiled by oracle/Makefile into
    oracle/_ref/shared.so) must return 1 on those pairs, 0 on a corrupted
    copy and -1 on a truncated copy.

Run:  python tests/golden/make_golden.py   (needs oracle/_ref/shared.so)
Each .npz holds plain int arrays only (loaded with allow_pickle=False).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import pyoracle as O  # noqa: E402

SEED = 0x5EED
I32_MIN, I32_MAX = -(1 << 31), (1 << 31) - 1
I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


def pin_i32(r, s, er, es):
    assert O.ref_available(), "oracle/_ref/shared.so missing: run make -C oracle"
    assert O.ref_check(r, s, er, es) == 1, "reference check() rejected the expected pairs"
    if len(er) > 0:
        bad_r = er.copy(); bad_r[0] = (bad_r[0] + 1) % max(1, len(r))
        if not O.same_multiset(bad_r, es, er, es):
            assert O.ref_check(r, s, bad_r, es) == 0
        assert O.ref_check(r, s, er[:-1], es[:-1]) == -1


def case_i32(name, r, s, H):
    r = np.asarray(r, np.int32); s = np.asarray(s, np.int32)
    v2 = O.chained_join_i32(r, s, H=H, variant=2)
    v1 = O.chained_join_i32(r, s, H=H, variant=1)
    nl = O.nested_loop_i32(r, s)
    assert O.same_multiset(*v2, *v1) and O.same_multiset(*v2, *nl), name
    pin_i32(r, s, *v2)
    exp = O.sorted_pairs(*v2)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), kind=np.array([32]), r=r, s=s,
                        expected=exp.astype(np.int64), H=np.array([H]))
    print(f"{name}: |R|={len(r)} |S|={len(s)} M={len(exp)} (H={H}, pinned by reference check())")


def case_i64(name, rk, rp, sk, sp, H):
    rk, rp, sk, sp = (np.asarray(a, np.int64) for a in (rk, rp, sk, sp))
    v2 = O.chained_join_i64(rk, rp, sk, sp, H=H, variant=2)
    v1 = O.chained_join_i64(rk, rp, sk, sp, H=H, variant=1)
    nl = O.nested_loop_i64(rk, rp, sk, sp)
    assert O.same_multiset(*v2, *v1) and O.same_multiset(*v2, *nl), name
    pinned = "nested-loop"
    fits = all(a.size == 0 or (a.min() >= I32_MIN and a.max() <= I32_MAX) for a in (rk, sk))
    rows = np.array_equal(rp, np.arange(len(rp))) and np.array_equal(sp, np.arange(len(sp)))
    if fits and rows:
        pin_i32(rk.astype(np.int32), sk.astype(np.int32), v2[0].astype(np.int32), v2[1].astype(np.int32))
        pinned = "reference check()"
    exp = O.sorted_pairs(*v2)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), kind=np.array([64]), rk=rk, rp=rp, sk=sk, sp=sp,
                        expected=exp, H=np.array([H]))
    print(f"{name}: |R|={len(rk)} |S|={len(sk)} M={len(exp)} (H={H}, pinned by {pinned})")


def main():
    # C0 plumbing: 1024 x 1024 i32 keys uniform in [1, 256].
    r = O.gen_uniform_i32(SEED, 1, 1, 256, 1024)
    s = O.gen_uniform_i32(SEED, 2, 1, 256, 1024)
    case_i32("c0_uniform_i32", r, s, H=10)              # chains of ~100 nodes, as join-performances.md:3
    # duplicate-heavy: 4 distinct keys
    case_i32("dup_heavy_i32", O.gen_uniform_i32(SEED, 3, 1, 4, 512), O.gen_uniform_i32(SEED, 4, 1, 4, 512), H=3)
    # empty result: disjoint key ranges
    case_i32("empty_result_i32", O.gen_uniform_i32(SEED, 5, 1, 100, 300),
             O.gen_uniform_i32(SEED, 6, 101, 200, 400), H=7)
    # all match: one key everywhere (|R| x |S| pairs)
    case_i32("all_match_i32", np.full(64, 7, np.int32), np.full(48, 7, np.int32), H=5)
    # ragged sizes + extreme i32 values (urem of negative keys, join_v2.mlir:231)
    ext = np.array([I32_MIN, -1, 0, 1, I32_MAX, -7, 1 << 30], np.int32)
    rr = np.concatenate([ext, O.gen_uniform_i32(SEED, 7, -50, 50, 993)])
    ss = np.concatenate([O.gen_uniform_i32(SEED, 8, -50, 50, 770), ext[::-1]])
    case_i32("ragged_extremes_i32", rr, ss, H=97)
    # sparse matches, the regime of the reference's [1, 1e9] range
    # (shared.cpp:13-14) scaled to fixture size: E[M] = 8192^2 / 2^20 = 64
    case_i32("sparse_i32", O.gen_uniform_i32(SEED, 9, 1, 1 << 20, 8192),
             O.gen_uniform_i32(SEED, 10, 1, 1 << 20, 8192), H=82)
    # int64 twin of C0 (payload = row id)
    k1, _ = O.gen_uniform_i64(SEED, 11, 1, 256, 1024)
    k2, _ = O.gen_uniform_i64(SEED, 12, 1, 256, 1024)
    case_i64("c0_uniform_i64", k1, np.arange(1024), k2, np.arange(1024), H=10)
    # int64 PK-FK with misses, arbitrary payloads
    rk, rp, sk, sp = O.gen_pkfk_i64(SEED, 2000, 3000, frac=0.75)
    case_i64("pkfk_i64", rk, rp * 3 + 11, sk, sp * -5, H=1 << 12)
    # int64 extremes incl. INT64_MIN (the table's EMPTY sentinel) and dups
    ext = np.array([I64_MIN, I64_MIN, -1, 0, I64_MAX, 1 << 40, -(1 << 40), I64_MIN + 1], np.int64)
    kr, _ = O.gen_uniform_i64(SEED, 13, -20, 20, 500)
    ks, _ = O.gen_uniform_i64(SEED, 14, -20, 20, 333)
    rk = np.concatenate([ext, kr]); sk = np.concatenate([ks, ext, ext[:3]])
    case_i64("extremes_i64", rk, np.arange(len(rk)) + 1000, sk, np.arange(len(sk)) - 77, H=31)

    # nested-loop.mlir @main known answer (nested-loop.mlir:195-289): tables
    # t[i][j] = i + j, 20x3 and 20x2; the join writes rows
    # x[g][0..3) ++ y[j][1..2) for matching keys (x = table 1 on ties).
    t1 = O.nested_init_i32(20, 3); t2 = O.nested_init_i32(20, 2)
    rows = O.nested_join_rows_i32(t1, t2)
    kat = np.array([[i, i + 1, i + 2, i + 1] for i in range(20)], np.int32)
    assert np.array_equal(rows, kat)
    np.savez_compressed(os.path.join(HERE, "nested_loop_kat.npz"), t1=t1, t2=t2, rows=rows)
    print("nested_loop_kat: 20 rows (hand-derived from nested-loop.mlir semantics)")
    # Experiments/selection.mlir @main (:159-193): 128 elements arr[i] = i,
    # predicate arr[i] < 80.0 -> 80 values 0..79 (hand-derived)
    a = O.selection_init_f32(128)
    vals, rows = O.select(a, "lt", 80.0)
    assert np.array_equal(vals, np.arange(80, dtype=np.float32)) and np.array_equal(rows, np.arange(80))
    np.savez_compressed(os.path.join(HERE, "selection_kat.npz"), input=a, value=np.float32(80.0), values=vals,
                        rows=rows)
    print("selection_kat: 80 of 128 (hand-derived from selection.mlir semantics)")


if __name__ == "__main__":
    main()
