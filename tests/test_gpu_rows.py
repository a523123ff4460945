"""GPU parity of the nested-loop.mlir row output.

nested-loop.mlir (:29-192) joins two row-major i32 tables on column 0 and
materialises rows [X row, Y cols 1..] with X the larger table.  The product
runs it as a hash join plus a row gather (hj_dev_join_rows_i32, the host
memref form hj_join_rows_i32 and _mlir_ciface_hj_join_rows_i32); the oracle
is the restated nested loop (oracle_nested_join_rows_i32).  Row order is
unspecified on both sides, so rows are compared sorted.
"""
import os

import numpy as np
import pytest
import torch

from hashjoin import HashJoin
from hashjoin import memref as M

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def hj():
    h = HashJoin(0)
    yield h
    h.close()


def sort_rows(a):
    a = np.asarray(a)
    if a.shape[0] == 0:
        return a
    return a[np.lexsort(a.T[::-1])]


def same_rows(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(sort_rows(a), sort_rows(b))


def table(seed, rows, cols, key_hi):
    rng = np.random.default_rng(seed)
    t = rng.integers(-(1 << 30), 1 << 30, size=(rows, cols), dtype=np.int64).astype(np.int32)
    t[:, 0] = rng.integers(0, key_hi, size=rows)
    return t


def test_kat_device(hj):
    with np.load(os.path.join(HERE, "golden", "nested_loop_kat.npz"), allow_pickle=False) as z:
        t1, t2, rows = z["t1"], z["t2"], z["rows"]
    out = hj.join_rows(torch.from_numpy(t1).cuda(), torch.from_numpy(t2).cuda()).cpu().numpy()
    assert same_rows(out, rows)


@pytest.mark.parametrize("shape", [(5000, 4, 3000, 3, 300), (3000, 2, 5000, 5, 200), (4000, 3, 4000, 1, 50),
                                   (1, 3, 7000, 2, 5), (20000, 1, 1, 1, 3)])
def test_random_tables_vs_oracle(hj, oracle, shape):
    r1, c1, r2, c2, hi = shape
    t1, t2 = table(r1 + c1, r1, c1, hi), table(r2 + c2 + 1, r2, c2, hi)
    exp = oracle.nested_join_rows_i32(t1, t2)
    out = hj.join_rows(torch.from_numpy(t1).cuda(), torch.from_numpy(t2).cuda()).cpu().numpy()
    assert out.shape[1] == c1 + c2 - 1
    assert same_rows(out, exp)


def test_empty_and_no_match(hj, oracle):
    e = np.empty((0, 3), np.int32)
    t = table(5, 100, 2, 10)
    for a, b in [(e, t), (t, e), (e, e)]:
        out = hj.join_rows(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
        assert out.shape == (0, a.shape[1] + b.shape[1] - 1)
    t2 = table(6, 50, 3, 10) + np.array([[1000, 0, 0]], np.int32)   # disjoint keys
    out = hj.join_rows(torch.from_numpy(t).cuda(), torch.from_numpy(t2).cuda()).cpu().numpy()
    assert out.shape[0] == 0 and oracle.nested_join_rows_i32(t, t2).shape[0] == 0


def test_strided_device_tables(hj, oracle):
    """Row stride > columns (a column slice of a wider table)."""
    w1, w2 = table(11, 3000, 6, 100), table(12, 2000, 5, 100)
    t1, t2 = w1[:, :3], w2[:, :2]
    exp = oracle.nested_join_rows_i32(np.ascontiguousarray(t1), np.ascontiguousarray(t2))
    d1, d2 = torch.from_numpy(w1).cuda()[:, :3], torch.from_numpy(w2).cuda()[:, :2]
    assert d1.stride(0) == 6
    out = hj.join_rows(d1, d2).cpu().numpy()
    assert same_rows(out, exp)


def test_host_memref_and_ciface(oracle):
    t1, t2 = table(21, 4000, 3, 400), table(22, 2500, 2, 400)
    exp = oracle.nested_join_rows_i32(t1, t2)
    assert M.count_rows_i32(t1, t2) == exp.shape[0]
    # a result memref larger than M (the reference allocates |X| * |Y| rows): only the first M written
    big = np.full((exp.shape[0] + 100, 4), -7, np.int32)
    m = M.join_rows_i32(t1, t2, big)
    assert m == exp.shape[0] and same_rows(big[:m], exp) and (big[m:] == -7).all()
    # strided views in and out
    wide = np.zeros((t1.shape[0], 5), np.int32); wide[:, ::2] = t1
    out_t = np.zeros((4, exp.shape[0]), np.int32)   # result viewed transposed (non-unit row stride)
    m = M.join_rows_i32(wide[:, ::2], t2, out_t.T)
    assert m == exp.shape[0] and same_rows(out_t.T, exp)
    assert same_rows(M.ciface_join_rows_i32(t1, t2), exp)
    # too small a result memref
    assert M.join_rows_i32(t1, t2, np.zeros((max(exp.shape[0] - 1, 0), 4), np.int32)) < 0
