"""GPU parity of the selection operator (Experiments/selection.mlir:34-155,
SURVEY 8(f) rank 4) against the restated oracle (oracle_select_*).

Selection is order-preserving on the GPU (per-tile counts, scan, ballot
compaction), so values and source rows compare exactly, in order."""
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


def test_kat(hj):
    with np.load(os.path.join(HERE, "golden", "selection_kat.npz"), allow_pickle=False) as z:
        a, c, vals, rows = z["input"], float(z["value"]), z["values"], z["rows"]
    v, r = hj.select(torch.from_numpy(a).cuda(), "lt", c, with_rows=True)
    assert np.array_equal(v.cpu().numpy(), vals) and np.array_equal(r.cpu().numpy(), rows)
    out = np.full(128, -1.0, np.float32)
    assert M.select_f32(a, c, out) == 80 and np.array_equal(out[:80], vals) and (out[80:] == -1).all()


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 4097, 1 << 20, (1 << 22) + 13])
@pytest.mark.parametrize("op", ["lt", "le", "gt", "ge", "eq", "ne"])
def test_f32_vs_oracle(hj, oracle, n, op):
    rng = np.random.default_rng(n + len(op))
    a = rng.integers(-8, 8, size=n).astype(np.float32) * 0.5
    if n > 40:
        a[::41] = np.nan; a[::43] = np.inf; a[::47] = -np.inf
    ev, er = oracle.select(a, op, 0.5)
    v, r = hj.select(torch.from_numpy(a).cuda(), op, 0.5, with_rows=True)
    assert np.array_equal(r.cpu().numpy(), er)
    assert np.array_equal(v.cpu().numpy(), ev, equal_nan=False)


@pytest.mark.parametrize("op", ["lt", "le", "gt", "ge", "eq", "ne"])
def test_i64_vs_oracle(hj, oracle, op):
    rng = np.random.default_rng(11)
    a = rng.integers(-(1 << 40), 1 << 40, size=300001)
    a[::7] = 12345
    ev, er = oracle.select(a, op, 12345)
    v = hj.select(torch.from_numpy(a).cuda(), op, 12345)
    assert np.array_equal(v.cpu().numpy(), ev)


def test_capacity_and_count(hj, oracle):
    a = np.arange(10000, dtype=np.int64)
    d = torch.from_numpy(a).cuda()
    out = torch.full((100,), -1, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    from hashjoin._lib import check, lib
    check(lib.hj_dev_select_i64(hj._ctx, d.data_ptr(), 10000, 0, 5000, out.data_ptr(), None, 100, cnt.data_ptr(),
                                None), "select")
    torch.cuda.synchronize()
    assert int(cnt.item()) == 5000 and np.array_equal(out.cpu().numpy(), a[:100])
    # host memref: result shorter than M is an error, strided input honoured
    base = np.arange(20000, dtype=np.float32)
    assert M.select_f32(base[::2], 100.0, np.zeros(10, np.float32)) < 0
    out2 = np.zeros(50, np.float32)
    assert M.select_f32(base[::2], 100.0, out2) == 50 and np.array_equal(out2, base[:100:2])
