"""HIP-graph capture of the device phases (the `hj_dev_*` phases
are graph-capturable once `hj_ctx_reserve*` has sized the workspace).

`build_table` + `probe_relation` are captured into ONE graph on a side
stream, then the graph is replayed over NEW contents of the same input
buffers -- PK-FK, PK-FK with misses, duplicate-heavy keys -- and every replay
is checked against the oracle's exact pair multiset.  The strategy and the
radix plan are fixed by the sizes at capture; every data-dependent choice
(join kernel, deferred items, the grouped join for repeated keys) is taken on
the device, so one graph serves any contents of its shapes."""
import numpy as np
import pytest
import torch

from hashjoin import HashJoin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hj():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    h = HashJoin(0)
    yield h
    h.close()


def _datasets_i64(O, n):
    dup_hi = max(1, n // 4)   # ~4 copies of a key per side: ~16 pairs per key
    return [
        ("pkfk", O.gen_pkfk_i64(91, n, n, 1.0)),
        ("pkfk_misses", O.gen_pkfk_i64(92, n, n, 0.5)),
        ("dups", O.gen_uniform_i64(93, 1, 1, dup_hi, n) + O.gen_uniform_i64(93, 2, 1, dup_hi, n)),
        ("pkfk_again", O.gen_pkfk_i64(94, n, n, 1.0)),
    ]


def _datasets_i32(O, n):
    return [
        ("uniform", (O.gen_uniform_i32(95, 1, 1, 4 * n, n), O.gen_uniform_i32(95, 2, 1, 4 * n, n))),
        ("dups", (O.gen_uniform_i32(96, 1, 1, max(1, n // 4), n), O.gen_uniform_i32(96, 2, 1, max(1, n // 4), n))),
        ("sparse", (O.gen_uniform_i32(97, 1, 1, 1 << 30, n), O.gen_uniform_i32(97, 2, 1, 1 << 30, n))),
    ]


@pytest.mark.parametrize("n,strategy,wide", [
    (1 << 12, "global", True),
    (1 << 16, "radix", True),
    (1 << 20, "auto", True),
    (1 << 12, "global", False),
    (1 << 16, "radix", False),
], ids=["i64-2^12-global", "i64-2^16-radix", "i64-2^20-auto", "i32-2^12-global", "i32-2^16-radix"])
def test_graph_replay_over_new_inputs(hj, oracle, n, strategy, wide):
    O = oracle
    kt = torch.int64 if wide else torch.int32
    rk = torch.empty(n, dtype=kt, device="cuda")
    sk = torch.empty(n, dtype=kt, device="cuda")
    rp = torch.empty(n, dtype=torch.int64, device="cuda") if wide else None
    sp = torch.empty(n, dtype=torch.int64, device="cuda") if wide else None
    sets = _datasets_i64(O, n) if wide else _datasets_i32(O, n)

    def load(data):
        if wide:
            a, b, c, d = data
            for t, x in ((rk, a), (rp, b), (sk, c), (sp, d)):
                t.copy_(torch.from_numpy(np.ascontiguousarray(x)))
        else:
            a, c = data
            rk.copy_(torch.from_numpy(np.ascontiguousarray(a)))
            sk.copy_(torch.from_numpy(np.ascontiguousarray(c)))
        torch.cuda.synchronize()

    hj.set_strategy(strategy)
    load(sets[0][1])
    bits = 64 if wide else 32
    hj.allocate_hash_table(n, bits)
    hj.build_table(rk, rp)
    hj.reserve_probe(n, bits)
    cap = 8 * n
    out_r = torch.empty(cap, dtype=kt, device="cuda")
    out_s = torch.empty_like(out_r)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):   # one eager step on the capture stream first
        hj.build_table(rk, rp)
        hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        hj.build_table(rk, rp)
        hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    try:
        for name, data in sets:
            load(data)
            out_r.fill_(-1)
            cnt.zero_()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            m = int(cnt.item())
            if wide:
                er, es = O.chained_join_i64(*data, H=n)
            else:
                er, es = O.chained_join_i32(data[0], data[1], H=n)
            assert m == len(er), (name, m, len(er))
            assert m <= cap, (name, m, cap)
            got_r = out_r[:m].cpu().numpy().astype(np.int64)
            got_s = out_s[:m].cpu().numpy().astype(np.int64)
            assert O.same_multiset(got_r, got_s, er, es), name
    finally:
        del g
        torch.cuda.synchronize()
