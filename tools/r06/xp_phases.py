"""EXPERIMENT: where a k_join_b item's time goes, per wave.  Needs a
libhj.so built with -DHJ_XP_PHASES (HJ_LIB=...); runs build + probe of a
bench config and prints the per-(workgroup, wave) phase cycles of the LAST
k_join_b launch (each wave's own s_memtime clock), averaged over waves.
    HJ_LIB=build/xpn/libhj.so python tools/r06/xp_phases.py C3
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "mlir-hashjoin_amd"))
import bench  # noqa: E402
import hashjoin  # noqa: E402

NAMES = ["table clear (+ barrier)", "build (R rows wait + LDS inserts)", "build barrier",
         "probe (S rows wait + bucket reads + ballots)", "claim (wave: LDS cursor + chunk; scan: barrier, scan, atomic, barrier)",
         "output stores issued", "(sub-chunk loop rest)", "end barrier (table reuse)",
         "loop top: R + S row loads issued", "loop top: s_next read + item claim issued", "loop top: next item's scalar loads"]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    NR, NS, distn, ktype, _ = bench.CONFIGS[cfg]

    class A:
        seed = 42
    rk, rp, sk, sp = bench.gen_inputs(hashjoin, A, NR, NS, distn, 0, NR, 0, NS)
    wide = ktype == "int64"
    hj = hashjoin.HashJoin(0)
    hj.allocate_hash_table(NR, 64 if wide else 32)
    hj.reserve_probe(NS, 64 if wide else 32)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    hj.build_table(rk, rp)
    hj.probe_relation(sk, sp, None, None, count=cnt)
    cap = max(int(cnt.item()), 1)
    odt = torch.int64 if wide else torch.int32
    out_r = torch.empty(cap, dtype=odt, device="cuda")
    out_s = torch.empty_like(out_r)
    for _ in range(3):
        hj.build_table(rk, rp)
        hj.probe_relation(sk, sp, out_r, out_s, count=cnt)
    torch.cuda.synchronize()
    L = C.CDLL(hashjoin._lib.LIB_PATH)
    n = 4096 * 16 * 16
    buf = (C.c_ulonglong * n)()
    assert L.hj_xp_read(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096 * 16, 16).astype(np.float64)
    a = a[a[:, 15] > 0]
    tot = a[:, :11].sum(axis=1)
    items = a[:, 15]
    print(f"{cfg} ({os.environ.get('HJ_LIB', 'product')}): {len(a)} waves, items/wave mean {items.mean():.1f}, "
          f"cycles/wave mean {tot.mean():.0f} (= {tot.mean() / 2.4e3:.1f} us at 2.4 GHz), per item {tot.sum() / items.sum():.0f} cycles")
    for k, nm in enumerate(NAMES):
        print(f"  {k} {nm:72s} {a[:, k].sum() / items.sum():8.0f} cycles/item  {a[:, k].sum() / tot.sum() * 100:5.1f} %")


if __name__ == "__main__":
    main()
