"""Summarise gpurun_out/r06a (tools/r06a_chan.sh): per buffer, the
pass-shaped write's time and its memory-side write requests split per L2
channel / per XCD, plus stall and DRAM/GMI counters, against a flat write."""
import collections
import csv
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r06a"


def load(f):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        e = d.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "c": {},
                                                  "t": (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))})
        e["c"][r["Counter_Name"]] = float(r["Counter_Value"])
    return d


def rows(f, keys):
    d = load(f"{D}/{f}/run_counter_collection.csv")
    pw = [v for v in d.values() if "k_passwrite" in v["name"]]
    fw = [v for v in d.values() if "k_flatwrite" in v["name"]]
    for b in list(range(len(pw) // 10)) + ["flat"]:
        v = pw[b * 5 + 2] if b != "flat" else fw[2]   # the median-position repeat of round 1
        yield b, (v["t"][1] - v["t"][0]) / 1e6, [v["c"][k] for k in keys]


print("per L2 channel (TCC instance, summed over XCDs): total write requests, max / mean, min / mean")
for b, t, vals in rows("pmc_inst", ["HJ_WR_I%d" % i for i in range(16)]):
    m = sum(vals) / 16
    print(f"  buf {b!s:>4}  {t:.3f} ms  {sum(vals):.4e}  max/mean {max(vals) / m:.4f}  min/mean {min(vals) / m:.4f}")
print("per XCD: write requests max / mean; TCC_EA0_WRREQ_STALL (all channels)")
for b, t, vals in rows("pmc_xcc", ["HJ_WR_X%d" % i for i in range(8)] + ["HJ_WRST_ALL"]):
    x = vals[:8]
    print(f"  buf {b!s:>4}  {t:.3f} ms  max/mean {max(x) / (sum(x) / 8):.4f}  stall {vals[8]:.4g}")
print("DRAM writes, GMI writes (32 B), DRAM credit stalls, GMI credit stalls")
ks = ["TCC_EA0_WRREQ_WRITE_DRAM_sum", "TCC_EA0_WRREQ_WRITE_GMI_32B_sum", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum",
      "TCC_EA0_WRREQ_GMI_CREDIT_STALL_sum"]
for b, t, vals in rows("pmc_dram", ks):
    print(f"  buf {b!s:>4}  {t:.3f} ms  " + "  ".join(f"{v:.4g}" for v in vals))
