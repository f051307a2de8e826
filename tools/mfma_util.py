"""Summarise a rocprofv3 `--pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE`
pass (counter_collection.csv) per kernel: dispatches, average duration, flops per dispatch
(MOPS x 512), MFMA pipe utilisation (rocprofv3's MfmaUtil: BUSY / (GRBM_GUI_ACTIVE per XCD
x SIMDs); GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md), the effective
clock (GRBM / 8 / duration) and TFLOP/s against the 2.5 PF dense f16 peak.

usage: python tools/mfma_util.py counter_collection.csv"""
import collections
import csv
import sys

SIMDS, XCDS, PEAK = 1024, 8, 2500.0
per = collections.defaultdict(dict)  # dispatch -> fields
for r in csv.DictReader(open(sys.argv[1])):
    d = per[r["Dispatch_Id"]]
    d["name"] = r["Kernel_Name"]
    d["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.Counter())
for d in per.values():
    if d.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0) <= 0:
        continue
    # one line per kernel and shape (flops per dispatch), so small spot-check passes stay apart
    a = agg[(d["name"].split("(")[0], round(d["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512 / 1e9, 1))]
    a["n"] += 1
    for k in ("dur", "SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
        a[k] += d[k]
print(f"{'kernel':66s} {'n':>4s} {'avg_us':>8s} {'GF/disp':>8s} {'util%':>6s} {'GHz':>5s} {'TF/s':>7s} {'%peak':>6s}")
tot_f = tot_t = 0.0
for (name, _), a in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU_MFMA_MOPS_F16"]):
    n = a["n"]
    flops = a["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512
    cyc = a["GRBM_GUI_ACTIVE"] / XCDS
    util = 100 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS)
    tf = flops / a["dur"] / 1e12
    tot_f += flops
    tot_t += a["dur"]
    print(f"{name[:66]:66s} {n:4d} {a['dur'] / n * 1e6:8.1f} {flops / n / 1e9:8.1f} {util:6.1f} "
          f"{cyc / a['dur'] / 1e9:5.2f} {tf:7.1f} {100 * tf / PEAK:6.1f}")
print(f"all MFMA kernels: {tot_f / tot_t / 1e12:.1f} TFLOP/s over their summed durations "
      f"({100 * tot_f / tot_t / 1e12 / PEAK:.1f}% of {PEAK:.0f})")
