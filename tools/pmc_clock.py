"""Effective clock and MFMA busy fraction per kernel of a rocprofv3 --pmc run
with GRBM_GUI_ACTIVE and SQ_VALU_MFMA_BUSY_CYCLES (MI355X_MICROARCH.md, 'DVFS
give-back': clock ~ GRBM_GUI_ACTIVE / 8 XCDs / wall; SQ_VALU_MFMA_BUSY_CYCLES
counts MFMA cycles summed over the SIMDs, so busy = MFMA / (clock cycles x 1024
SIMDs)).  Profiled runs clock a few % below un-profiled ones.
  python tools/pmc_clock.py <dir> [min_calls]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
min_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 1
disp = defaultdict(lambda: {"c": defaultdict(float)})
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        e = disp[int(r["Dispatch_Id"])]
        e["name"] = r["Kernel_Name"]
        e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
per = defaultdict(list)
for e in disp.values():
    per[e["name"]].append(e)
tot_ns = sum(e["ns"] for e in disp.values())
rows = []
for n, es in per.items():
    if len(es) < min_calls:
        continue
    ns = sum(e["ns"] for e in es)
    grbm = sum(e["c"]["GRBM_GUI_ACTIVE"] for e in es)
    mfma = sum(e["c"]["SQ_VALU_MFMA_BUSY_CYCLES"] for e in es)
    clk = grbm / 8 / ns if ns else 0.0        # GHz
    busy = mfma / (grbm / 8 * 1024) if grbm else 0.0
    rows.append((ns, n, len(es), clk, busy))
rows.sort(reverse=True)
print("%-62s %6s %9s %7s %8s %6s" % ("kernel", "calls", "mean us", "GHz", "MFMA busy", "share"))
for ns, n, k, clk, busy in rows[:25]:
    short = n.replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0][:62]
    print("%-62s %6d %9.1f %7.3f %8.3f %6.3f" % (short, k, ns / k / 1e3, clk, busy, ns / tot_ns))
