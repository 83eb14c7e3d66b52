"""Per-dispatch mean of every PMC counter for the kernels whose name contains
<substr>, over the rocprofv3 --pmc output directories <prefix>*.
  python tools/pmc_kernel.py <prefix> <substr>"""
import csv
import glob
import os
import sys
from collections import defaultdict

prefix, sub = sys.argv[1], sys.argv[2]
for d in sorted(p for p in glob.glob(prefix + "*") if os.path.isdir(p)):
    disp = defaultdict(lambda: {"c": defaultdict(float)})
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            e = disp[int(r["Dispatch_Id"])]
            e["name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    per = defaultdict(list)
    for e in disp.values():
        per[e["name"]].append(e)
    for n, es in per.items():
        ctr = sorted(es[0]["c"])
        print("%s %s: %d dispatches, %.1f us" % (os.path.basename(d), n, len(es), sum(e["ns"] for e in es) / len(es) / 1e3))
        for c in ctr:
            print("   %-28s %16.0f" % (c, sum(e["c"][c] for e in es) / len(es)))
